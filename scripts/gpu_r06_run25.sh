#!/bin/bash
# Round 6: per-wave stamps of the RS(16+4) bulk encode + sums (diagnostics 499 =
# Stamp<Rs164Bulk>: 5 pair-form hash waves + 6 encode waves) at 2 048 / 8 192 objects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SHAPE=16:4 NOBJ=2048,8192 VARIANTS=499 G=8 WPW=11 NHW=5 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_rs164.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_rs164.jsonl; exit 1; }
grep '^{' $OUT/stamps_rs164.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['ms'], d['clock_GHz'], [(p['wave'], p['role'], p['bar_frac'], p['load_frac']) for p in d['per_wave']], d.get('by_simd_mix'))"
echo run25 done
