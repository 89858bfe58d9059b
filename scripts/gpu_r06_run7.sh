#!/bin/bash
# Round 6: per-wave stamps of the RS(12+4) 1 KiB UA encode (diagnostics 484 = Rs124Ua1K
# with WT): which role paces the 16-drive default's encode + sums.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SHAPE=12:4 NOBJ=4096,16384 VARIANTS=484 G=4 WPW=8 NHW=4 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_rs124.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_rs124.jsonl; exit 1; }
grep '^{' $OUT/stamps_rs124.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['ms'], d['clock_GHz'], [(p['wave'], p['role'], p['bar_frac'], p['load_frac']) for p in d['per_wave']], d['by_simd_mix'])"

SWEEP_SHAPES=8:4:65536 SWEEP_VARIANTS=0,474 SWEEP_REPEAT=3 timeout -k 10 300 python -u scripts/sweep_variants.py \
    > $OUT/ab_pm4.jsonl 2>&1 || { tail -20 $OUT/ab_pm4.jsonl; exit 2; }
grep '^{' $OUT/ab_pm4.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'])"
echo run7b done
