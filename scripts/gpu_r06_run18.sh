#!/bin/bash
# Round 6: the 16-wave RS(8+4) encode + sums workgroup (32 stripes of 128-byte tiles, 12
# pair-form hash waves + 4 encode waves: every SIMD 3 hash + 1 encode; diagnostics
# 490 / 491 = PM 0 / 492 = stamped) against the product at 4 096 / 16 384 / 65 536 objects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=8:4:4096,8:4:16384,8:4:65536 SWEEP_VARIANTS=0,490,491 SWEEP_REPEAT=3 timeout -k 10 600 \
    python -u scripts/sweep_variants.py > $OUT/ab_g32.jsonl 2>&1 || { tail -20 $OUT/ab_g32.jsonl; exit 1; }
grep '^{' $OUT/ab_g32.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'])"
grep -q '"match": false' $OUT/ab_g32.jsonl && { echo MISMATCH; exit 2; }
SHAPE=8:4 NOBJ=65536 VARIANTS=492 G=32 WPW=16 NHW=12 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_g32.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_g32.jsonl; exit 3; }
grep '^{' $OUT/stamps_g32.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['ms'], d['clock_GHz'], [(p['wave'], p['role'], p['bar_frac'], p['load_frac']) for p in d['per_wave']], d.get('by_simd_mix'))"
echo run18 done
