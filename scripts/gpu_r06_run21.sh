#!/bin/bash
# Round 6: RS(12+4) 1 MiB encode + sums with two encode waves per SIMD (diagnostics 496 =
# Rs124Ua1K with 8-byte columns, 497 stamped) and the aligned-row shape on these rows (498)
# against the product, 4 096 / 16 384 objects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_VARIANTS=0,496,498 SWEEP_REPEAT=3 timeout -k 10 600 \
    python -u scripts/sweep_variants.py > $OUT/ab_rs124_cw8.jsonl 2>&1 || { tail -20 $OUT/ab_rs124_cw8.jsonl; exit 1; }
grep '^{' $OUT/ab_rs124_cw8.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'])"
grep -q '"match": false' $OUT/ab_rs124_cw8.jsonl && { echo MISMATCH; exit 2; }
SHAPE=12:4 NOBJ=4096 VARIANTS=497 G=4 WPW=12 NHW=4 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_rs124_cw8.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_rs124_cw8.jsonl; exit 3; }
grep '^{' $OUT/stamps_rs124_cw8.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['ms'], d['clock_GHz'], [(p['wave'], p['role'], p['bar_frac'], p['load_frac']) for p in d['per_wave']])"
echo run21 done
