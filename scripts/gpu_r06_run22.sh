#!/bin/bash
# Round 6: RS(12+4) 1 MiB encode + sums, the product (Rs124Ua1K) against 8 stripes of
# 512-byte tiles with the XCD-region order (diagnostics 498) from 2 048 to 32 768 objects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=12:4:2048,12:4:4096,12:4:8192,12:4:16384,12:4:32768 SWEEP_VARIANTS=0,498 SWEEP_REPEAT=3 timeout -k 10 600 \
    python -u scripts/sweep_variants.py > $OUT/ab_rs124_498.jsonl 2>&1 || { tail -20 $OUT/ab_rs124_498.jsonl; exit 1; }
grep '^{' $OUT/ab_rs124_498.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'])"
grep -q '"match": false' $OUT/ab_rs124_498.jsonl && { echo MISMATCH; exit 2; }
echo run22 done
