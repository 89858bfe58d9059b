#!/bin/bash
# Round 6: deeper encode-role prefetch on the headline (diagnostics 467-472).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=8:4:65536 SWEEP_VARIANTS=0,467,468,469,470 SWEEP_REPEAT=2 timeout -k 10 300 python -u scripts/sweep_variants.py \
    > $OUT/ab_pf.jsonl 2>&1 || { tail -20 $OUT/ab_pf.jsonl; exit 1; }
cat $OUT/ab_pf.jsonl
NOBJ=65536 VARIANTS=471,472 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_pf.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_pf.jsonl; exit 2; }
echo run4 done
