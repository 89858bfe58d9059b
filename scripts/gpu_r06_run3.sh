#!/bin/bash
# Round 6: issue priority by SIMD role mix on the headline (diagnostics 460-466).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=8:4:65536 SWEEP_VARIANTS=0,460,461,462,463,464 SWEEP_REPEAT=2 timeout -k 10 300 python -u scripts/sweep_variants.py \
    > $OUT/ab_prio.jsonl 2>&1 || { tail -20 $OUT/ab_prio.jsonl; exit 1; }
cat $OUT/ab_prio.jsonl
NOBJ=65536 VARIANTS=465,466 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_prio.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_prio.jsonl; exit 2; }
echo run3 done
