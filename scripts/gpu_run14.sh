#!/bin/bash
# RS(12+4) 4096 / 16384 x 1 MiB encode + sums: 4 stripes of 1 KiB tiles (391, 393-395) vs product
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,391,393,394,395 \
    timeout -k 10 400 python -u scripts/sweep_variants.py > gpurun_out/sweep_rs124_1k_b.jsonl 2>&1 || { tail gpurun_out/sweep_rs124_1k_b.jsonl; exit 1; }
grep -h '"k"' gpurun_out/sweep_rs124_1k_b.jsonl
