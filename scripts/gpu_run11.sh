#!/bin/bash
# RS(12+4) 4096 x 1 MiB encode + sums: product vs role ablations (334 no hash, 336 no GF,
# 338 neither) at the unaligned 1 MiB rows and at aligned rows of 12 x 87 392 bytes
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export SWEEP_SHAPES=12:4:4096 SWEEP_REPEAT=3
SWEEP_VARIANTS=0,334,336,338 timeout -k 10 300 python -u scripts/sweep_variants.py > gpurun_out/abl_rs124_ua.jsonl 2>&1 || { tail gpurun_out/abl_rs124_ua.jsonl; exit 1; }
SWEEP_BLEN=1048704 SWEEP_VARIANTS=0,330,334,336,338 timeout -k 10 300 python -u scripts/sweep_variants.py > gpurun_out/abl_rs124_al.jsonl 2>&1 || { tail gpurun_out/abl_rs124_al.jsonl; exit 1; }
grep -h '"k"' gpurun_out/abl_rs124_ua.jsonl gpurun_out/abl_rs124_al.jsonl
