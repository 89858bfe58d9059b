#!/bin/bash
# RS(16+4) encode + sums: the RS(12+4) round-4 recipe (366-368) vs product, 2048 / 8192 x 1 MiB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP_SHAPES=16:4:2048,16:4:8192 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,366,367,368,158 \
    timeout -k 10 400 python -u scripts/sweep_variants.py > gpurun_out/sweep_rs164_1k.jsonl 2>&1 || { tail gpurun_out/sweep_rs164_1k.jsonl; exit 1; }
grep -h '"k"' gpurun_out/sweep_rs164_1k.jsonl
