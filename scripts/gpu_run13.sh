#!/bin/bash
# RS(12+4) 4096 x 1 MiB: the memory pattern alone (ABL 7, no GF) of eight shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP_SHAPES=12:4:4096 SWEEP_REPEAT=2 SWEEP_VARIANTS=0,338,380,381,382,383,384,385,386,387 \
    timeout -k 10 400 python -u scripts/sweep_variants.py > gpurun_out/mem_rs124.jsonl 2>&1 || { tail gpurun_out/mem_rs124.jsonl; exit 1; }
grep -h '"k"' gpurun_out/mem_rs124.jsonl
