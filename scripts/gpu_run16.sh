#!/bin/bash
# RS(8+4) 4096 / 16384 x 1 MiB: 1 KiB-tile memory patterns (360-362) and real roles (363-365)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP_SHAPES=8:4:4096,8:4:16384 SWEEP_REPEAT=2 SWEEP_VARIANTS=0,312,360,361,362,363,364,365 \
    timeout -k 10 400 python -u scripts/sweep_variants.py > gpurun_out/sweep_rs84_1k.jsonl 2>&1 || { tail gpurun_out/sweep_rs84_1k.jsonl; exit 1; }
grep -h '"k"' gpurun_out/sweep_rs84_1k.jsonl
