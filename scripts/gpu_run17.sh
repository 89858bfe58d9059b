#!/bin/bash
# RS(12+4) 4096 x 1 MiB GET / heal: L2 prefetch by the hash waves (265 / 266 / 268) vs product
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
SHAPE=12:4:4096 VARIANTS=0,265,266,268 CASES="0,1,2;0,5;1,12;h0,5;h1,12;h0,1,2,3" timeout -k 10 300 python -u scripts/get_ab.py \
    >> gpurun_out/get_ab_k12_pfd.jsonl 2>&1 || { tail gpurun_out/get_ab_k12_pfd.jsonl; exit 1; }
done
grep -h '{' gpurun_out/get_ab_k12_pfd.jsonl
