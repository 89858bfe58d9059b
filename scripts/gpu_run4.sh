#!/bin/bash
# round-4 GPU batch 4: RS(12+4) UA encode stride variants; queue max_batch repeats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_VARIANTS=0,330,331 SWEEP_REPEAT=3 timeout -k 10 300 \
    python -u scripts/sweep_variants.py > gpurun_out/sweep_rs124_tsp.jsonl 2>&1 || { tail gpurun_out/sweep_rs124_tsp.jsonl; exit 1; }
for rep in 1 2; do
  T=16,64,256 PER=48 MB="128 64 32" MODES="1" scripts/queue_ab.sh >> gpurun_out/queue_ab3.jsonl 2>&1 || exit 2
done
