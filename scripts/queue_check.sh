#!/bin/bash
# Queue check: the GPU queue / block-size tests, then three A/B runs of tools/queue_bench
# (1/16/64/256 submitters, pinned mode 1 vs pageable, max_batch 256) -> gpurun_out/queue_ab6.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_queue.py tests/test_gpu_blocksize.py > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -2 gpurun_out/q_tests.log
for rep in 1 2 3; do
  T=1,16,64,256 PER=48 MB="256" MODES="1" scripts/queue_ab.sh >> gpurun_out/queue_ab6.jsonl 2>&1 || exit 2
done
grep -h '{' gpurun_out/queue_ab6.jsonl | cut -c1-200
