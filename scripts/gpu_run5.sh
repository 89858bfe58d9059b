#!/bin/bash
# round-4 GPU batch 5: queue with the pipelining cap (tests, then A/B at the shim's batch size)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_queue.py \
    tests/test_gpu_blocksize.py > gpurun_out/r5_tests.log 2>&1 || { tail -30 gpurun_out/r5_tests.log; exit 1; }
tail -2 gpurun_out/r5_tests.log
for rep in 1 2; do
  T=1,16,64,256 PER=48 MB="256 128" MODES="1" scripts/queue_ab.sh >> gpurun_out/queue_ab4.jsonl 2>&1 || exit 2
done
