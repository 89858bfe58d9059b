#!/bin/bash
# Round 6: streamed GET / heal tests (quad kernel through pattern groups, pinned per-row
# path, failed blocks), the queue tests, and the --gpus 2 same-device bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_stream_decode.py tests/test_gpu_queue.py tests/test_gpu_configs.py > $OUT/run5_tests.log 2>&1 \
    || { tail -40 $OUT/run5_tests.log; exit 1; }
tail -3 $OUT/run5_tests.log
ZS3_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu > $OUT/bench_gpus2_same_device.json 2>&1 \
    || { tail -20 $OUT/bench_gpus2_same_device.json; exit 2; }
tail -1 $OUT/bench_gpus2_same_device.json
echo run5 done
