#!/bin/bash
# Round 6: the streamed GET / heal with its per-block arrays staged through pinned memory
# (H2D of batch i+1 no longer waits for batch i's D2H), the queue at its new seal point:
# GPU tests, stream_get bench, a DMA timeline of stream_get, and the product queue_bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream_decode.py \
    tests/test_gpu_queue.py tests/test_gpu_configs.py > $OUT/run15_tests.log 2>&1 || { tail -30 $OUT/run15_tests.log; exit 1; }
tail -1 $OUT/run15_tests.log
PATHS=stream_get SG_GIB=1 timeout -k 10 300 python -u scripts/bench_paths.py > $OUT/stream_get2.jsonl 2>&1 \
    || { tail -20 $OUT/stream_get2.jsonl; exit 2; }
grep '"path"' $OUT/stream_get2.jsonl | cut -c1-200
rm -rf $OUT/dma_sg2
PATHS=stream_get SG_GIB=0.25 timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace -d $OUT/dma_sg2 -o run \
    --output-format csv -- python scripts/bench_paths.py > $OUT/dma_sg2.log 2>&1 || { tail -20 $OUT/dma_sg2.log; exit 3; }
: > $OUT/queue_product.jsonl
for pinned in 1 0; do
  timeout -k 10 200 tools/queue_bench 1,16,64,256 48 8 4 0 0 $pinned >> $OUT/queue_product.jsonl || exit 4
done
cat $OUT/queue_product.jsonl | cut -c1-200
echo run15 done
