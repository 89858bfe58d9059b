#!/bin/bash
# Round 6: the streamed GET / heal D2H of only the rebuilt rows (k_rows_copy) for rows
# that are not 256-byte aligned: GPU tests, stream_get bench, DMA timeline; the product
# queue at 64 / 256 submitters twice more (seal point 33 %, live count).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream_decode.py \
    > $OUT/run16_tests.log 2>&1 || { tail -30 $OUT/run16_tests.log; exit 1; }
tail -1 $OUT/run16_tests.log
PATHS=stream_get SG_GIB=1 timeout -k 10 300 python -u scripts/bench_paths.py > $OUT/stream_get3.jsonl 2>&1 \
    || { tail -20 $OUT/stream_get3.jsonl; exit 2; }
grep '"stream_decode"' $OUT/stream_get3.jsonl | cut -c1-200
rm -rf $OUT/dma_sg3
PATHS=stream_get SG_GIB=0.25 timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace -d $OUT/dma_sg3 -o run \
    --output-format csv -- python scripts/bench_paths.py > $OUT/dma_sg3.log 2>&1 || { tail -20 $OUT/dma_sg3.log; exit 3; }
: > $OUT/queue_product2.jsonl
for rep in 1 2; do
  for pinned in 1 0; do
    timeout -k 10 200 tools/queue_bench 64,256 48 8 4 0 0 $pinned | sed "s/^{/{\"rep\": $rep, /" >> $OUT/queue_product2.jsonl || exit 4
  done
done
cut -c1-230 $OUT/queue_product2.jsonl
echo run16 done
