#!/bin/bash
# Round 6: (1) the queue seal-point A/B of gpu_r06_run13.sh; (2) DMA timelines
# (rocprofv3 memory-copy + kernel trace) of the streamed GET / heal (zs3_stream_decode)
# and the encode stream (zs3_stream_encode), to see whether H2D and D2H overlap.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_r06_run13.sh || exit 1
rm -rf $OUT/dma_sg $OUT/dma_e2e
PATHS=stream_get SG_GIB=0.25 timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace -d $OUT/dma_sg -o run \
    --output-format csv -- python scripts/bench_paths.py > $OUT/dma_sg.log 2>&1 || { tail -20 $OUT/dma_sg.log; exit 2; }
grep '"path"' $OUT/dma_sg.log | cut -c1-220
PATHS=e2e E2E_GIB=1 timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace -d $OUT/dma_e2e -o run \
    --output-format csv -- python scripts/bench_paths.py > $OUT/dma_e2e.log 2>&1 || { tail -20 $OUT/dma_e2e.log; exit 3; }
grep '"path"' $OUT/dma_e2e.log | cut -c1-220
find $OUT/dma_sg $OUT/dma_e2e -name '*.csv' | head
echo run14 done
