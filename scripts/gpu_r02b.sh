#!/bin/bash
# Ring hand-off experiment: variant parity, queue tests, A/B sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_queue.py "tests/test_gpu_variants.py" -k "queue or 140 or 141 or 130 or 113 or 121 or 105" \
    > $OUT/t2.log 2>&1 || { tail -40 $OUT/t2.log; exit 4; }
tail -3 $OUT/t2.log
echo "sweep $(date +%T)"
SIZES=4096,16384,65536 VARIANTS=0,105,140,141 ROUNDS=4 REPS=6 \
    timeout -k 10 400 python scripts/sweep_sizes.py > $OUT/sweep_ring.log 2>&1 || { tail -20 $OUT/sweep_ring.log; exit 6; }
SIZES=512,1024,2048,4096,8192 VARIANTS=0,5,111,91,113 K=4 M=2 \
    timeout -k 10 400 python scripts/sweep_sizes.py > $OUT/sweep_rs42.log 2>&1 || { tail -20 $OUT/sweep_rs42.log; exit 7; }
SIZES=512,1024,2048,4096,8192 VARIANTS=0,5,120,121 K=16 M=4 \
    timeout -k 10 400 python scripts/sweep_sizes.py > $OUT/sweep_rs164.log 2>&1 || { tail -20 $OUT/sweep_rs164.log; exit 8; }
echo "done $(date +%T)"
