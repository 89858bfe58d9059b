#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_variants.py \
    tests/test_gpu_verify.py -k "122 or 123 or 124 or 216 or 217" > $OUT/t4.log 2>&1 || { tail -30 $OUT/t4.log; exit 4; }
tail -2 $OUT/t4.log
echo "sweep $(date +%T)"
SIZES=512,1024,2048,4096,8192 VARIANTS=120,122,123,121,124 ROUNDS=3 REPS=6 K=16 M=4 \
    timeit=1 timeout -k 10 300 python scripts/sweep_sizes.py > $OUT/sweep_nt164.log 2>&1 || { tail -20 $OUT/sweep_nt164.log; exit 6; }
echo "get $(date +%T)"
SHAPES=16,8 VARIANTS=0,200,216,217 timeout -k 10 300 python scripts/get_ab2.py > $OUT/get_ab.log 2>&1 || { tail -20 $OUT/get_ab.log; exit 7; }
echo "done $(date +%T)"
