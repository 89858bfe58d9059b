#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verify.py \
    tests/test_gpu_variants.py -k "ws or 155 or masks" > $OUT/t5.log 2>&1 || { tail -30 $OUT/t5.log; exit 4; }
tail -2 $OUT/t5.log
echo "get $(date +%T)"
SHAPES=8,16 VARIANTS=0,200,216 timeout -k 10 300 python scripts/get_ab2.py > $OUT/get_ab.log 2>&1 || { tail -20 $OUT/get_ab.log; exit 7; }
echo "sweep $(date +%T)"
SIZES=4096,65536 VARIANTS=0,151,155,105 ROUNDS=4 REPS=6 \
    timeout -k 10 300 python scripts/sweep_sizes.py > $OUT/sweep_st84.log 2>&1 || { tail -20 $OUT/sweep_st84.log; exit 6; }
echo "bench $(date +%T)"
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 5; }
grep metric $OUT/bench.log | cut -c1-400
echo "done $(date +%T)"
