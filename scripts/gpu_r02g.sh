#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verify.py \
    tests/test_gpu_queue.py > $OUT/t6.log 2>&1 || { tail -30 $OUT/t6.log; exit 4; }
tail -2 $OUT/t6.log
echo "get $(date +%T)"
SHAPES=4,8,16 VARIANTS=0,200,216 timeout -k 10 300 python scripts/get_ab2.py > $OUT/get_ab.log 2>&1 || { tail -20 $OUT/get_ab.log; exit 7; }
echo "done $(date +%T)"
