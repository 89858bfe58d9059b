#!/bin/bash
# Round-3 GPU batch: GET/heal tests on the new defaults, GET/heal and encode A/Bs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verify.py \
    > $OUT/verify_tests.log 2>&1 || { tail -30 $OUT/verify_tests.log; exit 3; }
tail -2 $OUT/verify_tests.log
echo "get ab $(date +%T)"
SHAPE=16:4:2048 VARIANTS=0,242 CASES="3;0,5;0,5,9;0,5,9,14;h3;h3,17;h0,5,17;h0,1,16,19" REPS=10 \
    timeout -k 10 300 python scripts/get_ab3.py > $OUT/get_ab_r03_16c.jsonl 2>&1 || exit 4
SHAPE=8:4:4096 VARIANTS=0,260,261,262,263 CASES="3;0,5;0,5,9;0,5,9,10;h3;h3,9;h0,5,9;h0,1,8,11" REPS=10 \
    timeout -k 10 300 python scripts/get_ab3.py > $OUT/get_ab_r03_84.jsonl 2>&1 || exit 5
echo "enc ab $(date +%T)"
SWEEP_SHAPES=8:4:65536 SWEEP_VARIANTS=0,191,192,193 SWEEP_REPEAT=2 timeout -k 10 300 python scripts/sweep_variants.py \
    > $OUT/sweep_prio.jsonl 2>&1 || exit 6
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_VARIANTS=0,195,196,197 SWEEP_REPEAT=2 timeout -k 10 300 python scripts/sweep_variants.py \
    > $OUT/sweep_rs124.jsonl 2>&1 || exit 7
VARIANTS=194 NOBJ=16384 timeout -k 10 200 python scripts/stamps3.py > $OUT/stamps194.txt 2>&1 || exit 8
echo "done $(date +%T)"
