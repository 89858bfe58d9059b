#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_variants.py \
    -k "153 or 154 or 114 or 115 or 116" > $OUT/t3.log 2>&1 || { tail -30 $OUT/t3.log; exit 4; }
tail -2 $OUT/t3.log
echo "sweep $(date +%T)"
SIZES=4096,16384,65536 VARIANTS=105,151,153 ROUNDS=4 REPS=6 \
    timeout -k 10 300 python scripts/sweep_sizes.py > $OUT/sweep_nt84.log 2>&1 || { tail -20 $OUT/sweep_nt84.log; exit 6; }
SIZES=1024,4096,8192 VARIANTS=111,116,113,114,115 ROUNDS=3 REPS=6 K=4 M=2 \
    timeout -k 10 300 python scripts/sweep_sizes.py > $OUT/sweep_nt42.log 2>&1 || { tail -20 $OUT/sweep_nt42.log; exit 7; }
echo "profile $(date +%T)"
bash scripts/profile_paths.sh || exit 8
echo "done $(date +%T)"
