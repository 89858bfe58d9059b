#!/bin/bash
# Round-2 first GPU pass: smoke, the new parity tests, the bench, the batch-size sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 3; }
echo "tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_configs.py tests/test_gpu_bitrot.py "tests/test_gpu_verify.py::test_verify_reconstruct_ws_rs164" \
    "tests/test_gpu_verify.py::test_heal_ws_rs164" "tests/test_gpu_verify.py::test_reconstruct_batch_masks" \
    "tests/test_gpu_verify.py::test_verify_reconstruct_batch_masks" > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 4; }
tail -3 $OUT/t1.log
echo "bench $(date +%T)"
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 5; }
grep metric $OUT/bench.log
echo "sweep $(date +%T)"
SIZES=256,512,1000,1024,2047,2048,3001,4096,8192,16384 VARIANTS=0,105,130,131,132,5 \
    timeout -k 10 400 python scripts/sweep_sizes.py > $OUT/sweep.log 2>&1 || { tail -20 $OUT/sweep.log; exit 6; }
echo "done $(date +%T)"
