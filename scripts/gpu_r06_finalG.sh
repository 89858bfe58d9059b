#!/bin/bash
# Round 6 closing run G on the final HEAD: the full GPU suite, smoke(), the bench, and the
# --gpus 2 same-device rehearsal of the N > 1 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; P=$OUT/profile/r06g; mkdir -p $P; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/final_tests.log 2>&1 \
    || { tail -30 $OUT/final_tests.log; exit 1; }
tail -1 $OUT/final_tests.log | tee $P/gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/final_smoke.log 2>&1 \
    || { tail -20 $OUT/final_smoke.log; exit 2; }
tail -1 $OUT/final_smoke.log | tee $P/smoke.txt
timeout -k 10 300 python bench.py > $OUT/final_bench.json 2>&1 || { tail $OUT/final_bench.json; exit 3; }
grep '"metric"' $OUT/final_bench.json > $P/bench.json
cut -c1-300 $P/bench.json
ZS3_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu > $OUT/bench_gpus2.json 2>&1 \
    || { tail -20 $OUT/bench_gpus2.json; exit 4; }
grep '"metric"' $OUT/bench_gpus2.json > $P/bench_gpus2_same_device.json
cut -c1-200 $P/bench_gpus2_same_device.json
echo finalG done
