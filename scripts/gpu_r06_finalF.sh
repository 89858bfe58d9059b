#!/bin/bash
# Round 6 closing run F, after adopting the 64-bit nibble splits (S64) in the RS(8+4) bulk,
# RS(12+4) 1 KiB and RS(4+4) bulk encode shapes: the full GPU suite, smoke(), the bench,
# the rocprofv3 kernel trace / stats of the bench, the headline kernel's PMC traffic for
# every per-GPU share, every path's roofline + traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; P=$OUT/profile/r06f; mkdir -p $P; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/final_tests.log 2>&1 \
    || { tail -30 $OUT/final_tests.log; exit 1; }
tail -1 $OUT/final_tests.log | tee $P/gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/final_smoke.log 2>&1 \
    || { tail -20 $OUT/final_smoke.log; exit 2; }
tail -1 $OUT/final_smoke.log | tee $P/smoke.txt
timeout -k 10 300 python bench.py > $OUT/final_bench.json 2>&1 || { tail $OUT/final_bench.json; exit 3; }
grep '"metric"' $OUT/final_bench.json > $P/bench.json
cut -c1-300 $P/bench.json
rm -rf $OUT/trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python bench.py --no-cpu > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 4; }
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $P/kernel_stats.csv
grep '"metric"' $OUT/trace.log > $P/bench_under_rocprof.json
head -3 $P/kernel_stats.csv | cut -c1-250
ROUND=r06f bash scripts/profile_traffic_shares.sh > $OUT/final_traffic.log 2>&1 || { tail -20 $OUT/final_traffic.log; exit 5; }
tail -4 $OUT/final_traffic.log
ROUND=r06f bash scripts/profile_paths.sh > $OUT/final_paths.log 2>&1 || { tail -20 $OUT/final_paths.log; exit 6; }
tail -2 $OUT/final_paths.log
echo finalF done
