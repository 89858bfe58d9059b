#!/bin/bash
# Round 5 closing run: the full GPU suite, smoke(), the bench, the rocprofv3 kernel trace /
# stats of the bench, every path's roofline (scripts/profile_paths.sh: times, kernel stats,
# FETCH / WRITE traffic) and the GET / encode compute counters (scripts/pmc_compute.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; P=$OUT/profile/r05; mkdir -p $P; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/final_tests.log 2>&1 \
    || { tail -30 $OUT/final_tests.log; exit 1; }
tail -1 $OUT/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/final_smoke.log 2>&1 \
    || { tail -20 $OUT/final_smoke.log; exit 2; }
tail -1 $OUT/final_smoke.log
timeout -k 10 300 python bench.py > $OUT/final_bench.json 2>&1 || { tail $OUT/final_bench.json; exit 3; }
tail -1 $OUT/final_bench.json | cut -c1-300
rm -rf $OUT/trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python bench.py --no-cpu > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 4; }
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $P/kernel_stats.csv
grep '"metric"' $OUT/trace.log > $P/bench_under_rocprof.json
ROUND=r05 bash scripts/profile_paths.sh > $OUT/final_paths.log 2>&1 || { tail -20 $OUT/final_paths.log; exit 5; }
ROUND=r05 PATHS=get bash scripts/pmc_compute.sh > $OUT/final_pmc_compute.log 2>&1 || { tail -8 $OUT/final_pmc_compute.log; exit 6; }
echo final done
