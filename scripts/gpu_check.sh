#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprofv3 kernel trace.
# Stops at the first GPU fault / abort / timeout (exit >= 2 from pytest, or any
# nonzero from the others); a pytest exit of 1 (test failures) still lets the
# bench run so the numbers are seen.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "=== $1 ($(date +%T))"; }

step pytest
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -30 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ge 2 ]; then exit $rc; fi

step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
cat $OUT/smoke.log

step bench
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 || { cat $OUT/bench.log; exit 4; }
cat $OUT/bench.log

if [ "${PROF:-1}" = "1" ]; then
  step rocprof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 5; }
  tail -3 $OUT/prof.log
  find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \; | head -20
fi
echo "=== done"
