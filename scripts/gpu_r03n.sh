#!/bin/bash
# End-of-session check: full GPU suite, smoke, bench, then every path's kernel stats + PMC
# traffic + compute counters on the final defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 5; }
echo "smoke ok"
timeout -k 10 300 python bench.py > $OUT/bench_final.log 2>&1 || exit 9
grep metric $OUT/bench_final.log | cut -c1-200
rm -rf $OUT/profile/r03s
ROUND=r03s bash scripts/profile_paths.sh || exit 6
ROUND=r03s bash scripts/pmc_compute.sh || exit 7
echo "all done $(date +%T)"
