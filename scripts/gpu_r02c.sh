#!/bin/bash
# Memory-policy variants A/B (interleaved, one process), then the full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "sweep $(date +%T)"
SIZES=16384,65536 VARIANTS=105,150,151,152,0 ROUNDS=4 REPS=6 \
    timeout -k 10 300 python scripts/sweep_sizes.py > $OUT/sweep_mem.log 2>&1 || { tail -20 $OUT/sweep_mem.log; exit 6; }
echo "tests $(date +%T)"
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    > $OUT/tests_full.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/tests_full.log | tail -3
grep -E "FAILED|ERROR" $OUT/tests_full.log | head -30
echo "done $(date +%T) rc=$rc"
exit $rc
