#!/bin/bash
# Full GPU test suite on one box (one pytest process, per-test timeout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "tests $(date +%T)"
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} \
    > $OUT/tests_full.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/tests_full.log | tail -5
grep -E "FAILED|ERROR" $OUT/tests_full.log | head -30
echo "done $(date +%T) rc=$rc"
exit $rc
