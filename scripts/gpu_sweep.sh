#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "=== pytest $(date +%T)"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ge 2 ]; then exit $rc; fi
echo "=== sweep $(date +%T)"
timeout -k 10 600 python scripts/sweep_variants.py > $OUT/sweep.log 2>&1; rc=$?
cat $OUT/sweep.log | grep -v amdgpu.ids; echo "sweep rc=$rc"
