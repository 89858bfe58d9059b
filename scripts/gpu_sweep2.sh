#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "=== sweep $(date +%T)"
SWEEP_SHAPES=${SWEEP_SHAPES:-8:4:4096,16:4:2048} SWEEP_VARIANTS=${SWEEP_VARIANTS:-5,9,10,11,12,13,14,15,16} \
  timeout -k 10 600 python scripts/sweep_variants.py > $OUT/sweep.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/sweep.log; echo "sweep rc=$rc"
