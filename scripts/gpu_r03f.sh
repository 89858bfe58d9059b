#!/bin/bash
# Round-3 evidence refresh: RS(12+4) alignment A/B, then every path's kernel stats + PMC
# traffic (profile_paths.sh) and the compute counters of the encode / GET kernels
# (pmc_compute.sh) on the current defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT/profile/r03; export TMPDIR=/tmp
for a in 0 1; do
  for bl in 1048576 1048704; do
    SWEEP_SHAPES=12:4:4096 SWEEP_VARIANTS=0 SWEEP_REPEAT=1 SWEEP_BLEN=$bl SWEEP_ALIAS=$a \
      timeout -k 10 120 python scripts/sweep_variants.py >> $OUT/profile/r03/ab_rs124_align.jsonl 2>>$OUT/sweep.err || exit 3
  done
done
SWEEP_SHAPES=16:4:4096,8:4:4096,4:4:4096 SWEEP_VARIANTS=0 SWEEP_REPEAT=1 \
  timeout -k 10 120 python scripts/sweep_variants.py >> $OUT/profile/r03/ab_rs124_align.jsonl 2>>$OUT/sweep.err || exit 3
grep -v amdgpu.ids $OUT/profile/r03/ab_rs124_align.jsonl | cut -c1-200
ROUND=r03 bash scripts/profile_paths.sh || exit 4
grep -v amdgpu.ids $OUT/profile/r03/bench_paths.jsonl | cut -c1-160
ROUND=r03 bash scripts/pmc_compute.sh || exit 5
echo "all done $(date +%T)"
