#!/bin/bash
# RS(12+4) on 1 MiB blocks (UA rows): every diagnostics shape, now that variants reach it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_VARIANTS=0,175,176,177,178,195,196,197,198,199,165,166 SWEEP_REPEAT=2 \
  timeout -k 10 300 python scripts/sweep_variants.py > $OUT/ab_rs124_ua_variants.jsonl 2>$OUT/sweep.err || { tail $OUT/sweep.err; exit 3; }
grep -v amdgpu.ids $OUT/ab_rs124_ua_variants.jsonl | cut -c1-170
