#!/bin/bash
# Unaligned encode-only parity + RS(12+4) GET shape A/B + encode paths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_measured.py \
  -k "unaligned or any_geometry or rs124 or server_default" > $OUT/tenc.log 2>&1 || { tail -30 $OUT/tenc.log; exit 2; }
tail -2 $OUT/tenc.log
bash scripts/gpu_r03l.sh || exit 3
PATHS=encode timeout -k 10 300 python scripts/bench_paths.py > $OUT/bp_enc.jsonl 2>$OUT/bp.err || { tail $OUT/bp.err; exit 4; }
grep -v amdgpu $OUT/bp_enc.jsonl | cut -c1-150
