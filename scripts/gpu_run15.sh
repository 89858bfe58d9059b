#!/bin/bash
# RS(12+4) product shape change: parity tests, then bench_paths RS(12+4) encode lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_measured.py tests/test_gpu_parity.py \
    -k "12 or rs124 or server_default" > gpurun_out/t15.txt 2>&1 || { tail -30 gpurun_out/t15.txt; exit 1; }
tail -3 gpurun_out/t15.txt
