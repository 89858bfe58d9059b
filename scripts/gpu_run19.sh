#!/bin/bash
# generic-geometry encode parity after the RS(5+4) / RS(6+4) shape change
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_measured.py \
    -k "default_geometries" > gpurun_out/t19.txt 2>&1 || { tail -30 gpurun_out/t19.txt; exit 1; }
tail -3 gpurun_out/t19.txt
