#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_measured.py \
    -k 'default_geometries' > gpurun_out/r10_tests.log 2>&1 || { tail -30 gpurun_out/r10_tests.log; exit 1; }
tail -2 gpurun_out/r10_tests.log
GEOMS=2:2,3:2,3:3,4:3 PATHS=geom timeout -k 10 400 python -u scripts/bench_paths.py > gpurun_out/geom_r10.jsonl 2>&1 || exit 2
