#!/bin/bash
# generic-geometry encode shapes: parity tests, then the geometry bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_measured.py \
    -k 'default_geometries or config4' > gpurun_out/r9_tests.log 2>&1 || { tail -30 gpurun_out/r9_tests.log; exit 1; }
tail -2 gpurun_out/r9_tests.log
PATHS=geom timeout -k 10 400 python -u scripts/bench_paths.py > gpurun_out/geom_r9.jsonl 2>&1 || exit 2
for g in 2:2 3:2 3:3 5:4 6:4 7:4; do
  SHAPE=${g}:4096 VARIANTS=0,350,351 CASES="0,1;h0,1" timeout -k 10 200 python -u scripts/get_ab.py >> gpurun_out/get_ab_gen.jsonl 2>&1 || exit 3
done
