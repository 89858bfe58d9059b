#!/bin/bash
# round-4 GPU batch 3: buffer-addressed GET / heal instances (parity, then A/B and the
# path benches), config 2 on a warmed clock.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_measured.py \
    tests/test_gpu_verify.py tests/test_gpu_parity.py -k 'get or heal or verify or masks or reconstruct' > gpurun_out/r3_tests.log 2>&1 \
    || { tail -30 gpurun_out/r3_tests.log; exit 1; }
tail -2 gpurun_out/r3_tests.log
PATHS=encode,get,geom timeout -k 10 400 python -u scripts/bench_paths.py > gpurun_out/bench_paths_r3.jsonl 2>&1 || exit 2
SHAPE=16:4:2048 VARIANTS=0,247 CASES="1,7,15;0,5,9,14;h3,17;h1,7,15;h0,1,16,19" timeout -k 10 300 \
    python -u scripts/get_ab.py > gpurun_out/get_ab_k16_buf.jsonl 2>&1 || exit 3
SHAPE=8:4:4096 VARIANTS=0,247 CASES="0,5,6;1,2,5,7;h1,3,8;h1,3,8,11" timeout -k 10 300 \
    python -u scripts/get_ab.py > gpurun_out/get_ab_k8_buf.jsonl 2>&1 || exit 4
