#!/bin/bash
# round-4 GPU batch 2: queue modes (tests + A/B), GET instances (RS(4+m) product, RS(16+4)
# candidates), then the round profile of the headline (rocprof trace/stats + PMC passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_queue.py \
    tests/test_gpu_measured.py -k 'queue or default_geometries_ws_get_heal or get_heal_profiled' > gpurun_out/r2_tests.log 2>&1 \
    || { tail -30 gpurun_out/r2_tests.log; exit 1; }
tail -2 gpurun_out/r2_tests.log
MB="256 64 32" MODES="1 2" scripts/queue_ab.sh > gpurun_out/queue_ab2.jsonl 2>&1 || { tail gpurun_out/queue_ab2.jsonl; exit 2; }
SHAPE=16:4:2048 VARIANTS=0,273,274,275 CASES="1,7,15;0,5,9,14;h3,17;h1,7,15;h0,1,16,19" timeout -k 10 300 \
    python -u scripts/get_ab.py > gpurun_out/get_ab_k16.jsonl 2>&1 || exit 3
PATHS=get timeout -k 10 300 python -u scripts/bench_paths.py > gpurun_out/bench_paths_get.jsonl 2>&1 || exit 4
ROUND=r04 timeout -k 10 900 bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -20 gpurun_out/profile_round.log; exit 5; }
tail -3 gpurun_out/profile_round.log
