#!/bin/bash
# Round 5 A/B set 1: the GPU suite (after the named-shape refactor and the pruned
# diagnostics build), then the conflict-free LDS stride (TSP 1) and the region-interleaved
# workgroup order (XMAP) on every other bulk encode shape and on the GET / heal shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r05_suite2.log 2>&1
tail -3 gpurun_out/r05_suite2.log
grep -q "failed\|error" gpurun_out/r05_suite2.log && grep FAILED gpurun_out/r05_suite2.log | head -20
SWEEP_SHAPES=4:4:4096,4:4:16384 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,400,402 timeout -k 10 200 python scripts/sweep_variants.py > gpurun_out/r05_ab_enc.jsonl 2>&1 || exit 2
SWEEP_SHAPES=16:4:2048,16:4:8192 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,401,415 timeout -k 10 200 python scripts/sweep_variants.py >> gpurun_out/r05_ab_enc.jsonl 2>&1 || exit 3
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,416 timeout -k 10 200 python scripts/sweep_variants.py >> gpurun_out/r05_ab_enc.jsonl 2>&1 || exit 4
SHAPE=8:4:4096 VARIANTS=0,420,421 CASES="0;0,5;0,5,6;1,2,5,7;h1,8;h1,3,8,11" timeout -k 10 200 python scripts/get_ab.py > gpurun_out/r05_ab_get.jsonl 2>&1 || exit 5
SHAPE=16:4:2048 VARIANTS=0,420,421 CASES="0;1,7;1,7,15;0,5,9,14;h3,17;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py >> gpurun_out/r05_ab_get.jsonl 2>&1 || exit 6
SHAPE=12:4:4096 VARIANTS=0,420 CASES="0,5;0,1,2,3;h0,5;h0,1,2,3" timeout -k 10 200 python scripts/get_ab.py >> gpurun_out/r05_ab_get.jsonl 2>&1 || exit 7
echo ab done
