#!/bin/bash
# Round 5 run 4: GET / heal per-wave stamps (variant 424), XMAP on the RS(12+4) GET, the
# RS(8+4) ablations with the XMAP order (the new pattern roof), multi-stream split on the
# new product, config 5 end-to-end at 10 GiB, the queue single- vs multi-device, GET/heal
# compute counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verify.py -k "424 or heal_ws_rs164 or large_batch" > gpurun_out/r05_t4.log 2>&1 || { tail -30 gpurun_out/r05_t4.log; exit 1; }
tail -1 gpurun_out/r05_t4.log
( SHAPE=16:4:2048 CASES="h0,1,16,19" WPW=11 NHW=5 timeout -k 10 120 python scripts/stamps_get.py &&
  SHAPE=16:4:2048 CASES="0,5,9,14" WPW=12 NHW=4 timeout -k 10 120 python scripts/stamps_get.py &&
  SHAPE=12:4:4096 CASES="h0,5;0,5" WPW=12 NHW=4 timeout -k 10 120 python scripts/stamps_get.py ) > gpurun_out/r05_stamps_get.jsonl 2>&1 || { tail -5 gpurun_out/r05_stamps_get.jsonl; exit 2; }
SHAPE=12:4:4096 VARIANTS=0,421 CASES="0,5;0,1,2,3;h0,5;h0,1,2,3" timeout -k 10 200 python scripts/get_ab.py > gpurun_out/r05_ab_get12_xmap.jsonl 2>&1 || exit 3
SWEEP_SHAPES=8:4:65536,8:4:16384 SWEEP_REPEAT=2 SWEEP_VARIANTS=0,310,311,312,409 timeout -k 10 300 python scripts/sweep_variants.py > gpurun_out/r05_abl84.jsonl 2>&1 || exit 4
NOBJ=65536 PARTS=1,2,4 REPS=2 timeout -k 10 200 python scripts/ab_streams.py > gpurun_out/r05_ab_streams2.jsonl 2>&1 || exit 5
PATHS=e2e E2E_GIB=10 timeout -k 10 500 python -u scripts/bench_paths.py > gpurun_out/r05_e2e10.jsonl 2>&1 || { tail -5 gpurun_out/r05_e2e10.jsonl; exit 6; }
bash scripts/queue_r05.sh > gpurun_out/r05_queue.jsonl 2>&1 || { tail -5 gpurun_out/r05_queue.jsonl; exit 7; }
ROUND=r05 PATHS=get bash scripts/pmc_compute.sh > gpurun_out/r05_pmc_compute.log 2>&1 || { tail -8 gpurun_out/r05_pmc_compute.log; exit 8; }
echo run4 done
