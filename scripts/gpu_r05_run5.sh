#!/bin/bash
# Round 5 run 5: GET / heal occupancy and priority shapes (diagnostics 425-428): parity
# first, then the A/B against the product on RS(16+4) and RS(12+4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verify.py -k "rs164 or rs124_large" > gpurun_out/r05_t5.log 2>&1 || { tail -30 gpurun_out/r05_t5.log; exit 1; }
tail -1 gpurun_out/r05_t5.log
SHAPE=16:4:2048 VARIANTS=0,425,426,427,428 CASES="1,7;0,5,9,14;h3,17;h0,1,16,19" timeout -k 10 300 python scripts/get_ab.py > gpurun_out/r05_ab_get_occ16.jsonl 2>&1 || { tail -5 gpurun_out/r05_ab_get_occ16.jsonl; exit 2; }
SHAPE=12:4:4096 VARIANTS=0,425,426,427,428 CASES="0,5;h0,5" timeout -k 10 300 python scripts/get_ab.py > gpurun_out/r05_ab_get_occ12.jsonl 2>&1 || { tail -5 gpurun_out/r05_ab_get_occ12.jsonl; exit 3; }
echo run5 done
