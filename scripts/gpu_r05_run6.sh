#!/bin/bash
# Round 5 run 6: issue priority.  GET / heal: the rebuild role at s_setprio 1 (now the
# product) vs 429 (the round-4 instances, no priority) on every GET geometry; encode: PM
# variants 403-407 on the bulk shapes.  Parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verify.py tests/test_gpu_variants.py > gpurun_out/r05_t6.log 2>&1 || { tail -30 gpurun_out/r05_t6.log; exit 1; }
tail -1 gpurun_out/r05_t6.log
O=gpurun_out/r05_ab_prio_get.jsonl
SHAPE=8:4:4096 VARIANTS=0,429 CASES="0;0,5;0,5,6;1,2,5,7;h1,8;h1,3,8,11" timeout -k 10 200 python scripts/get_ab.py > $O 2>&1 || exit 2
SHAPE=16:4:2048 VARIANTS=0,429 CASES="0;1,7;1,7,15;0,5,9,14;h3,17;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 3
SHAPE=16:4:2048 VARIANTS=0,430 CASES="h0,1,16,19;h0,5,17" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 3
SHAPE=12:4:4096 VARIANTS=0,429 CASES="0,5;0,1,2,3;h0,5;h0,1,2,3" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 4
SHAPE=4:2:8192 VARIANTS=0,429 CASES="0;1;0,5;h1;h0,5" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 5
SHAPE=6:4:4096 VARIANTS=0,429 CASES="0,5;h0,5;h0,1,6,9" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 6
SHAPE=2:2:8192 VARIANTS=0,429 CASES="0;h1,3" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 7
O=gpurun_out/r05_ab_prio_enc.jsonl
SWEEP_SHAPES=16:4:2048,16:4:8192 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,403,407 timeout -k 10 200 python scripts/sweep_variants.py > $O 2>&1 || exit 8
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,404,408 timeout -k 10 200 python scripts/sweep_variants.py >> $O 2>&1 || exit 9
SWEEP_SHAPES=8:4:65536,8:4:16384 SWEEP_REPEAT=2 SWEEP_VARIANTS=0,405,406 timeout -k 10 300 python scripts/sweep_variants.py >> $O 2>&1 || exit 10
ROUND=r05 VARIANTS=0,408 bash scripts/traffic_rs124.sh > gpurun_out/r05_traffic124.log 2>&1 || { tail -5 gpurun_out/r05_traffic124.log; exit 11; }
cat gpurun_out/r05_traffic124.log
echo run6 done
