#!/bin/bash
# Round 5 run 7: the adopted priorities (GET rebuild role PRIO 1 on pair-form shapes,
# RS(16+4) encode PM 1) under the parity tests, the bench, and HBM traffic by request size
# (scripts/traffic_req.sh) for the headline and the RS(12+4) encode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verify.py tests/test_gpu_variants.py tests/test_gpu_parity.py > gpurun_out/r05_t7.log 2>&1 || { tail -30 gpurun_out/r05_t7.log; exit 1; }
tail -1 gpurun_out/r05_t7.log
timeout -k 10 300 python bench.py > gpurun_out/r05_bench7.json 2>&1 || { tail gpurun_out/r05_bench7.json; exit 2; }
tail -1 gpurun_out/r05_bench7.json | cut -c1-300
TAG=rs84 CMD="python bench.py --objects 65536 --steps 3 --warmup 1 --no-cpu" bash scripts/traffic_req.sh || exit 3
TAG=rs124 SWEEP_SHAPES=12:4:4096 SWEEP_REPEAT=1 SWEEP_VARIANTS=0 CMD="python scripts/sweep_variants.py" bash scripts/traffic_req.sh || exit 4
TAG=rs164 SWEEP_SHAPES=16:4:8192 SWEEP_REPEAT=1 SWEEP_VARIANTS=0 CMD="python scripts/sweep_variants.py" bash scripts/traffic_req.sh || exit 5
O=gpurun_out/r05_ab_prio_get2.jsonl
SHAPE=4:2:8192 VARIANTS=0,429 CASES="1;h1;h0,5" timeout -k 10 200 python scripts/get_ab.py > $O 2>&1 || exit 6
SHAPE=2:2:8192 VARIANTS=0,429 CASES="0;h1,3" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 7
SHAPE=16:4:2048 VARIANTS=0,429 CASES="0,5,9,14;h3,17;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 8
SWEEP_SHAPES=16:4:2048,16:4:8192 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,403 timeout -k 10 200 python scripts/sweep_variants.py > gpurun_out/r05_ab_prio_enc2.jsonl 2>&1 || exit 9
echo run7 done
