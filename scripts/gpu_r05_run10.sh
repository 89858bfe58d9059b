#!/bin/bash
# Round 5 run 10: SPL adopted on RS(16+4) rebuild 3-4 / heal and RS(8+4) rebuild 3-4
# (parity), RS(12+4) encode cache policies (time + request-size traffic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verify.py tests/test_gpu_variants.py > gpurun_out/r05_t10.log 2>&1 || { tail -30 gpurun_out/r05_t10.log; exit 1; }
tail -1 gpurun_out/r05_t10.log
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,408,435,436 timeout -k 10 300 python scripts/sweep_variants.py > gpurun_out/r05_ab_ntm124.jsonl 2>&1 || exit 2
grep '^{' gpurun_out/r05_ab_ntm124.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['k'], d['objects'], d['variant'], d['ms'])"
TAG=rs124ntm SWEEP_SHAPES=12:4:4096 SWEEP_REPEAT=1 SWEEP_VARIANTS=0,408,435,436 CMD="python scripts/sweep_variants.py" bash scripts/traffic_req.sh || exit 3
SHAPE=16:4:2048 VARIANTS=0,434 CASES="0,5,9,14;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py > gpurun_out/r05_ab_spl2.jsonl 2>&1 || exit 4
grep '^{' gpurun_out/r05_ab_spl2.jsonl | cut -c1-200
echo run10 done
