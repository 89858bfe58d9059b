#!/bin/bash
# Round 5 run 11: the headline shape with the LDS-counter hand-off (437) / L2 prefetch
# (438, 439), the RS(12+4) UA shape with prefetch distance 1 / 3 and XMAP 16 (440-442).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_variants.py > gpurun_out/r05_t11.log 2>&1 || { tail -30 gpurun_out/r05_t11.log; exit 1; }
tail -1 gpurun_out/r05_t11.log
O=gpurun_out/r05_ab_enc3.jsonl
SWEEP_SHAPES=8:4:65536,8:4:16384 SWEEP_REPEAT=2 SWEEP_VARIANTS=0,437,438,439 timeout -k 10 300 python scripts/sweep_variants.py > $O 2>&1 || exit 2
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,440,441,442 timeout -k 10 300 python scripts/sweep_variants.py >> $O 2>&1 || exit 3
grep '^{' $O | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['k'], d['objects'], d['variant'], d['ms'])"
echo run11 done
