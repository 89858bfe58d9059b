#!/bin/bash
# Round 5 run 16: RS(12+4) 1 MiB encode + sums on the pair-form 8 x 512 UA shape without /
# with XMAP (445 / 446) against the 1 KiB quad-form product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_variants.py -k "rs124" > gpurun_out/r05_t16.log 2>&1 || { tail -30 gpurun_out/r05_t16.log; exit 1; }
tail -1 gpurun_out/r05_t16.log
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,445,446 timeout -k 10 300 python scripts/sweep_variants.py > gpurun_out/r05_ab_rs124pair.jsonl 2>&1 || exit 2
grep '^{' gpurun_out/r05_ab_rs124pair.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['k'], d['objects'], d['variant'], d['ms'])"
echo run16 done
