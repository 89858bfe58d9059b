#!/bin/bash
# Round 5 run 17: the survivor-quad kernel on 8 stripes (product) vs 4 stripes per
# workgroup, two workgroups per CU (445); parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_verify.py -k "rs164 or large_batch" > gpurun_out/r05_t17.log 2>&1 || { tail -30 gpurun_out/r05_t17.log; exit 1; }
tail -1 gpurun_out/r05_t17.log
O=gpurun_out/r05_ab_quad5.jsonl
SHAPE=16:4:2048 VARIANTS=0,445 CASES="0,5,9,14;h0,1,16,19;h2,7,16,18" timeout -k 10 200 python scripts/get_ab.py > $O 2>&1 || exit 2
SHAPE=16:4:8192 VARIANTS=0,445 CASES="0,5,9,14;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 3
grep '^{' $O | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['round'], d['objects'], d['erased'], d['heal'], d['variant'], d['ms'], d['frac'], d['path'], d['bad'])"
echo run17 done
