#!/bin/bash
# Round 5 run 9: survivor splits before the first table wait (diagnostics 434) vs the
# product on the scalar-table GET / heal shapes; parity of 434 first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verify.py -k "434" > gpurun_out/r05_t9.log 2>&1 || { tail -30 gpurun_out/r05_t9.log; exit 1; }
tail -1 gpurun_out/r05_t9.log
O=gpurun_out/r05_ab_spl.jsonl
SHAPE=16:4:2048 VARIANTS=0,434 CASES="1,7;1,7,15;0,5,9,14;h3,17;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py > $O 2>&1 || exit 2
SHAPE=12:4:4096 VARIANTS=0,434 CASES="0,5;h0,5;0,1,2,3" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 3
SHAPE=8:4:4096 VARIANTS=0,434 CASES="0,5,6;1,2,5,7;h1,8;h1,3,8,11" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 4
grep '^{' $O | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['round'], d['k'], d['erased'], d['heal'], d['variant'], d['ms'], d['frac'])"
echo run9 done
