#!/bin/bash
# Round 5 run 8: GET / heal timing ablations (diagnostics 431 no scalar table loads in the
# loop, 433 no HighwayHash arithmetic) on RS(16+4) rebuild / heal 4 and RS(12+4) rebuild /
# heal 2.  (The first attempt also ran a GF-free ablation, 432: its heal-4 launch faulted
# on the box, so it was removed and is not run again.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r05_abl_get.jsonl
SHAPE=16:4:2048 VARIANTS=0,431,433 CASES="0,5,9,14" timeout -k 10 200 python scripts/get_ab.py > $O 2>&1 || exit 1
SHAPE=16:4:2048 VARIANTS=0,431,433 CASES="h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 1
SHAPE=12:4:4096 VARIANTS=0,431,433 CASES="0,5" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 2
SHAPE=12:4:4096 VARIANTS=0,431,433 CASES="h0,5" timeout -k 10 200 python scripts/get_ab.py >> $O 2>&1 || exit 2
grep '^{' $O | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['k'], d['erased'], d['heal'], d['variant'], d['ms'], d['frac'])"
echo run8 done
