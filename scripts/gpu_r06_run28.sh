#!/bin/bash
# Round 6: RS(12+4) 1 MiB encode + sums with the hash waves re-touching each row's next-tile edge line (diagnostics 503)
# against the product: time at 4 096 / 16 384, HBM traffic by request
# size at 4 096.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT; export TMPDIR=/tmp
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_VARIANTS=0,503 SWEEP_REPEAT=3 timeout -k 10 300 python -u scripts/sweep_variants.py \
    > $OUT/ab_rs124_pfe.jsonl 2>&1 || { tail -20 $OUT/ab_rs124_pfe.jsonl; exit 1; }
grep '^{' $OUT/ab_rs124_pfe.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'])"
grep -q '"match": false' $OUT/ab_rs124_pfe.jsonl && { echo MISMATCH; exit 2; }
for v in 503; do
  ROUND=r06 TAG=rs124_v$v CMD="python scripts/sweep_variants.py" SWEEP_SHAPES=12:4:4096 SWEEP_VARIANTS=$v SWEEP_REPEAT=1 SWEEP_STEPS=3 \
      bash scripts/traffic_req.sh > $OUT/tq_$v.log 2>&1 || { tail -5 $OUT/tq_$v.log; exit 3; }
  tail -3 $OUT/tq_$v.log
done
echo run28 done
