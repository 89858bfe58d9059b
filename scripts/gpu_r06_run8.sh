#!/bin/bash
# Round 6: RS(12+4) 1 MiB encode + sums with aligned data-row loads realigned in registers
# (diagnostics 485 = Rs124Ua1K + ALN 6; 486 stamped): bit-exactness vs the product,
# time, HBM traffic by request size, stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT; export TMPDIR=/tmp
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_VARIANTS=0,485 SWEEP_REPEAT=3 timeout -k 10 300 python -u scripts/sweep_variants.py \
    > $OUT/ab_aln.jsonl 2>&1 || { tail -20 $OUT/ab_aln.jsonl; exit 1; }
grep '^{' $OUT/ab_aln.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'], d['path'])"
grep -q '"match": false' $OUT/ab_aln.jsonl && { echo MISMATCH; exit 2; }
for v in 0 485; do
  ROUND=r06 TAG=rs124_v$v CMD="python scripts/sweep_variants.py" SWEEP_SHAPES=12:4:4096 SWEEP_VARIANTS=$v SWEEP_REPEAT=1 SWEEP_STEPS=3 \
      bash scripts/traffic_req.sh > $OUT/tq_$v.log 2>&1 || { tail -5 $OUT/tq_$v.log; exit 3; }
  tail -3 $OUT/tq_$v.log
done
SHAPE=12:4 NOBJ=4096 VARIANTS=486 G=4 WPW=8 NHW=4 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_aln.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_aln.jsonl; exit 4; }
grep '^{' $OUT/stamps_aln.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['ms'], d['clock_GHz'], [(p['wave'], p['role'], p['bar_frac'], p['load_frac']) for p in d['per_wave']])"
echo run8 done
