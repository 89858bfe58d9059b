#!/bin/bash
# Round 6: RS(16+4) rebuild 4 / heal 4 on k_vr_quad with the XCD-region workgroup order
# (diagnostics 446) and rebuild-quad priority 2 (447) against the product, 2 048 / 8 192.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
: > $OUT/ab_quad_x8.jsonl
for rep in 1 2; do
  for n in 2048 8192; do
    SHAPE=16:4:$n VARIANTS=0,446,447 CASES="0,5,9,14;h0,1,16,19;h2,7,16,18" timeout -k 10 300 python -u scripts/get_ab.py \
        >> $OUT/ab_quad_x8.jsonl 2>&1 || { tail -20 $OUT/ab_quad_x8.jsonl; exit 1; }
  done
done
cat $OUT/ab_quad_x8.jsonl | cut -c1-160
echo run23 done
