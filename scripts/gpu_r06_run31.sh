#!/bin/bash
# Round 6: the headline encode with the dyadic nibble splits of dword pairs done by 64-bit
# shifts (diagnostics 504 = Split64<Rs84Bulk>: v_lshrrev_b64 ~4.5 cycles against 2 x 2.8
# for two 32-bit shifts, profiles/r06/opcost.txt) against the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=8:4:65536,8:4:16384 SWEEP_VARIANTS=0,504 SWEEP_REPEAT=4 timeout -k 10 600 \
    python -u scripts/sweep_variants.py > $OUT/ab_split64.jsonl 2>&1 || { tail -20 $OUT/ab_split64.jsonl; exit 1; }
grep '^{' $OUT/ab_split64.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'])"
grep -q '"match": false' $OUT/ab_split64.jsonl && { echo MISMATCH; exit 2; }
echo run31 done
