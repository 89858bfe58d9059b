#!/bin/bash
# Round 6: 64-bit nibble splits on the other dyadic M = 4 shapes: RS(12+4) 1 KiB UA (506),
# RS(8+4) mid (507, <= 2048 stripes), RS(4+4) bulk (508).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=12:4:4096,12:4:16384,8:4:2048,4:4:4096,4:4:16384 SWEEP_VARIANTS=0,506,507,508 SWEEP_REPEAT=3 timeout -k 10 600 \
    python -u scripts/sweep_variants.py > $OUT/ab_split64b.jsonl 2>&1 || { tail -20 $OUT/ab_split64b.jsonl; exit 1; }
grep '^{' $OUT/ab_split64b.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['k'], d['m'], d['objects'], d['variant'], d['ms'], d['match'], d.get('path'))"
grep -q '"match": false' $OUT/ab_split64b.jsonl && { echo MISMATCH; exit 2; }
echo run32 done
