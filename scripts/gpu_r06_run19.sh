#!/bin/bash
# Round 6: BASELINE config 3's encode (RS(8+4) 4 096 x 1 MiB): the bulk shape (one launch
# wave of 256 workgroups) against the <= 2048-stripe shape Rs84Mid (1 024 workgroups of 4
# stripes; diagnostics 494, 495 = with the XCD-region order), also at 2 048 / 8 192.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=8:4:2048,8:4:4096,8:4:8192 SWEEP_VARIANTS=0,494,495 SWEEP_REPEAT=3 timeout -k 10 600 \
    python -u scripts/sweep_variants.py > $OUT/ab_cfg3.jsonl 2>&1 || { tail -20 $OUT/ab_cfg3.jsonl; exit 1; }
grep '^{' $OUT/ab_cfg3.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'], d.get('path'))"
echo run19 done
