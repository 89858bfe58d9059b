#!/bin/bash
# Round 6: start stagger of the headline encode's workgroups (diagnostics 487-489): does
# the lockstep of one launch wave (every workgroup at the same row offset) cost HBM time?
# 4 096 objects = one wave of 256 workgroups (BASELINE config 3), 16 384, 65 536.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=8:4:4096,8:4:16384,8:4:65536 SWEEP_VARIANTS=0,487,488,489 SWEEP_REPEAT=3 timeout -k 10 600 \
    python -u scripts/sweep_variants.py > $OUT/ab_stagger.jsonl 2>&1 || { tail -20 $OUT/ab_stagger.jsonl; exit 1; }
grep '^{' $OUT/ab_stagger.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'])"
echo run17 done
