#!/bin/bash
# Round 6: the headline encode with its nibble-split masks in SGPRs instead of 32-bit
# literals (diagnostics 509 = Smk<Rs84Bulk>: 4-byte instead of 8-byte VALU encodings)
# against the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=8:4:65536,8:4:16384 SWEEP_VARIANTS=0,509 SWEEP_REPEAT=4 timeout -k 10 600 \
    python -u scripts/sweep_variants.py > $OUT/ab_smk.jsonl 2>&1 || { tail -20 $OUT/ab_smk.jsonl; exit 1; }
grep '^{' $OUT/ab_smk.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['objects'], d['variant'], d['ms'], d['match'])"
grep -q '"match": false' $OUT/ab_smk.jsonl && { echo MISMATCH; exit 2; }
echo run33 done
