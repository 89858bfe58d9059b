#!/bin/bash
# Round 6, first box: the headline bench on round-5 code, per-wave stamps of the headline
# encode (variant 313) at 65 536 / 16 384 objects, and the pattern-roof ablations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench_start.json 2>&1 || { tail -20 $OUT/bench_start.json; exit 1; }
tail -1 $OUT/bench_start.json | cut -c1-400
NOBJ=65536,16384 VARIANTS=313 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_enc.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_enc.jsonl; exit 2; }
SWEEP_SHAPES=8:4:65536 SWEEP_VARIANTS=0,310,311,312 SWEEP_REPEAT=2 timeout -k 10 300 python -u scripts/sweep_variants.py \
    > $OUT/abl84.jsonl 2>&1 || { tail -20 $OUT/abl84.jsonl; exit 3; }
cat $OUT/abl84.jsonl
echo run1 done
