#!/bin/bash
# Round 6: the balanced mixed-role encode (ehx_mx.hpp, diagnostics 450-457) against the
# product on 65 536 x 1 MiB RS(8+4), with stamps of each G (SIMD placement, barrier waits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
SWEEP_SHAPES=8:4:65536 SWEEP_VARIANTS=0,450,451,452,456,457 SWEEP_REPEAT=2 timeout -k 10 300 python -u scripts/sweep_variants.py \
    > $OUT/ab_mix.jsonl 2>&1 || { tail -20 $OUT/ab_mix.jsonl; exit 1; }
cat $OUT/ab_mix.jsonl
NOBJ=65536 VARIANTS=453 G=16 WPW=6 NHW=0 timeout -k 10 300 python -u scripts/stamps_enc.py > $OUT/stamps_mix.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_mix.jsonl; exit 2; }
NOBJ=65536 VARIANTS=454 G=8 WPW=3 NHW=0 timeout -k 10 300 python -u scripts/stamps_enc.py >> $OUT/stamps_mix.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_mix.jsonl; exit 3; }
NOBJ=65536 VARIANTS=455 G=32 WPW=12 NHW=0 timeout -k 10 300 python -u scripts/stamps_enc.py >> $OUT/stamps_mix.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_mix.jsonl; exit 4; }
NOBJ=65536 VARIANTS=313 timeout -k 10 300 python -u scripts/stamps_enc.py >> $OUT/stamps_mix.jsonl 2>&1 \
    || { tail -20 $OUT/stamps_mix.jsonl; exit 5; }
echo run2 done
