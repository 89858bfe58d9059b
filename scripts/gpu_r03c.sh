#!/bin/bash
# Round-3 GPU batch: full GPU suite, then the RS(12+4) 16-byte-column encode A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit $?
echo "enc ab $(date +%T)"
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_VARIANTS=0,198,199 SWEEP_REPEAT=2 timeout -k 10 300 python scripts/sweep_variants.py \
    > $OUT/sweep_rs124b.jsonl 2>&1 || exit 7
cat $OUT/sweep_rs124b.jsonl
