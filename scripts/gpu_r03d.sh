#!/bin/bash
# Round-3 GPU batch: full GPU suite, then encode A/Bs (RS(12+4) 16-byte columns,
# RS(8+4) mid batches) and one bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit $?
echo "enc ab $(date +%T)"
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_VARIANTS=0,198,199,165,166 SWEEP_REPEAT=2 \
    timeout -k 10 300 python scripts/sweep_variants.py > $OUT/sweep_rs124b.jsonl 2>&1 || exit 7
SWEEP_SHAPES=8:4:700,8:4:1024 SWEEP_VARIANTS=0,187,197,198,199 SWEEP_REPEAT=2 \
    timeout -k 10 300 python scripts/sweep_variants.py > $OUT/sweep_rs84_mid.jsonl 2>&1 || exit 8
timeout -k 10 300 python bench.py > $OUT/bench_r03d.log 2>&1 || exit 9
grep -v amdgpu.ids $OUT/sweep_rs124b.jsonl $OUT/sweep_rs84_mid.jsonl
grep metric $OUT/bench_r03d.log | cut -c1-400
echo "done $(date +%T)"
