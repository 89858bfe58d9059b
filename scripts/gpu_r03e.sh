#!/bin/bash
# Round-3 GPU batch: full GPU suite, smoke, bench, size sweep of the product dispatch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 5; }
echo "smoke ok"
timeout -k 10 300 python bench.py > $OUT/bench_r03e.log 2>&1 || exit 9
grep metric $OUT/bench_r03e.log | cut -c1-300
SWEEP_SHAPES=8:4:64,8:4:129,8:4:700,8:4:1025,8:4:2048,8:4:2049,8:4:4096 SWEEP_VARIANTS=0 SWEEP_REPEAT=1 \
    timeout -k 10 300 python scripts/sweep_variants.py > $OUT/sweep_rs84_product.jsonl 2>&1 || exit 8
grep -v amdgpu.ids $OUT/sweep_rs84_product.jsonl | cut -c1-120
echo "done $(date +%T)"
