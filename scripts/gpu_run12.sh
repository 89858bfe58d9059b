#!/bin/bash
# aligned-row RS(12+4) dispatch: parity tests, then product vs diagnostics 330 at 12 x 87 392
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_measured.py \
    -k "server_default_geometries or rs124" > gpurun_out/t12.txt 2>&1 || { tail -30 gpurun_out/t12.txt; exit 1; }
tail -3 gpurun_out/t12.txt
SWEEP_SHAPES=12:4:4096,12:4:16384 SWEEP_REPEAT=3 SWEEP_BLEN=1048704 SWEEP_VARIANTS=0,330 \
    timeout -k 10 300 python -u scripts/sweep_variants.py > gpurun_out/rs124_al_ab.jsonl 2>&1 || { tail gpurun_out/rs124_al_ab.jsonl; exit 1; }
grep -h '"k"' gpurun_out/rs124_al_ab.jsonl
