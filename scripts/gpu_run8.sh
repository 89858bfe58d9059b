#!/bin/bash
# general-matrix encode + sums shape candidates (diagnostics 340-344) on 4096 x 1 MiB
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SWEEP_SHAPES=3:3:4096,3:2:4096,5:4:4096,6:4:4096,10:4:4096 SWEEP_VARIANTS=0,340,341,342,343,344 SWEEP_REPEAT=2 \
    timeout -k 10 500 python -u scripts/sweep_variants.py > gpurun_out/sweep_gen.jsonl 2>&1 || { tail gpurun_out/sweep_gen.jsonl; exit 1; }
