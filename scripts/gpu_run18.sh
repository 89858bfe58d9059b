#!/bin/bash
# RS(5+4) / RS(6+4) 4096 x 1 MiB encode + sums: 4 stripes of 1 KiB tiles (345 / 346) vs product
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP_SHAPES=${SHAPES:-5:4:4096,6:4:4096} SWEEP_REPEAT=3 SWEEP_VARIANTS=0,345,346 \
    timeout -k 10 400 python -u scripts/sweep_variants.py > gpurun_out/${OUTF:-sweep_gen_1k.jsonl} 2>&1 || { tail gpurun_out/${OUTF:-sweep_gen_1k.jsonl}; exit 1; }
grep -h '"k"' gpurun_out/${OUTF:-sweep_gen_1k.jsonl}
