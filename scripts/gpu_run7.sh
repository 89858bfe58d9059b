#!/bin/bash
# RS(12+4) UA encode cache policy: time, then FETCH/WRITE traffic of each variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SWEEP_SHAPES=12:4:4096 SWEEP_VARIANTS=0,332,333 SWEEP_REPEAT=3 timeout -k 10 300 \
    python -u scripts/sweep_variants.py > gpurun_out/sweep_rs124_nt.jsonl 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  SWEEP_SHAPES=12:4:4096 SWEEP_VARIANTS=0,332,333 SWEEP_REPEAT=1 SWEEP_STEPS=2 timeout -s KILL 200 rocprofv3 --pmc $c \
      -d gpurun_out/pmc_nt_$c -o p --output-format csv -- python scripts/sweep_variants.py > gpurun_out/pmc_nt_$c.log 2>&1 || exit 2
done
python scripts/pmc_summary.py $(find gpurun_out/pmc_nt_FETCH_SIZE -name '*counter_collection.csv' | head -1) > gpurun_out/pmc_nt.txt
python scripts/pmc_summary.py $(find gpurun_out/pmc_nt_WRITE_SIZE -name '*counter_collection.csv' | head -1) >> gpurun_out/pmc_nt.txt
