#!/bin/bash
# What bounds the fused RS(8+4) launch: per-kernel SQ stall/issue counters and the
# effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time), against HBM and with the
# bytes L2-resident (ALIAS=1), for the variants in VARS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_ws; mkdir -p $OUT; export TMPDIR=/tmp
VARS=${VARS:-105 140}
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for v in $VARS; do
  for al in 0 1; do
    tag=v${v}_a${al}
    echo "pmc $tag $(date +%T)"
    SIZES=${N:-16384} VARIANTS=$v ROUNDS=1 REPS=4 ALIAS=$al timeout -s KILL 120 rocprofv3 --pmc $SQ -d $OUT/$tag -o p \
        --output-format csv -- python scripts/sweep_sizes.py > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 3; }
    f=$(find $OUT/$tag -name '*counter_collection.csv' | head -1)
    python scripts/pmc_summary.py $f | grep -i "ehx\|encode" | tee $OUT/$tag.txt
    grep '"ms"' $OUT/$tag.log | tail -1
  done
done
echo "done $(date +%T)"
