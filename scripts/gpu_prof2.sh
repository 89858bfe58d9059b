#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "=== isa rates"; timeout -k 10 120 ./scripts/ubench/isa_rate || exit 3
i=0
for pmc in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM" \
           "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "TA_BUSY_avr TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_SMEM SQ_INSTS_BRANCH" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1)); echo "=== pmc $i: $pmc"
  timeout -k 10 300 rocprofv3 --pmc $pmc -d $OUT/pmcb$i -o p --output-format csv -- python scripts/microbench.py > $OUT/pmcb$i.log 2>&1 || { tail -5 $OUT/pmcb$i.log; continue; }
  f=$(find $OUT/pmcb$i -name '*counter_collection.csv' | head -1); [ -n "$f" ] && python scripts/pmc_summary.py "$f" | grep -E "encode|hash"
done
