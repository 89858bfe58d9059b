#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "=== microbench $(date +%T)"
timeout -k 10 300 python scripts/microbench.py 2>&1 | grep -v amdgpu.ids || exit 3
echo "=== counters list"
rocprofv3 -L > $OUT/counters.txt 2>&1; grep -o '^[A-Za-z_0-9]*' $OUT/counters.txt | sort -u | tr '\n' ' ' | head -c 6000; echo
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"; do
  i=$((i+1))
  echo "=== pmc $i: $pmc"
  timeout -k 10 300 rocprofv3 --pmc $pmc -d $OUT/pmc$i -o p --output-format csv -- python scripts/microbench.py > $OUT/pmc$i.log 2>&1 || { tail -5 $OUT/pmc$i.log; continue; }
  f=$(find $OUT/pmc$i -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && python scripts/pmc_summary.py "$f"
done
echo "=== done"
