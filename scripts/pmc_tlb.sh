#!/bin/bash
# Address-translation / latency PMC passes over scripts/pmc_probe.py (encode-only
# stream kernel vs fused encode+hash kernel), one rocprofv3 run per counter group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tlb; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum" \
           "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/p$i -o p --output-format csv -- python scripts/pmc_probe.py > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 5; }
  python scripts/pmc_summary.py $(find $OUT/p$i -name '*counter_collection.csv' | head -1) | grep -v k_fill | tee -a $OUT/summary.txt
done
