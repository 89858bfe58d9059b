#!/bin/bash
# Round profile: bench line + rocprofv3 kernel trace/stats + FETCH/WRITE PMC passes.
# Copies the summaries into $P/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r01}
OUT=gpurun_out; P=$OUT/profile/$ROUND; mkdir -p $OUT $P; export TMPDIR=/tmp
echo "=== trace $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python bench.py --no-cpu > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 5; }
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $P/kernel_stats.csv
grep '"metric"' $OUT/trace.log > $P/bench_under_rocprof.json
cat $P/kernel_stats.csv
echo "=== pmc FETCH_SIZE"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf -o p --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmcf.log 2>&1 || { tail -5 $OUT/pmcf.log; exit 6; }
echo "=== pmc WRITE_SIZE"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw -o p --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmcw.log 2>&1 || { tail -5 $OUT/pmcw.log; exit 7; }
python scripts/pmc_traffic.py $(find $OUT/pmcf -name '*counter_collection.csv' | head -1) \
    $(find $OUT/pmcw -name '*counter_collection.csv' | head -1) $P/pmc_traffic.json 65536
echo "=== pmc VALU"
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS \
    -d $OUT/pmcv -o p --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmcv.log 2>&1 || { tail -5 $OUT/pmcv.log; exit 8; }
python scripts/pmc_summary.py $(find $OUT/pmcv -name '*counter_collection.csv' | head -1) | tee $P/pmc_valu.txt
echo "=== pmc LDS"
timeout -k 10 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES \
    -d $OUT/pmcl -o p --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmcl.log 2>&1 || { tail -5 $OUT/pmcl.log; exit 9; }
python scripts/pmc_summary.py $(find $OUT/pmcl -name '*counter_collection.csv' | head -1) | tee $P/pmc_lds.txt
echo "=== bench $(date +%T)"
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { cat $OUT/bench.log; exit 4; }
grep '"metric"' $OUT/bench.log | tee $P/bench.json
