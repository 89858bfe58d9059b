#!/bin/bash
# Compute-side counters for the encode and GET / heal kernels:
# one rocprofv3 pass per counter group (SQ <= 8, GRBM <= 2 per pass), each its own run,
# over scripts/bench_paths.py PATHS=${PATHS:-encode,get}; joined per kernel by
# scripts/pmc_compute_join.py with the kernel-trace average duration.
# Output: gpurun_out/profile/$ROUND/pmc_compute*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r03}
OUT=gpurun_out; P=$OUT/profile/$ROUND; mkdir -p $P; export TMPDIR=/tmp
export PATHS=${PATHS:-encode,get}
export REPS=${REPS:-2}
timeout -s KILL 60 rocprofv3 -L > $P/rocprofv3_counters.txt 2>&1 || true
echo "trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ctrace -o run --output-format csv -- \
    python scripts/bench_paths.py > $OUT/ctrace.log 2>&1 || { tail -20 $OUT/ctrace.log; exit 4; }
cp $(find $OUT/ctrace -name '*kernel_stats.csv' | head -1) $P/pmc_compute_kernel_stats.csv
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_COUNT"; do
    i=$((i + 1))
    echo "pmc pass $i $(date +%T)"
    timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/cpmc$i -o p --output-format csv -- \
        python scripts/bench_paths.py > $OUT/cpmc$i.log 2>&1 || { tail -5 $OUT/cpmc$i.log; exit 5; }
    cp $(find $OUT/cpmc$i -name '*counter_collection.csv' | head -1) $P/pmc_compute_pass$i.csv
done
python scripts/pmc_compute_join.py $P/pmc_compute_kernel_stats.csv $P/pmc_compute_pass*.csv > $P/pmc_compute.json
echo "done $(date +%T)"
