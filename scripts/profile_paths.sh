#!/bin/bash
# rocprofv3 evidence for every kernel family bench_paths.py measures: kernel trace +
# stats, and FETCH_SIZE / WRITE_SIZE passes (separate runs, counters only) -> per-kernel
# HBM bytes per launch.  Output under gpurun_out/profile/$ROUND/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r02}
OUT=gpurun_out; P=$OUT/profile/$ROUND; mkdir -p $P; export TMPDIR=/tmp
export PATHS=${PATHS:-encode,rec,get,hash,deep,digest}
echo "plain $(date +%T)"
timeout -k 10 300 python scripts/bench_paths.py > $P/bench_paths.jsonl 2>$OUT/bp.err || { tail $OUT/bp.err; exit 3; }
echo "trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ptrace -o run --output-format csv -- \
    python scripts/bench_paths.py > $OUT/ptrace.log 2>&1 || { tail -20 $OUT/ptrace.log; exit 4; }
cp $(find $OUT/ptrace -name '*kernel_stats.csv' | head -1) $P/paths_kernel_stats.csv
echo "pmc fetch $(date +%T)"
REPS=3 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/ppf -o p --output-format csv -- \
    python scripts/bench_paths.py > $OUT/ppf.log 2>&1 || { tail -5 $OUT/ppf.log; exit 5; }
echo "pmc write $(date +%T)"
REPS=3 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/ppw -o p --output-format csv -- \
    python scripts/bench_paths.py > $OUT/ppw.log 2>&1 || { tail -5 $OUT/ppw.log; exit 6; }
python scripts/pmc_paths.py $(find $OUT/ppf -name '*counter_collection.csv' | head -1) \
    $(find $OUT/ppw -name '*counter_collection.csv' | head -1) $P/paths_kernel_stats.csv $P/paths_pmc_traffic.json
python scripts/paths_traffic_join.py $(find $OUT/ppf -name '*counter_collection.csv' | head -1) \
    $(find $OUT/ppw -name '*counter_collection.csv' | head -1) $P/bench_paths.jsonl $P/bench_paths_roofline.jsonl
echo "done $(date +%T)"
