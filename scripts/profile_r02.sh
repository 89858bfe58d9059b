#!/bin/bash
# Round-2 final evidence: every kernel family of bench_paths.py (trace + PMC), the
# bench line under rocprofv3 (trace/stats, FETCH/WRITE per per-GPU share of N=1/2/4/8,
# VALU), the plain bench, and the queue / end-to-end sections.  Copies into
# gpurun_out/profile/r02/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; P=$OUT/profile/r02; mkdir -p $P; export TMPDIR=/tmp
ROUND=r02 bash scripts/profile_paths.sh || exit $?
echo "bench trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python bench.py --no-cpu > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 11; }
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $P/bench_kernel_stats.csv
grep '"metric"' $OUT/trace.log > $P/bench_under_rocprof.json
rm -f $P/pmc_traffic.json
for n in 65536 32768 16384 8192; do
  echo "bench pmc $n $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf$n -o p --output-format csv -- \
      python bench.py --total-objects $n --steps 3 --warmup 1 --no-cpu > $OUT/pmcf$n.log 2>&1 || { tail -5 $OUT/pmcf$n.log; exit 12; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw$n -o p --output-format csv -- \
      python bench.py --total-objects $n --steps 3 --warmup 1 --no-cpu > $OUT/pmcw$n.log 2>&1 || { tail -5 $OUT/pmcw$n.log; exit 13; }
  python scripts/pmc_traffic.py $(find $OUT/pmcf$n -name '*counter_collection.csv' | head -1) \
      $(find $OUT/pmcw$n -name '*counter_collection.csv' | head -1) $P/pmc_traffic.json $n > /dev/null || exit 14
done
echo "bench pmc valu $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    -d $OUT/pmcv -o p --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmcv.log 2>&1 || { tail -5 $OUT/pmcv.log; exit 15; }
python scripts/pmc_summary.py $(find $OUT/pmcv -name '*counter_collection.csv' | head -1) > $P/pmc_valu.txt
cp $P/pmc_traffic.json profiles/r02/pmc_traffic.json 2>/dev/null
echo "bench $(date +%T)"
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { cat $OUT/bench.log; exit 16; }
grep '"metric"' $OUT/bench.log | tee $P/bench.json
echo "native queue $(date +%T)"
timeout -k 10 200 tools/queue_bench 1,4,16,64,256 32 > $P/queue_native.jsonl || exit 18
echo "size sweeps $(date +%T)"
SIZES=1,64,256,512,640,641,1000,2047,2048,2304,2305,3001,4096,8192,16384 VARIANTS=0 ROUNDS=2 REPS=7 \
    timeout -k 10 300 python -u scripts/sweep_sizes.py > $P/sweep_sizes_final_rs84.jsonl || exit 19
K=16 M=4 SIZES=1,64,256,384,385,1024,2047,2048,4096,8192 VARIANTS=0 ROUNDS=2 REPS=7 \
    timeout -k 10 300 python -u scripts/sweep_sizes.py > $P/sweep_sizes_final_rs164.jsonl || exit 20
K=4 M=2 SIZES=1,64,256,1024,2048,2049,4096,8192 VARIANTS=0 ROUNDS=2 REPS=7 \
    timeout -k 10 300 python -u scripts/sweep_sizes.py > $P/sweep_sizes_final_rs42.jsonl || exit 21
echo "GET small batches $(date +%T)"
for n in 1 64 512; do
  NOBJ=$n VARIANTS=0,231 SHAPES=4,8,16 timeout -k 10 200 python -u scripts/get_ab2.py >> $P/get_small_batches.jsonl || exit 22
done
echo "queue + e2e $(date +%T)"
PATHS=queue,e2e timeout -k 10 600 python scripts/bench_paths.py > $P/bench_paths_host.jsonl 2>$OUT/bph.err || { tail $OUT/bph.err; exit 17; }
echo "done $(date +%T)"
