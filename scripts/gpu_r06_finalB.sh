#!/bin/bash
# Round 6 closing run, part B: the headline kernel's PMC traffic for every per-GPU share,
# every path's roofline + traffic (bench_paths), and the GET / encode compute counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; P=$OUT/profile/r06; mkdir -p $P; export TMPDIR=/tmp
ROUND=r06 bash scripts/profile_traffic_shares.sh > $OUT/final_traffic.log 2>&1 || { tail -20 $OUT/final_traffic.log; exit 1; }
tail -4 $OUT/final_traffic.log
ROUND=r06 bash scripts/profile_paths.sh > $OUT/final_paths.log 2>&1 || { tail -20 $OUT/final_paths.log; exit 2; }
tail -2 $OUT/final_paths.log
ROUND=r06 PATHS=get bash scripts/pmc_compute.sh > $OUT/final_pmc_compute.log 2>&1 || { tail -8 $OUT/final_pmc_compute.log; exit 3; }
echo finalB done
