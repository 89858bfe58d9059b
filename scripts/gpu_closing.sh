#!/bin/bash
# Round-closing run on one box (ROUND, default r04): GPU suite + smoke + bench, the headline profile
# (trace/stats + PMC passes), every path's profile, the server-default geometries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_final.sh || exit 1
ROUND=${ROUND:-r04} bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -20 gpurun_out/profile_round.log; exit 2; }
tail -3 gpurun_out/profile_round.log
ROUND=${ROUND:-r04} bash scripts/profile_paths.sh > gpurun_out/profile_paths.log 2>&1 || { tail -20 gpurun_out/profile_paths.log; exit 3; }
tail -2 gpurun_out/profile_paths.log
PATHS=geom timeout -k 10 400 python -u scripts/bench_paths.py > gpurun_out/geom_final.jsonl 2>&1 || { tail gpurun_out/geom_final.jsonl; exit 4; }
echo geom done
