#!/bin/bash
# Round 5 run 3: full GPU suite on HEAD (TSP 1 GET shapes, RS(16+4) bulk TSP + XMAP,
# pooled stream staging), STH A/B on the GET / heal shapes, the bench, the streamed
# GET / heal and end-to-end measurements, and the per-share headline traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r05_suite3.log 2>&1 || { tail -30 gpurun_out/r05_suite3.log; exit 1; }
tail -1 gpurun_out/r05_suite3.log
timeout -k 10 300 python bench.py > gpurun_out/r05_bench3.json 2>&1 || { tail gpurun_out/r05_bench3.json; exit 2; }
tail -1 gpurun_out/r05_bench3.json | cut -c1-300
SHAPE=16:4:2048 VARIANTS=0,423 CASES="1,7;0,5,9,14;h3,17;h0,1,16,19" timeout -k 10 200 python scripts/get_ab.py > gpurun_out/r05_ab_sth.jsonl 2>&1 || exit 3
SHAPE=8:4:4096 VARIANTS=0,423 CASES="0,5,6;1,2,5,7;h1,8;h1,3,8,11" timeout -k 10 200 python scripts/get_ab.py >> gpurun_out/r05_ab_sth.jsonl 2>&1 || exit 4
SHAPE=12:4:4096 VARIANTS=0,423,420 CASES="0,5;0,1,2,3;h0,5;h0,1,2,3" timeout -k 10 200 python scripts/get_ab.py >> gpurun_out/r05_ab_sth.jsonl 2>&1 || exit 5
PATHS=stream_get,e2e E2E_GIB=4 timeout -k 10 500 python -u scripts/bench_paths.py > gpurun_out/r05_stream3.jsonl 2>&1 || { tail -5 gpurun_out/r05_stream3.jsonl; exit 6; }
ROUND=r05 bash scripts/profile_traffic_shares.sh > gpurun_out/r05_traffic.log 2>&1 || { tail -8 gpurun_out/r05_traffic.log; exit 7; }
tail -5 gpurun_out/r05_traffic.log
echo run3 done
