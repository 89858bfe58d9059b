#!/bin/bash
# Round 6: heal 4 on k_vr_quad in the XCD-region order (product now; 446 = the round-5
# order): GET / heal GPU tests, A/B, and the GET paths of bench_paths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_verify.py \
    tests/test_gpu_measured.py tests/test_gpu_stream_decode.py > $OUT/run24_tests.log 2>&1 || { tail -30 $OUT/run24_tests.log; exit 1; }
tail -1 $OUT/run24_tests.log
: > $OUT/ab_quad_heal.jsonl
for rep in 1 2; do
  for n in 2048 8192; do
    SHAPE=16:4:$n VARIANTS=0,446 CASES="0,5,9,14;h0,1,16,19;h2,7,16,18" timeout -k 10 300 python -u scripts/get_ab.py \
        >> $OUT/ab_quad_heal.jsonl 2>&1 || { tail -20 $OUT/ab_quad_heal.jsonl; exit 2; }
  done
done
PATHS=get timeout -k 10 300 python -u scripts/bench_paths.py > $OUT/paths_get.jsonl 2>&1 || { tail -20 $OUT/paths_get.jsonl; exit 3; }
grep 'RS(16+4)' $OUT/paths_get.jsonl | cut -c1-200
echo run24 done
