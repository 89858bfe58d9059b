#!/bin/bash
# Round 5 run 2: the new stream-decode / multi-device queue / variant tests, the bench on
# HEAD (XMAP product shapes), A/B of the remaining XMAP / TSP candidates, the streamed
# GET / heal and end-to-end measurements, and the LDS-conflict counters of the GET
# instances with and without the conflict-free stride (diagnostics 420).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream_decode.py tests/test_gpu_queue.py tests/test_gpu_variants.py > gpurun_out/r05_t2.log 2>&1 || { tail -30 gpurun_out/r05_t2.log; exit 1; }
tail -1 gpurun_out/r05_t2.log
timeout -k 10 300 python bench.py > gpurun_out/r05_bench_xmap.json 2>&1 || { tail gpurun_out/r05_bench_xmap.json; exit 2; }
tail -1 gpurun_out/r05_bench_xmap.json | cut -c1-400
SWEEP_SHAPES=16:4:2048,16:4:8192 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,401,415,417 timeout -k 10 200 python scripts/sweep_variants.py > gpurun_out/r05_ab_enc2.jsonl 2>&1 || exit 3
SWEEP_SHAPES=4:4:4096,4:4:16384,4:2:4096 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,418 timeout -k 10 200 python scripts/sweep_variants.py >> gpurun_out/r05_ab_enc2.jsonl 2>&1 || exit 4
SWEEP_SHAPES=6:4:4096,10:4:4096,3:2:4096,4:3:4096 SWEEP_REPEAT=3 SWEEP_VARIANTS=0,419 timeout -k 10 300 python scripts/sweep_variants.py >> gpurun_out/r05_ab_enc2.jsonl 2>&1 || exit 5
SWEEP_SHAPES=8:4:65536,8:4:32768,8:4:16384,8:4:8192 SWEEP_REPEAT=2 SWEEP_VARIANTS=0,409,413 timeout -k 10 300 python scripts/sweep_variants.py > gpurun_out/r05_xmap84_shares.jsonl 2>&1 || exit 6
PATHS=stream_get,e2e E2E_GIB=4 timeout -k 10 500 python -u scripts/bench_paths.py > gpurun_out/r05_stream.jsonl 2>&1 || { tail -5 gpurun_out/r05_stream.jsonl; exit 7; }
SHAPE=16:4:2048 VARIANTS=0,420 CASES="0;1,7;0,5,9,14;h3,17;h0,1,16,19" REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc_lds_get -o p --output-format csv -- python scripts/get_ab.py > gpurun_out/r05_pmc_lds_get.log 2>&1 || { tail -5 gpurun_out/r05_pmc_lds_get.log; exit 8; }
echo run2 done
