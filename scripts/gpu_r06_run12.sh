#!/bin/bash
# Round 6: the two-rank partition test at the bulk size, queue / stream GPU tests on the
# split copy streams, and the queue's seal point (ZS3_QUEUE_PIPE_PCT 50 / 33 / 25) with
# split streams at 16 / 64 / 256 submitters (tools/queue_bench_diag).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py \
    tests/test_gpu_queue.py tests/test_gpu_stream_decode.py tests/test_gpu_configs.py > $OUT/run12_tests.log 2>&1 \
    || { tail -30 $OUT/run12_tests.log; exit 1; }
tail -1 $OUT/run12_tests.log
: > $OUT/queue_pipe.jsonl
for rep in 1 2; do
  for pct in 50 33 25; do
    ZS3_QUEUE_PIPE_PCT=$pct timeout -k 10 200 tools/queue_bench_diag 16,64,256 48 8 4 0 0 1 \
        | sed "s/^{/{\"rep\": $rep, \"pipe_pct\": $pct, /" >> $OUT/queue_pipe.jsonl || exit 2
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r06/queue_pipe.jsonl'):
    d=json.loads(l)
    if d['path']=='queue_timers': print('   timers', d['pipe_pct'], d['threads'], 'busy', d['gpu_busy'], 'sum', d['gpu_sum'], 'lock', d['sub_lock'])
    else: print(d['rep'], d['pipe_pct'], d['threads'], d['GiBps'], d['block_latency_us_p50'], d['blocks_per_batch'], d['errors'])
PY
echo run12 done
