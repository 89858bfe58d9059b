#!/bin/bash
# Round 6: the queue with split copy streams (one H2D and one D2H stream per lane, the
# slot's stream for kernels only) against one stream per slot: GPU queue tests, then
# tools/queue_bench_diag with ZS3_QUEUE_SPLIT=1 / 0 and the product tools/queue_bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_queue.py \
    > $OUT/run10_tests.log 2>&1 || { tail -30 $OUT/run10_tests.log; exit 1; }
tail -1 $OUT/run10_tests.log
: > $OUT/queue_split.jsonl
for rep in 1 2; do
  for split in 1 0; do
    for pinned in 1 0; do
      ZS3_QUEUE_SPLIT=$split timeout -k 10 200 tools/queue_bench_diag 16,64,256 48 8 4 0 0 $pinned \
          | sed "s/^{/{\"rep\": $rep, \"split\": $split, /" >> $OUT/queue_split.jsonl || exit 2
    done
  done
done
for pinned in 1 0; do
  timeout -k 10 200 tools/queue_bench 1,16,64,256 48 8 4 0 0 $pinned | sed "s/^{/{\"build\": \"product\", /" >> $OUT/queue_split.jsonl || exit 3
done
python - <<'PY'
import json
for l in open('gpurun_out/r06/queue_split.jsonl'):
    d=json.loads(l)
    if d['path']=='queue_timers': print('   timers', d.get('split'), d['pinned'], d['threads'], 'busy', d['gpu_busy'], 'sum', d['gpu_sum'], 'lock', d['sub_lock'])
    else: print(d.get('rep'), d.get('split', d.get('build')), d['pinned'], d['threads'], d['GiBps'], d['block_latency_us_p50'], d['blocks_per_batch'], d['errors'])
PY
echo run10 done
