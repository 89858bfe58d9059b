#!/bin/bash
# Round 6: the queue's seal point below a third now that the live count includes parked
# submitters (ZS3_QUEUE_PIPE_LIVE=1): 33 / 25 / 20 % with 4 / 6 slots, 16 / 64 / 256
# synchronous submitters, pinned (tools/queue_bench_diag).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
: > $OUT/queue_pipe2.jsonl
for rep in 1 2; do
  for cfg in "33 4" "25 4" "25 6" "20 6"; do
    set -- $cfg
    ZS3_QUEUE_PIPE_LIVE=1 ZS3_QUEUE_PIPE_PCT=$1 timeout -k 10 200 tools/queue_bench_diag 16,64,256 48 8 4 0 $2 1 \
        | sed "s/^{/{\"rep\": $rep, \"pipe_pct\": $1, \"slots\": $2, /" >> $OUT/queue_pipe2.jsonl || exit 1
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r06/queue_pipe2.jsonl'):
    d=json.loads(l)
    if d['path']=='queue_timers': continue
    print(d['rep'], d['pipe_pct'], d['slots'], d['threads'], d['GiBps'], d['block_latency_us_p50'], d['block_latency_us_p99'], d['blocks_per_batch'], d['errors'])
PY
echo run30 done
