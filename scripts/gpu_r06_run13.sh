#!/bin/bash
# Round 6: the queue's seal point counted over every live block of the device
# (ZS3_QUEUE_PIPE_LIVE=1, submitters parked on backpressure included) against the open +
# launched blocks only (0), at seal 50 / 33 % and 4 / 6 slots, split copy streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
: > $OUT/queue_pipe_live.jsonl
for rep in 1 2; do
  for cfg in "0 50 4" "1 50 4" "1 33 4" "1 33 6"; do
    set -- $cfg
    ZS3_QUEUE_PIPE_LIVE=$1 ZS3_QUEUE_PIPE_PCT=$2 timeout -k 10 200 tools/queue_bench_diag 16,64,256 48 8 4 0 $3 1 \
        | sed "s/^{/{\"rep\": $rep, \"pipe_live\": $1, \"pipe_pct\": $2, \"slots\": $3, /" >> $OUT/queue_pipe_live.jsonl || exit 2
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r06/queue_pipe_live.jsonl'):
    d=json.loads(l)
    if d['path']=='queue_timers': continue
    print(d['rep'], d['pipe_live'], d['pipe_pct'], d['slots'], d['threads'], d['GiBps'], d['block_latency_us_p50'], d['blocks_per_batch'], d['errors'])
PY
echo run13 done
