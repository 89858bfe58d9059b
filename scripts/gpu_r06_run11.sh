#!/bin/bash
# Round 6: split copy streams with 4 / 6 / 8 slots per lane at 64 / 256 synchronous
# submitters, pinned and pageable (tools/queue_bench_diag, host phase timers).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
: > $OUT/queue_split_slots.jsonl
for rep in 1 2; do
  for slots in 4 6 8; do
    for pinned in 1 0; do
      timeout -k 10 200 tools/queue_bench_diag 64,256 48 8 4 0 $slots $pinned \
          | sed "s/^{/{\"rep\": $rep, \"slots\": $slots, /" >> $OUT/queue_split_slots.jsonl || exit 1
    done
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r06/queue_split_slots.jsonl'):
    d=json.loads(l)
    if d['path']=='queue_timers': print('   timers', d['slots'], d['pinned'], d['threads'], 'busy', d['gpu_busy'], 'sum', d['gpu_sum'], 'lock', d['sub_lock'], 'copy', d['sub_copy'], d['copy_out'])
    else: print(d['rep'], d['slots'], d['pinned'], d['threads'], d['GiBps'], d['block_latency_us_p50'], d['blocks_per_batch'], d['errors'])
PY
echo run11 done
