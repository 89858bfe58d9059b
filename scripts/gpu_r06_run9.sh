#!/bin/bash
# Round 6: queue slots per lane (4 = the shim's default, 6, 8) at 64 / 256 synchronous
# submitters, pinned and pageable, with the host phase timers (tools/queue_bench_diag).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT
: > $OUT/queue_slots.jsonl
for rep in 1 2; do
  for slots in 4 6 8; do
    for pinned in 1 0; do
      timeout -k 10 200 tools/queue_bench_diag 64,256 48 8 4 0 $slots $pinned | sed "s/^{/{\"rep\": $rep, \"slots\": $slots, /" >> $OUT/queue_slots.jsonl || exit 1
    done
  done
done
grep queue_encode $OUT/queue_slots.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['rep'], d['slots'], d['pinned'], d['threads'], d['GiBps'], d['block_latency_us_p50'], d['blocks_per_batch'])"
echo run9 done
