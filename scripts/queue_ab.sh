#!/bin/bash
# Queue A/B (round 4): tools/queue_bench (encode, 1 MiB RS(8+4), synchronous submit + wait
# per block) at 1/16/64/256 submitters, for several max_batch values, pageable callers
# vs pinned callers in the zero-copy modes of queue.hip (ZS3_QUEUE_ZC: 1 = first block of
# a batch, the default; 2 = every block by its own DMA; 3 = copy-list kernels).
# Output: one JSON line per run, tagged with the mode and max_batch.
#   MB="256 128 64 32" MODES="1 2" scripts/queue_ab.sh > gpurun_out/queue_ab.jsonl
set -o pipefail
T=${T:-1,16,64,256}
PER=${PER:-32}
for mb in ${MB:-256 128 64 32}; do
  for mode in pageable ${MODES:-1 2}; do
    pinned=1; [ $mode = pageable ] && pinned=0
    if [ $pinned = 1 ]; then export ZS3_QUEUE_ZC=$mode; else unset ZS3_QUEUE_ZC; fi
    timeout -k 10 120 tools/queue_bench $T $PER 8 4 $mb 0 $pinned | \
        sed "s/^{/{\"zc_mode\": \"$mode\", \"max_batch\": $mb, /" || exit 1
  done
done
