#!/bin/bash
# queue seal threshold sweep (ZS3_QUEUE_PIPE_PCT), pinned mode 1 and pageable, max_batch 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for pct in 35 50 67 80; do
  for rep in 1 2; do
    ZS3_QUEUE_PIPE_PCT=$pct T=16,64,256 PER=48 MB="256" MODES="1" scripts/queue_ab.sh | sed "s/^{/{\"pipe_pct\": $pct, /" >> gpurun_out/queue_ab5.jsonl || exit 1
  done
done
