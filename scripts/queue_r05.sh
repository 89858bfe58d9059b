#!/bin/bash
# Round 5 queue check (tools/queue_bench, 1 MiB RS(8+4), synchronous submit + wait per
# block): one device vs the same device listed twice (the multi-device queue's two parts
# on one GPU), pageable and pinned callers, 1 / 16 / 64 / 256 submitters, two runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for devs in 0 0,0; do
    for pinned in 0 1; do
      timeout -k 10 150 tools/queue_bench 1,16,64,256 48 8 4 0 0 $pinned $devs | sed "s/^{/{\"rep\": $rep, /" || exit 1
    done
  done
done
