#!/bin/bash
# Round 5: bench.py --gpus 2 on the final code: two self-launched ranks sharing the box's
# one GPU (test-only ZS3_BENCH_SAME_DEVICE=1), and the refusal without it (exit 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ZS3_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 > gpurun_out/r05_gpus2_same.json 2> gpurun_out/r05_gpus2_same.err || { tail gpurun_out/r05_gpus2_same.err; exit 1; }
tail -1 gpurun_out/r05_gpus2_same.json | cut -c1-240
rc=0
timeout -k 10 120 python bench.py --gpus 2 > gpurun_out/r05_gpus2_refused.out 2> gpurun_out/r05_gpus2_refused.err || rc=$?
echo "exit status without the override: $rc" | tee -a gpurun_out/r05_gpus2_refused.err
tail -2 gpurun_out/r05_gpus2_refused.err
[ "$rc" = 2 ] || exit 2
