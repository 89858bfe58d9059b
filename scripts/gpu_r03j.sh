#!/bin/bash
# Unaligned-row reconstruct: parity, then reconstruct / GET timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_measured.py tests/test_gpu_parity.py tests/test_gpu_verify.py tests/test_gpu_reference_tables.py \
  > $OUT/tua.log 2>&1 || { tail -30 $OUT/tua.log; exit 2; }
tail -2 $OUT/tua.log
PATHS=rec,get timeout -k 10 300 python scripts/bench_paths.py > $OUT/bp_ua.jsonl 2>$OUT/bp.err || { tail $OUT/bp.err; exit 3; }
python - <<'PY'
import json
for l in open("gpurun_out/bp_ua.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["what"][:80], d["ms"], d["roofline"]["frac"], d["kernel_path"])
PY
