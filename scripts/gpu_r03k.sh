#!/bin/bash
# RS(12+4) UA fused GET: parity (GET / heal / masks / reference tables), then timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_measured.py tests/test_gpu_verify.py tests/test_gpu_reference_tables.py tests/test_gpu_queue.py \
  > $OUT/tget.log 2>&1 || { tail -30 $OUT/tget.log; exit 2; }
tail -2 $OUT/tget.log
PATHS=get timeout -k 10 300 python scripts/bench_paths.py > $OUT/bp_get.jsonl 2>$OUT/bp.err || { tail $OUT/bp.err; exit 3; }
python - <<'PY'
import json
for l in open("gpurun_out/bp_get.jsonl"):
    if l.startswith("{") and ("12+4" in l or "4+4" in l):
        d = json.loads(l); print(d["what"][:80], d["ms"], d["roofline"]["frac"], d["kernel_path"])
PY
