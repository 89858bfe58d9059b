#!/bin/bash
# RS(12+4) UA: parity of every variant, then the prefetch-distance sweep on the 512-byte-tile shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_variants.py -k rs124 > $OUT/t124.log 2>&1 || { tail -30 $OUT/t124.log; exit 2; }
tail -2 $OUT/t124.log
SWEEP_SHAPES=12:4:4096,12:4:16384,12:4:2048 SWEEP_VARIANTS=0,196,175,179,180,181 SWEEP_REPEAT=2 \
  timeout -k 10 300 python scripts/sweep_variants.py > $OUT/ab_rs124_pfd.jsonl 2>$OUT/sweep.err || { tail $OUT/sweep.err; exit 3; }
python - <<'PY'
import json
for l in open("gpurun_out/ab_rs124_pfd.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["objects"], d["variant"], d["ms"], round(d["hbm_GBps"] / 8000, 3), d["match"])
PY
