#!/bin/bash
# New RS(12+4) UA default: measured-shape parity; RS(16+4) L2-prefetch A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_measured.py tests/test_gpu_variants.py -k "rs124 or server_default or any_geometry" > $OUT/t124b.log 2>&1 || { tail -30 $OUT/t124b.log; exit 2; }
tail -2 $OUT/t124b.log
SWEEP_SHAPES=16:4:2048,16:4:4096,16:4:8192,12:4:4096 SWEEP_VARIANTS=0,158,159 SWEEP_REPEAT=2 \
  timeout -k 10 300 python scripts/sweep_variants.py > $OUT/ab_rs164_pfd.jsonl 2>$OUT/sweep.err || { tail $OUT/sweep.err; exit 3; }
python - <<'PY'
import json
for l in open("gpurun_out/ab_rs164_pfd.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["k"], d["objects"], d["variant"], d["ms"], round(d["hbm_GBps"] / 8000, 3), d["match"])
PY
