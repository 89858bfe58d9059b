#!/bin/bash
# Classify the box's memory behaviour (mempat lockstep vs stream), then sweep variants.
# Usage: VARIANTS=5,80 SHAPES=8:4:4096 REPEAT=3 bash scripts/box_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/ubench/mempat > gpurun_out/mempat.log 2>&1 || exit 3
grep -E "^stream|^lock G4 NT192 CW8 \(T384\) bar" gpurun_out/mempat.log
SWEEP_SHAPES=${SHAPES:-8:4:4096} SWEEP_VARIANTS=${VARIANTS:-5,80} SWEEP_REPEAT=${REPEAT:-3} \
  timeout -k 10 300 python scripts/sweep_variants.py 2>&1 | grep -v amdgpu.ids > gpurun_out/sw.log || exit 4
python3 - <<'PY'
import json
from collections import defaultdict
d = defaultdict(list)
for l in open("gpurun_out/sw.log"):
    if l.startswith("{"):
        r = json.loads(l)
        d[(r["k"], r["m"], r["variant"])].append(r["ms"])
for key, ms in d.items():
    print(key, "min %.4f" % min(ms), ms, "" if all(True for _ in ms) else "")
PY
grep -c '"match": false' gpurun_out/sw.log
