#!/bin/bash
# RS(12+4) unaligned GET with temporal survivor loads: parity + timing + traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_measured.py \
  -k "any_geometry or masks or unaligned" > $OUT/to.log 2>&1 || { tail -30 $OUT/to.log; exit 2; }
tail -1 $OUT/to.log
bash scripts/gpu_r03l.sh > $OUT/getab2.log 2>&1 || exit 3
grep '"variant": 0' $OUT/get_ab_rs124.jsonl
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/of -o p --output-format csv -- python scripts/gpu_ab_one.py > $OUT/of.log 2>&1 || { tail -5 $OUT/of.log; exit 4; }
python - <<'PY'
import csv, glob
rows = [r for r in csv.DictReader(open(glob.glob("gpurun_out/of/**/*counter_collection.csv", recursive=True)[0])) if "k_vr_ws<12" in r["Kernel_Name"]]
vals = [float(r["Counter_Value"]) for r in rows]
print("k_vr_ws<12,...> FETCH_SIZE KiB per launch:", sorted(vals)[len(vals)//2], "launches", len(vals), "algo survivor bytes KiB:", 4096 * 12 * 87382 / 1024)
PY
