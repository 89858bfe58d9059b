#!/bin/bash
# HBM traffic of the RS(12+4) unaligned GET (rebuild 2) with temporal survivor loads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/of -o p --output-format csv -- python scripts/gpu_ab_one.py > $OUT/of.log 2>&1 || { tail -5 $OUT/of.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/ow -o p --output-format csv -- python scripts/gpu_ab_one.py > $OUT/ow.log 2>&1 || { tail -5 $OUT/ow.log; exit 5; }
python - <<'PY' | tee $OUT/rs124_get_traffic.json
import csv, glob, json
def med(d):
    rows = [r for r in csv.DictReader(open(glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0])) if "k_vr_ws<12" in r["Kernel_Name"]]
    v = sorted(float(r["Counter_Value"]) for r in rows)
    return v[len(v) // 2], rows[0]["Kernel_Name"] if rows else ""
f, name = med("of"); w, _ = med("ow")
S = 87382; nb = 4096
algo = nb * (12 * S + 2 * S + 32 * 12)
traffic = (2 * f + w) * 1024  # gfx950 correction, MI355X_MICROARCH.md
print(json.dumps({"kernel": name, "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "traffic": traffic, "algo": algo, "traffic_over_algo": round(traffic / algo, 4)}))
PY
