"""Per-kernel HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE) over scripts/bench_paths.py, with the gfx950 correction of
MI355X_MICROARCH.md §HBM (FETCH_SIZE in KiB and half the bytes of wide streaming reads,
so doubled; WRITE_SIZE in KiB), joined with the kernel-trace stats (average duration).

  python scripts/pmc_paths.py FETCH.csv WRITE.csv kernel_stats.csv out.json
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
stats = {}
with open(sys.argv[3]) as f:
    for row in csv.DictReader(f):
        stats[row["Name"]] = row
out = {}
for name in sorted(fetch):
    f = sum(fetch[name]) / len(fetch[name])
    w = sum(write.get(name, [0])) / max(1, len(write.get(name, [0])))
    st = stats.get(name, {})
    out[name] = {"FETCH_SIZE_KiB": round(f, 1), "WRITE_SIZE_KiB": round(w, 1),
                 "hbm_bytes_per_launch": int((2 * f + w) * 1024),
                 "launches_in_pmc_pass": len(fetch[name]),
                 "avg_duration_ns": float(st["AverageNs"]) if st else None,
                 "calls_in_trace": int(st["Calls"]) if st else None}
json.dump(out, open(sys.argv[4], "w"), indent=1)
for n, v in out.items():
    print(f"{v['hbm_bytes_per_launch']/1e9:9.3f} GB  {v['avg_duration_ns'] or 0:12.0f} ns  {n[:150]}")
