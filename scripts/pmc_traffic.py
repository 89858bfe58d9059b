"""Per-launch HBM traffic of the bench kernel from two rocprofv3 PMC passes.

MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports exactly half the bytes of a wide coalesced streaming read (16 B/lane loads),
so it is doubled; WRITE_SIZE reads the bytes exactly for 16-B streaming stores.
Usage: pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv out.json [objects]
With `objects` (the bench's objects per launch) the entries are keyed "<kernel> @ <objects>
objects", carry workload.objects (bench.py's committed_traffic lookup) and are merged into
an existing out.json, so one file holds the per-GPU shares of N = 1/2/4/8.
"""
import os
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
objects = int(sys.argv[4]) if len(sys.argv) > 4 else None
out = json.load(open(sys.argv[3])) if objects is not None and os.path.exists(sys.argv[3]) else {}
for name in fetch:
    if "encode" not in name and "k_ehx" not in name:
        continue
    f = sum(fetch[name]) / len(fetch[name])
    w = sum(write.get(name, [0])) / max(1, len(write.get(name, [0])))
    key = f"{name} @ {objects} objects" if objects is not None else name
    out[key] = {
        "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
        "hbm_bytes_per_launch": (2 * f + w) * 1024,
        "note": "(2*FETCH_SIZE + WRITE_SIZE) * 1024: gfx950 FETCH_SIZE counts half of wide streaming reads",
        "launches": len(fetch[name]),
    }
    if objects is not None:
        out[key]["workload"] = {"objects": objects}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
