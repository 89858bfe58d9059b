"""Per-kernel HBM bytes per launch from request-size counters (scripts/traffic_req.sh).
Usage: traffic_req.py reads_counter_collection.csv writes_counter_collection.csv out.json
Only the encode / GET kernels (k_ehx_ws, k_vr_ws, k_vr_quad) are kept; values are means over launches."""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(lambda: defaultdict(float))
    seen = defaultdict(set)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if "k_ehx_ws" not in name and "k_vr_ws" not in name and "k_vr_quad" not in name:
                continue
            per[name][row["Counter_Name"]] += float(row["Counter_Value"])
            seen[name].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    return per, {k: len(v) for k, v in seen.items()}


rd, nr = load(sys.argv[1])
wr, nw = load(sys.argv[2])
out = {}
for name, c in rd.items():
    n = max(1, nr[name])
    req, r32, r64, r128 = (c[k] / n for k in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum",
                                               "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"))
    rest = max(0.0, req - r32 - r64 - r128)
    w = wr.get(name, {})
    m = max(1, nw.get(name, 1))
    wreq, w64 = w.get("TCC_EA0_WRREQ_sum", 0.0) / m, w.get("TCC_EA0_WRREQ_64B_sum", 0.0) / m
    rbytes = 32 * r32 + 64 * r64 + 128 * r128 + 64 * rest
    wbytes = 32 * (wreq - w64) + 64 * w64
    out[name] = {"read_bytes": rbytes, "write_bytes": wbytes, "hbm_bytes_per_launch": rbytes + wbytes,
                 "rdreq": req, "rdreq_32b": r32, "rdreq_64b": r64, "rdreq_128b": r128, "rdreq_other": rest,
                 "wrreq": wreq, "wrreq_64b": w64, "launches": n,
                 "note": "bytes by request size: 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (+64 per other RDREQ); "
                         "32*(WRREQ-WRREQ_64B) + 64*WRREQ_64B"}
json.dump(out, open(sys.argv[3], "w"), indent=1)
for name, v in out.items():
    print(json.dumps({"kernel": name, "read_GB": round(v["read_bytes"] / 1e9, 4), "write_GB": round(v["write_bytes"] / 1e9, 4),
                      "rdreq_128b_frac": round(v["rdreq_128b"] / max(1, v["rdreq"]), 4),
                      "rdreq_other": v["rdreq_other"], "launches": v["launches"]}))
