"""Compact DMA / kernel timeline of a rocprofv3 run (--memory-copy-trace --kernel-trace):
the events of at least MIN_US microseconds in the first TRACE_WINDOW_MS milliseconds after
the first host -> device copy, as JSON lines (start / end ms, kind, stream), then one
summary line: busy time of the H2D copies, of the device -> host copy kernels (the HIP
runtime's __amd_rocclr_copyBuffer and k_rows_copy) and of both at once.
Usage: python scripts/dma_timeline.py <memory_copy_trace.csv> <kernel_trace.csv>"""
import csv
import json
import os
import sys

MIN_US = float(os.environ.get("MIN_US", "50"))
WINDOW_MS = float(os.environ.get("TRACE_WINDOW_MS", "120"))


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(u, v):
    i = j = tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        tot += max(0, b - a)
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    mc = list(csv.DictReader(open(sys.argv[1])))
    kt = list(csv.DictReader(open(sys.argv[2])))
    h2d = [r for r in mc if "HOST_TO_DEVICE" in r["Direction"]]
    t0 = min(int(r["Start_Timestamp"]) for r in h2d)
    t1 = t0 + WINDOW_MS * 1e6
    ev = []
    for r in mc:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"].replace("MEMORY_COPY_", ""),
                   r["Stream_Id"]))
    for r in kt:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel " + r["Kernel_Name"][:70],
                   r["Stream_Id"]))
    ev = sorted(e for e in ev if t0 <= e[0] <= t1)
    for a, b, what, st in ev:
        if b - a >= MIN_US * 1e3:
            print(json.dumps({"start_ms": round((a - t0) / 1e6, 3), "end_ms": round((b - t0) / 1e6, 3), "what": what,
                              "stream": st}))
    up = union([(a, b) for a, b, w, _ in ev if w == "HOST_TO_DEVICE"])
    down = union([(a, b) for a, b, w, _ in ev if "copyBuffer" in w or "k_rows_copy" in w or w == "DEVICE_TO_HOST"])
    print(json.dumps({"summary": True, "window_ms": WINDOW_MS, "h2d_busy_ms": round(sum(b - a for a, b in up) / 1e6, 3),
                      "d2h_busy_ms": round(sum(b - a for a, b in down) / 1e6, 3),
                      "both_ms": round(inter(up, down) / 1e6, 3)}))


if __name__ == "__main__":
    main()
