"""DMA timeline of a rocprofv3 --memory-copy-trace run: per direction the union of the
copy intervals, the bytes moved, the rate while copying, and how long H2D and D2H copies
ran at the same time.  Usage: python scripts/dma_overlap.py <memory_copy_trace.csv> [t0 t1]
(optional window in seconds from the first copy).  Prints one JSON line."""
import csv
import json
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(u, v):
    i = j = 0
    tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if b > a:
            tot += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    if not rows:
        print(json.dumps({"copies": 0}))
        return
    cols = rows[0].keys()
    cs = next(c for c in cols if "Start" in c)
    ce = next(c for c in cols if "End" in c)
    cd = next((c for c in cols if c in ("Direction", "Operation", "Kind") and any(
        "HOST_TO_DEVICE" in r[c] or "DEVICE_TO_HOST" in r[c] for r in rows[:50])), None)
    cb = next((c for c in cols if "Size" in c or "Bytes" in c), None)
    t_first = min(int(r[cs]) for r in rows)
    w0 = float(sys.argv[2]) * 1e9 if len(sys.argv) > 2 else 0
    w1 = float(sys.argv[3]) * 1e9 if len(sys.argv) > 3 else float("inf")
    by = {}
    for r in rows:
        a, b = int(r[cs]) - t_first, int(r[ce]) - t_first
        if b < w0 or a > w1:
            continue
        d = r[cd] if cd else "?"
        d = "H2D" if "HOST_TO_DEVICE" in d else "D2H" if "DEVICE_TO_HOST" in d else d
        x = by.setdefault(d, {"iv": [], "bytes": 0, "n": 0})
        x["iv"].append((a, b))
        x["bytes"] += int(r[cb]) if cb and r[cb].isdigit() else 0
        x["n"] += 1
    out = {"columns": list(cols)[:16]}
    us = {}
    for d, x in by.items():
        u = union(x["iv"])
        busy = sum(b - a for a, b in u)
        us[d] = u
        span = u[-1][1] - u[0][0]
        out[d] = {"copies": x["n"], "bytes": x["bytes"], "busy_ms": round(busy / 1e6, 3), "span_ms": round(span / 1e6, 3),
                  "GBps_while_busy": round(x["bytes"] / busy, 2) if busy else None,
                  "GBps_over_span": round(x["bytes"] / span, 2) if span else None}
    if "H2D" in us and "D2H" in us:
        out["overlap_ms"] = round(inter(us["H2D"], us["D2H"]) / 1e6, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
