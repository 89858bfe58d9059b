"""Attach measured HBM traffic to every bench_paths.py measurement line.

The two PMC passes (FETCH_SIZE, WRITE_SIZE) run bench_paths.py with REPS=3, so each
measurement is 1 + 3 launches of its kernel; helper dispatches (k_fill, runtime
copies/fills, torch reductions, k_any_rows) interleave and single setup launches (the
encode that builds a GET / hash input) sit between measurements.  Consecutive
dispatches of one kernel (helpers skipped) form runs; runs of 4·j launches are the j
measurements, in bench_paths order.  Traffic per launch = mean over the 3 timed
launches of (2·FETCH_SIZE + WRITE_SIZE)·1024 (gfx950 correction, MI355X_MICROARCH.md).
The join refuses to write anything if the chunk count differs from the line count.

  python scripts/paths_traffic_join.py FETCH.csv WRITE.csv bench_paths.jsonl out.jsonl
"""
import csv
import json
import sys

HELPERS = ("k_fill", "__amd_rocclr", "at::native", "k_any_rows")
PER = 4  # 1 warm + REPS=3 timed launches per measurement


def dispatches(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in rows
            if not any(h in r["Kernel_Name"] for h in HELPERS)]


def chunks(seq):
    runs = []
    for name, v in seq:
        if runs and runs[-1][0] == name:
            runs[-1][1].append(v)
        else:
            runs.append([name, [v]])
    out = []
    for name, vals in runs:
        if len(vals) % PER == 1:
            vals = vals[1:]  # a setup launch (input encode / warm-up) ahead of the measurement(s)
        if len(vals) % PER:
            continue
        for i in range(0, len(vals), PER):
            out.append((name, vals[i + 1:i + PER]))
    return out


def main():
    f = chunks(dispatches(sys.argv[1], "FETCH_SIZE"))
    w = chunks(dispatches(sys.argv[2], "WRITE_SIZE"))
    lines = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")]
    # the part-digest lines time 1 + 2 launches (long single-lane chains): not joined
    lines = [d for d in lines if "roofline" in d and not d["path"].endswith("_parts")]
    if not (len(f) == len(w) == len(lines)):
        sys.exit(f"chunk count mismatch: fetch {len(f)}, write {len(w)}, lines {len(lines)}")
    with open(sys.argv[4], "w") as out:
        for d, (fn, fv), (wn, wv) in zip(lines, f, w):
            assert fn == wn, (fn, wn)
            t = (2 * sum(fv) / len(fv) + sum(wv) / len(wv)) * 1024
            d["kernel"] = fn
            d["roofline"]["traffic"] = int(t)
            d["roofline"]["traffic_over_algo"] = round(t / d["roofline"]["algo_bytes_per_launch"], 4)
            out.write(json.dumps(d) + "\n")
            print(f"{d['roofline']['traffic_over_algo']:7.4f} {d['path'][:20]:20s} {d['what'][:60]:60s} {fn[:60]}")


if __name__ == "__main__":
    main()
