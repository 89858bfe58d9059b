"""Join rocprofv3 counter passes per kernel: mean counter value per launch, the
kernel-trace average duration, and derived fractions (VALU issue share of SIMD cycles,
wait shares of wave cycles).

  python scripts/pmc_compute_join.py kernel_stats.csv pass1.csv [pass2.csv ...] > out.json

VALU issue share = SQ_INSTS_VALU x 2 cycles (one wave64 VALU instruction occupies a
SIMD-32 for 2 cycles, MI355X_MICROARCH.md 'Wave scheduling') / (1024 SIMDs x the
kernel's duration x the clock GRBM_GUI_ACTIVE implies: GRBM_GUI_ACTIVE is summed over
the 8 XCDs, so clock = GRBM_GUI_ACTIVE / 8 / duration).
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    stats = {}
    with open(sys.argv[1]) as f:
        for row in csv.DictReader(f):
            stats[row["Name"]] = float(row["AverageNs"])
    vals = defaultdict(lambda: defaultdict(list))
    for path in sys.argv[2:]:
        per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> sum over dims
        with open(path) as f:
            for row in csv.DictReader(f):
                key = (row["Kernel_Name"], row.get("Dispatch_Id", row.get("Correlation_Id", "")))
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
        for (name, _), cs in per.items():
            for c, v in cs.items():
                vals[name][c].append(v)
    out = {}
    for name, cs in vals.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        ns = stats.get(name)
        rec = {"avg_ns": ns, **{c: round(v, 1) for c, v in sorted(d.items())}}
        if ns and d.get("GRBM_GUI_ACTIVE"):
            ghz = d["GRBM_GUI_ACTIVE"] / 8 / ns
            rec["clock_GHz"] = round(ghz, 3)
            if "SQ_INSTS_VALU" in d:
                rec["valu_issue_frac"] = round(d["SQ_INSTS_VALU"] * 2 / (1024 * ns * ghz), 3)
        wc = d.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in d:
                    rec[c.replace("SQ_", "").lower() + "_frac_of_wave_cycles"] = round(d[c] / wc, 3)
        out[name] = rec
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
