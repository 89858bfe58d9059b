"""Average each PMC counter per kernel from a rocprofv3 counter_collection.csv."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
with open(sys.argv[1]) as f:
    for row in csv.DictReader(f):
        name = row.get("Kernel_Name", "?")
        short = name.split("(")[0][-60:]
        acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for kname, cs in acc.items():
    print(kname, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in cs.items()))
