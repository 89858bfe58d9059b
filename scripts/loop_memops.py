#!/usr/bin/env python3
"""Print the LDS / wait / barrier instructions of a kernel's hottest loop (the backward
branch whose body holds the most v_perm_b32), with their instruction index.
  python scripts/loop_memops.py k.s <kernel-name-substring>"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(sys.argv[2]) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
labels = {}
best = None
for i in range(start, end):
    m = re.match(r"^(\.LBB\d+_\d+):", lines[i])
    if m:
        labels[m.group(1)] = i
    m = re.search(r"s_cbranch\w*\s+(\.LBB\d+_\d+)", lines[i])
    if m and m.group(1) in labels:
        body = lines[labels[m.group(1)]:i + 1]
        n = sum("v_perm_b32" in l for l in body)
        if best is None or n > best[0]:
            best = (n, body)
n = 0
for l in best[1]:
    if re.search(r"^\s+(v_|s_|ds_|global_|buffer_)", l):
        n += 1
    if re.search(r"ds_|s_waitcnt|s_barrier|global_|buffer_", l):
        print(n, l.strip())
