"""Generate tests/golden/golden.json from the KAT-pinned oracles.

Both independent restatements (oracle/zs3_oracle.c via ctypes and
oracle/pyoracle.py) must agree on every vector before it is written.
Vectors: per (k, m, block_len, seed) the SHA-256 of all k+m shards, the k+m
HighwayHash-256 bitrot sums, and the full parity bytes for small blocks; plus
HH-256 (bitrot magic key) of fill() messages of every length 0..96 (all
remainder branches).  Inputs are oracle.fill(seed, obj=0, block_len).
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402

from oracle import oracle_c as oc  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

KEY = po.MAGIC_HH256_KEY
CASES = [(4, 2, 1 << 20, 1), (8, 4, 1 << 20, 2), (16, 4, 1 << 20, 3), (12, 4, 1 << 20, 4),
         (8, 4, (1 << 20) + 1, 5), (8, 4, 17, 6), (5, 3, 1000, 7), (4, 2, 1, 8), (6, 2, 3072, 9),
         (3, 3, 256, 10), (2, 2, 4096, 11), (20, 12, 5000, 12), (8, 4, 384, 13), (7, 5, 4099, 14)]


def main():
    out = {"generator": "tests/golden/make_golden.py", "key": KEY.hex(), "encode": [], "hh256": []}
    for k, m, n, seed in CASES:
        data = oc.fill(seed, 0, n)
        a = oc.encode_data(k, m, data)
        if n <= 1 << 16:
            b = po.encode_data(k, m, data.tobytes())
            assert np.array_equal(a, b), (k, m, n)
        sums = oc.hh256_rows(KEY, a)
        if a.shape[1] <= 4096:
            for i in range(k + m):
                assert po.hh256(KEY, a[i].tobytes()) == sums[i].tobytes()
        rec = {"k": k, "m": m, "block_len": n, "seed": seed, "shard_size": int(a.shape[1]),
               "shards_sha256": hashlib.sha256(a.tobytes()).hexdigest(),
               "sums": [s.tobytes().hex() for s in sums]}
        if n <= 4096:
            rec["parity_hex"] = a[k:].tobytes().hex()
        out["encode"].append(rec)
    msg = oc.fill(99, 3, 96)
    for L in range(0, 97):
        h = oc.hh256(KEY, msg[:L])
        assert h == po.hh256(KEY, msg[:L].tobytes())
        out["hh256"].append({"len": L, "sum": h.hex()})
    json.dump(out, open(os.path.join(HERE, "golden.json"), "w"), indent=0)
    print("wrote", len(out["encode"]), "encode vectors and", len(out["hh256"]), "hash vectors")


if __name__ == "__main__":
    main()
