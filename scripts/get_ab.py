"""A/B of GET / heal launches (product vs diagnostics variants) on 1 MiB stripes:
verify the k survivors + rebuild e rows (+ hash them for heal), median of REPS launches,
% of 8 TB/s on the algorithmic bytes k*S + e*S + 32*k (+ 32*e).

  SHAPE=16:4:2048 VARIANTS=0,250,251 CASES="0,5;0,5,9,14;h3,17;h0,1,16,19" python scripts/get_ab.py
(a case is a comma list of erased shards; a leading 'h' = heal)
"""
import contextlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

MiB = 1 << 20
REPS = int(os.environ.get("REPS", "10"))
k, m, n = (int(x) for x in os.environ.get("SHAPE", "16:4:2048").split(":"))
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0").split(",")]
CASES = []
for c in os.environ.get("CASES", "0,5;h3,17").split(";"):
    heal = c.startswith("h")
    CASES.append(([int(x) for x in c.lstrip("h").split(",")], heal))
R = k + m
S = -(-MiB // k)
stride = R * S
d = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
z.fill_batch(d, stride, MiB, n, seed=3)
sums = torch.zeros(n * R * 32, dtype=torch.uint8, device="cuda")
z.Codec(k, m, MiB).encode_batch(d, stride, MiB, n, parity=d, parity_offset=k * S, parity_stride=stride, sums=sums)
bad = torch.zeros(n * R, dtype=torch.int32, device="cuda")
hs = torch.zeros_like(sums)
st = torch.cuda.current_stream()
for rnd in range(2):
    for erased, heal in CASES:
        pres = [i not in erased for i in range(R)]
        e = len(erased) if heal else len([i for i in erased if i < k])
        ab = n * (k * S + e * S + 32 * k + (32 * e if heal else 0))
        for v in VARIANTS:
            with (z.diag(v) if v else contextlib.nullcontext()):
                c = z.Codec(k, m, MiB)

                def f():
                    c.verify_reconstruct_batch(d, stride, S, n, pres, not heal, sums, bad, sums_out=hs if heal else None)
                f()
                torch.cuda.synchronize()
                ts = []
                for _ in range(REPS):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    f()
                    b.record(st)
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b))
                ms = sorted(ts)[REPS // 2]
                print(json.dumps({"round": rnd, "k": k, "m": m, "objects": n, "erased": erased, "heal": heal,
                                  "variant": v, "ms": round(ms, 4), "frac": round(ab / (ms * 1e-3) / 8e12, 4),
                                  "path": z.last_path(), "bad": int(bad.sum())}), flush=True)
