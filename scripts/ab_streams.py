"""A/B: one encode launch over the whole batch vs the batch split into P parts launched
concurrently on P streams (fork / join through events), BASELINE config 4 shape
(RS(8+4), 1 MiB blocks, in-place layout).  Prints one JSON line per (P, repeat):
ms per whole batch (HIP events on the joining stream) and GiB/s of object bytes.

    NOBJ=65536 PARTS=1,2,3,4 REPS=3 python scripts/ab_streams.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k, m, blen = int(os.environ.get("K", 8)), int(os.environ.get("M", 4)), 1 << 20
nobj = int(os.environ.get("NOBJ", 65536))
parts = [int(x) for x in os.environ.get("PARTS", "1,2,3,4").split(",")]
reps = int(os.environ.get("REPS", 3))
steps = int(os.environ.get("STEPS", 10))
S = -(-blen // k)
stride = (k + m) * S
codec = z.Codec(k, m, blen)
buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, stride, blen, nobj, seed=1234)
torch.cuda.synchronize()
main = torch.cuda.current_stream()
side = [torch.cuda.Stream() for _ in range(max(parts))]


def run(P):
    bounds = [nobj * i // P for i in range(P + 1)]
    if P == 1:
        codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
        return
    fork = torch.cuda.Event()
    fork.record(main)
    joins = []
    for i in range(P):
        st = side[i]
        st.wait_event(fork)
        lo, hi = bounds[i], bounds[i + 1]
        codec.encode_batch(buf, stride, blen, hi - lo, parity=buf, parity_offset=lo * stride + k * S,
                           parity_stride=stride, sums=sums[lo * (k + m) * 32:], data_offset=lo * stride, stream=st)
        e = torch.cuda.Event()
        e.record(st)
        joins.append(e)
    for e in joins:
        main.wait_event(e)


for rep in range(reps):
    for P in parts:
        for _ in range(3):
            run(P)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main)
        for _ in range(steps):
            run(P)
        b.record(main)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / steps
        print(json.dumps({"k": k, "m": m, "objects": nobj, "parts": P, "rep": rep, "ms": round(ms, 4),
                          "GiBps": round(nobj * blen / (ms * 1e-3) / 2 ** 30, 1),
                          "frac_8TBps": round(nobj * (blen + m * S + 32 * (k + m)) / (ms * 1e-3) / 8e12, 4)}),
              flush=True)
