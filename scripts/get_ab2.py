"""A/B of the GET / heal launches for the RS(4+2), RS(8+4) and RS(16+4) shapes
(variant 0 = product default dispatch; others forced through the diagnostics build,
e.g. 200 = first-generation kernel, 216/217 = scalar coefficient tables), interleaved
rounds.  SHAPES=4,8,16 selects the shapes, CASES=heal filters the case names, NOBJ=n
overrides the batch size."""
import contextlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402


def timeit(fn, steps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


variants = [int(v) for v in os.environ.get("VARIANTS", "0,200").split(",")]
shapes = [int(x) for x in os.environ.get("SHAPES", "4,8,16").split(",")]
only = os.environ.get("CASES")  # e.g. CASES=heal: substring filter on the case names
ALL = ((4, 2, 2048, (("verify 4", [], False), ("verify + rebuild 2", [0, 3], False),
                     ("verify + rebuild 1", [1], False), ("heal 2", [1, 5], True))),
       (8, 4, 4096, (("verify 8", [], False), ("verify + rebuild 1", [3], False),
                     ("verify + rebuild 2", [0, 5], False), ("verify + rebuild 3", [0, 5, 6], False),
                     ("verify + rebuild 4", [1, 2, 5, 7], False), ("heal 1", [4], True), ("heal 2", [2, 10], True),
                     ("heal 3", [0, 6, 9], True), ("heal 4", [1, 3, 8, 11], True))),
       (16, 4, 2048, (("verify 16", [], False), ("verify + rebuild 1", [6], False), ("verify + rebuild 2", [0, 9], False),
                      ("verify + rebuild 3", [1, 7, 15], False), ("verify + rebuild 4", [1, 7, 14, 15], False),
                      ("heal 1", [5], True), ("heal 2", [0, 17], True), ("heal 3", [2, 11, 18], True),
                      ("heal 4", [1, 7, 15, 19], True))))


def ctx(v):
    return contextlib.nullcontext() if v == 0 else z.diag(v)


for k, m, nobj, cases in [c for c in ALL if c[0] in shapes]:
    nobj = int(os.environ.get("NOBJ", nobj))  # e.g. NOBJ=16: the small-batch regime
    blen = 1 << 20
    S = blen // k
    R = k + m
    stride = R * S
    codec = z.Codec(k, m)
    with z.diag():
        dcodec = z.Codec(k, m)
    buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
    z.fill_batch(buf, stride, blen, nobj, seed=3)
    sums = torch.zeros(nobj * R * 32, dtype=torch.uint8, device="cuda")
    codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
    bad = torch.zeros((nobj, R), dtype=torch.int32, device="cuda")
    out = torch.zeros_like(sums)
    for rnd in range(2):
        for name, erased, heal in cases:
            if only and only not in name:
                continue
            present = [i not in erased for i in range(R)]
            for v in variants:
                c = codec if v == 0 else dcodec
                with ctx(v):
                    ms = timeit(lambda: c.verify_reconstruct_batch(buf, stride, S, nobj, present, not heal, sums, bad,
                                                                   sums_out=out if heal else None))
                    path = z.last_path()
                nre = len([e for e in erased if e < k or heal])
                nbytes = nobj * (k + nre) * S
                print(json.dumps({"round": rnd, "k": k, "case": name, "variant": v, "path": path, "ms": round(ms, 4),
                                  "hbm_frac": round(nbytes / ms / 1e-3 / 8e12, 3),
                                  "bad": int(bad.sum())}), flush=True)
    del buf, sums, bad, out
    torch.cuda.empty_cache()
