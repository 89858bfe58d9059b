"""A/B of the GET / heal kernel launch shapes on one device (variant 0 = default,
200 = small-workgroup launch), interleaved rounds."""
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


k, m, blen, nobj = 8, 4, 1 << 20, 4096
S = blen // k
stride = (k + m) * S
codec = z.Codec(k, m)
buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, stride, blen, nobj, seed=3)
sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
vbad = torch.empty(nobj * (k + m), dtype=torch.int32, device="cuda")
hsum = torch.empty_like(sums)
cases = [([], True, False, "verify 8"), ([0, 5], True, False, "verify 8 + rebuild 2"),
         ([2, 10], False, True, "heal 1d+1p")]
variants = [int(v) for v in os.environ.get("VARIANTS", "0,200").split(",")]
for rnd in range(3):
    for erased, data_only, heal, label in cases:
        pres = [i not in erased for i in range(k + m)]
        for v in variants:
            with (z.diag(v) if v else contextlib.nullcontext()):
                cv = z.Codec(k, m)  # a codec belongs to the library (product / diagnostics) that made it
                ms = timeit(lambda: cv.verify_reconstruct_batch(buf, stride, S, nobj, pres, data_only, sums, vbad,
                                                                sums_out=hsum if heal else None))
            e = len(erased)
            ab = nobj * (k * S + e * S + 32 * k + (32 * e if heal else 0))
            print(json.dumps({"round": rnd, "case": label, "variant": v, "ms": round(ms, 4),
                              "hbm_frac": round(ab / ms / 1e6 / 8000, 3), "bad": int(vbad.sum())}), flush=True)
