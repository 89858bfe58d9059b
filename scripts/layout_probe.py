"""Does the DRAM address pattern of the parity/data streams matter?  Times the fused
RS(8+4) kernel (and its no-hash ablation) with parity in place, in a separate buffer,
and in a separate buffer whose per-stripe stride is skewed off the 128 KiB grid."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k, m, blen, nobj = 8, 4, 1 << 20, 4096
S = blen // k
codec = z.Codec(k, m)


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


VARS = [int(v) for v in os.environ.get('LP_VARIANTS', '0,44').split(',')]
DSKEWS = [int(v) for v in os.environ.get('LP_DSKEW', '0,4352').split(',')]
PSKEWS = [None if v == 'in' else int(v) for v in os.environ.get('LP_PSKEW', 'in,0,4352,73984').split(',')]
for dskew in DSKEWS:
    dstride = (k + m) * S + dskew
    buf = torch.empty(nobj * dstride, dtype=torch.uint8, device="cuda")
    z.fill_batch(buf, dstride, blen, nobj, seed=5)
    sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
    for pskew in PSKEWS:
        if pskew is None:
            par, poff, pstride = buf, k * S, dstride
        else:
            pstride = m * S + pskew
            par, poff = torch.empty(nobj * pstride, dtype=torch.uint8, device="cuda"), 0
        for v in VARS:
            z.set_variant(v)
            ms = timeit(lambda: codec.encode_batch(buf, dstride, blen, nobj, parity=par, parity_offset=poff,
                                                    parity_stride=pstride, sums=sums))
            print(json.dumps({"data_skew": dskew, "parity": "inplace" if pskew is None else f"sep+{pskew}",
                              "variant": v, "ms": round(ms, 4)}), flush=True)
        if pskew is not None:
            del par
    del buf
    torch.cuda.empty_cache()
z.set_variant(0)
