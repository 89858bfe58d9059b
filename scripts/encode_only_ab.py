"""A/B of the encode-only launch (zs3_encode_batch without sums: Split + Encode of
klauspost EncodeData, k_encode_only) on the BASELINE shapes, interleaved rounds.
Variant 0 = product build; 98 = the diagnostics build with plain (temporal) loads and
stores.  VARIANTS=0,98"""
import contextlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

variants = [int(v) for v in os.environ.get("VARIANTS", "0,98").split(",")]
for k, m, nobj in ((4, 2, 1024), (8, 4, 4096), (16, 4, 2048)):
    blen = 1 << 20
    S = blen // k
    stride = (k + m) * S
    buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
    z.fill_batch(buf, stride, blen, nobj, seed=5)
    codecs = {0: z.Codec(k, m)}
    with z.diag():
        codecs[1] = z.Codec(k, m)
    for rnd in range(3):
        for v in variants:
            c = codecs[0 if v == 0 else 1]
            with (contextlib.nullcontext() if v == 0 else z.diag(v)):
                fn = lambda: c.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S,  # noqa: E731
                                            parity_stride=stride)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            nbytes = nobj * (blen + m * S)
            print(json.dumps({"round": rnd, "k": k, "m": m, "n": nobj, "variant": v, "ms": round(ms, 4),
                              "frac": round(nbytes / ms / 1e-3 / 8e12, 4)}), flush=True)
    del buf
    torch.cuda.empty_cache()
