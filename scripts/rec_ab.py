"""A/B of the reconstruct kernel launch shapes (BASELINE config 3: RS(8+4), 4096 x 1 MiB,
erased {0, 5} and {2, 10}), interleaved rounds; variant 0 = product dispatch, others
through the diagnostics build (220/221: 2/4 columns per thread, 222: non-temporal
loads and stores).  VARIANTS=0,220,221,222"""
import contextlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k, m, blen, nobj = 8, 4, 1 << 20, 4096
S = blen // k
stride = (k + m) * S
codec = z.Codec(k, m)
with z.diag():
    dcodec = z.Codec(k, m)  # a codec handle belongs to the library that made it
buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, stride, blen, nobj, seed=3)
codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride)
ref = buf.clone()
variants = [int(v) for v in os.environ.get("VARIANTS", "0,220,221").split(",")]
for rnd in range(3):
    for erased in ([0, 5], [2, 10]):
        present = [i not in erased for i in range(k + m)]
        for v in variants:
            with (contextlib.nullcontext() if v == 0 else z.diag(v)):
                c = codec if v == 0 else dcodec
                fn = lambda: c.reconstruct_batch(buf, stride, S, nobj, present, True)  # noqa: E731
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            ok = bool(torch.equal(buf, ref))
            nbytes = nobj * (k + len([e for e in erased if e < k])) * S
            print(json.dumps({"round": rnd, "erased": erased, "variant": v, "ms": round(ms, 4),
                              "hbm_frac": round(nbytes / ms / 1e-3 / 8e12, 3), "ok": ok}), flush=True)
