"""Decompose the fused RS(8+4)+HH256 step: encode-only, hash-only, fused and a
plain HBM copy on the same 4096 x 1 MiB batch (device-resident)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k, m, blen, nobj = 8, 4, 1 << 20, int(os.environ.get("MB_OBJ", "4096"))
S = blen // k
stride = (k + m) * S
_V = int(os.environ.get("MB_VARIANT", "0"))
if _V:
    z.diag(_V).__enter__()  # this thread runs on the diagnostics build with variant _V
codec = z.Codec(k, m)
buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, stride, blen, nobj, seed=5)


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


def fused():
    codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)


def enc_only():
    codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride)


def hash_only():
    z.hh256_batch(buf, S, S, nobj * (k + m), sums)


src = buf[: nobj * blen]
dst = torch.empty_like(src)


def copy():
    dst.copy_(src)


res = {}
for name, fn, nbytes in [("copy_4GiB", copy, 2 * nobj * blen),
                         ("encode_only", enc_only, nobj * (blen + m * S)),
                         ("hash_only_6GiB", hash_only, nobj * (k + m) * S),
                         ("fused", fused, nobj * (blen + m * S + 32 * (k + m)))]:
    ms = timeit(fn)
    res[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}
    print(json.dumps({name: res[name]}), flush=True)
