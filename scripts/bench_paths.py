"""Secondary measurements: reconstruct (BASELINE config 3),
hash-only and verify (GET path), and the end-to-end host->device->host stream
(config 5, PCIe-inclusive).  Prints one JSON line per measurement."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
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


def out(**kw):
    print(json.dumps(kw), flush=True)


# ---- config 3: RS(8+4) 4096 x 1 MiB encode, then reconstruct with 2 erased
k, m, blen, nobj = 8, 4, 1 << 20, 4096
S = blen // k
stride = (k + m) * S
codec = z.Codec(k, m)
buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, stride, blen, nobj, seed=3)
codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride)
torch.cuda.synchronize()
for erased, data_only, label in (([0, 5], True, "ReconstructData, data shards 0+5 erased"),
                                 ([2, 10], False, "Reconstruct, 1 data + 1 parity erased")):
    pres = [i not in erased for i in range(k + m)]
    ms = timeit(lambda: codec.reconstruct_batch(buf, stride, S, nobj, pres, data_only))
    ab = nobj * (k * S + len(erased) * S)
    out(path="reconstruct", shape="RS(8+4)", objects=nobj, what=label, ms=round(ms, 4),
        GiBps_object=round(nobj * blen / ms / 1e-3 / 2**30, 1), hbm_GBps=round(ab / ms / 1e6, 1),
        hbm_frac=round(ab / ms / 1e6 / 8000, 3))

# ---- GET / heal fused pass (zs3_verify_reconstruct_batch): verify the k survivors
# against stored sums and rebuild the missing shards; heal also hashes the rebuilt rows
sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
vbad = torch.empty(nobj * (k + m), dtype=torch.int32, device="cuda")
hsum = torch.empty_like(sums)
for erased, data_only, heal, label in (([], True, False, "GET, all data shards present: verify 8"),
                                       ([0, 5], True, False, "GET, data 0+5 lost: verify 8 + rebuild 2"),
                                       ([2, 10], False, True, "heal 1 data + 1 parity: verify 8, rebuild+hash 2")):
    pres = [i not in erased for i in range(k + m)]
    ms = timeit(lambda: codec.verify_reconstruct_batch(buf, stride, S, nobj, pres, data_only, sums, vbad,
                                                       sums_out=hsum if heal else None))
    e = len(erased)
    ab = nobj * (k * S + e * S + 32 * k + (32 * e if heal else 0))
    out(path="verify_reconstruct", shape="RS(8+4)", objects=nobj, what=label, ms=round(ms, 4),
        GiBps_object=round(nobj * blen / ms / 1e-3 / 2**30, 1), hbm_GBps=round(ab / ms / 1e6, 1),
        hbm_frac=round(ab / ms / 1e6 / 8000, 3), bad=int(vbad.sum()))

# ---- GET-side hash-only and verify over all 12 shards of every stripe
ms = timeit(lambda: z.hh256_batch(buf, S, S, nobj * (k + m), sums))
out(path="hh256_batch", msgs=nobj * (k + m), msg_len=S, ms=round(ms, 4),
    hbm_GBps=round(nobj * (k + m) * S / ms / 1e6, 1))
bad = torch.empty(nobj * (k + m), dtype=torch.int32, device="cuda")
ms = timeit(lambda: z.hh256_verify_batch(buf, S, S, nobj * (k + m), sums, bad))
out(path="hh256_verify_batch", msgs=nobj * (k + m), msg_len=S, ms=round(ms, 4),
    hbm_GBps=round(nobj * (k + m) * S / ms / 1e6, 1), bad=int(bad.sum()))
# ---- PUT-stream object digests: S3 ETag (MD5) and content SHA-256
# of 4096 x 1 MiB device-resident objects, one lane per object (serial chains)
for name, fn, width in (("md5_batch", z.md5_batch, 16), ("sha256_batch", z.sha256_batch, 32)):
    dout = torch.empty(nobj * width, dtype=torch.uint8, device="cuda")
    ms = timeit(lambda: fn(buf, stride, blen, nobj, dout), steps=3)
    out(path=name, objects=nobj, object_bytes=blen, ms=round(ms, 3),
        GiBps=round(nobj * blen / ms / 1e-3 / 2**30, 1))
import hashlib  # noqa: E402
sample = np.frombuffer(os.urandom(64 << 20), dtype=np.uint8)
for name, h in (("md5_cpu_1thread", hashlib.md5), ("sha256_cpu_1thread", hashlib.sha256)):
    t0 = time.perf_counter()
    h(sample.tobytes()).digest()
    dt = time.perf_counter() - t0
    out(path=name, bytes=len(sample), GiBps=round(len(sample) / dt / 2**30, 2))
del buf, sums, bad
torch.cuda.empty_cache()

# ---- config 5: end-to-end stream incl. pinned / pageable host buffers and PCIe
gib = float(os.environ.get("E2E_GIB", "10"))
for (k, m) in ((16, 4), (8, 4)):
    bs = 1 << 20
    total = int(gib * (1 << 30))
    nblk = total // bs
    S = bs // k
    codec = z.Codec(k, m, bs)
    for pinned in (True, False):
        if pinned:
            src, par, sums = z.HostBuffer(total), z.HostBuffer(nblk * m * S), z.HostBuffer(nblk * (k + m) * 32)
            src.array[:] = 7
        else:
            src = np.full(total, 7, dtype=np.uint8)
            par = np.zeros(nblk * m * S, np.uint8)
            sums = np.zeros(nblk * (k + m) * 32, np.uint8)
        codec.stream_encode(src, 64 * bs, par, sums, batch_blocks=64)  # warm
        t0 = time.perf_counter()
        codec.stream_encode(src, total, par, sums, batch_blocks=512)
        dt = time.perf_counter() - t0
        out(path="stream_encode_e2e", shape=f"RS({k}+{m})", GiB=gib, host_buffers="pinned" if pinned else "pageable",
            seconds=round(dt, 3), GiBps=round(total / dt / 2**30, 2),
            pcie_GBps=round((total + nblk * (m * S + 32 * (k + m))) / dt / 1e9, 1))
        if pinned:
            for x in (src, par, sums):
                x.free()
        del src, par, sums
