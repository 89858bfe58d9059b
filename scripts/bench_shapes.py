"""Encode + bitrot and GET timings for the server's default geometries and the BASELINE
shapes: getDefaultParityBlocks gives RS(12+4) for 16-drive sets and
RS(4+4) for 8-drive sets (cmd/format-erasure.go:870-881); the parity upgrade of
cmd/erasure-object.go:724-775 gives (11+5), (10+6), ...  Each line: device-resident
batch of 1 MiB objects, median of REPS launches (HIP events), % of 8 TB/s on the
algorithmic bytes, the kernel family that ran, and a cpu_ref check of sampled blocks.

  SHAPES=12:4:4096,4:4:4096 python scripts/bench_shapes.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402
from oracle import cpuref, oracle_c  # noqa: E402

MiB = 1 << 20
REPS = int(os.environ.get("REPS", "10"))
SHAPES = [tuple(int(x) for x in t.split(":")) for t in
          os.environ.get("SHAPES", "12:4:4096,4:4:4096,8:4:4096,16:4:2048,4:2:1024,11:5:4096,10:6:4096").split(",")]
KEY = z.MAGIC_HH256_KEY


def med(fn):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[REPS // 2]


for k, m, n in SHAPES:
    R = k + m
    S = -(-MiB // k)
    stride = R * S
    codec = z.Codec(k, m, MiB)
    d = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    z.fill_batch(d, stride, MiB, n, seed=3)
    sums = torch.zeros(n * R * 32, dtype=torch.uint8, device="cuda")

    def enc():
        codec.encode_batch(d, stride, MiB, n, parity=d, parity_offset=k * S, parity_stride=stride, sums=sums)

    ms = med(enc)
    path = z.last_path()
    ab = n * (MiB + m * S + 32 * R)
    # check 8 sampled blocks against cpu_ref (pinned to the oracle)
    mat = oracle_c.build_matrix(k, m)
    ok = True
    for b in np.linspace(0, n - 1, 8).astype(int).tolist():
        blk = d[b * stride:(b + 1) * stride].cpu().numpy()
        par = np.empty(m * S, np.uint8)
        sr = np.empty(R * 32, np.uint8)
        cpuref.encode_hash(k, m, mat, blk, MiB, 1, stride, par, m * S, sr, KEY, 4)
        ok &= bool(np.array_equal(blk[k * S:], par)) and bool(np.array_equal(sums[b * R * 32:(b + 1) * R * 32].cpu().numpy(), sr))
    print(json.dumps({"what": "encode_hash", "k": k, "m": m, "objects": n, "S": S, "ms": round(ms, 4),
                      "frac": round(ab / (ms * 1e-3) / 8e12, 4), "path": path, "ok": ok}), flush=True)
    # GET: verify k survivors + rebuild 2 data rows; heal 2 (1 data + 1 parity)
    bad = torch.zeros(n * R, dtype=torch.int32, device="cuda")
    hs = torch.zeros_like(sums)
    for erased, data_only, heal in (([0, 1], True, False), ([1, k], False, True)):
        pres = [i not in erased for i in range(R)]
        e = len(erased)
        ms = med(lambda: codec.verify_reconstruct_batch(d, stride, S, n, pres, data_only, sums, bad,
                                                        sums_out=hs if heal else None))
        ab = n * (k * S + e * S + 32 * k + (32 * e if heal else 0))
        print(json.dumps({"what": "heal" if heal else "get", "k": k, "m": m, "objects": n, "erased": erased,
                          "ms": round(ms, 4), "frac": round(ab / (ms * 1e-3) / 8e12, 4), "path": z.last_path(),
                          "bad": int(bad.sum())}), flush=True)
    del d, sums, bad, hs
    torch.cuda.empty_cache()
