"""Serial-chain latency floor: hh256_batch over n messages of S bytes (one chain each)
and the encode launch at small batch sizes per variant (diagnostics build).  Median of
REPS launches, HIP events."""
import contextlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

MiB = 1 << 20


def med(fn, reps=9):
    st = torch.cuda.current_stream()
    fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[reps // 2] * 1e3


S = 128 << 10
buf = torch.empty(4096 * S, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, S, S, 4096, seed=3)
out = torch.empty(4096 * 32, dtype=torch.uint8, device="cuda")
for n in (1, 12, 96, 768, 3072):
    us = med(lambda: z.hh256_batch(buf, S, S, n, out))
    print(json.dumps({"what": "hh256_batch", "messages": n, "bytes": S, "us": round(us, 1),
                      "ns_per_packet": round(us * 1e3 / (S / 32), 1)}), flush=True)
k, m = 8, 4
R, Sh = k + m, MiB // k
eb = torch.empty(256 * R * Sh, dtype=torch.uint8, device="cuda")
sums = torch.empty(256 * R * 32, dtype=torch.uint8, device="cuda")
z.fill_batch(eb, R * Sh, MiB, 256, seed=4)
codecs = {}
for v in [int(x) for x in os.environ.get("VARIANTS", "0,5,30,31,32,33,34,131,132").split(",")]:
    with (contextlib.nullcontext() if v == 0 else z.diag(v)):
        c = codecs.setdefault(v != 0, z.Codec(k, m))
        for n in (1, 16, 64, 256):
            us = med(lambda: c.encode_batch(eb, R * Sh, MiB, n, parity=eb, parity_offset=k * Sh,
                                            parity_stride=R * Sh, sums=sums))
            print(json.dumps({"what": "encode_batch", "variant": v, "blocks": n, "us": round(us, 1),
                              "path": z.last_path()}), flush=True)
