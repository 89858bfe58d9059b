"""Where a single queued 1 MiB RS(8+4) block's latency goes: the device launch alone
(n blocks already in HBM, HIP events), pinned H2D / D2H of the block, and the queue's
encode_data round trip at 1 submitter.  One JSON line per measurement."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

MiB = 1 << 20
k, m = 8, 4
S = MiB // k
R = k + m
codec = z.Codec(k, m)
buf = torch.empty(64 * R * S, dtype=torch.uint8, device="cuda")
sums = torch.empty(64 * R * 32, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, R * S, MiB, 64, seed=1)
st = torch.cuda.current_stream()
for n in (1, 2, 4, 8, 16, 64):
    ts = []
    for _ in range(12):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        codec.encode_batch(buf, R * S, MiB, n, parity=buf, parity_offset=k * S, parity_stride=R * S, sums=sums)
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    print(json.dumps({"what": "encode_batch launch", "blocks": n, "us_p50": round(ts[6] * 1e3, 1),
                      "path": z.last_path()}), flush=True)
h = torch.empty(MiB, dtype=torch.uint8).pin_memory()
d = torch.empty(MiB, dtype=torch.uint8, device="cuda")
for what, fn in (("H2D 1 MiB pinned", lambda: d.copy_(h, non_blocking=True)),
                 ("D2H 1 MiB pinned", lambda: h.copy_(d, non_blocking=True))):
    ts = []
    for _ in range(12):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(json.dumps({"what": what, "us_p50": round(ts[6] * 1e6, 1)}), flush=True)
q = z.Queue(codec, max_batch=128, max_wait_us=200)
blk = np.zeros(R * S, np.uint8)
blk[:MiB] = np.frombuffer(os.urandom(MiB), np.uint8)
ts = []
for _ in range(40):
    t0 = time.perf_counter()
    q.encode_data(blk, MiB)
    ts.append(time.perf_counter() - t0)
ts.sort()
print(json.dumps({"what": "queue encode_data, 1 submitter", "us_p50": round(ts[20] * 1e6, 1),
                  "us_min": round(ts[0] * 1e6, 1)}), flush=True)
t0 = time.perf_counter()
for _ in range(20):
    blk2 = blk.copy()
dt = (time.perf_counter() - t0) / 20
print(json.dumps({"what": "host memcpy 1.5 MiB pageable", "us": round(dt * 1e6, 1)}), flush=True)
q.close()
