"""Per-phase cycle breakdown of the fused kernel (diagnostic stamped variants)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k, m, blen, nobj = 8, 4, 1 << 20, 4096
S = blen // k
stride = (k + m) * S
codec = z.Codec(k, m)
buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, stride, blen, nobj, seed=5)
for v in [int(x) for x in os.environ.get('STAMP_VARIANTS', '17,24').split(',')]:
    dbg = torch.zeros(1024 * 8 * 5, dtype=torch.int64, device="cuda")
    z.set_debug_buffer(dbg)
    z.set_variant(v)
    for _ in range(3):
        codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
    e1.record()
    torch.cuda.synchronize()
    d = dbg.view(-1, 5).double()
    d = d[d.sum(1) > 0]
    mean = d.mean(0).tolist()
    tot = sum(mean)
    names = ["encode+store", "prefetch-issue", "barrier1", "hash", "barrier2"]
    print(f"variant {v}: {e0.elapsed_time(e1):.3f} ms, waves={d.shape[0]}, mean cycles/wave total={tot:.3e}")
    for n, x in zip(names, mean):
        print(f"   {n:15s} {x:12.4g} cycles  {100*x/tot:5.1f}%")
z.set_debug_buffer(None)
z.set_variant(0)
