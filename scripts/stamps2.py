"""Residency/clock check for the stamped pipelined variant (24)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k, m, blen, nobj = 8, 4, 1 << 20, int(os.environ.get("NOBJ", "4096"))
S = blen // k
stride = (k + m) * S
codec = z.Codec(k, m)
buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, stride, blen, nobj, seed=5)
dbg = torch.zeros(nobj // 4 * 8 * 5, dtype=torch.int64, device="cuda")
z.set_debug_buffer(dbg)
z.set_variant(24)
for _ in range(3):
    codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
d = dbg.view(-1, 5)
d = d[d[:, 3] > 0].double()
rt_start, rt_end, cyc = d[:, 1], d[:, 3], d[:, 4]
life_us = (rt_end - rt_start) / 100.0
span_us = (rt_end.max() - rt_start.min()).item() / 100.0
clk = (cyc / (rt_end - rt_start) * 100e6 / 1e9)
st = (rt_start - rt_start.min()) / 100.0
print(f"kernel {ms:.3f} ms; stamp span {span_us:.1f} us; waves {d.shape[0]}")
print(f"wave lifetime us: min {life_us.min():.1f} mean {life_us.mean():.1f} max {life_us.max():.1f}")
print(f"clock GHz: mean {clk.mean():.3f} min {clk.min():.3f} max {clk.max():.3f}")
print(f"start offset us: quantiles {[round(float(x),1) for x in torch.quantile(st, torch.tensor([0,0.25,0.5,0.75,0.9,1.0],dtype=torch.float64))]}")
z.set_debug_buffer(None)
z.set_variant(0)
