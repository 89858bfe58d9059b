"""Driver for PMC comparisons between the stream-pattern encode-only kernel and the
fused encode+hash kernel on the headline shape (RS(8+4), 4096 x 1 MiB), 3 launches each:
  rocprofv3 --pmc <counters> -- python scripts/pmc_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k, m, nobj, blen = 8, 4, 4096, 1 << 20
S = blen // k
stride = (k + m) * S
codec = z.Codec(k, m)
buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, stride, blen, nobj, seed=5)
for v in [int(x) for x in os.environ.get("PROBE_VARIANTS", "0").split(",")]:
    z.set_variant(v)
    for _ in range(3):
        codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
        codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride)
torch.cuda.synchronize()
z.set_variant(0)
