"""One RS(12+4) 4096 x 1 MiB GET (rebuild 2) launch series for a PMC pass."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import zs3server_amd as z  # noqa: E402
MiB = 1 << 20
k, m, nb = 12, 4, 4096
R = k + m
S = -(-MiB // k)
buf = torch.empty(nb * R * S, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, R * S, MiB, nb, seed=3)
sums = torch.empty(nb * R * 32, dtype=torch.uint8, device="cuda")
c = z.Codec(k, m, MiB)
c.encode_batch(buf, R * S, MiB, nb, parity=buf, parity_offset=k * S, parity_stride=R * S, sums=sums)
bad = torch.empty(nb * R, dtype=torch.int32, device="cuda")
for _ in range(4):
    c.verify_reconstruct_batch(buf, R * S, S, nb, [i not in (0, 5) for i in range(R)], True, sums, bad)
torch.cuda.synchronize()
