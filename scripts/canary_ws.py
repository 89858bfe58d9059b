import os, sys
sys.path.insert(0, "/root/repo") if os.path.exists("/root/repo") else None
import torch
import zs3server_amd as z
k, m, blen = 8, 4, 1 << 20
S = blen // k; stride = (k + m) * S
codec = z.Codec(k, m)
for nobj in (33, 4096):
    for v in (100, 102, 103, 104):
        guard = 1 << 22
        big = torch.full((guard + nobj * stride + guard,), 0x5A, dtype=torch.uint8, device="cuda")
        buf = big[guard: guard + nobj * stride]
        sums = torch.zeros(nobj * (k + m) * 32 + 4096, dtype=torch.uint8, device="cuda")
        z.fill_batch(buf, stride, blen, nobj, seed=5)
        dbg = torch.zeros(nobj // 16 * 12 * 5 + 64, dtype=torch.int64, device="cuda")
        z.set_variant(v)
        z.set_debug_buffer(dbg)
        codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
        torch.cuda.synchronize()
        z.set_debug_buffer(None)
        g0 = int((big[:guard] != 0x5A).sum()); g1 = int((big[guard + nobj * stride:] != 0x5A).sum())
        st = int((sums[nobj * (k + m) * 32:] != 0).sum())
        d = dbg.view(-1)[: nobj // 16 * 12 * 5].view(-1, 5).cpu()
        bad = int(((d[:, 1] - d[:, 0]) <= 0).sum()) if nobj % 16 == 0 else -1
        print(f"nobj {nobj} v{v}: guard_lo {g0} guard_hi {g1} sums_tail {st} dbg_bad {bad} sig {int(buf.view(torch.int64).sum())} {int(sums.view(torch.int64).sum())}", flush=True)
        del big, buf, sums, dbg
z.set_variant(0)
