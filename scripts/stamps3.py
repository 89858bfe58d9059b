"""Per-wave lifetime, in-kernel clock and placement (CU / XCD) of a fused_v2 variant.
Usage: VARIANT=50 python scripts/stamps3.py"""
import os
import sys
from collections import Counter

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
# STAMP_ALIAS=1: strides 0 (every block reads stripe 0: L2-resident, compute-bound)
ALIAS = os.environ.get("STAMP_ALIAS", "0") == "1"
st = 0 if ALIAS else stride
G = 4
nwave = nobj // G * 3
dbg = torch.zeros(nwave * 5, dtype=torch.int64, device="cuda")
for v in [int(x) for x in os.environ.get("VARIANTS", "50").split(",")]:
    ctx = z.diag(v)
    ctx.__enter__()
    codec = z.Codec(k, m)  # a codec belongs to the library that made it
    z.set_debug_buffer(None)
    for _ in range(3):
        codec.encode_batch(buf, st, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=st, sums=sums)
    dbg.zero_()
    z.set_debug_buffer(dbg)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    codec.encode_batch(buf, st, blen, nobj, parity=buf, parity_offset=k * S, parity_stride=st, sums=sums)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    d = dbg.view(-1, 5).cpu()
    wid = torch.arange(d.shape[0]) % 12  # wave index within a 12-wave workgroup
    wid = wid[d[:, 1] > 0]
    d = d[d[:, 1] > 0]
    rt0, rt1, cyc = d[:, 0].double(), d[:, 1].double(), d[:, 2].double()
    life = (rt1 - rt0) / 100.0
    start = (rt0 - rt0.min()) / 100.0
    end = (rt1 - rt0.min()) / 100.0
    clk = cyc / (rt1 - rt0) * 100e6 / 1e9
    hw = d[:, 3].long()
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    xcc = d[:, 4].long() & 0xF
    q = torch.tensor([0, 0.1, 0.5, 0.9, 1.0], dtype=torch.float64)
    print(f"variant {v}{' (alias)' if ALIAS else ''}: kernel {ms:.3f} ms, waves {d.shape[0]}")
    print("  lifetime us q0/10/50/90/100:", [round(float(x), 1) for x in torch.quantile(life, q)])
    print("  start us   q0/10/50/90/100:", [round(float(x), 1) for x in torch.quantile(start, q)])
    print("  end us     q0/10/50/90/100:", [round(float(x), 1) for x in torch.quantile(end, q)])
    print("  clock GHz  q0/10/50/90/100:", [round(float(x), 3) for x in torch.quantile(clk, q)])
    cukey = [(int(a), int(b), int(c), int(e)) for a, b, c, e in zip(xcc, se, sh, cu)]
    per_cu = Counter(cukey)
    print("  waves per CU histogram:", sorted(Counter(per_cu.values()).items()))
    simdkey = Counter([(a, b, c, e, int(f)) for (a, b, c, e), f in zip(cukey, simd)])
    print("  waves per SIMD histogram:", sorted(Counter(simdkey.values()).items()))
    print("  (wave index in a 12-wave workgroup, SIMD) counts:", sorted(Counter(zip(wid.tolist(), simd.tolist())).items())[:24])
    wait = ((d[:, 4] >> 8) & 0xFFFFFFF).double()  # barrier-wait shader cycles (variants built with WT)
    vwait = (d[:, 4] >> 36).double()  # encode role: cycles waiting for its tile's loads (WT)
    for r in range(12):
        sel = wid == r
        if sel.any():
            print(f"  wave {r:2d}: life mean {float(life[sel].mean()):.1f} us, clock {float(clk[sel].mean()):.3f} GHz, "
                  f"barrier wait {float((wait[sel] / cyc[sel]).mean()) * 100:.1f} %, load wait "
                  f"{float((vwait[sel] / cyc[sel]).mean()) * 100:.1f} % of cycles")
    for x in sorted(set(int(t) for t in xcc)):
        sel = xcc == x
        print(f"  xcc {x}: waves {int(sel.sum())} life mean {float(life[sel].mean()):.1f} end max {float(end[sel].max()):.1f}")
    # lifetime vs waves on the wave's CU
    load = torch.tensor([per_cu[k_] for k_ in cukey], dtype=torch.float64)
    for n in sorted(set(int(t) for t in load)):
        sel = load == n
        print(f"  CUs with {n} waves: wave life mean {float(life[sel].mean()):.1f} us")
    z.set_debug_buffer(None)
    ctx.__exit__(None, None, None)
