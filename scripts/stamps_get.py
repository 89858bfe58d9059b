"""Per-wave stamps of the GET / heal kernel (k_vr_ws with diagnostics variant 424 = the
product shape + WT): for every wave its lifetime, shader clock, and the share of its
cycles spent in workgroup barriers and (rebuild waves) waiting for survivor loads,
summarised per role (hash waves: the first NH/64 waves of a workgroup).  Settles whether
a GET / heal instance is paced by its rebuild waves (VALU: they rarely wait, the hash
waves wait at barriers) or by memory (the rebuild waves wait for loads).

  SHAPE=16:4:2048 CASES="h0,1,16,19" WPW=11 NHW=5 python scripts/stamps_get.py
(WPW / NHW: waves per workgroup and hash waves of the instance the case runs)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

MiB = 1 << 20
k, m, n = (int(x) for x in os.environ.get("SHAPE", "16:4:2048").split(":"))
CASES = []
for c in os.environ.get("CASES", "h0,1,16,19;0,5,9,14").split(";"):
    CASES.append(([int(x) for x in c.lstrip("h").split(",")], c.startswith("h")))
R = k + m
S = -(-MiB // k)
stride = R * S
d = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
z.fill_batch(d, stride, MiB, n, seed=3)
sums = torch.zeros(n * R * 32, dtype=torch.uint8, device="cuda")
z.Codec(k, m, MiB).encode_batch(d, stride, MiB, n, parity=d, parity_offset=k * S, parity_stride=stride, sums=sums)
bad = torch.zeros(n * R, dtype=torch.int32, device="cuda")
hs = torch.zeros_like(sums)
dbg = torch.zeros(n * 16 * 5, dtype=torch.int64, device="cuda")  # >= waves of any GET launch
for erased, heal in CASES:
    pres = [i not in erased for i in range(R)]
    e = len(erased) if heal else len([i for i in erased if i < k])
    with z.diag(424):
        codec = z.Codec(k, m, MiB)
        run = lambda: codec.verify_reconstruct_batch(d, stride, S, n, pres, not heal, sums, bad,  # noqa: E731
                                                     sums_out=hs if heal else None)
        z.set_debug_buffer(None)
        for _ in range(3):
            run()
        dbg.zero_()
        z.set_debug_buffer(dbg)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        torch.cuda.synchronize()
        z.set_debug_buffer(None)
        path = z.last_path()
    ms = a.elapsed_time(b)
    st = dbg.view(-1, 5).cpu()
    live = st[:, 1] > 0
    # waves per workgroup: the launch's NT / 64; a workgroup's waves are consecutive rows
    idx = torch.nonzero(live).flatten()
    rows = st[live]
    rt0, rt1, cyc = rows[:, 0].double(), rows[:, 1].double(), rows[:, 2].double()
    wbar = ((rows[:, 4] >> 8) & 0xFFFFFFF).double()
    wvm = (rows[:, 4] >> 36).double()
    wpw = int(os.environ["WPW"])  # waves per workgroup of the instance (NT / 64)
    nhw = int(os.environ["NHW"])  # of which hash waves
    out = {"k": k, "m": m, "objects": n, "erased": erased, "heal": heal, "e": e, "ms": round(ms, 4), "path": path,
           "waves_per_wg": wpw, "hash_waves": nhw, "clock_GHz": round(float((cyc / ((rt1 - rt0) / 100.0)).mean()) / 1e3, 3)}
    # per wave-slot position inside the workgroup: barrier and load-wait fractions
    pos = idx % wpw
    per = []
    for p in range(wpw):
        sel = pos == p
        if sel.any():
            per.append({"wave": p, "role": "hash" if p < nhw else "rebuild", "bar_frac": round(float((wbar[sel] / cyc[sel]).mean()), 3),
                        "vm_frac": round(float((wvm[sel] / cyc[sel]).mean()), 3)})
    out["per_wave"] = per
    print(json.dumps(out), flush=True)
