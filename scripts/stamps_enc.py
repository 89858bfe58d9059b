"""Per-wave stamps of the headline encode + bitrot kernel (k_ehx_ws<8, 4, Rs84Bulk> built
with WT: diagnostics variant 313): for every wave its lifetime, shader
clock, hardware SIMD, and the share of its cycles spent in the per-step workgroup barrier
and (encode waves) waiting for its tile's loads.  Summarised per wave slot of the
12-wave workgroup (slots 0-5 hash, 6-11 encode) and per (role mix, SIMD), so it says which
role paces a step under the XCD-region order: the pacing waves are the ones that wait
least at the barrier.

  NOBJ=65536 VARIANTS=313 python scripts/stamps_enc.py
(VARIANTS: stamped instances; WPW / NHW: waves per workgroup and hash waves; G: stripes
per workgroup of the instance)
"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k, m = (int(x) for x in os.environ.get("SHAPE", "8:4").split(":"))
blen = 1 << 20
S = -(-blen // k)
stride = (k + m) * S
G = int(os.environ.get("G", "16"))
WPW = int(os.environ.get("WPW", "12"))
NHW = int(os.environ.get("NHW", "6"))
ALIAS = os.environ.get("STAMP_ALIAS", "0") == "1"  # every block reads stripe 0 (L2-resident)
for nobj in [int(x) for x in os.environ.get("NOBJ", "65536").split(",")]:
    buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
    sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
    z.fill_batch(buf, stride, blen, nobj, seed=5)
    st = 0 if ALIAS else stride
    nwg = -(-nobj // G)
    dbg = torch.zeros(nwg * WPW * 5, dtype=torch.int64, device="cuda")
    for v in [int(x) for x in os.environ.get("VARIANTS", "313").split(",")]:
        with z.diag(v):
            codec = z.Codec(k, m)
            run = lambda: codec.encode_batch(buf, st, blen, nobj, parity=buf, parity_offset=k * S,  # noqa: E731
                                             parity_stride=st, sums=sums)
            z.set_debug_buffer(None)
            for _ in range(5):
                run()
            dbg.zero_()
            z.set_debug_buffer(dbg)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            z.set_debug_buffer(None)
            path = z.last_path()
        ms = e0.elapsed_time(e1)
        d = dbg.view(-1, 5).cpu()
        live = d[:, 1] > 0
        idx = torch.nonzero(live).flatten()
        rows = d[live]
        rt0, rt1, cyc = rows[:, 0].double(), rows[:, 1].double(), rows[:, 2].double()
        wbar = ((rows[:, 4] >> 8) & 0xFFFFFFF).double()
        wvm = (rows[:, 4] >> 36).double()
        hw = rows[:, 3].long()
        simd = ((hw >> 4) & 0x3).tolist()
        pos = (idx % WPW).tolist()
        clk = cyc / ((rt1 - rt0) / 100.0) / 1e3  # GHz (s_memrealtime ticks at 100 MHz)
        out = {"k": k, "m": m, "objects": nobj, "variant": v, "alias": ALIAS, "ms": round(ms, 4), "path": path,
               "waves": int(live.sum()), "waves_per_wg": WPW, "hash_waves": NHW,
               "clock_GHz": round(float(clk.median()), 3),
               "life_us_median": round(float(((rt1 - rt0) / 100.0).median()), 1)}
        per = []
        for p in range(WPW):
            sel = torch.tensor([q == p for q in pos])
            if sel.any():
                sims = sorted(set(s for s, q in zip(simd, pos) if q == p))
                per.append({"wave": p, "role": "hash" if p < NHW else "encode", "simd": sims,
                            "bar_frac": round(float((wbar[sel] / cyc[sel]).mean()), 4),
                            "load_frac": round(float((wvm[sel] / cyc[sel]).mean()), 4)})
        out["per_wave"] = per
        # the mix of roles on each SIMD of a workgroup (hash / encode waves) and the mean
        # barrier fraction of each role on SIMDs of that mix
        wg = (idx // WPW).tolist()
        mix = defaultdict(lambda: [0, 0])
        for w, p, s in zip(wg, pos, simd):
            mix[(w, s)][0 if p < NHW else 1] += 1
        agg = defaultdict(list)
        for i, (w, p, s) in enumerate(zip(wg, pos, simd)):
            h, e = mix[(w, s)]
            agg[(f"{h}H+{e}E", "hash" if p < NHW else "encode")].append(float(wbar[i] / cyc[i]))
        out["by_simd_mix"] = [{"mix": a, "role": r, "waves": len(x), "bar_frac": round(sum(x) / len(x), 4)}
                              for (a, r), x in sorted(agg.items())]
        # SIMD balance of the CU's resident waves (several workgroups per CU): per CU, the
        # wave-time each SIMD hosted; max / mean over the CU's 4 SIMDs (1.0 = balanced)
        cu = ((rows[:, 4] & 0xF) << 8 | ((hw >> 13) & 0x7) << 5 | ((hw >> 12) & 0x1) << 4 | ((hw >> 8) & 0xF)).tolist()
        life = ((rt1 - rt0) / 100.0).tolist()
        per_cu = defaultdict(lambda: [0.0, 0.0, 0.0, 0.0])
        for c, s_, lt in zip(cu, simd, life):
            per_cu[c][s_] += lt
        imb = sorted(max(v) / (sum(v) / 4) for v in per_cu.values() if sum(v) > 0)
        out["simd_time_imbalance_q10_50_90"] = [round(imb[int(q * (len(imb) - 1))], 4) for q in (0.1, 0.5, 0.9)]
        out["cus"] = len(per_cu)
        print(json.dumps(out), flush=True)
    del buf, sums, dbg
    torch.cuda.empty_cache()
