"""Batch-size sweep of the fused encode + HighwayHash-256 launch (one device, one process).

For every batch size n and every launch shape (variant 0 = product default dispatch;
others forced through the diagnostics build), interleaved rounds: median kernel time
of `reps` back-to-back launches (HIP events on the launch stream), GiB/s of object
bytes and the fraction of the 8 TB/s HBM spec the algorithmic bytes reach.

  SIZES=256,512,...  VARIANTS=0,105,130,131,132,5  K=8 M=4  python scripts/sweep_sizes.py
One JSON line per (round, n, variant).
"""
import contextlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

k = int(os.environ.get("K", "8"))
m = int(os.environ.get("M", "4"))
sizes = [int(x) for x in os.environ.get("SIZES", "256,512,1000,1024,2047,2048,3001,4096,8192,16384").split(",")]
variants = [int(x) for x in os.environ.get("VARIANTS", "0").split(",")]
rounds = int(os.environ.get("ROUNDS", "3"))
# ALIAS=1: every block reads stripe 0 and writes its parity there (data_stride =
# parity_stride = 0): the same instruction stream with the bytes L2-resident, i.e.
# the launch's compute-bound time (timing only; output is meaningless)
alias = os.environ.get("ALIAS", "0") == "1"
reps = int(os.environ.get("REPS", "10"))
B = 1 << 20
S = B // k
R = k + m
abytes = B + m * S + 32 * R

nmax = max(sizes)
buf = torch.empty(nmax * R * S, dtype=torch.uint8, device="cuda")
sums = torch.empty(nmax * R * 32, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, R * S, B, nmax, seed=7)
torch.cuda.synchronize()
codecs = {}


def ctx(v):
    return contextlib.nullcontext() if v == 0 else z.diag(v)


for rnd in range(rounds):
    for n in sizes:
        for v in variants:
            with ctx(v):
                key = (v != 0)
                if key not in codecs:
                    codecs[key] = z.Codec(k, m, B)
                c = codecs[key]
                st = torch.cuda.current_stream()
                bs = 0 if alias else R * S
                for _ in range(2):
                    c.encode_batch(buf, bs, B, n, parity=buf, parity_offset=k * S, parity_stride=bs, sums=sums)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
                for a, b in ev:
                    a.record(st)
                    c.encode_batch(buf, bs, B, n, parity=buf, parity_offset=k * S, parity_stride=bs, sums=sums)
                    b.record(st)
                torch.cuda.synchronize()
                path = z.last_path()
            ts = sorted(a.elapsed_time(b) for a, b in ev)
            ms = ts[len(ts) // 2]
            print(json.dumps({"round": rnd, "k": k, "m": m, "n": n, "variant": v, "alias": alias, "path": path,
                              "ms": round(ms, 4),
                              "min_ms": round(ts[0], 4), "GiBps": round(n * B / ms / 1e-3 / 2**30, 1),
                              "frac": round(n * abytes / (ms * 1e-3) / 8e12, 4)}), flush=True)
