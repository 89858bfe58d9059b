#!/bin/bash
# RS(12+4) UA GET / heal shapes: product vs 264 / 267, 4096 x 1 MiB, e = 1..4, heal 1..4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u - > $OUT/get_ab_rs124.jsonl 2>$OUT/getab.err <<'PY' || { tail $OUT/getab.err; exit 3; }
import json, contextlib, torch, zs3server_amd as z
MiB = 1 << 20
k, m, nb = 12, 4, 4096
R = k + m; S = -(-MiB // k)
buf = torch.empty(nb * R * S, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, R * S, MiB, nb, seed=3)
sums = torch.empty(nb * R * 32, dtype=torch.uint8, device="cuda")
z.Codec(k, m, MiB).encode_batch(buf, R * S, MiB, nb, parity=buf, parity_offset=k * S, parity_stride=R * S, sums=sums)
bad = torch.empty(nb * R, dtype=torch.int32, device="cuda"); hs = torch.empty_like(sums)
cases = [([3], False), ([0, 5], False), ([1, 7, 13], False), ([0, 1, 2, 3], False),
         ([2], True), ([1, 12], True), ([0, 6, 15], True), ([1, 2, 13, 14], True)]
for erased, heal in cases:
    for v in (0, 264, 267):
        with (z.diag(v) if v else contextlib.nullcontext()):
            c = z.Codec(k, m, MiB)
            pres = [i not in erased for i in range(R)]
            f = lambda: c.verify_reconstruct_batch(buf, R * S, S, nb, pres, not heal, sums, bad, sums_out=hs if heal else None)
            f(); torch.cuda.synchronize(); path = z.last_path()
            ok = int(bad.sum()) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): f()
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            e = len(erased) if heal else len([i for i in erased if i < k])
            ab = nb * (k * S + e * S + 32 * k + (32 * e if heal else 0))
            print(json.dumps({"erased": erased, "heal": heal, "variant": v, "ms": round(ms, 4), "frac": round(ab / ms / 1e6 / 8000, 4), "path": path, "ok": ok}), flush=True)
PY
cat $OUT/get_ab_rs124.jsonl
