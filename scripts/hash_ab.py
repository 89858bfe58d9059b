"""A/B of the standalone HighwayHash-256 kernel (k_hash_batch): hash and verify of the
49 152 shard rows (128 KiB) of 4096 RS(8+4) stripes, and the deep scan of 512 shard
files ([sum|chunk]* x 64), interleaved rounds.  Variant 0 = product build, others
through the diagnostics build (the non-temporal-load variant measured slower and was removed).  VARIANTS=0,223"""
import contextlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

variants = [int(v) for v in os.environ.get("VARIANTS", "0").split(",")]


def timeit(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


S, n = 131072, 4096 * 12
buf = torch.empty(n * S, dtype=torch.uint8, device="cuda")
z.fill_batch(buf, S, S, n, seed=7)
sums = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
z.hh256_batch(buf, S, S, n, sums)
bad = torch.empty(n, dtype=torch.int32, device="cuda")
shard, chunks, nfiles = 131072, 64, 512
part = shard * chunks
want = z.bitrot_shard_file_size(part, shard)
files = torch.empty(nfiles * want, dtype=torch.uint8, device="cuda")
z.fill_batch(files, want, want, nfiles, seed=9)
fbad = torch.empty(nfiles * chunks, dtype=torch.int32, device="cuda")
ffile = torch.empty(nfiles, dtype=torch.int32, device="cuda")
work = {
    "hh256_batch": (lambda: z.hh256_batch(buf, S, S, n, sums), n * (S + 32)),
    "hh256_verify_batch": (lambda: z.hh256_verify_batch(buf, S, S, n, sums, bad), n * (S + 36)),
    "bitrot_verify_file_batch": (lambda: z.bitrot_verify_file_batch(files, want, nfiles, want, part, shard, fbad,
                                                                     ffile), nfiles * (want + 4 * chunks + 4)),
}
for rnd in range(3):
    for name, (fn, nbytes) in work.items():
        for v in variants:
            with (contextlib.nullcontext() if v == 0 else z.diag(v)):
                ms = timeit(fn)
            print(json.dumps({"round": rnd, "path": name, "variant": v, "ms": round(ms, 4),
                              "frac": round(nbytes / ms / 1e-3 / 8e12, 4)}), flush=True)
