#!/usr/bin/env python3
"""Benchmark: device-resident RS(8+4) encode + HighwayHash-256 bitrot, 1 MiB blocks.

Metric (BASELINE.json): GiB/s of input object bytes, device-resident, at 1/2/4/8 GPUs.
A "step" = one pass of the hot path (zs3_encode_batch: Split + Encode + k+m HH256
sums, fused) over one batch of `--objects` 1 MiB blocks already resident in HBM
(BASELINE config 3's batch: 4096 objects per GPU).  Objects are independent: each
rank encodes its own batch (disjoint object ids), no data-path collective; gloo is
used only for the timing barrier and the max-over-ranks reduction -> "scaling": "weak".

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 TB/s measured copy)
KEY = bytes.fromhex("4be734fa8e238acd263e83e6bb968552040f935da39f441497e09d1322de36a0")


def algo_bytes_per_block(k: int, m: int, blen: int) -> int:
    """B + B*m/k + 32*(k+m): data read + parity written + sums written."""
    S = -(-blen // k)
    return blen + m * S + 32 * (k + m)


def cpu_baseline(k: int, m: int, blen: int, seconds: float, threads: int) -> dict:
    """C++ restatement of the reference CPU encode structure (oracle/cpu_ref.cpp):
    per block Split -> Encode split over T threads -> k+m HH256; blocks sequential."""
    import numpy as np

    from oracle import oracle_c

    so = os.path.join(ROOT, "oracle", "libcpuref.so")
    if not os.path.exists(so):
        oracle_c.build()
    L = C.CDLL(so)
    L.cpuref_isa.restype = C.c_char_p
    L.cpuref_encode_hash.restype = C.c_int64
    L.cpuref_encode_hash.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                     C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int]
    mat = oracle_c.build_matrix(k, m)
    S = -(-blen // k)
    nb = 64  # BASELINE config 1 sample size: 64 x 1 MiB
    data = np.concatenate([oracle_c.fill(0, b, blen) for b in range(nb)])
    par = np.zeros(nb * m * S, dtype=np.uint8)
    sums = np.zeros(nb * (k + m) * 32, dtype=np.uint8)
    kb = C.create_string_buffer(KEY, 32)

    def run(T):
        reps, t0 = 0, time.perf_counter()
        while True:
            L.cpuref_encode_hash(k, m, mat.ctypes.data, data.ctypes.data, blen, nb, blen, par.ctypes.data,
                                 m * S, sums.ctypes.data, kb, T)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                return reps * nb * blen / dt / 2 ** 30, reps

    v1, r1 = run(1)
    vt, rt = run(threads) if threads > 1 else (v1, r1)
    best_t, best_v = (threads, vt) if vt >= v1 else (1, v1)
    return {
        "value": round(best_v, 3), "unit": "GiB/s", "cores": best_t, "kind": "port",
        "sample": f"RS({k}+{m}) encode+HH256 of {nb} x {blen} B blocks (seed 0), blocks sequential, "
                  f"repeated ~{seconds:.0f}s per thread count; C++ restatement of klauspost/reedsolomon "
                  f"v1.11.8 + minio/highwayhash v1.0.2 structure ({L.cpuref_isa().decode()}); "
                  f"T=1: {v1:.3f} GiB/s, T={threads}: {vt:.3f} GiB/s",
    }


def committed_traffic(k: int, m: int, nobj: int, blen: int):
    """Per-launch HBM bytes measured by scripts/profile_round.sh (two rocprofv3 PMC
    passes, FETCH_SIZE doubled per the gfx950 correction) for this workload, if the
    committed profile was taken on the same shape."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        for name, v in d.items():
            if f"<{k}, {m}," in name and v.get("workload", {}).get("objects", nobj) == nobj:
                best = (v["hbm_bytes_per_launch"], os.path.relpath(path, ROOT))
    return best if best else (None, None)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--objects", type=int, default=4096, help="1 MiB blocks per GPU per step")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per launch from a rocprofv3 PMC pass; default: the committed "
                         "profiles/*/pmc_traffic.json entry for the kernel that runs, if any")
    args = ap.parse_args()

    from zs3server_amd.dist import max_over_ranks, object_range, rank_env

    world, rank, local = rank_env()
    if world > 1:
        dist.init_process_group("gloo")  # control only: barrier + max of timings
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import zs3server_amd as z

    k, m, blen, nobj = args.k, args.m, args.block, args.objects
    S = -(-blen // k)
    stride = (k + m) * S  # reference in-place layout: [k data rows | m parity rows] per block
    codec = z.Codec(k, m, blen)
    buf = torch.empty(nobj * stride, dtype=torch.uint8, device=dev)
    sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device=dev)
    obj_lo, _ = object_range(rank, nobj)  # disjoint object ids per rank
    z.fill_batch(buf, stride, blen, nobj, seed=1234, obj0=obj_lo)
    torch.cuda.synchronize()

    def step():
        codec.encode_batch(buf, stride, blen, nobj, parity=buf, parity_offset=k * S,
                           parity_stride=stride, sums=sums)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    fast = z.last_path()

    elapsed, kern_ms = max_over_ranks([elapsed, kern_ms], world)

    traffic, traffic_src = args.traffic, None
    if traffic is None:
        traffic, traffic_src = committed_traffic(k, m, nobj, blen)

    total_bytes = world * nobj * blen * args.steps
    value = total_bytes / elapsed / 2 ** 30
    abytes = nobj * algo_bytes_per_block(k, m, blen)
    achieved = abytes / (kern_ms * 1e-3) / 1e9
    if rank == 0:
        out = {
            "metric": f"GiB/s device-resident RS({k}+{m}) encode+bitrot, 1 MiB blocks, at 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 counter stream per object id), device-resident in HBM",
            "config": {"workload": f"RS({k}+{m}) Split+Encode+HighwayHash256S bitrot sums of {nobj} x {blen} B "
                                   f"blocks per GPU, in-place bpool layout (BASELINE config 3 batch)",
                       "objects_per_gpu": nobj, "block_bytes": blen, "k": k, "m": m,
                       "parallelism": f"objects partitioned over {world} GPU(s), no collectives",
                       "kernel_path": "specialised" if fast == 1 else "generic"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel_ms": round(kern_ms, 4),
                         "algo_bytes_per_launch": abytes},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(k, m, blen, args.cpu_seconds,
                                               min(args.cpu_threads, os.cpu_count() or 1))
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
