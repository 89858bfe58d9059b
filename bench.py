#!/usr/bin/env python3
"""Benchmark: device-resident RS(8+4) encode + HighwayHash-256 bitrot, 1 MiB blocks.

Metric (BASELINE.json): GiB/s of input object bytes, device-resident, at 1/2/4/8 GPUs.
Workload (BASELINE config 4): a 64 GiB stream of 65 536 independent 1 MiB objects,
partitioned contiguously over the N GPUs (zs3server_amd.dist.split_range; 65 536 /
32 768 / 16 384 / 8 192 objects per GPU at N = 1 / 2 / 4 / 8), each GPU's share
resident in HBM in the reference's in-place layout ([k data | m parity] rows per
block, 1.5 MiB per object).  A "step" = one pass of the hot path over the share: one
zs3_encode_batch launch doing Split + Encode + the k+m HighwayHash-256 bitrot sums of
every block (cmd/erasure-coding.go:77-91 + cmd/bitrot-streaming.go:47-49, fused).
Total work is fixed as N grows -> "scaling": "strong".  No data-path collective: gloo
carries only the timing barrier and the max-over-ranks reduction.  --objects N
switches to weak scaling (N objects per GPU).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU).
"""
from __future__ import annotations

import argparse
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


def _cpu_rate(k: int, m: int, blen: int, nb: int, seconds: float, threads: int) -> float:
    """GiB/s of object bytes of oracle/cpu_ref.cpp over nb blocks (seed 0), repeated
    for ~`seconds`."""
    import numpy as np

    from oracle import cpuref, oracle_c

    mat = oracle_c.build_matrix(k, m)
    S = -(-blen // k)
    data = np.concatenate([oracle_c.fill(0, b, blen) for b in range(nb)])
    par = np.zeros(nb * m * S, dtype=np.uint8)
    sums = np.zeros(nb * (k + m) * 32, dtype=np.uint8)
    reps, t0 = 0, time.perf_counter()
    while True:
        cpuref.encode_hash(k, m, mat, data, blen, nb, blen, par, m * S, sums, KEY, threads)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return reps * nb * blen / dt / 2 ** 30


def cpu_baseline(k: int, m: int, blen: int, seconds: float) -> dict:
    """C++ restatement of the reference CPU encode structure (oracle/cpu_ref.cpp): per
    block Split -> Encode split over T threads -> k+m HH256; blocks sequential.  Timed
    at T = 1 and T = every host thread this process may use, on 64 x 1 MiB blocks
    (BASELINE config 1's sample size) of the bench's RS(k+m), and on config 1 itself
    (RS(4+2))."""
    from oracle import cpuref

    tall = cpuref.threads_available()
    nb = 64
    v1 = _cpu_rate(k, m, blen, nb, seconds, 1)
    vt = _cpu_rate(k, m, blen, nb, seconds, tall) if tall > 1 else v1
    c1 = _cpu_rate(4, 2, blen, nb, seconds / 2, 1)
    ct = _cpu_rate(4, 2, blen, nb, seconds / 2, tall) if tall > 1 else c1
    best_t, best_v = (tall, vt) if vt >= v1 else (1, v1)
    nproc = os.cpu_count()
    return {
        "value": round(best_v, 3), "unit": "GiB/s", "cores": best_t, "kind": "port",
        "sample": f"RS({k}+{m}) encode+HH256 of {nb} x {blen} B blocks (seed 0), blocks sequential, "
                  f"repeated ~{seconds:.0f}s per thread count; C++ restatement of klauspost/reedsolomon "
                  f"v1.11.8 + minio/highwayhash v1.0.2 structure ({cpuref.isa()}); "
                  f"T=1: {v1:.3f} GiB/s, T={tall}: {vt:.3f} GiB/s; host: os.cpu_count()={nproc}, "
                  f"threads available to this process (affinity, OMP_NUM_THREADS)={tall}",
        "t1": round(v1, 3), "t_all": round(vt, 3), "threads_all": tall, "nproc": nproc,
        "config1": {"workload": f"RS(4+2) encode+HH256 of {nb} x {blen} B blocks (BASELINE config 1)",
                    "t1": round(c1, 3), "t_all": round(ct, 3), "unit": "GiB/s"},
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
            if f"<{k}, {m}," in name and v.get("workload", {}).get("objects") == nobj:
                best = (v["hbm_bytes_per_launch"], os.path.relpath(path, ROOT))
    return best if best else (None, None)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--total-objects", type=int, default=65536,
                    help="strong scaling: 1 MiB objects of the whole stream, split over the GPUs "
                         "(BASELINE config 4: 64 GiB)")
    ap.add_argument("--objects", type=int, default=None,
                    help="weak scaling instead: 1 MiB objects per GPU per step")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per launch from a rocprofv3 PMC pass; default: the committed "
                         "profiles/*/pmc_traffic.json entry for this kernel and batch, if any")
    args = ap.parse_args()

    from zs3server_amd.dist import max_over_ranks, object_range, rank_env, split_range

    world, rank, local = rank_env()
    if world > 1:
        dist.init_process_group("gloo")  # control only: barrier + max of timings
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import zs3server_amd as z

    k, m, blen = args.k, args.m, args.block
    if args.objects is not None:
        nobj = args.objects
        obj_lo, _ = object_range(rank, nobj)  # disjoint object ids per rank
        total_objects, scaling = nobj * world, "weak"
    else:
        obj_lo, obj_hi = split_range(args.total_objects, world, rank)
        nobj = obj_hi - obj_lo
        total_objects, scaling = args.total_objects, "strong"
    S = -(-blen // k)
    stride = (k + m) * S  # reference in-place layout: [k data rows | m parity rows] per block
    codec = z.Codec(k, m, blen)
    buf = torch.empty(nobj * stride, dtype=torch.uint8, device=dev)
    sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device=dev)
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
    stream = torch.cuda.current_stream()  # the stream encode_batch launches on
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
    path = z.last_path()

    elapsed, kern_ms = max_over_ranks([elapsed, kern_ms], world)

    traffic, traffic_src = args.traffic, None
    if traffic is None:
        traffic, traffic_src = committed_traffic(k, m, nobj, blen)

    total_bytes = total_objects * blen * args.steps
    value = total_bytes / elapsed / 2 ** 30
    abytes = nobj * algo_bytes_per_block(k, m, blen)
    achieved = abytes / (kern_ms * 1e-3) / 1e9
    if rank == 0:
        wl = (f"RS({k}+{m}) Split+Encode+HighwayHash256S bitrot sums, in-place bpool layout, "
              + (f"{total_objects} x {blen} B objects ({total_objects * blen / 2**30:.0f} GiB stream, BASELINE "
                 f"config 4) split over {world} GPU(s): {nobj} objects resident per GPU, one launch per step"
                 if scaling == "strong" else f"{nobj} x {blen} B objects per GPU (weak scaling)"))
        out = {
            "metric": f"GiB/s device-resident RS({k}+{m}) encode+bitrot, 1 MiB blocks, at 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 counter stream per object id), device-resident in HBM",
            "config": {"workload": wl, "total_objects": total_objects, "objects_per_gpu": nobj,
                       "block_bytes": blen, "k": k, "m": m,
                       "parallelism": f"objects partitioned over {world} GPU(s), no collectives",
                       "kernel_path": {0: "generic", 1: "first-generation", 2: "warp-specialised",
                                       3: "mixed-wave", 4: "small-batch latency"}.get(path, str(path))},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel_ms": round(kern_ms, 4),
                         "algo_bytes_per_launch": abytes},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(k, m, blen, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
