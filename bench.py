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

Launch: python bench.py [--gpus N --steps K --warmup W].  For N > 1 either under
torch.distributed.run (one rank per GPU, WORLD_SIZE must equal N), or plain: the process
then spawns the N ranks itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* per child,
before any GPU call in the parent) and relays rank 0's line.  It exits non-zero when
fewer than N devices are visible or WORLD_SIZE disagrees with --gpus: it never reports
N GPUs it did not use.  Test-only switches (the JSON line says so): ZS3_BENCH_SAME_DEVICE=1
puts every rank on device 0 (rehearsing N ranks on a 1-GPU box), ZS3_BENCH_DRY_RUN=1
runs the launcher, rendezvous, barriers and max-over-ranks on CPU with no GPU work
(value null).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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


# The kernel instance each bench launch runs (fused_v2.hip launch_ehx_default: n > 2048
# stripes of RS(8+4) at 1 MiB take the named shape Rs84Bulk).  committed_traffic matches
# this full name, so counters of an older instance are never attached to the current one;
# scripts/profile_round.sh checks that the traced kernel carries this name.
HEADLINE_KERNEL = {(8, 4, 1 << 20): "void zs3k::k_ehx_ws<8, 4, zs3k::shape::Rs84Bulk>(zs3k::EncArgs)"}
HEADLINE_MIN_OBJECTS = 2049


def headline_kernel(k: int, m: int, blen: int, nobj: int):
    if nobj < HEADLINE_MIN_OBJECTS:
        return None
    return HEADLINE_KERNEL.get((k, m, blen))


def committed_traffic(k: int, m: int, nobj: int, blen: int):
    """Per-launch HBM bytes measured by scripts/profile_round.sh (two rocprofv3 PMC
    passes, FETCH_SIZE doubled per the gfx950 correction) for exactly this kernel
    instance (full name) and objects per launch; the newest round's entry wins."""
    import glob
    want = headline_kernel(k, m, blen, nobj)
    if want is None:
        return None, None
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        for name, v in d.items():
            kname = name.split(" @ ")[0]
            if kname == want and v.get("workload", {}).get("objects") == nobj:
                best = (v["hbm_bytes_per_launch"], os.path.relpath(path, ROOT))
    return best if best else (None, None)


def roofline_block(k: int, m: int, blen: int, nobj: int, total_objects: int, world: int, kern_ms: float,
                   traffic, traffic_src) -> dict:
    """The line's `roofline` object.  Every rank launches the same kernel on its own share
    (nobj objects), so the roofline is a per-GPU quantity: `achieved` / `frac` (alias
    `frac_per_gpu`) = one GPU's algorithmic bytes per launch / the slowest rank's average
    kernel time, against one GPU's HBM peak; `traffic` is per launch on one GPU.  The
    whole-job view sits beside it: `aggregate_achieved` = the bytes of all ranks' launches /
    the slowest rank's kernel time, against `aggregate_peak` = N x one GPU's peak."""
    abytes = nobj * algo_bytes_per_block(k, m, blen)
    achieved = abytes / (kern_ms * 1e-3) / 1e9
    agg_bytes = total_objects * algo_bytes_per_block(k, m, blen)
    agg = agg_bytes / (kern_ms * 1e-3) / 1e9
    return {"bound": "hbm", "scope": "per_gpu", "n_gpus": world,
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "frac_per_gpu": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic, "traffic_scope": "per_gpu_per_launch", "traffic_source": traffic_src,
            "kernel": headline_kernel(k, m, blen, nobj),
            "kernel_ms": round(kern_ms, 4), "kernel_ms_scope": "max_over_ranks",
            "algo_bytes_per_launch": abytes,
            "aggregate_achieved": round(agg, 1), "aggregate_peak": HBM_PEAK_GBS * world,
            "aggregate_frac": round(agg / (HBM_PEAK_GBS * world), 4), "aggregate_algo_bytes": agg_bytes}


def _free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int, argv: list) -> int:
    """Spawn the N ranks of `bench.py --gpus N` (the parent never touches a GPU: counting
    devices does not initialise HIP on this image).  Rank 0's stdout is relayed; the
    exit code is the worst of the children's."""
    same = os.environ.get("ZS3_BENCH_SAME_DEVICE") == "1"
    dry = os.environ.get("ZS3_BENCH_DRY_RUN") == "1"
    if not (same or dry):
        vis = torch.cuda.device_count()
        if vis < n:
            print(f"bench.py: --gpus {n} needs {n} visible devices, found {vis} "
                  f"(set ZS3_BENCH_SAME_DEVICE=1 only to rehearse the ranks on one device)", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ZS3_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    for p in procs:
        c = p.wait()
        if c != 0 and rc == 0:
            rc = c
            for q in procs:  # one rank failed: the others would wait at a barrier forever
                if q.poll() is None:
                    q.terminate()
    return rc if rc >= 0 else 1


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

    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1, got {args.gpus}")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = rank_env()
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a different N")
    same_dev = os.environ.get("ZS3_BENCH_SAME_DEVICE") == "1"
    dry = os.environ.get("ZS3_BENCH_DRY_RUN") == "1"
    if world > 1:
        dist.init_process_group("gloo")  # control only: barrier + max of timings
    if dry:
        return dry_run(args, world, rank)
    if torch.cuda.device_count() < (1 if same_dev else world):
        sys.exit(f"bench.py: rank {rank} needs device {local}, {torch.cuda.device_count()} visible")
    local = 0 if same_dev else local
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
                       "parallelism": f"objects partitioned over {world} GPU(s), no collectives"
                                      + (" (TEST: all ranks on device 0)" if same_dev else ""),
                       "kernel_path": {0: "generic", 1: "first-generation", 2: "warp-specialised",
                                       3: "mixed-wave", 4: "small-batch latency"}.get(path, str(path))},
            "roofline": roofline_block(k, m, blen, nobj, total_objects, world, kern_ms, traffic, traffic_src),
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(k, m, blen, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dry_run(args, world: int, rank: int) -> None:
    """ZS3_BENCH_DRY_RUN=1 (tests only): the launcher, rendezvous, barriers and the
    max-over-ranks reduction without any GPU work; value is null."""
    from zs3server_amd.dist import max_over_ranks
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    if world > 1:
        dist.barrier()
    elapsed, = max_over_ranks([time.perf_counter() - t0], world)
    if rank == 0:
        print(json.dumps({"metric": "dry run (launcher test, no GPU work)", "value": None, "unit": "GiB/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed * 1e3, 3), "dry_run": True,
                          "ranks_seen": world, "pid": os.getpid(),
                          "roofline": roofline_block(args.k, args.m, args.block, args.total_objects // world,
                                                     args.total_objects, world, elapsed * 1e3, None, None)}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
