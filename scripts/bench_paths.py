"""Secondary measurements: every kernel family of the path at the
BASELINE shapes, each as one JSON line with its roofline (algorithmic HBM bytes per
launch / median launch time, against the 8 TB/s HBM3E spec), plus the batching queue
and the end-to-end host stream.

  PATHS=encode,geom,rec,get,hash,deep,digest,queue,e2e,stream_get  python scripts/bench_paths.py
(default: all).  Kernel-only sections (encode..digest) are what scripts/profile_paths.sh
runs under rocprofv3; queue and e2e include host copies and PCIe.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import zs3server_amd as z  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E spec
MiB = 1 << 20
KEY = z.MAGIC_HH256_KEY
PATHS = set(os.environ.get("PATHS", "encode,geom,rec,get,hash,deep,digest,queue,e2e").split(","))
REPS = int(os.environ.get("REPS", "10"))


def timeit(fn, reps=REPS):
    """Median of `reps` launches timed with HIP events on the launch stream."""
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def out(path, what, ms, algo_bytes, objects=None, **kw):
    ach = algo_bytes / (ms * 1e-3) / 1e9
    d = {"path": path, "what": what, "ms": round(ms, 4), "kernel_path": z.last_path()}
    if objects:
        d["objects"] = objects
        d["GiBps_object"] = round(objects * MiB / (ms * 1e-3) / 2**30, 1)
    d["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK, "unit": "GB/s",
                     "frac": round(ach / PEAK, 4), "algo_bytes_per_launch": int(algo_bytes)}
    d.update(kw)
    print(json.dumps(d), flush=True)


def encoded(k, m, nobj, seed):
    S = -(-MiB // k)
    stride = (k + m) * S
    codec = z.Codec(k, m)
    buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
    sums = torch.empty(nobj * (k + m) * 32, dtype=torch.uint8, device="cuda")
    z.fill_batch(buf, stride, MiB, nobj, seed=seed)
    codec.encode_batch(buf, stride, MiB, nobj, parity=buf, parity_offset=k * S, parity_stride=stride, sums=sums)
    torch.cuda.synchronize()
    return codec, buf, sums, S, stride


def warm_clock(seconds=0.5):
    """Run back-to-back launches first so that the first measured path is not timed on the
    GPU's clock ramp (a process's first launches run slower: config 2 0.43-0.48 ms there
    vs 0.36-0.40 warmed)."""
    buf = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(8):
            z.fill_batch(buf, MiB, MiB, 1024, seed=0)
        torch.cuda.synchronize()
    del buf
    torch.cuda.empty_cache()


warm_clock()

# ---- encode + bitrot sums (BASELINE configs 2, 3, RS(16+4)) and encode only
if "encode" in PATHS:
    for k, m, nobj, label in ((4, 2, 1024, "config 2: RS(4+2) 1024 x 1 MiB"),
                              (8, 4, 4096, "config 3: RS(8+4) 4096 x 1 MiB"),
                              (16, 4, 2048, "RS(16+4) 2048 x 1 MiB"),
                              (12, 4, 4096, "RS(12+4) 4096 x 1 MiB (16-drive default)"),
                              (4, 4, 4096, "RS(4+4) 4096 x 1 MiB (8-drive default)")):
        codec, buf, sums, S, stride = encoded(k, m, nobj, 1)
        ms = timeit(lambda: codec.encode_batch(buf, stride, MiB, nobj, parity=buf, parity_offset=k * S,
                                               parity_stride=stride, sums=sums))
        out("encode_hash", label, ms, nobj * (MiB + m * S + 32 * (k + m)), objects=nobj)
        ms = timeit(lambda: codec.encode_batch(buf, stride, MiB, nobj, parity=buf, parity_offset=k * S,
                                               parity_stride=stride))
        out("encode_only", label, ms, nobj * (MiB + m * S), objects=nobj)
        del buf, sums
        torch.cuda.empty_cache()

# ---- the server's other default geometries (getDefaultParityBlocks,
# cmd/format-erasure.go:870-881: set size 4..16 -> RS(2+2), (3+2), (3+3), (4+3), (4+4),
# (5+4), ..., (12+4)): encode + sums, encode only, GET rebuild 2 and heal 2 at 4096 x 1 MiB
# (PATHS=geom; GEOMS="6:4,10:4" selects)
if "geom" in PATHS:
    geoms = [tuple(int(x) for x in g.split(":")) for g in os.environ.get(
        "GEOMS", "2:2,3:2,3:3,4:3,5:4,6:4,7:4,9:4,10:4,11:4").split(",")]
    for k, m in geoms:
        nobj = 4096
        codec, buf, sums, S, stride = encoded(k, m, nobj, 11)
        R = k + m
        label = f"RS({k}+{m}) {nobj} x 1 MiB (default for {R}-drive sets)"
        ms = timeit(lambda: codec.encode_batch(buf, stride, MiB, nobj, parity=buf, parity_offset=k * S,
                                               parity_stride=stride, sums=sums))
        out("encode_hash", label, ms, nobj * (MiB + m * S + 32 * R), objects=nobj)
        ms = timeit(lambda: codec.encode_batch(buf, stride, MiB, nobj, parity=buf, parity_offset=k * S,
                                               parity_stride=stride))
        out("encode_only", label, ms, nobj * (MiB + m * S), objects=nobj)
        vbad = torch.empty(nobj * R, dtype=torch.int32, device="cuda")
        hsum = torch.empty_like(sums)
        for erased, heal in (([0, 1], False), ([0, k], True)):
            pres = [i not in erased for i in range(R)]
            e = len(erased)
            ms = timeit(lambda: codec.verify_reconstruct_batch(buf, stride, S, nobj, pres, not heal, sums, vbad,
                                                               sums_out=hsum if heal else None))
            out("verify_reconstruct", f"RS({k}+{m}) {nobj} x 1 MiB: verify {k} + rebuild {e}" +
                (" + hash rebuilt (heal)" if heal else ""), ms,
                nobj * (k * S + e * S + 32 * k + (32 * e if heal else 0)), objects=nobj, bad=int(vbad.sum()))
        del buf, sums, vbad, hsum
        torch.cuda.empty_cache()

# ---- reconstruct (ReconstructData / Reconstruct), BASELINE config 3 and RS(16+4)
if "rec" in PATHS:
    for k, m, nobj, cases in ((8, 4, 4096, (([0, 5], True), ([2, 10], False))),
                              (16, 4, 2048, (([0, 5], True), ([0, 5, 9, 14], True), ([3, 17], False))),
                              (12, 4, 4096, (([0, 5], True), ([1, 13], False)))):
        codec, buf, sums, S, stride = encoded(k, m, nobj, 3)
        for erased, data_only in cases:
            pres = [i not in erased for i in range(k + m)]
            e = len([i for i in erased if i < k or not data_only])
            ms = timeit(lambda: codec.reconstruct_batch(buf, stride, S, nobj, pres, data_only))
            out("reconstruct", f"RS({k}+{m}) {nobj} x 1 MiB, erased {erased}, "
                f"{'ReconstructData' if data_only else 'Reconstruct'}", ms, nobj * (k * S + e * S), objects=nobj)
        del buf, sums
        torch.cuda.empty_cache()

# ---- GET / heal fused pass: verify the k survivors, rebuild, (heal) hash the rebuilt rows
if "get" in PATHS:
    for k, m, nobj, cases in (
            (8, 4, 4096, (([], True, False), ([3], True, False), ([0, 5], True, False), ([0, 5, 6], True, False),
                          ([1, 2, 5, 7], True, False), ([4], False, True), ([2, 10], False, True))),
            (4, 2, 2048, (([], True, False), ([1], True, False), ([0, 3], True, False), ([0, 5], False, True))),
            (16, 4, 2048, (([], True, False), ([6], True, False), ([0, 5], True, False), ([1, 7, 15], True, False),
                           ([0, 5, 9, 14], True, False), ([5], False, True), ([3, 17], False, True),
                           ([0, 1, 16, 19], False, True))),
            (12, 4, 4096, (([], True, False), ([0, 5], True, False), ([1, 12], False, True))),
            (4, 4, 4096, (([], True, False), ([0, 1], True, False), ([1, 4], False, True)))):
        codec, buf, sums, S, stride = encoded(k, m, nobj, 5)
        R = k + m
        vbad = torch.empty(nobj * R, dtype=torch.int32, device="cuda")
        hsum = torch.empty_like(sums)
        for erased, data_only, heal in cases:
            pres = [i not in erased for i in range(R)]
            e = len(erased) if heal else len([i for i in erased if i < k or not data_only])
            ms = timeit(lambda: codec.verify_reconstruct_batch(buf, stride, S, nobj, pres, data_only, sums, vbad,
                                                               sums_out=hsum if heal else None))
            what = (f"RS({k}+{m}) {nobj} x 1 MiB: verify {k}" + (f" + rebuild {e}" if e else "") +
                    (" + hash rebuilt (heal)" if heal and e else ""))
            out("verify_reconstruct", what, ms, nobj * (k * S + e * S + 32 * k + (32 * e if heal else 0)),
                objects=nobj, bad=int(vbad.sum()))
        del buf, sums, vbad, hsum
        torch.cuda.empty_cache()

# ---- hash-only / verify over all 12 shard rows of 4096 RS(8+4) stripes
if "hash" in PATHS:
    k, m, nobj = 8, 4, 4096
    codec, buf, sums, S, stride = encoded(k, m, nobj, 7)
    n = nobj * (k + m)
    ms = timeit(lambda: z.hh256_batch(buf, S, S, n, sums))
    out("hh256_batch", f"{n} x {S} B messages", ms, n * (S + 32))
    bad = torch.empty(n, dtype=torch.int32, device="cuda")
    ms = timeit(lambda: z.hh256_verify_batch(buf, S, S, n, sums, bad))
    out("hh256_verify_batch", f"{n} x {S} B messages", ms, n * (S + 32 + 4), bad=int(bad.sum()))
    del buf, sums, bad
    torch.cuda.empty_cache()

# ---- deep scan: bitrotVerify over whole shard files ([sum|chunk]* in place)
if "deep" in PATHS:
    shard, chunks, nfiles = 131072, 64, 512        # 512 RS(8+4) shard files of a 64 MiB part
    part = shard * chunks
    want = z.bitrot_shard_file_size(part, shard)
    files = torch.empty(nfiles * want, dtype=torch.uint8, device="cuda")
    z.fill_batch(files, want, want, nfiles, seed=9)
    bad = torch.empty(nfiles * chunks, dtype=torch.int32, device="cuda")
    fbad = torch.empty(nfiles, dtype=torch.int32, device="cuda")
    ms = timeit(lambda: z.bitrot_verify_file_batch(files, want, nfiles, want, part, shard, bad, fbad, key=KEY))
    out("bitrot_verify_file_batch", f"{nfiles} shard files x {chunks} chunks of {shard} B", ms,
        nfiles * (want + 4 * chunks + 4))
    del files, bad, fbad
    torch.cuda.empty_cache()

# ---- PUT-stream object digests: S3 ETag (MD5) and content SHA-256
if "digest" in PATHS:
    nobj = 4096
    buf = torch.empty(nobj * MiB, dtype=torch.uint8, device="cuda")
    z.fill_batch(buf, MiB, MiB, nobj, seed=2)
    for name, fn, width in (("md5_batch", z.md5_batch, 16), ("sha256_batch", z.sha256_batch, 32)):
        dout = torch.empty(nobj * width, dtype=torch.uint8, device="cuda")
        ms = timeit(lambda: fn(buf, MiB, MiB, nobj, dout), reps=3)
        # per-block latency of one lane's chain: the launch is one 1 MiB message long
        # (16 385 blocks with the padding block); the roof is the compression wave's
        # VALU count per block x 4 cycles (digest.hip header)
        blk = MiB // 64 + 1
        out(name, f"{nobj} x 1 MiB objects, one lane per object", ms, nobj * (MiB + width), objects=nobj,
            us_per_block=round(ms * 1e3 / blk, 4))
    # the parts of multipart uploads: one 5 MiB part alone (the latency of one part), and
    # 256 parts of 5 MiB at arbitrary offsets in one launch (zs3_*_parts)
    part = 5 * MiB
    pbuf = torch.empty(256 * part + 4096, dtype=torch.uint8, device="cuda")
    z.fill_batch(pbuf, part, part, 256, seed=3)
    for nparts in (1, 256):
        offs = torch.arange(nparts, dtype=torch.int64, device="cuda") * (part + 7)
        lens = torch.full((nparts,), part, dtype=torch.int64, device="cuda")
        for name, fn, width in (("md5_parts", z.md5_parts, 16), ("sha256_parts", z.sha256_parts, 32)):
            dout = torch.empty(nparts * width, dtype=torch.uint8, device="cuda")
            ms = timeit(lambda: fn(pbuf, offs, lens, nparts, dout), reps=2)
            out(name, f"{nparts} x 5 MiB parts at unaligned offsets, one launch", ms, nparts * (part + width),
                objects=nparts, us_per_block=round(ms * 1e3 / (part // 64 + 1), 4))
    del buf, pbuf
    torch.cuda.empty_cache()


# ---- batching queue: T concurrent submitters (goroutines in cgo), per-block latency and
# aggregate rate, next to the reference CPU structure at the same concurrency
def queue_run(k, m, T, per_thread, q, cpu):
    from oracle import cpuref, oracle_c
    R = k + m
    S = MiB // k
    mat = oracle_c.build_matrix(k, m)
    bufs = [np.zeros((per_thread, R * S), np.uint8) for _ in range(T)]
    for t in range(T):
        bufs[t][:, :MiB] = np.frombuffer(os.urandom(MiB), np.uint8)
    sums = [np.zeros((per_thread, R * 32), np.uint8) for _ in range(T)]
    lat = [[] for _ in range(T)]

    def work(t):
        for i in range(per_thread):
            t0 = time.perf_counter()
            if cpu:
                par = bufs[t][i, k * S:]
                cpuref.encode_hash(k, m, mat, bufs[t][i], MiB, 1, MiB, par, m * S, sums[t][i], KEY, 1)
            else:
                q.encode_data(bufs[t][i], MiB)
            lat[t].append(time.perf_counter() - t0)

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    allv = sorted(v for lt in lat for v in lt)
    return T * per_thread * MiB / dt / 2**30, allv[len(allv) // 2] * 1e6, allv[int(len(allv) * 0.99)] * 1e6


if "queue" in PATHS:
    from oracle import cpuref
    k, m = 8, 4
    codec = z.Codec(k, m)
    q = z.Queue(codec, max_batch=128, max_wait_us=200)
    queue_run(k, m, 4, 4, q, False)  # warm
    for T in [int(x) for x in os.environ.get("QUEUE_T", "1,4,16,64").split(",")]:
        per = 32 if T <= 16 else 16
        b0, n0 = q.stats()
        g, p50, p99 = queue_run(k, m, T, per, q, False)
        b1, n1 = q.stats()
        c, cp50, cp99 = (queue_run(k, m, T, max(2, per // 4), None, True) if os.environ.get("QUEUE_CPU", "1") == "1"
                         else (0.0, 0.0, 0.0))
        print(json.dumps({"path": "queue_encode", "what": f"RS(8+4) 1 MiB blocks, {T} concurrent submitters",
                          "GiBps": round(g, 2), "block_latency_us_p50": round(p50, 1),
                          "block_latency_us_p99": round(p99, 1), "blocks_per_batch": round((n1 - n0) / max(1, b1 - b0), 1),
                          "cpu_ref_same_concurrency": {"GiBps": round(c, 2), "block_latency_us_p50": round(cp50, 1),
                                                       "threads": T, "cores_available": cpuref.threads_available()}}),
              flush=True)
    q.close()

# ---- config 5: end-to-end stream incl. pinned / pageable host buffers and PCIe
if "e2e" in PATHS:
    gib = float(os.environ.get("E2E_GIB", "10"))
    for (k, m) in ((16, 4), (8, 4), (12, 4)):
        bs = MiB
        total = int(gib * (1 << 30))
        nblk = total // bs
        S = -(-bs // k)
        codec = z.Codec(k, m, bs)
        for pinned in (True, False):
            if pinned:
                src, par, sums = z.HostBuffer(total), z.HostBuffer(nblk * m * S), z.HostBuffer(nblk * (k + m) * 32)
                src.array[:] = 7
            else:
                src = np.full(total, 7, dtype=np.uint8)
                par = np.zeros(nblk * m * S, np.uint8)
                sums = np.zeros(nblk * (k + m) * 32, np.uint8)
            # warm: the same batch size, so the timed call reuses the pooled staging
            codec.stream_encode(src, 1024 * bs, par, sums, batch_blocks=512)
            t0 = time.perf_counter()
            codec.stream_encode(src, total, par, sums, batch_blocks=512)
            dt = time.perf_counter() - t0
            print(json.dumps({"path": "stream_encode_e2e", "what": f"RS({k}+{m}) {gib:g} GiB stream, 1 MiB blocks",
                              "driver": "zs3_stream_encode -> zs3_stream_encode_multi, 1 device",
                              "host_buffers": "pinned" if pinned else "pageable", "seconds": round(dt, 3),
                              "GiBps": round(total / dt / 2**30, 2),
                              "pcie_GBps": round((total + nblk * (m * S + 32 * (k + m))) / dt / 1e9, 1)}), flush=True)
            if pinned:
                for x in (src, par, sums):
                    x.free()
            del src, par, sums
    # the same stream split over two device entries (zs3_stream_encode_multi; on a 1-GPU
    # box both are device 0: the split, threads and slots of an N-device run, one HBM)
    k, m, bs = 16, 4, MiB
    total = int(gib * (1 << 30))
    nblk = total // bs
    S = bs // k
    codec = z.Codec(k, m, bs)
    src, par, sums = z.HostBuffer(total), z.HostBuffer(nblk * m * S), z.HostBuffer(nblk * (k + m) * 32)
    src.array[:] = 7
    devs = [int(x) for x in os.environ.get("E2E_DEVICES", "0,0").split(",")]
    codec.stream_encode_multi(devs, src, min(2048 * bs, total), par, sums, batch_blocks=512)
    t0 = time.perf_counter()
    codec.stream_encode_multi(devs, src, total, par, sums, batch_blocks=512)
    dt = time.perf_counter() - t0
    print(json.dumps({"path": "stream_encode_multi_e2e", "what": f"RS({k}+{m}) {gib:g} GiB stream, 1 MiB blocks",
                      "devices": devs, "host_buffers": "pinned", "seconds": round(dt, 3),
                      "GiBps": round(total / dt / 2**30, 2),
                      "pcie_GBps": round((total + nblk * (m * S + 32 * (k + m))) / dt / 1e9, 1)}), flush=True)
    for x in (src, par, sums):
        x.free()

# ---- one large GET / heal (Erasure.Decode / Erasure.Heal block loops) streamed through
# the device (zs3_stream_decode) vs the per-block queue path of a lone caller and the CPU
if "stream_get" in PATHS:
    from oracle import cpuref, oracle_c
    gib = float(os.environ.get("SG_GIB", "1"))
    for (k, m, lost) in ((12, 4, [1, 12]), (8, 4, [2, 9])):
        R = k + m
        S = -(-MiB // k)
        E = R * S
        nblk = int(gib * 1024)
        codec = z.Codec(k, m, MiB)
        for pinned in (True, False):
            st_h = z.HostBuffer(nblk * E) if pinned else None
            st = st_h.array if pinned else np.empty(nblk * E, np.uint8)
            st[:] = 0
            d = torch.empty(nblk * E, dtype=torch.uint8, device="cuda")
            z.fill_batch(d, E, MiB, nblk, seed=17)
            sums_d = torch.empty(nblk * R * 32, dtype=torch.uint8, device="cuda")
            codec.encode_batch(d, E, MiB, nblk, parity=d, parity_offset=k * S, parity_stride=E, sums=sums_d)
            st[:] = d.cpu().numpy()
            sums = sums_d.cpu().numpy().reshape(nblk, R, 32)
            del d, sums_d
            present = np.ones((nblk, R), bool)
            present[:, lost] = False
            bad = np.zeros((nblk, R), np.int32)
            for heal in (False, True):
                outs = np.zeros((nblk, R, 32), np.uint8) if heal else None
                arg = st_h if pinned else st
                codec.stream_decode(arg, 64 * MiB, present[:64], not heal, expect=sums[:64], bad=bad[:64],
                                    sums_out=outs[:64] if heal else None, batch_blocks=64)
                ts = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    n = codec.stream_decode(arg, nblk * MiB, present, not heal, expect=sums, bad=bad, sums_out=outs,
                                            batch_blocks=128)
                    ts.append(time.perf_counter() - t0)
                    assert n == nblk and not bad.any(), n
                dt = sorted(ts)[1]
                e = len(lost) if heal else len([i for i in lost if i < k])
                pcie = nblk * ((k if not heal else k) * S + e * S + R * 32 * (2 if heal else 1))
                print(json.dumps({"path": "stream_decode", "what": f"RS({k}+{m}) lone {'heal' if heal else 'GET'} of "
                                  f"{nblk} x 1 MiB blocks, lost {lost}", "host_buffers": "pinned" if pinned else "pageable",
                                  "seconds": round(dt, 4), "GiBps_object": round(nblk * MiB / dt / 2**30, 2),
                                  "us_per_block": round(dt / nblk * 1e6, 1)}), flush=True)
            if st_h is not None:
                st_h.free()
            del st
        # CPU reference structure for the same heal (verify k survivors, rebuild e rows,
        # hash them): cpu_ref's encode + hash with the e rebuild rows as the coding rows
        # (GF cost is value-independent), 64 blocks repeated, T = 1 and T = all
        e = len(lost)
        mat = oracle_c.build_matrix(k, e)
        nb = 64
        data = np.concatenate([oracle_c.fill(0, b, MiB) for b in range(nb)])
        par = np.zeros(nb * e * S, np.uint8)
        sm = np.zeros(nb * (k + e) * 32, np.uint8)
        for T in (1, cpuref.threads_available()):
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < 3.0:
                cpuref.encode_hash(k, e, mat, data, MiB, nb, MiB, par, e * S, sm, KEY, T)
                reps += 1
            dt = time.perf_counter() - t0
            print(json.dumps({"path": "cpu_heal_ref", "what": f"RS({k}+{m}) heal {e} rows (verify {k} + rebuild {e} + "
                              f"hash {e}) on the host, cpu_ref ({cpuref.isa()})", "threads": T,
                              "GiBps_object": round(reps * nb * MiB / dt / 2**30, 2),
                              "us_per_block": round(dt / (reps * nb) * 1e6, 1)}), flush=True)
        # the per-block queue path of a lone synchronous caller (round 4: ~306 us per block)
        q = z.Queue(codec, max_wait_us=200)
        sh_ = np.zeros((R, S), np.uint8)
        pres = np.ones(R, bool)
        pres[lost] = False
        t0 = time.perf_counter()
        nq = 200
        for _ in range(nq):
            q.decode(sh_, pres, False, sums_out=np.zeros((R, 32), np.uint8))
        dt = time.perf_counter() - t0
        print(json.dumps({"path": "queue_lone_heal", "what": f"RS({k}+{m}) heal {len(lost)}, one block per call",
                          "GiBps_object": round(nq * MiB / dt / 2**30, 2), "us_per_block": round(dt / nq * 1e6, 1)}),
              flush=True)
        q.close()
