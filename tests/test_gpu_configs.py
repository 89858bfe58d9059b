"""BASELINE configs 4 and 5 at full size, every output byte
checked.

* Config 4: RS(8+4) encode of a 64 GiB stream of 1 MiB objects partitioned over 2/4/8
  GPUs.  Each GPU's share (16 384 objects at N = 4, 8 192 at N = 8) goes through the
  default dispatch in one launch; sampled blocks against the scalar oracle, and the
  SHA-256 of the whole output (parity rows and bitrot sums of every block) against the
  SHA-256 of the same output computed on the host by oracle/cpu_ref.cpp (the threaded
  SIMD restatement, itself cross-checked against the scalar oracle).
* Config 5: RS(16+4) multipart stream with 1 MiB blocks through zs3_stream_encode
  (pinned and pageable host buffers, ragged last block), and the full 10 GiB stream.

Reference: cmd/erasure-encode.go:83-111 (independent 1 MiB blocks), cmd/erasure-coding.go:77-91.
"""
import hashlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import zs3server_amd as z  # noqa: E402
from oracle import cpuref  # noqa: E402

KEY = z.MAGIC_HH256_KEY
DEV = "cuda:0"
MiB = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z.lib()


def digest_check(oracle, k, m, d, sums, nb, S, seed, chunk=1024):
    """SHA-256 of every block's parity rows + sums as the GPU wrote them vs as cpu_ref
    computes them from the same data rows; data rows of sampled blocks vs oracle_fill."""
    R = k + m
    mat = oracle.build_matrix(k, m)
    T = cpuref.threads_available()
    h_gpu, h_ref = hashlib.sha256(), hashlib.sha256()
    for b0 in range(0, nb, chunk):
        n = min(chunk, nb - b0)
        blk = d[b0 * R * S:(b0 + n) * R * S].cpu().numpy()
        sm = sums[b0 * R * 32:(b0 + n) * R * 32].cpu().numpy()
        par = np.empty(n * m * S, np.uint8)
        sref = np.empty(n * R * 32, np.uint8)
        cpuref.encode_hash(k, m, mat, blk, k * S, n, R * S, par, m * S, sref, KEY, T)
        h_gpu.update(np.ascontiguousarray(blk.reshape(n, R, S)[:, k:]))
        h_gpu.update(sm)
        h_ref.update(par)
        h_ref.update(sref)
    assert h_gpu.hexdigest() == h_ref.hexdigest()
    for b in (0, nb // 3, nb - 1):
        v = d[b * R * S:(b + 1) * R * S].cpu().numpy().reshape(R, S)
        want = oracle.encode_data(k, m, oracle.fill(seed, b, k * S), mat)
        assert np.array_equal(v, want), b
        assert np.array_equal(sums[b * R * 32:(b + 1) * R * 32].cpu().numpy().reshape(R, 32),
                              oracle.hh256_rows(KEY, want)), b
    return h_gpu.hexdigest()


@pytest.mark.parametrize("nb", [8192, 16384])
def test_config4_per_gpu_share(oracle, nb):
    """One GPU's share of config 4 (N = 8 and N = 4), default dispatch, full check."""
    k, m = 8, 4
    S = MiB // k
    R = k + m
    codec = z.Codec(k, m)
    d = torch.empty(nb * R * S, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, MiB, nb, seed=4, obj0=0)
    sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, R * S, MiB, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    assert z.last_path() == 2, "config 4 runs on the warp-specialised kernel"
    digest_check(oracle, k, m, d, sums, nb, S, seed=4)
    del d, sums
    torch.cuda.empty_cache()


@pytest.mark.parametrize("nb", [1, 7, 128, 129, 256, 511, 512, 640, 641, 1000, 1024, 1025, 2047, 2048, 2049, 2304,
                                3001, 4096, 4097, 8192 + 5])
def test_rs84_batch_sizes_no_cliff(oracle, nb):
    """Every batch size runs a specialised kernel (the launch shape follows the batch:
    the small-batch latency path up to 128 stripes, warp-specialised at 4 (129-2048) or
    16 stripes per workgroup above), bit-exact over the whole output."""
    k, m = 8, 4
    S = MiB // k
    R = k + m
    codec = z.Codec(k, m)
    d = torch.empty(nb * R * S, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, MiB, nb, seed=nb, obj0=0)
    sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, R * S, MiB, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    assert z.last_path() == (2 if nb > 128 else 4)
    digest_check(oracle, k, m, d, sums, nb, S, seed=nb)
    del d, sums
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pinned", [False, True])
def test_config5_stream_rs164_1mib_ragged(oracle, pinned):
    """zs3_stream_encode, RS(16+4), 1 MiB blocks (BASELINE config 5 shape), several
    double-buffered batches and a ragged last block; every block vs cpu_ref, the last
    block and two sampled blocks vs the scalar oracle."""
    k, m = 16, 4
    R = k + m
    S = MiB // k
    nfull, tail, batch = 70, (1 << 20) // 3 + 5, 16
    total = nfull * MiB + tail
    nblk = nfull + 1
    codec = z.Codec(k, m, MiB)
    dsrc = torch.empty(nblk * MiB, dtype=torch.uint8, device=DEV)
    z.fill_batch(dsrc, MiB, MiB, nblk, seed=55, obj0=0)
    data = dsrc.cpu().numpy()[:total]
    bufs = []
    if pinned:
        src = z.HostBuffer(total)
        src.array[:] = data
        par = z.HostBuffer(nblk * m * S)
        sm = z.HostBuffer(nblk * R * 32)
        bufs = [src, par, sm]
        par_a, sums_a = par.array, sm.array
    else:
        src, par_a, sums_a = data.copy(), np.zeros(nblk * m * S, np.uint8), np.zeros(nblk * R * 32, np.uint8)
        par, sm = par_a, sums_a
    assert codec.stream_encode(src, total, par, sm, batch_blocks=batch) == nblk
    mat = oracle.build_matrix(k, m)
    pref = np.empty(nfull * m * S, np.uint8)
    sref = np.empty(nfull * R * 32, np.uint8)
    cpuref.encode_hash(k, m, mat, data, MiB, nfull, MiB, pref, m * S, sref, KEY, cpuref.threads_available())
    assert np.array_equal(par_a[:nfull * m * S], pref)
    assert np.array_equal(sums_a[:nfull * R * 32], sref)
    for b in (0, nfull // 2, nfull):
        blk = data[b * MiB:min((b + 1) * MiB, total)]
        want = oracle.encode_data(k, m, blk, mat)
        Sb = want.shape[1]
        assert np.array_equal(par_a[b * m * S: b * m * S + m * Sb].reshape(m, Sb), want[k:]), b
        assert np.array_equal(sums_a[b * R * 32:(b + 1) * R * 32].reshape(R, 32), oracle.hh256_rows(KEY, want)), b
    for x in bufs:
        x.free()


def test_config5_full_10gib_stream(oracle):
    """BASELINE config 5 at full size on one GPU: a 10 GiB RS(16+4) stream (10 240 x
    1 MiB) from pinned host memory through zs3_stream_encode; SHA-256 of all parity and
    sums vs cpu_ref's."""
    k, m = 16, 4
    R = k + m
    S = MiB // k
    nb = 10240
    codec = z.Codec(k, m, MiB)
    src = z.HostBuffer(nb * MiB)
    par = z.HostBuffer(nb * m * S)
    sm = z.HostBuffer(nb * R * 32)
    step = 1024
    dtmp = torch.empty(step * MiB, dtype=torch.uint8, device=DEV)
    for b0 in range(0, nb, step):
        z.fill_batch(dtmp, MiB, MiB, step, seed=10, obj0=b0)
        torch.cuda.synchronize()
        src.array[b0 * MiB:(b0 + step) * MiB] = dtmp.cpu().numpy()
    del dtmp
    assert codec.stream_encode(src, nb * MiB, par, sm, batch_blocks=256) == nb
    mat = oracle.build_matrix(k, m)
    T = cpuref.threads_available()
    h_gpu, h_ref = hashlib.sha256(), hashlib.sha256()
    for b0 in range(0, nb, step):
        pref = np.empty(step * m * S, np.uint8)
        sref = np.empty(step * R * 32, np.uint8)
        cpuref.encode_hash(k, m, mat, src.array[b0 * MiB:], MiB, step, MiB, pref, m * S, sref, KEY, T)
        h_ref.update(pref)
        h_ref.update(sref)
        h_gpu.update(par.array[b0 * m * S:(b0 + step) * m * S])
        h_gpu.update(sm.array[b0 * R * 32:(b0 + step) * R * 32])
    assert h_gpu.hexdigest() == h_ref.hexdigest()
    want = oracle.encode_data(k, m, oracle.fill(10, nb - 1, MiB), mat)
    assert np.array_equal(par.array[(nb - 1) * m * S:].reshape(m, S), want[k:])
    for x in (src, par, sm):
        x.free()


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("pinned", [False, True])
def test_stream_encode_multi_device_driver(oracle, devices, pinned):
    """zs3_stream_encode_multi: the config-5 driver with its stream split over n
    device threads (here n threads sharing device 0: the same split, per-thread
    streams and pinned slots, reassembly at the stream offsets); RS(16+4) 1 MiB blocks
    with a ragged tail, every block vs cpu_ref, the tail vs the scalar oracle."""
    k, m = 16, 4
    R = k + m
    S = MiB // k
    nfull, tail, batch = 29, 12345, 4
    total = nfull * MiB + tail
    nblk = nfull + 1
    codec = z.Codec(k, m, MiB)
    dsrc = torch.empty(nblk * MiB, dtype=torch.uint8, device=DEV)
    z.fill_batch(dsrc, MiB, MiB, nblk, seed=77, obj0=0)
    data = dsrc.cpu().numpy()[:total]
    bufs = []
    if pinned:
        src = z.HostBuffer(total)
        src.array[:] = data
        par = z.HostBuffer(nblk * m * S)
        sm = z.HostBuffer(nblk * R * 32)
        bufs = [src, par, sm]
        par_a, sums_a = par.array, sm.array
    else:
        src, par_a, sums_a = data.copy(), np.zeros(nblk * m * S, np.uint8), np.zeros(nblk * R * 32, np.uint8)
        par, sm = par_a, sums_a
    assert codec.stream_encode_multi(devices, src, total, par, sm, batch_blocks=batch) == nblk
    mat = oracle.build_matrix(k, m)
    pref = np.empty(nfull * m * S, np.uint8)
    sref = np.empty(nfull * R * 32, np.uint8)
    cpuref.encode_hash(k, m, mat, data, MiB, nfull, MiB, pref, m * S, sref, KEY, cpuref.threads_available())
    assert np.array_equal(par_a[:nfull * m * S], pref)
    assert np.array_equal(sums_a[:nfull * R * 32], sref)
    want = oracle.encode_data(k, m, data[nfull * MiB:], mat)
    St = want.shape[1]
    assert np.array_equal(par_a[nfull * m * S: nfull * m * S + m * St].reshape(m, St), want[k:])
    assert np.array_equal(sums_a[nfull * R * 32:].reshape(R, 32), oracle.hh256_rows(KEY, want))
    for x in bufs:
        x.free()
