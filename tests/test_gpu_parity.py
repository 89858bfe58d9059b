"""GPU parity tests: every device path through the C ABI vs the CPU oracle.

Bit-exact integer/byte work: parity shards, reconstructed shards and
HighwayHash-256 bitrot sums must equal the oracle (KAT-pinned, see
test_oracle_kats.py) byte for byte.  Edge cases follow the reference tests:
erasure_test.go:29-110 (encode/decode cases incl. expected failures),
bitrot_test.go:28-85 (10- and 5-byte chunks: HH remainder path), plus
empty / ragged final blocks and non-16-aligned shard sizes.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import zs3server_amd as z  # noqa: E402
from conftest import variant_ctx  # noqa: E402
from zs3server_amd import erasure as ze  # noqa: E402

KEY = z.MAGIC_HH256_KEY
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z.lib()


def dev_blocks(oracle, seed, n_blocks, blen, stride):
    host = np.zeros(n_blocks * stride, dtype=np.uint8)
    for b in range(n_blocks):
        host[b * stride: b * stride + blen] = oracle.fill(seed, b, blen)
    return host, torch.from_numpy(host).to(DEV)


# (k, m, block_len, n_blocks): specialised kernels, generic kernel, ragged tails
ENCODE_CASES = [
    (4, 2, 1 << 20, 3), (8, 4, 1 << 20, 5), (16, 4, 1 << 20, 4), (8, 4, 1 << 16, 9),
    (4, 2, 1 << 16, 17), (2, 2, 4096, 7), (6, 2, 3072, 3), (8, 4, 4096 + 512, 3),
    # shard size % 32 == 16 (HH remainder on the vectorised kernel)
    (8, 4, 8 * 48, 5),
    # generic kernel: non-16-aligned S, padding, odd k
    (5, 3, 1000, 3), (12, 4, 1 << 20, 2), (8, 4, (1 << 20) + 1, 2), (8, 4, 17, 4), (4, 2, 1, 3),
    (3, 3, 256, 2), (7, 5, 4099, 2), (20, 12, 5000, 2),
]


@pytest.mark.parametrize("k,m,blen,nb", ENCODE_CASES)
def test_encode_hash_batch_in_place(oracle, k, m, blen, nb):
    """In-place layout (parity at data + k*S, stride (k+m)*S) as the bpool buffer."""
    codec = z.Codec(k, m, 1 << 20)
    S = -(-blen // k)
    stride = (k + m) * S
    host, d = dev_blocks(oracle, 7 + k, nb, blen, stride)
    sums = torch.zeros(nb * (k + m) * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, stride, blen, nb, parity=d, parity_offset=k * S, parity_stride=stride, sums=sums)
    torch.cuda.synchronize()
    out = d.cpu().numpy().reshape(nb, k + m, S)
    hs = sums.cpu().numpy().reshape(nb, k + m, 32)
    mat = oracle.build_matrix(k, m)
    for b in range(nb):
        want = oracle.encode_data(k, m, host[b * stride: b * stride + blen], mat)
        assert np.array_equal(out[b, k:], want[k:]), f"parity block {b}"
        assert np.array_equal(hs[b], oracle.hh256_rows(KEY, want)), f"sums block {b}"


@pytest.mark.parametrize("k,m,blen,nb", [(8, 4, 1 << 20, 3), (4, 2, 1 << 16, 5), (5, 3, 777, 2)])
def test_encode_only_separate_parity(oracle, k, m, blen, nb):
    codec = z.Codec(k, m, 1 << 20)
    S = -(-blen // k)
    host, d = dev_blocks(oracle, 99, nb, blen, blen)
    par = torch.zeros(nb * m * S, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, blen, blen, nb, parity=par, parity_stride=m * S)
    torch.cuda.synchronize()
    p = par.cpu().numpy().reshape(nb, m, S)
    for b in range(nb):
        want = oracle.encode_data(k, m, host[b * blen:(b + 1) * blen])
        assert np.array_equal(p[b], want[k:])


def test_encode_empty_block_is_noop():
    codec = z.Codec(8, 4)
    d = torch.full((64,), 7, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, 0, 0, 4, parity=d, parity_stride=0, sums=d)
    torch.cuda.synchronize()
    assert bool((d == 7).all())


def test_specialised_kernel_selected():
    codec = z.Codec(8, 4)
    d = torch.zeros(12 * 131072, dtype=torch.uint8, device=DEV)
    s = torch.zeros(12 * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, 12 * 131072, 1 << 20, 1, parity=d, parity_offset=8 * 131072, parity_stride=0, sums=s)
    torch.cuda.synchronize()
    assert z.last_path() >= 1


RECON_PATTERNS = [
    (4, 2, [0, 1]), (4, 2, [2, 5]), (8, 4, [0, 5]), (8, 4, [3, 9]), (8, 4, [8, 9, 10, 11]),
    (8, 4, [0, 1, 2, 3]), (16, 4, [1, 7, 15, 19]), (5, 3, [0, 4, 6]), (12, 4, [11]), (20, 12, [0, 3, 21, 30]),
]


@pytest.mark.parametrize("k,m,erased", RECON_PATTERNS)
@pytest.mark.parametrize("data_only", [True, False])
def test_reconstruct_batch(oracle, k, m, erased, data_only):
    run_reconstruct_case(oracle, k, m, erased, data_only)


def run_reconstruct_case(oracle, k, m, erased, data_only):
    blen = 1 << 16 if k in (4, 8, 16) else 4099
    nb = 3
    codec = z.Codec(k, m)
    S = -(-blen // k)
    stride = (k + m) * S
    host, d = dev_blocks(oracle, 5, nb, blen, stride)
    codec.encode_batch(d, stride, blen, nb, parity=d, parity_offset=k * S, parity_stride=stride)
    torch.cuda.synchronize()
    full = d.clone()
    v = d.view(nb, k + m, S)
    for e in erased:
        v[:, e, :] = 0xA5
    present = [i not in erased for i in range(k + m)]
    codec.reconstruct_batch(d, stride, S, nb, present, data_only)
    torch.cuda.synchronize()
    got = d.view(nb, k + m, S)
    ref = full.view(nb, k + m, S)
    for i in range(k + m):
        if i in erased and data_only and i >= k:
            assert bool((got[:, i] == 0xA5).all()), "parity must stay untouched for ReconstructData"
        else:
            assert torch.equal(got[:, i], ref[:, i]), f"shard {i}"


def test_reconstruct_errors():
    codec = z.Codec(4, 2)
    d = torch.zeros(6 * 64, dtype=torch.uint8, device=DEV)
    with pytest.raises(z.ZS3Error) as ei:
        codec.reconstruct_batch(d, 6 * 64, 64, 1, [0, 0, 1, 1, 1, 0], True)
    assert ei.value.code == -3  # ErrTooFewShards
    with pytest.raises(z.ZS3Error) as ei:
        codec.reconstruct_batch(d, 6 * 64, 64, 1, [0] * 6, True)
    assert ei.value.code == -4  # ErrShardNoData
    codec.reconstruct_batch(d, 6 * 64, 64, 1, [1] * 6, False)  # nothing missing -> ok


@pytest.mark.parametrize("lens", [list(range(0, 161)), [10, 10, 10, 5], [1 << 20, 131072, 131072 + 17, 999]])
def test_hh256_batch_lengths(oracle, lens):
    """Every HH remainder branch (size_mod32 = 0..31, & 16, & 3) vs the oracle, on
    unaligned and 16-byte aligned strides."""
    for align in (3, 16):
        _hh256_lengths(oracle, lens, align)


def _hh256_lengths(oracle, lens, align):
    rng = np.random.default_rng(len(lens))
    for L in sorted(set(lens)):
        n = 5
        stride = max(L, 1) + 3 if align == 3 else -(-max(L, 1) // 16) * 16  # unaligned / aligned stride
        host = rng.integers(0, 256, n * stride, dtype=np.uint8)
        d = torch.from_numpy(host).to(DEV)
        out = torch.zeros(n * 32, dtype=torch.uint8, device=DEV)
        z.hh256_batch(d, stride, L, n, out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().reshape(n, 32)
        for i in range(n):
            assert got[i].tobytes() == oracle.hh256(KEY, host[i * stride: i * stride + L].tobytes()), (L, i)


def test_hh256_verify_flags_corruption(oracle):
    """streamingBitrotReader.ReadAt: per-chunk errFileCorrupt, not whole-batch."""
    n, L = 200, 4096
    rng = np.random.default_rng(1)
    host = rng.integers(0, 256, n * L, dtype=np.uint8)
    want = np.stack([np.frombuffer(oracle.hh256(KEY, host[i * L:(i + 1) * L].tobytes()), np.uint8) for i in range(n)])
    bad_idx = [0, 17, 63, 64, 199]
    for i in bad_idx:
        host[i * L + (i * 7) % L] ^= 0x40
    d = torch.from_numpy(host).to(DEV)
    w = torch.from_numpy(want.reshape(-1).copy()).to(DEV)
    bad = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    z.hh256_verify_batch(d, L, L, n, w, bad)
    torch.cuda.synchronize()
    flags = bad.cpu().numpy()
    assert sorted(np.nonzero(flags)[0].tolist()) == bad_idx
    assert set(flags.tolist()) <= {0, 1}


def test_selftests_on_device():
    z.selftest()  # erasureSelfTest (60 KATs) + bitrotSelfTest through the GPU


def test_hh256_host_kats():
    pi100 = b"1415926535897932384626433832795028841971693993751058209749445923078164062862089986280348253421170679"
    assert z.hh256(pi100, key=bytes(32)) == KEY  # cmd/bitrot.go:36-37
    assert z.hh256(b"") == bytes.fromhex(
        z.hh256(b"").hex())  # smoke of the empty message path


@pytest.mark.parametrize("k,m,n", [(4, 2, 256), (8, 4, 1 << 20), (5, 3, 1000), (12, 4, 4097), (2, 2, 1)])
def test_host_encode_data_in_place(oracle, k, m, n):
    codec = z.Codec(k, m)
    buf = np.zeros(2 * max(n, 1 << 10) + 64 * (k + m), dtype=np.uint8)
    data = oracle.fill(3, 1, n)
    buf[:n] = data
    buf[n:] = 0xEE  # Split must zero [n, k*S)
    S, sums = codec.encode_data(buf, n, sums=True)
    want = oracle.encode_data(k, m, data)
    assert S == want.shape[1]
    assert np.array_equal(buf[:(k + m) * S].reshape(k + m, S), want)
    assert np.array_equal(sums, oracle.hh256_rows(KEY, want))


def test_erasure_encode_decode_reference_cases(oracle):
    """cmd/erasure_test.go:29-110 — TestErasureEncodeDecode's ten cases."""
    cases = [
        (2, 2, 0, 0, True, False), (3, 3, 1, 0, True, False), (4, 4, 2, 0, False, False),
        (5, 5, 0, 1, True, False), (6, 6, 0, 2, True, False), (7, 7, 1, 1, False, False),
        (8, 8, 3, 2, False, False), (2, 2, 2, 1, True, True), (4, 2, 2, 2, False, True),
        (8, 4, 2, 2, False, False),
    ]
    data = np.random.default_rng(0).integers(0, 256, 256, dtype=np.uint8).tobytes()
    for i, (k, m, md, mp, recon_parity, should_fail) in enumerate(cases):
        er = ze.NewErasure(k, m, ze.BLOCK_SIZE_V2)
        buffer = bytearray(data) + bytearray(len(data))  # len 256, cap 512
        encoded = er.EncodeData(buffer, len(data))
        for j in range(md):
            encoded[j] = None
        for j in range(k, k + mp):
            encoded[j] = None
        err = None
        try:
            if recon_parity:
                er.DecodeDataAndParityBlocks(encoded)
            else:
                er.DecodeDataBlocks(encoded)
        except z.ZS3Error as e:
            err = e
        assert (err is not None) == should_fail, f"case {i}: {err}"
        if not should_fail:
            if recon_parity:
                assert all(s is not None for s in encoded), i
            got = ze.write_data_blocks(encoded, k, 0, len(data))
            assert got == data, f"case {i}"


def test_bitrot_stream_roundtrip_reference_case(oracle):
    """cmd/bitrot_test.go:28-85 — 35 bytes in chunks of 10 (shardSize 10)."""
    from zs3server_amd import bitrot as zb
    w = zb.StreamingBitrotWriter(shard_size=10)
    for chunk in (b"a" * 10, b"a" * 10, b"a" * 10, b"a" * 5):
        w.Write(chunk)
    blob = w.getvalue()
    assert len(blob) == z.bitrot_shard_file_size(35, 10)
    # framing is [HH256(chunk)][chunk]
    assert blob[:32] == oracle.hh256(KEY, b"a" * 10)
    assert blob[-37:-5] == oracle.hh256(KEY, b"a" * 5)
    r = zb.StreamingBitrotReader(blob, till_offset=35, shard_size=10)
    assert r.ReadAt(10, 0) == b"a" * 10
    assert r.ReadAt(10, 10) == b"a" * 10
    assert r.ReadAt(10, 20) == b"a" * 10
    assert r.ReadAt(5, 30) == b"a" * 5
    # corruption -> errFileCorrupt (bitrot-streaming.go:182-185)
    bad = bytearray(blob)
    bad[32 + 3] ^= 1
    r2 = zb.StreamingBitrotReader(bytes(bad), till_offset=35, shard_size=10)
    with pytest.raises(z.ZS3Error) as ei:
        r2.ReadAt(10, 0)
    assert ei.value.code == -7
    assert zb.bitrot_verify(blob, 35 + 4 * 32, 35, 10) is None
    with pytest.raises(z.ZS3Error):
        zb.bitrot_verify(bytes(bad), 35 + 4 * 32, 35, 10)


def test_full_size_rs84_properties(oracle):
    """BASELINE config 3 at full size: RS(8+4), 4096 x 1 MiB, encode, then reconstruct
    with 2 erased data shards (0 and 5) and with 1 data + 1 parity erased; checked by
    round trip on every block and against the oracle on sampled blocks."""
    k, m, blen, nb = 8, 4, 1 << 20, 4096
    S = blen // k
    stride = (k + m) * S
    codec = z.Codec(k, m)
    d = torch.empty(nb * stride, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, stride, blen, nb, seed=2024)
    sums = torch.zeros(nb * (k + m) * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, stride, blen, nb, parity=d, parity_offset=k * S, parity_stride=stride, sums=sums)
    torch.cuda.synchronize()
    v = d.view(nb, k + m, S)
    hs = sums.view(nb, k + m, 32)
    mat = oracle.build_matrix(k, m)
    for b in (0, 1, 777, 2048, 4095):
        want = oracle.encode_data(k, m, oracle.fill(2024, b, blen), mat)
        assert np.array_equal(v[b].cpu().numpy(), want)
        assert np.array_equal(hs[b].cpu().numpy(), oracle.hh256_rows(KEY, want))
    # re-hash all shards with the standalone hash kernel: sums must agree everywhere
    sums2 = torch.zeros_like(sums)
    z.hh256_batch(d, S, S, nb * (k + m), sums2)
    torch.cuda.synchronize()
    assert torch.equal(sums, sums2)
    ref = d.clone()
    for erased, data_only in (([0, 5], True), ([2, 10], False)):
        for e in erased:
            v[:, e, :] = 0
        codec.reconstruct_batch(d, stride, S, nb, [i not in erased for i in range(k + m)], data_only)
        torch.cuda.synchronize()
        assert torch.equal(d, ref), erased
    del d, ref, sums, sums2
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k,m,nb", [(4, 2, 1024), (16, 4, 2048)])
def test_full_size_ws_defaults(oracle, k, m, nb):
    """BASELINE config 2 (RS(4+2), 1024 x 1 MiB) and RS(16+4) 2048 x 1 MiB at full size
    through the default launches (warp-specialised kernels); sampled blocks against the
    oracle, every parity byte and sum against cpu_ref (pinned to the oracle by
    tests/test_cpuref_pin.py)."""
    blen = 1 << 20
    S = blen // k
    stride = (k + m) * S
    codec = z.Codec(k, m)
    d = torch.empty(nb * stride, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, stride, blen, nb, seed=42)
    sums = torch.zeros(nb * (k + m) * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, stride, blen, nb, parity=d, parity_offset=k * S, parity_stride=stride, sums=sums)
    torch.cuda.synchronize()
    v = d.view(nb, k + m, S)
    hs = sums.view(nb, k + m, 32)
    mat = oracle.build_matrix(k, m)
    for b in (0, 3, nb // 2 - 1, nb - 1):
        want = oracle.encode_data(k, m, oracle.fill(42, b, blen), mat)
        assert np.array_equal(v[b].cpu().numpy(), want)
        assert np.array_equal(hs[b].cpu().numpy(), oracle.hh256_rows(KEY, want))
    from oracle import cpuref
    R = k + m
    host = d.cpu().numpy().reshape(nb, R * S)
    par = np.empty(nb * m * S, np.uint8)
    sref = np.empty(nb * R * 32, np.uint8)
    cpuref.encode_hash(k, m, mat, np.ascontiguousarray(host), blen, nb, R * S, par, m * S, sref, KEY,
                       cpuref.threads_available())
    assert np.array_equal(host[:, k * S:], par.reshape(nb, m * S))
    assert np.array_equal(sums.cpu().numpy(), sref)
    del d, sums
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k,m,bs,nfull,tail,batch,pinned", [
    (4, 2, 1 << 16, 5, 1000, 2, False), (8, 4, 1 << 16, 7, 0, 3, True), (16, 4, 1 << 16, 3, 17, 8, False),
    (8, 4, 1 << 20, 4, (1 << 19) + 3, 2, True),
])
def test_stream_encode_end_to_end(oracle, k, m, bs, nfull, tail, batch, pinned):
    """zs3_stream_encode: host stream -> H2D -> fused kernel -> D2H, multiple
    double-buffered batches plus a partial last block (erasure-encode.go:83-111)."""
    codec = z.Codec(k, m, bs)
    total = nfull * bs + tail
    S = -(-bs // k)
    nblk = nfull + (1 if tail else 0)
    data = np.concatenate([oracle.fill(31, b, bs) for b in range(nblk)])[:total]
    bufs = []
    if pinned:
        src = z.HostBuffer(max(total, 1))
        src.array[:total] = data
        par = z.HostBuffer(nblk * m * S)
        sums = z.HostBuffer(nblk * (k + m) * 32)
        bufs = [src, par, sums]
        par_a, sums_a = par.array, sums.array
    else:
        src, par_a, sums_a = data.copy(), np.zeros(nblk * m * S, np.uint8), np.zeros(nblk * (k + m) * 32, np.uint8)
        par, sums = par_a, sums_a
    assert codec.stream_encode(src, total, par, sums, batch_blocks=batch) == nblk
    mat = oracle.build_matrix(k, m)
    for b in range(nblk):
        blk = data[b * bs: min((b + 1) * bs, total)]
        want = oracle.encode_data(k, m, blk, mat)
        Sb = want.shape[1]
        got_p = par_a[b * m * S: b * m * S + m * Sb].reshape(m, Sb)
        assert np.array_equal(got_p, want[k:]), b
        assert np.array_equal(sums_a[b * (k + m) * 32:(b + 1) * (k + m) * 32].reshape(k + m, 32),
                              oracle.hh256_rows(KEY, want)), b
    for x in bufs:
        x.free()
