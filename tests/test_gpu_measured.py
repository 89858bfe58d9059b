"""Parity on exactly the workloads the measured numbers come from (bench.py).

* BASELINE config 4 as bench.py runs it: the N = 1 share (65 536 x 1 MiB RS(8+4)
  objects, one launch, seed 1234) and an N = 2 share (32 768 objects starting at object
  32 768), every parity byte and bitrot sum compared chunk by chunk with cpu_ref
  (itself pinned to the scalar oracle by tests/test_cpuref_pin.py), three blocks per
  share against the scalar oracle.
* The profiled GET / heal shapes: 1 MiB blocks, RS(8+4) x 4 096 and RS(16+4) x 2 048
  stripes through the product dispatch (k_vr_ws): verify + rebuild 2, heal 2 and
  heal 4, every rebuilt row and heal sum against oracle stripes.
* SURVEY.md §8(d) synthetic edge inputs: all-zero and all-0xFF batches at the BASELINE
  shapes RS(4+2) x 1 024, RS(8+4) x 4 096 and RS(16+4) x 2 048, encode + sums and a
  reconstruct round trip.
* Per-block erasure patterns on the warp-specialised GET kernel (block-id lists through
  k_vr_ws, groups larger than the small-batch path takes).

Reference: cmd/erasure-encode.go:83-111, cmd/erasure-coding.go:77-119,
cmd/bitrot-streaming.go:43-65, 142-189, cmd/erasure-decode.go:165-179, 287-332.
"""
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


@pytest.fixture(autouse=True)
def _release_cache():
    yield
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # the tests' multi-GiB buffers are garbage once they return


def chunked_check(oracle, k, m, d, sums, nb, S, seed, obj0, chunk=1024, samples=3):
    """Every block's parity rows and sums vs cpu_ref on the same data rows, chunk by
    chunk (np.array_equal), plus `samples` blocks vs the scalar oracle from oracle_fill."""
    R = k + m
    mat = oracle.build_matrix(k, m)
    T = cpuref.threads_available()
    for b0 in range(0, nb, chunk):
        n = min(chunk, nb - b0)
        blk = d[b0 * R * S:(b0 + n) * R * S].cpu().numpy()
        sm = sums[b0 * R * 32:(b0 + n) * R * 32].cpu().numpy()
        par = np.empty(n * m * S, np.uint8)
        sref = np.empty(n * R * 32, np.uint8)
        cpuref.encode_hash(k, m, mat, blk, k * S, n, R * S, par, m * S, sref, KEY, T)
        assert np.array_equal(blk.reshape(n, R, S)[:, k:], par.reshape(n, m, S)), f"parity, blocks {b0}..{b0 + n}"
        assert np.array_equal(sm, sref), f"sums, blocks {b0}..{b0 + n}"
    for b in np.linspace(0, nb - 1, samples).astype(int).tolist():
        v = d[b * R * S:(b + 1) * R * S].cpu().numpy().reshape(R, S)
        want = oracle.encode_data(k, m, oracle.fill(seed, obj0 + b, k * S), mat)
        assert np.array_equal(v, want), b
        assert np.array_equal(sums[b * R * 32:(b + 1) * R * 32].cpu().numpy().reshape(R, 32),
                              oracle.hh256_rows(KEY, want)), b


@pytest.mark.parametrize("nb,obj0", [(65536, 0), (32768, 32768)], ids=["N1-share", "N2-rank1-share"])
def test_config4_bench_share(oracle, nb, obj0):
    """bench.py's own sequence (fill_batch seed 1234 at the rank's first object, one
    encode_batch over the share in the in-place layout) on the N = 1 and N = 2 shares."""
    k, m = 8, 4
    S = MiB // k
    R = k + m
    codec = z.Codec(k, m, MiB)
    d = torch.empty(nb * R * S, dtype=torch.uint8, device=DEV)
    sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, MiB, nb, seed=1234, obj0=obj0)
    codec.encode_batch(d, R * S, MiB, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    assert z.last_path() == 2, "config 4 runs on the warp-specialised kernel"
    chunked_check(oracle, k, m, d, sums, nb, S, 1234, obj0)


@pytest.mark.parametrize("k,m,nb", [(4, 2, 1024), (16, 4, 2048), (8, 4, 4096)])
def test_profiled_encode_shapes_full_check(oracle, k, m, nb):
    """BASELINE config 2 (RS(4+2) x 1 024), RS(16+4) x 2 048 and config 3's encode
    (RS(8+4) x 4 096) as profiled: every parity byte and sum vs cpu_ref."""
    S = MiB // k
    R = k + m
    codec = z.Codec(k, m, MiB)
    d = torch.empty(nb * R * S, dtype=torch.uint8, device=DEV)
    sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, MiB, nb, seed=42, obj0=0)
    codec.encode_batch(d, R * S, MiB, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    assert z.last_path() == 2
    chunked_check(oracle, k, m, d, sums, nb, S, 42, 0)


# Distinct oracle stripes per batch: prime, so the period is coprime with every
# workgroup's stripe count G (4 / 8 / 16) and with the tile loops: a kernel that reads or
# writes the wrong stripe (shifted by any multiple of G) cannot land on an identical copy.
PERIOD = 61


def _tiled_stripes(oracle, k, m, blen, nb, seed, distinct=PERIOD):
    """`distinct` oracle stripes (+ their sums) and the device index of the stripe each of
    the nb batch positions holds (position b holds stripe b % distinct)."""
    R = k + m
    S = -(-blen // k)
    mat = oracle.build_matrix(k, m)
    base = np.stack([oracle.encode_data(k, m, oracle.fill(seed, b, blen), mat).reshape(R, S)
                     for b in range(distinct)])
    bsum = np.stack([oracle.hh256_rows(KEY, s) for s in base])
    idx = torch.arange(nb, device=DEV) % distinct
    return base, bsum, idx


@pytest.mark.parametrize("k,m,nb,erased,heal", [
    (8, 4, 4096, [0, 5], False), (8, 4, 4096, [2, 10], True), (8, 4, 4096, [1, 3, 8, 11], True),
    (16, 4, 2048, [0, 5], False), (16, 4, 2048, [3, 17], True), (16, 4, 2048, [0, 1, 16, 19], True),
    (16, 4, 2048, [2, 7, 9, 12], False),
], ids=lambda v: str(v))
def test_get_heal_profiled_shape(oracle, k, m, nb, erased, heal):
    """GET (verify the survivors + rebuild the lost data rows) and heal (rebuild every
    lost row + hash it) at the profiled shape: 1 MiB blocks, product dispatch, one
    rotted survivor flagged exactly."""
    R = k + m
    base, bsum, idx = _tiled_stripes(oracle, k, m, MiB, nb, seed=17)
    S = base.shape[2]
    codec = z.Codec(k, m, MiB)
    ref = torch.from_numpy(base).to(DEV)
    refs = torch.from_numpy(bsum).to(DEV)
    d = ref[idx].contiguous()
    for e in erased:
        d[:, e, :] = 0x5A
    surv = [i for i in range(R) if i not in erased][:k]
    bad_blk, bad_row = nb - 3, surv[-1]
    d[bad_blk, bad_row, 12345] ^= 1
    exp = refs[idx].contiguous()
    bad = torch.full((nb, R), 7, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    present = [i not in erased for i in range(R)]
    codec.verify_reconstruct_batch(d, R * S, S, nb, present, not heal, exp, bad, sums_out=out)
    torch.cuda.synchronize()
    assert z.last_path() == 2, "profiled shape runs k_vr_ws"
    want_bad = np.zeros((nb, R), np.int32)
    want_bad[bad_blk, bad_row] = 1
    assert np.array_equal(bad.cpu().numpy(), want_bad)
    rebuilt = [i for i in erased if i < k or heal]
    ok = torch.ones(nb, dtype=torch.bool, device=DEV)
    ok[bad_blk] = False  # rebuilt from a rotted survivor: garbage by design
    for i in rebuilt:
        same = (d[:, i, :] == ref[idx, i, :]).all(dim=1)
        assert bool(same[ok].all()), f"rebuilt shard {i}"
        if heal:
            assert bool((out[:, i, :] == refs[idx, i, :]).all(dim=1)[ok].all()), f"heal sum of shard {i}"
    for i in range(R):
        if i in erased and i not in rebuilt:
            assert bool((d[:, i, :] == 0x5A).all()), "ReconstructData leaves lost parity untouched"
        elif i not in erased:
            assert bool((d[:, i, :] == ref[idx, i, :]).all(dim=1)[ok].all()), f"survivor {i} untouched"


@pytest.mark.parametrize("fillv", [0x00, 0xFF], ids=["zero", "ff"])
@pytest.mark.parametrize("k,m,nb", [(4, 2, 1024), (8, 4, 4096), (16, 4, 2048), (8, 4, 300)])
def test_constant_input_batches(oracle, k, m, nb, fillv):
    """All-zero and all-0xFF objects through the default encode dispatch
    of each BASELINE shape, then ReconstructData of two lost data rows and heal of a
    lost parity row; every block equals the oracle's encode of one such block."""
    R = k + m
    S = MiB // k
    codec = z.Codec(k, m, MiB)
    d = torch.full((nb, R, S), fillv, dtype=torch.uint8, device=DEV)
    d[:, k:, :] = 0x3C
    sums = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, R * S, MiB, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    want = oracle.encode_data(k, m, np.full(MiB, fillv, np.uint8))
    wsum = oracle.hh256_rows(KEY, want)
    wt = torch.from_numpy(want).to(DEV)
    assert bool((d == wt[None]).all()), "parity"
    assert bool((sums == torch.from_numpy(wsum).to(DEV)[None]).all()), "sums"
    erased = [1, k - 1]
    for e in erased:
        d[:, e, :] = 0x11
    codec.reconstruct_batch(d, R * S, S, nb, [i not in erased for i in range(R)], True)
    d[:, k, :] = 0x22
    codec.reconstruct_batch(d, R * S, S, nb, [i != k for i in range(R)], False)
    torch.cuda.synchronize()
    assert bool((d == wt[None]).all()), "reconstruct round trip"


@pytest.mark.parametrize("k,m,blen", [(8, 4, 1 << 16), (16, 4, 1 << 16), (12, 4, 12 * 5000 + 6)])
@pytest.mark.parametrize("heal", [False, True])
def test_masks_on_ws_kernel(oracle, k, m, blen, heal):
    """Per-block patterns whose groups exceed the small-batch path (> 2 048 blocks per
    pattern), so every group runs k_vr_ws with its block-id list: three
    interleaved patterns over 7 680 blocks, one rotted survivor flagged exactly."""
    R = k + m
    nb = 7680
    base, bsum, idx = _tiled_stripes(oracle, k, m, blen, nb, seed=23)
    S = base.shape[2]
    pats_list = [[0, 5], [k, R - 1], [2]] if not heal else [[0, 5], [k, R - 1], [2, k + 1]]
    rng = np.random.default_rng(k + heal)
    which = rng.integers(0, len(pats_list), nb)
    pats = np.ones((nb, R), dtype=bool)
    for b in range(nb):
        pats[b, pats_list[which[b]]] = False
    d = torch.from_numpy(base).to(DEV)[idx].contiguous()
    pt = torch.from_numpy(pats).to(DEV)
    d[~pt] = 0x66
    rb = 4000
    surv = [i for i in range(R) if pats[rb, i]][:k]
    d[rb, surv[0], S - 1] ^= 0x80
    exp = torch.from_numpy(bsum).to(DEV)[idx].contiguous()
    bad = torch.full((nb, R), 9, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    codec = z.Codec(k, m, blen)
    status = np.full(nb, 99, np.int32)
    rc = codec.verify_reconstruct_batch_masks(d, R * S, S, nb, pats, not heal, exp, bad, sums_out=out, status=status)
    torch.cuda.synchronize()
    assert rc == 0 and not status.any()
    assert z.last_path() == 2, "large pattern groups run k_vr_ws"
    want_bad = np.zeros((nb, R), np.int32)
    want_bad[rb, surv[0]] = 1
    assert np.array_equal(bad.cpu().numpy(), want_bad)
    ref = torch.from_numpy(base).to(DEV)[idx]
    ok = torch.ones(nb, dtype=torch.bool, device=DEV)
    ok[rb] = False
    rows_ok = (d == ref).all(dim=2)  # [nb, R]
    expect_rows = pt.clone()
    expect_rows[:, :k] = True
    if heal:
        expect_rows[:] = True
    assert bool(rows_ok[ok][expect_rows[ok]].all()), "rebuilt rows"
    if heal:
        lost = ~pt
        eq = (out == exp).all(dim=2)
        assert bool(eq[ok][lost[ok]].all()), "heal sums of the rebuilt rows"


@pytest.mark.parametrize("k,m,nb,blen", [(12, 4, 4096, MiB), (12, 4, 2051, MiB), (12, 4, 1025, MiB), (12, 4, 1024, MiB),
                                         (12, 4, 5, MiB), (12, 4, 1031, 12 * 87392), (4, 4, 4096, MiB),
                                         (4, 4, 1024, MiB), (4, 4, 3, MiB)])
def test_server_default_geometries(oracle, k, m, nb, blen):
    """The server's default erasure geometries (getDefaultParityBlocks,
    cmd/format-erasure.go:870-881): RS(12+4) for 16-drive sets (1 MiB blocks: S = 87 382,
    rows 2-byte aligned, 8 bytes of Split padding, 22-byte HighwayHash remainder) and
    RS(4+4) for 8-drive sets, through the default dispatch; every block vs cpu_ref.  Blocks
    of 12 x 87 392 bytes give RS(12+4) 16-byte-aligned rows (the aligned-row dispatch)."""
    R = k + m
    S = -(-blen // k)
    codec = z.Codec(k, m, blen)
    d = torch.zeros(nb * R * S, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, blen, nb, seed=77, obj0=0)
    if k * S > blen:  # bytes past the object: Split must read them as zero
        d.view(nb, R * S)[:, blen:k * S] = 0xEE
    sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, R * S, blen, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    if nb >= 1024:
        assert z.last_path() == 2, "warp-specialised kernel"
    mat = oracle.build_matrix(k, m)
    host = d.cpu().numpy().reshape(nb, R * S)
    hs = sums.cpu().numpy()
    for b0 in range(0, nb, 1024):
        n = min(1024, nb - b0)
        par = np.empty(n * m * S, np.uint8)
        sref = np.empty(n * R * 32, np.uint8)
        blk = np.ascontiguousarray(host[b0:b0 + n])
        cpuref.encode_hash(k, m, mat, blk, blen, n, R * S, par, m * S, sref, KEY, cpuref.threads_available())
        assert np.array_equal(blk[:, k * S:], par.reshape(n, m * S)), f"parity, blocks {b0}.."
        assert np.array_equal(hs[b0 * R * 32:(b0 + n) * R * 32], sref), f"sums, blocks {b0}.."
    want = oracle.encode_data(k, m, oracle.fill(77, nb - 1, blen), mat)
    assert np.array_equal(host[nb - 1, k * S:].reshape(m, S), want[k:])


@pytest.mark.parametrize("blen", [MiB + 12 * 7, 12 * 384 * 3 + 200, 12 * 999 + 5, MiB - 4000])
def test_rs124_ragged_blocks(oracle, blen):
    """RS(12+4) on other block lengths: the unaligned-row kernel where the Split padding
    fits its tail tile, the generic kernel otherwise; bit-exact either way."""
    k, m, nb = 12, 4, 37
    R = k + m
    S = -(-blen // k)
    codec = z.Codec(k, m, MiB)
    d = torch.full((nb * R * S,), 0xEE, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, blen, nb, seed=5, obj0=0)
    sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, R * S, blen, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    host = d.cpu().numpy().reshape(nb, R, S)
    hs = sums.cpu().numpy().reshape(nb, R, 32)
    mat = oracle.build_matrix(k, m)
    for b in range(nb):
        want = oracle.encode_data(k, m, oracle.fill(5, b, blen), mat)
        assert np.array_equal(host[b, k:], want[k:]), b
        assert np.array_equal(hs[b], oracle.hh256_rows(KEY, want)), b


@pytest.mark.parametrize("k,m,nb", [(11, 5, 1024), (10, 6, 1024), (5, 4, 512), (7, 3, 300), (9, 7, 256), (13, 3, 64)])
def test_any_geometry_encode(oracle, k, m, nb):
    """Geometries of other set sizes and parity upgrades (cmd/erasure-object.go:724-775):
    the any-geometry encode (8-byte columns at unaligned row offsets) + the batched hash
    in stripe mode; 1 MiB blocks, every block vs cpu_ref, Split padding bytes poisoned."""
    R = k + m
    S = -(-MiB // k)
    codec = z.Codec(k, m, MiB)
    d = torch.zeros(nb * R * S, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, MiB, nb, seed=k * 10 + m, obj0=0)
    if k * S > MiB:
        d.view(nb, R * S)[:, MiB:k * S] = 0xEE
    sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, R * S, MiB, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    mat = oracle.build_matrix(k, m)
    host = d.cpu().numpy().reshape(nb, R * S)
    par = np.empty(nb * m * S, np.uint8)
    sref = np.empty(nb * R * 32, np.uint8)
    cpuref.encode_hash(k, m, mat, np.ascontiguousarray(host), MiB, nb, R * S, par, m * S, sref, KEY,
                       cpuref.threads_available())
    assert np.array_equal(host[:, k * S:], par.reshape(nb, m * S))
    assert np.array_equal(sums.cpu().numpy(), sref)


@pytest.mark.parametrize("k,m,erased,heal", [(12, 4, [0, 5], False), (12, 4, [3, 13], True),
                                             (12, 4, [0, 1, 2, 15], True), (12, 4, [], False), (12, 4, [7], False),
                                             (12, 4, [2, 9, 14], False), (12, 4, [1, 2, 3, 4], False),
                                             (12, 4, [6], True), (12, 4, [0, 11, 12], True),
                                             (11, 5, [1, 4, 12], True),
                                             (10, 6, [0, 9], False), (5, 4, [4, 5, 6, 7], True)])
def test_any_geometry_get_heal(oracle, k, m, erased, heal):
    """GET / heal at unaligned shard sizes on 1 MiB blocks: RS(12+4) (S = 87 382) on the
    warp-specialised kernel in UA mode (round 3), the other geometries as survivors
    verified in one stripe-mode hash launch, the rebuild, rebuilt rows hashed in one
    launch; one rotted survivor flagged exactly; 512 stripes of 61 distinct oracle
    stripes."""
    R = k + m
    nb = 512
    base, bsum, idx = _tiled_stripes(oracle, k, m, MiB, nb, seed=31)
    S = base.shape[2]
    codec = z.Codec(k, m, MiB)
    ref = torch.from_numpy(base).to(DEV)
    refs = torch.from_numpy(bsum).to(DEV)
    d = ref[idx].contiguous()
    for e in erased:
        d[:, e, :] = 0x5A
    surv = [i for i in range(R) if i not in erased][:k]
    bad_blk, bad_row = 77, surv[2]
    d[bad_blk, bad_row, S - 1] ^= 4
    exp = refs[idx].contiguous()
    bad = torch.full((nb, R), 7, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    codec.verify_reconstruct_batch(d, R * S, S, nb, [i not in erased for i in range(R)], not heal, exp, bad,
                                   sums_out=out)
    torch.cuda.synchronize()
    if k == 12 and 1 <= len(erased) <= 4:
        assert z.last_path() == 2, z.last_path()
    want_bad = np.zeros((nb, R), np.int32)
    want_bad[bad_blk, bad_row] = 1
    assert np.array_equal(bad.cpu().numpy(), want_bad)
    ok = torch.ones(nb, dtype=torch.bool, device=DEV)
    ok[bad_blk] = False
    for i in erased:
        if i < k or heal:
            assert bool((d[:, i, :] == ref[idx, i, :]).all(dim=1)[ok].all()), f"rebuilt shard {i}"
            if heal:
                assert bool((out[:, i, :] == refs[idx, i, :]).all(dim=1)[ok].all()), f"heal sum {i}"
        else:
            assert bool((d[:, i, :] == 0x5A).all())
    for i in range(R):  # nothing written outside the rebuilt rows (ragged last column)
        if i not in erased:
            assert bool((d[:, i, :] == ref[idx, i, :]).all(dim=1)[ok].all()), f"survivor {i}"


@pytest.mark.parametrize("k,m,blen,erased,data_only", [
    (12, 4, MiB, [0, 5], True), (12, 4, MiB, [1, 13, 14, 15], False), (12, 4, MiB, [0, 1, 2, 3], True),
    (10, 6, MiB, [0, 1, 2, 3], True), (6, 3, MiB, [2, 7], False), (5, 4, MiB, [4], True),
    (4, 2, MiB + 7, [0, 5], False), (8, 4, 8 * 1000 + 3, [3, 9, 10], False), (2, 1, 21, [0], True)],
    ids=lambda v: str(v))
def test_reconstruct_unaligned_rows(oracle, k, m, blen, erased, data_only):
    """ReconstructData / Reconstruct at shard sizes that are not a multiple of 16 (1 MiB
    blocks of RS(12+4), RS(10+6), RS(5+4); ragged block lengths): the specialised
    reconstruct kernel with unaligned rows and a byte-wise last column, every byte of
    every block vs the oracle's encode (rows outside the rebuilt ones untouched)."""
    R = k + m
    nb = 9
    S = -(-blen // k)
    mat = oracle.build_matrix(k, m)
    base = np.stack([oracle.encode_data(k, m, oracle.fill(41, b, blen), mat).reshape(R, S) for b in range(nb)])
    d = torch.from_numpy(base).to(DEV).contiguous()
    for e in erased:
        d[:, e, :] = 0xA5
    z.Codec(k, m, MiB).reconstruct_batch(d, R * S, S, nb, [i not in erased for i in range(R)], data_only)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    for i in range(R):
        if i in erased and i >= k and data_only:
            assert (got[:, i, :] == 0xA5).all(), f"row {i} written"
        else:
            assert np.array_equal(got[:, i, :], base[:, i, :]), f"row {i}"


@pytest.mark.parametrize("k,m,blen", [(12, 4, MiB), (10, 4, MiB), (8, 4, 8 * 1000 + 3), (4, 2, MiB + 7),
                                      (16, 4, 16 * 777 + 1), (2, 1, 21), (6, 3, 6 * 40 + 1)],
                         ids=lambda v: str(v))
def test_encode_only_unaligned_rows(oracle, k, m, blen):
    """EncodeData without sums at shard sizes that are not a multiple of 16 and with Split
    padding (RS(12+4) / RS(10+4) on 1 MiB blocks, ragged lengths): the specialised
    encode-only kernel in UA mode (round 4); padding bytes poisoned in memory must read as
    zero, every parity byte vs the oracle."""
    R = k + m
    nb = 9
    S = -(-blen // k)
    d = torch.zeros(nb * R * S, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, blen, nb, seed=k * 7 + m, obj0=0)
    if k * S > blen:
        d.view(nb, R * S)[:, blen:k * S] = 0xEE
    z.Codec(k, m, MiB).encode_batch(d, R * S, blen, nb, parity=d, parity_offset=k * S, parity_stride=R * S)
    torch.cuda.synchronize()
    host = d.cpu().numpy().reshape(nb, R * S)
    mat = oracle.build_matrix(k, m)
    for b in range(nb):
        want = oracle.encode_data(k, m, oracle.fill(k * 7 + m, b, blen), mat).reshape(-1)
        assert np.array_equal(host[b, k * S:], want[k * S:]), f"parity, block {b}"
        assert np.array_equal(host[b, :blen], want[:blen]), f"data, block {b}"


GEN_GEOMS = [(2, 2), (3, 2), (3, 3), (4, 3), (5, 4), (6, 4), (7, 4), (9, 4), (10, 4), (11, 4)]


@pytest.mark.parametrize("nb", [1024, 1031])
@pytest.mark.parametrize("k,m", GEN_GEOMS, ids=lambda v: str(v))
def test_default_geometries_ws_encode(oracle, k, m, nb):
    """The server's non-dyadic default geometries (getDefaultParityBlocks,
    cmd/format-erasure.go:870-881: 4-7 and 9-15-drive sets) on the warp-specialised
    kernel with a general coding matrix (fused_v2_gen.hip, round 4): 1 MiB blocks, Split
    padding poisoned in memory, a last workgroup with dead stripes (nb = 1031), every
    parity byte and bitrot sum vs cpu_ref, two blocks vs the scalar oracle."""
    R = k + m
    S = -(-MiB // k)
    codec = z.Codec(k, m, MiB)
    d = torch.zeros(nb * R * S, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, MiB, nb, seed=k * 31 + m, obj0=0)
    if k * S > MiB:
        d.view(nb, R * S)[:, MiB:k * S] = 0xEE
    sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, R * S, MiB, nb, parity=d, parity_offset=k * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    assert z.last_path() == 2, "warp-specialised kernel (general matrix)"
    mat = oracle.build_matrix(k, m)
    host = d.cpu().numpy().reshape(nb, R * S)
    hs = sums.cpu().numpy()
    par = np.empty(nb * m * S, np.uint8)
    sref = np.empty(nb * R * 32, np.uint8)
    cpuref.encode_hash(k, m, mat, np.ascontiguousarray(host), MiB, nb, R * S, par, m * S, sref, KEY,
                       cpuref.threads_available())
    assert np.array_equal(host[:, k * S:], par.reshape(nb, m * S)), "parity"
    assert np.array_equal(hs, sref), "sums"
    for b in (0, nb - 1):
        want = oracle.encode_data(k, m, oracle.fill(k * 31 + m, b, MiB), mat)
        assert np.array_equal(host[b, k * S:].reshape(m, S), want[k:]), b
        assert np.array_equal(hs[b * R * 32:(b + 1) * R * 32].reshape(R, 32), oracle.hh256_rows(KEY, want)), b


def _gen_get_cases():
    cases = []
    for k, m in GEN_GEOMS:
        R = k + m
        e = min(m, 4)
        # every parity row + the lowest data rows lost, healed; two data rows rebuilt
        cases.append((k, m, sorted(list(range(k, R))[: e - 1] + [0]), True))
        cases.append((k, m, [k // 2, k - 1] if k > 2 else [0, 1], False))
    cases += [(5, 4, [1], False), (11, 4, [2, 12, 13], False), (3, 3, [1], True), (2, 2, [3], True)]
    # RS(4+4), the 8-drive default: 1, 3 and 4 lost rows (round 4 instances)
    cases += [(4, 4, [0, 2, 5], True), (4, 4, [0, 1, 2, 3], False), (4, 4, [1, 4, 6, 7], True), (4, 4, [3], True),
              (4, 4, [1, 2, 7], False)]
    return cases


@pytest.mark.parametrize("k,m,erased,heal", _gen_get_cases(), ids=lambda v: str(v))
def test_default_geometries_ws_get_heal(oracle, k, m, erased, heal):
    """GET / heal of the non-dyadic server-default geometries on the warp-specialised
    k_vr_ws (fused_v2_get_gen.hip, round 4; UA mode for every k but 2) and RS(4+4) with
    1, 3 or 4 lost rows (fused_v2_get.hip, round 4): 1 MiB blocks,
    1031 stripes (a last workgroup with dead stripes) tiled from 61 distinct oracle
    stripes, one rotted survivor flagged exactly, every rebuilt byte and heal sum vs the
    oracle, survivors and lost parity (ReconstructData) untouched."""
    R = k + m
    nb = 1031
    base, bsum, idx = _tiled_stripes(oracle, k, m, MiB, nb, seed=k * 13 + m)
    S = base.shape[2]
    codec = z.Codec(k, m, MiB)
    ref = torch.from_numpy(base).to(DEV)
    refs = torch.from_numpy(bsum).to(DEV)
    d = ref[idx].contiguous()
    for e in erased:
        d[:, e, :] = 0x5A
    surv = [i for i in range(R) if i not in erased][:k]
    bad_blk, bad_row = nb - 2, surv[-1]
    d[bad_blk, bad_row, S - 1] ^= 0x10
    exp = refs[idx].contiguous()
    bad = torch.full((nb, R), 7, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    codec.verify_reconstruct_batch(d, R * S, S, nb, [i not in erased for i in range(R)], not heal, exp, bad,
                                   sums_out=out)
    torch.cuda.synchronize()
    if k != 4 or m == 4:
        assert z.last_path() == 2, z.last_path()
    want_bad = np.zeros((nb, R), np.int32)
    want_bad[bad_blk, bad_row] = 1
    assert np.array_equal(bad.cpu().numpy(), want_bad)
    ok = torch.ones(nb, dtype=torch.bool, device=DEV)
    ok[bad_blk] = False
    for i in erased:
        if i < k or heal:
            assert bool((d[:, i, :] == ref[idx, i, :]).all(dim=1)[ok].all()), f"rebuilt shard {i}"
            if heal:
                assert bool((out[:, i, :] == refs[idx, i, :]).all(dim=1)[ok].all()), f"heal sum {i}"
        else:
            assert bool((d[:, i, :] == 0x5A).all())
    for i in range(R):
        if i not in erased:
            assert bool((d[:, i, :] == ref[idx, i, :]).all(dim=1)[ok].all()), f"survivor {i}"


@pytest.mark.parametrize("k,m", GEN_GEOMS + [(12, 4)], ids=lambda v: str(v))
def test_default_geometries_encode_only(oracle, k, m):
    """EncodeData without sums for the server-default geometries on 1 MiB blocks (UA mode
    of the specialised encode-only kernel for every unaligned k, round 4): 1031 stripes,
    Split padding poisoned in memory, every parity byte vs cpu_ref, two blocks vs the
    scalar oracle."""
    R = k + m
    nb = 1031
    S = -(-MiB // k)
    d = torch.zeros(nb * R * S, dtype=torch.uint8, device=DEV)
    z.fill_batch(d, R * S, MiB, nb, seed=k * 17 + m, obj0=0)
    if k * S > MiB:
        d.view(nb, R * S)[:, MiB:k * S] = 0xEE
    z.Codec(k, m, MiB).encode_batch(d, R * S, MiB, nb, parity=d, parity_offset=k * S, parity_stride=R * S)
    torch.cuda.synchronize()
    assert z.last_path() == 1, z.last_path()
    mat = oracle.build_matrix(k, m)
    host = d.cpu().numpy().reshape(nb, R * S)
    clean = host.copy()
    clean[:, MiB:k * S] = 0
    par = np.empty(nb * m * S, np.uint8)
    cpuref.encode_hash(k, m, mat, np.ascontiguousarray(clean), MiB, nb, R * S, par, m * S, None, KEY,
                       cpuref.threads_available())
    assert np.array_equal(host[:, k * S:], par.reshape(nb, m * S)), "parity"
    assert (host[:, MiB:k * S] == 0xEE).all(), "Split padding left as it was"
    for b in (0, nb - 1):
        want = oracle.encode_data(k, m, oracle.fill(k * 17 + m, b, MiB), mat)
        assert np.array_equal(host[b, k * S:].reshape(m, S), want[k:]), b


@pytest.mark.parametrize("erased,heal", [([0, 5], False), ([3, 13], True), ([1, 2, 14, 15], True)],
                         ids=lambda v: str(v))
def test_rs124_aligned_rows_get_heal(oracle, erased, heal):
    """RS(12+4) at a 16-byte-aligned shard size (blocks of 12 x 65 536 bytes): GET / heal
    on the warp-specialised kernel (round 4: the UA instances serve aligned rows too; the
    first-generation kernel before), 1 401 stripes (past the small-batch latency path's
    1 GiB, a last workgroup with dead stripes) of 61 distinct oracle stripes, one rotted
    survivor flagged exactly."""
    k, m, blen = 12, 4, 12 * 65536
    R = k + m
    nb = 1401
    base, bsum, idx = _tiled_stripes(oracle, k, m, blen, nb, seed=97)
    S = base.shape[2]
    assert S % 16 == 0
    codec = z.Codec(k, m, blen)
    ref = torch.from_numpy(base).to(DEV)
    refs = torch.from_numpy(bsum).to(DEV)
    d = ref[idx].contiguous()
    for e in erased:
        d[:, e, :] = 0x5A
    surv = [i for i in range(R) if i not in erased][:k]
    bad_blk, bad_row = 500, surv[4]
    d[bad_blk, bad_row, 777] ^= 0x40
    exp = refs[idx].contiguous()
    bad = torch.full((nb, R), 7, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    codec.verify_reconstruct_batch(d, R * S, S, nb, [i not in erased for i in range(R)], not heal, exp, bad,
                                   sums_out=out)
    torch.cuda.synchronize()
    assert z.last_path() == 2, z.last_path()
    want_bad = np.zeros((nb, R), np.int32)
    want_bad[bad_blk, bad_row] = 1
    assert np.array_equal(bad.cpu().numpy(), want_bad)
    ok = torch.ones(nb, dtype=torch.bool, device=DEV)
    ok[bad_blk] = False
    for i in erased:
        if i < k or heal:
            assert bool((d[:, i, :] == ref[idx, i, :]).all(dim=1)[ok].all()), f"rebuilt shard {i}"
            if heal:
                assert bool((out[:, i, :] == refs[idx, i, :]).all(dim=1)[ok].all()), f"heal sum {i}"
        else:
            assert bool((d[:, i, :] == 0x5A).all())
    for i in range(R):
        if i not in erased:
            assert bool((d[:, i, :] == ref[idx, i, :]).all(dim=1)[ok].all()), f"survivor {i}"
