"""GPU parity for the GET / heal pass (zs3_verify_reconstruct_batch).

Reference semantics: streamingBitrotReader.ReadAt (bitrot-streaming.go:171-186) compares
each chunk's HighwayHash-256 with the stored 32-byte sum and returns errFileCorrupt for
that shard only; parallelReader (erasure-decode.go:165-179) then treats the shard as
missing and reads the next one; DecodeDataBlocks / DecodeDataAndParityBlocks
(erasure-coding.go:96-119) rebuild from the first k shards read.  The oracle supplies
the shards (encode), the stored sums (hh256 per shard) and the expected rebuilt rows.
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


def stripes(oracle, k, m, blen, nb, seed=11):
    """Oracle-encoded stripes [nb][k+m][S] and their stored bitrot sums [nb][k+m][32]."""
    S = -(-blen // k)
    mat = oracle.build_matrix(k, m)
    sh = np.zeros((nb, k + m, S), dtype=np.uint8)
    sums = np.zeros((nb, k + m, 32), dtype=np.uint8)
    for b in range(nb):
        sh[b] = oracle.encode_data(k, m, oracle.fill(seed, b, blen), mat).reshape(k + m, S)
        sums[b] = oracle.hh256_rows(KEY, sh[b])
    return sh, sums


# (k, m, block_len, erased): fused kernel (S % 16 == 0, k in 2/4/6/8/10/12/16) and the
# fallback (any other k or shard size); no erasure = verify-only GET.
CASES = [
    (8, 4, 1 << 16, []), (8, 4, 1 << 16, [0, 5]), (8, 4, 1 << 16, [3, 9]), (8, 4, 1 << 16, [8, 9, 10, 11]),
    (8, 4, 1 << 16, [0, 1, 2, 3]), (8, 4, 8 * 48, [2, 11]), (4, 2, 1 << 16, [1]), (4, 2, 1 << 16, [0, 5]),
    (16, 4, 1 << 16, [1, 7, 15, 19]), (16, 4, 1 << 16, []), (6, 3, 6 * 4096, [0, 2, 7]), (12, 4, 1 << 16, [11]),
    (5, 3, 1000, [0, 4, 6]), (8, 4, 1000, [1, 10]), (8, 4, 17, [0]), (3, 3, 256, []),
]


@pytest.mark.parametrize("k,m,blen,erased", CASES)
@pytest.mark.parametrize("data_only", [True, False])
@pytest.mark.parametrize("heal", [False, True])
@pytest.mark.parametrize("variant", [0, 200, 230])
def test_verify_reconstruct(oracle, k, m, blen, erased, data_only, heal, variant):
    """variant 0 = default dispatch (k_vr_ws for RS(8+4)-shaped verify / rebuild-2),
    200 = k_verify_reconstruct for every shape, 230 = the small-batch latency path
    (k_reconstruct, then one chain per quad verifying / hashing)."""
    with variant_ctx(variant):
        run_verify_case(oracle, k, m, blen, erased, data_only, heal)


# warp-specialised GET / heal kernel (fused_v2.hip k_vr_ws, RS(8+4)-shaped, e = 0 or 2):
# tile edges (no full tile, one tile, ragged tails) and dead stripes of the 16-stripe
# workgroup
WS_CASES = [(8, 4, 1 << 16, []), (8, 4, 1 << 16, [0, 5]), (8, 4, 1 << 16, [3, 9]), (8, 4, 8 * 48, [2, 11]),
            (8, 4, 8 * 256, [1, 4]), (8, 4, 8 * (256 * 3 + 16), [0, 7]), (8, 4, 8 * (256 * 2 + 48), []),
            (8, 4, 1 << 16, [6]), (8, 4, 8 * (256 * 3 + 16), [2]), (8, 4, 1 << 16, [0, 5, 6]),
            (8, 4, 8 * (256 * 2 + 48), [1, 2, 3]), (8, 4, 1 << 16, [1, 2, 5, 7]), (8, 4, 8 * 48, [0, 3, 4, 7]),
            (8, 4, 1 << 16, [4, 9])]


@pytest.mark.parametrize("k,m,blen,erased", WS_CASES)
@pytest.mark.parametrize("data_only", [True, False])
@pytest.mark.parametrize("heal", [False, True])
@pytest.mark.parametrize("variant", [0, 230, 231, 246, 247, 420, 423, 424, 429, 434])
def test_verify_reconstruct_ws(oracle, k, m, blen, erased, data_only, heal, variant):
    """Variant 0: the product dispatch; at 17 blocks it takes the small-batch latency
    path (k_reconstruct + one chain per quad; 230 forces it).  231 = the product dispatch
    without that path, asserted to run k_vr_ws for every RS(8+4) GET and heal with 0-4
    rebuilt rows (zs3_last_path); 246 / 247 / 420 / 423 = the product shapes with
    plain survivor loads / 64-bit addresses / the round-4 LDS row stride / the tables'
    high dwords from LDS, 424 per-wave stamps, 429 the other rebuild-role priority, 434
    the other split placement (fused_v2.hpp launch_vr_ws_t)."""
    want = {0: 4, 230: 4}.get(variant, 2)
    with variant_ctx(variant):
        run_verify_case(oracle, k, m, blen, erased, data_only, heal, nb=17, want_path=want)


WS4_CASES = [(4, 2, 1 << 16, []), (4, 2, 1 << 16, [1]), (4, 2, 1 << 16, [0, 5]), (4, 2, 4 * 48, [2, 3]),
             (4, 2, 4 * (256 * 3 + 16), [1, 4]), (4, 2, 4 * 256, [0])]


@pytest.mark.parametrize("k,m,blen,erased", WS4_CASES)
@pytest.mark.parametrize("data_only", [True, False])
@pytest.mark.parametrize("heal", [False, True])
@pytest.mark.parametrize("variant", [0, 231, 429])
def test_verify_reconstruct_ws_rs42(oracle, k, m, blen, erased, data_only, heal, variant):
    """RS(4+2)-shaped GET / heal on k_vr_ws (quad-form hash waves): tile edges and dead
    stripes; 231 = the product dispatch asserted to run the warp-specialised kernel."""
    with variant_ctx(variant):
        run_verify_case(oracle, k, m, blen, erased, data_only, heal, nb=11, want_path=2 if variant == 231 else None)


WS16_HEAL_CASES = [(16, 4, 1 << 16, [0, 5]), (16, 4, 1 << 16, [3, 17]), (16, 4, 16 * 48, [2, 19]),
                   (16, 4, 16 * 1536, [3, 17]), (16, 4, 16 * 1536, [0, 1, 16, 19]), (16, 4, 16 * 768, [5]),
                   (16, 4, 16 * (256 * 3 + 16), [0, 1, 16, 19]), (16, 4, 16 * 256, [4, 5, 6, 7]),
                   (16, 4, 16 * (256 * 2 + 48), [15, 18]), (16, 4, 1 << 16, [7]), (16, 4, 16 * 48, [18]),
                   (16, 4, 16 * (256 * 3 + 16), [16]), (16, 4, 16 * (256 * 2 + 48), [2, 9, 19]),
                   (16, 4, 16 * 256, [0, 8, 17])]


@pytest.mark.parametrize("k,m,blen,erased", WS16_HEAL_CASES)
@pytest.mark.parametrize("variant", [0, 231, 246, 247, 420, 423, 424, 429, 434, 440, 442, 443, 444])
def test_heal_ws_rs164(oracle, k, m, blen, erased, variant):
    """RS(16+4) heal (rebuild 1-4 shards and hash them) on k_vr_ws: the product shapes
    (231 = the product dispatch without the small-batch latency path that variant 0 takes
    at 11 blocks) and their memory-policy / layout variants (246 plain loads, 247 64-bit
    addresses, 420 round-4 LDS stride, 423 high table
    dwords from LDS, 424 per-wave stamps, 429 the rebuild role without issue priority, 434
    survivor splits before the first table wait, 440 the k_vr_ws instance instead of the
    survivor-quad kernel (vr_quad.hpp) that the product runs for heal 4).  The
    launched family is asserted: tile edges, ragged tails and dead stripes of the
    8-stripe workgroup."""
    want = 4 if variant == 0 else 2
    with variant_ctx(variant):
        run_verify_case(oracle, k, m, blen, erased, False, True, nb=11, want_path=want)


# RS(16+4) GET on the default k_vr_ws (8-byte rebuild columns, e = 2 and e = 4): tile
# edges, ragged tails and dead stripes of the 8-stripe workgroup (nb = 11)
WS16_GET_CASES = [(16, 4, blen, erased, data_only)
                  for blen in (1 << 16, 16 * 48, 16 * (256 * 3 + 16), 16 * (256 * 2 + 48), 16 * 1536)
                  for erased, data_only in (([0, 5], True), ([4, 15], True), ([3, 17], False),
                                            ([0, 1, 16, 19], False), ([2, 7, 9, 12], True), ([6], True),
                                            ([1, 7, 15], True), ([5, 18], True), ([0, 13, 16], False))]


@pytest.mark.parametrize("k,m,blen,erased,data_only", WS16_GET_CASES)
@pytest.mark.parametrize("variant", [0, 231, 246, 247, 420, 423, 424, 429, 434, 440, 442, 443, 444])
def test_verify_reconstruct_ws_rs164(oracle, k, m, blen, erased, data_only, variant):
    """The RS(16+4) rebuild-1..4 defaults (231: without the small-batch latency path
    that variant 0 takes at 11 blocks) run the warp-specialised kernel (asserted through
    zs3_last_path) and are bit-exact vs the oracle; 216 = the rebuild role with scalar
    (SGPR) coefficient tables, 217 = 4-byte rebuild columns (twice the rebuild waves)."""
    with variant_ctx(variant):
        run_verify_case(oracle, k, m, blen, erased, data_only, False, nb=11, want_path=4 if variant == 0 else 2)


def run_verify_case(oracle, k, m, blen, erased, data_only, heal, nb=3, want_path=None):
    sh, sums = stripes(oracle, k, m, blen, nb)
    S = sh.shape[2]
    R = k + m
    codec = z.Codec(k, m)
    d = torch.from_numpy(sh.copy()).to(DEV)
    for e in erased:
        d[:, e, :] = 0xA5
    exp = torch.from_numpy(sums).to(DEV)
    bad = torch.full((nb, R), 7, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    present = [i not in erased for i in range(R)]
    codec.verify_reconstruct_batch(d, R * S, S, nb, present, data_only, exp, bad, sums_out=out)
    torch.cuda.synchronize()
    if want_path is not None:
        assert z.last_path() == want_path, f"kernel family {z.last_path()} ran, expected {want_path}"
    got = d.cpu().numpy()
    assert not bad.cpu().numpy().any(), "no survivor is corrupt"
    rebuilt = [i for i in erased if i < k or not data_only]
    for i in range(R):
        if i in erased and i not in rebuilt:
            assert (got[:, i] == 0xA5).all(), "ReconstructData leaves missing parity untouched"
        else:
            assert np.array_equal(got[:, i], sh[:, i]), f"shard {i}"
    if heal and rebuilt:
        o = out.cpu().numpy()
        for i in rebuilt:
            assert np.array_equal(o[:, i], sums[:, i]), f"heal sum of shard {i}"


@pytest.mark.parametrize("k,m,blen,erased", [(8, 4, 1 << 16, [0, 5]), (8, 4, 1 << 16, []), (5, 3, 1000, [6]),
                                             (16, 4, 1 << 16, [19])])
def test_verify_flags_only_the_corrupt_survivor(oracle, k, m, blen, erased):
    """One flipped byte in survivor j of block 1 flags exactly (1, j): per-shard
    errFileCorrupt, never a whole-batch failure."""
    nb = 3
    sh, sums = stripes(oracle, k, m, blen, nb, seed=3)
    S = sh.shape[2]
    R = k + m
    survivors = [i for i in range(R) if i not in erased][:k]
    j = survivors[len(survivors) // 2]
    bad_sh = sh.copy()
    bad_sh[1, j, S // 2] ^= 0x40
    codec = z.Codec(k, m)
    d = torch.from_numpy(bad_sh).to(DEV)
    exp = torch.from_numpy(sums).to(DEV)
    bad = torch.zeros((nb, R), dtype=torch.int32, device=DEV)
    codec.verify_reconstruct_batch(d, R * S, S, nb, [i not in erased for i in range(R)], True, exp, bad)
    torch.cuda.synchronize()
    want = np.zeros((nb, R), dtype=np.int32)
    want[1, j] = 1
    assert np.array_equal(bad.cpu().numpy(), want)


def test_get_retry_reads_next_shard(oracle):
    """The reference's recovery: a corrupt survivor is dropped and the block decoded
    from the next shard (erasure-decode.go:165-179) — Erasure.decode_verified."""
    k, m, blen, nb = 8, 4, 1 << 16, 4
    sh, sums = stripes(oracle, k, m, blen, nb, seed=21)
    S = sh.shape[2]
    corrupt = sh.copy()
    corrupt[2, 3, 100] ^= 1          # data shard 3 of block 2 rotted on disk
    d = torch.from_numpy(corrupt).to(DEV)
    d[:, 0, :] = 0                   # shard 0 offline for every block
    e = ze.NewErasure(k, m, blen)
    bad = e.decode_verified(d, S, nb, [i != 0 for i in range(k + m)], torch.from_numpy(sums).to(DEV))
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    for b in range(nb):
        assert np.array_equal(got[b, :k], sh[b, :k]), f"block {b} data"
    assert bad == {(2, 3)}


def test_verify_reconstruct_errors():
    codec = z.Codec(4, 2)
    d = torch.zeros(6 * 64, dtype=torch.uint8, device=DEV)
    exp = torch.zeros(6 * 32, dtype=torch.uint8, device=DEV)
    bad = torch.zeros(6, dtype=torch.int32, device=DEV)
    with pytest.raises(z.ZS3Error) as ei:
        codec.verify_reconstruct_batch(d, 6 * 64, 64, 1, [0, 0, 1, 1, 1, 0], True, exp, bad)
    assert ei.value.code == -3  # ErrTooFewShards
    with pytest.raises(z.ZS3Error) as ei:
        codec.verify_reconstruct_batch(d, 6 * 64, 64, 1, [0] * 6, True, exp, bad)
    assert ei.value.code == -4  # ErrShardNoData


def test_fused_kernel_selected():
    codec = z.Codec(8, 4)
    R, S = 12, 1 << 14
    d = torch.zeros(R * S, dtype=torch.uint8, device=DEV)
    exp = torch.zeros(R * 32, dtype=torch.uint8, device=DEV)
    bad = torch.zeros(R, dtype=torch.int32, device=DEV)
    codec.verify_reconstruct_batch(d, R * S, S, 1, [i != 2 for i in range(R)], True, exp, bad)
    torch.cuda.synchronize()
    assert z.last_path() >= 1


@pytest.mark.parametrize("k,m,blen,erased,heal", [(8, 4, 8 * 640, [], False), (8, 4, 8 * 640, [0, 5], False),
                                                  (8, 4, 8 * 640, [2, 10], True), (4, 2, 4 * 512, [1], True),
                                                  (16, 4, 16 * 256, [3, 17], False),
                                                  (16, 4, 16 * 256, [3, 17], True),
                                                  (16, 4, 16 * 768, [0, 1, 16, 19], True),
                                                  (16, 4, 16 * 512, [0, 5, 9, 14], False)])
@pytest.mark.parametrize("variant", [0, 200, 420, 423, 429, 440, 442, 443, 444])
def test_verify_reconstruct_large_batch(oracle, k, m, blen, erased, heal, variant):
    """4096 stripes through the default launch (k_vr_ws where it applies), the
    first-generation kernel (200, any variant the product GET dispatch does not serve) and
    the product shapes with the round-4 LDS row stride (420) / the high table dwords from
    LDS (423) / the other rebuild-role priority (429) / the k_vr_ws instances instead of
    the survivor-quad kernel the product runs for RS(16+4) rebuild and heal 4 (440);
    every stripe checked against the oracle, one corrupt survivor flagged."""
    nb = 4096
    R = k + m
    S = -(-blen // k)
    mat = oracle.build_matrix(k, m)
    base = np.stack([oracle.encode_data(k, m, oracle.fill(5, b, blen), mat).reshape(R, S) for b in range(64)])
    sh = np.concatenate([base] * (nb // 64))  # 64 distinct stripes, repeated
    sums = np.stack([oracle.hh256_rows(KEY, s) for s in base])
    sums = np.concatenate([sums] * (nb // 64))
    d = torch.from_numpy(sh.copy()).to(DEV)
    for e in erased:
        d[:, e, :] = 0x5A
    survivors = [i for i in range(R) if i not in erased][:k]
    bad_blk, bad_row = 4093, survivors[-1]
    d[bad_blk, bad_row, 7] ^= 1
    exp = torch.from_numpy(sums).to(DEV)
    bad = torch.full((nb, R), 7, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    present = [i not in erased for i in range(R)]
    with variant_ctx(variant):
        codec = z.Codec(k, m)
        codec.verify_reconstruct_batch(d, R * S, S, nb, present, not heal, exp, bad, sums_out=out)
        torch.cuda.synchronize()
    b = bad.cpu().numpy()
    want_bad = np.zeros((nb, R), dtype=np.int32)
    want_bad[bad_blk, bad_row] = 1
    assert np.array_equal(b, want_bad)
    got = d.cpu().numpy()
    rebuilt = [i for i in erased if i < k or heal]
    ok = np.ones(nb, dtype=bool)
    ok[bad_blk] = False  # rebuilt from a corrupt survivor: garbage by design
    for i in rebuilt:
        assert np.array_equal(got[ok, i], sh[ok, i]), f"rebuilt shard {i}"
    if heal:
        o = out.cpu().numpy()
        for i in rebuilt:
            assert np.array_equal(o[ok, i], sums[ok, i]), f"heal sums of shard {i}"


# ---- per-block erasure patterns (zs3_*_batch_masks) ---------------------------------

MASK_SHAPES = [(8, 4, 1 << 16), (4, 2, 4 * (256 * 3 + 16)), (16, 4, 16 * 256), (5, 3, 1000)]


def random_patterns(rng, nb, k, m, allow_fail=False):
    R = k + m
    pats = np.ones((nb, R), dtype=bool)
    for b in range(nb):
        e = int(rng.integers(0, m + (2 if allow_fail else 1)))
        pats[b, rng.choice(R, size=min(e, R), replace=False)] = False
    return pats


@pytest.mark.parametrize("k,m,blen", MASK_SHAPES)
@pytest.mark.parametrize("data_only", [True, False])
def test_reconstruct_batch_masks(oracle, k, m, blen, data_only):
    """Every block of one batch decoded with its own erasure pattern (the reference
    decodes each block with the shards its readers returned, erasure-decode.go:166-179),
    including patterns with too few shards: those blocks get ErrTooFewShards in their
    status and are left untouched, the others are rebuilt bit-exact."""
    nb = 37
    rng = np.random.default_rng(k * 100 + m)
    sh, _ = stripes(oracle, k, m, blen, nb, seed=9)
    S = sh.shape[2]
    R = k + m
    pats = random_patterns(rng, nb, k, m, allow_fail=True)
    d = torch.from_numpy(sh.copy()).to(DEV)
    dv = d.view(nb, R, S)
    for b in range(nb):
        for i in np.nonzero(~pats[b])[0]:
            dv[b, int(i)] = 0x3C
    codec = z.Codec(k, m)
    status = np.full(nb, 99, np.int32)
    rc = codec.reconstruct_batch_masks(d, R * S, S, nb, pats, data_only, status=status)
    torch.cuda.synchronize()
    got = d.cpu().numpy().reshape(nb, R, S)
    fail = pats.sum(axis=1) < k
    assert rc == (-3 if fail.any() else 0)
    assert np.array_equal(status, np.where(fail, -3, 0).astype(np.int32))
    for b in range(nb):
        for i in range(R):
            if pats[b, i]:
                assert np.array_equal(got[b, i], sh[b, i])
            elif fail[b] or (data_only and i >= k):
                assert (got[b, i] == 0x3C).all(), (b, i)
            else:
                assert np.array_equal(got[b, i], sh[b, i]), (b, i)


@pytest.mark.parametrize("k,m,blen", MASK_SHAPES)
@pytest.mark.parametrize("heal", [False, True])
@pytest.mark.parametrize("variant", [0, 231])
def test_verify_reconstruct_batch_masks(oracle, k, m, blen, heal, variant):
    """GET / heal pass with per-block patterns: survivors verified per block (one rotted
    survivor flagged exactly), missing shards rebuilt, heal sums of the rebuilt shards.
    231: the product dispatch without the small-batch path, so the block-id lists of
    the RS(8+4) / RS(16+4) groups go through k_vr_ws."""
    nb = 41
    rng = np.random.default_rng(k * 7 + m)
    sh, sums = stripes(oracle, k, m, blen, nb, seed=13)
    S = sh.shape[2]
    R = k + m
    pats = random_patterns(rng, nb, k, m)
    bad_sh = sh.copy()
    rb = 5
    surv = [i for i in range(R) if pats[rb, i]][:k]
    bad_sh[rb, surv[0], S - 1] ^= 0x80
    d = torch.from_numpy(bad_sh).to(DEV)
    dv = d.view(nb, R, S)
    for b in range(nb):
        for i in np.nonzero(~pats[b])[0]:
            dv[b, int(i)] = 0x77
    codec = z.Codec(k, m)
    exp = torch.from_numpy(sums).to(DEV)
    bad = torch.full((nb, R), 9, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    status = np.full(nb, 99, np.int32)
    with variant_ctx(variant):
        if variant:
            codec = z.Codec(k, m)
        rc = codec.verify_reconstruct_batch_masks(d, R * S, S, nb, pats, not heal, exp, bad, sums_out=out,
                                                  status=status)
        torch.cuda.synchronize()
    assert rc == 0 and not status.any()
    want_bad = np.zeros((nb, R), np.int32)
    want_bad[rb, surv[0]] = 1
    assert np.array_equal(bad.cpu().numpy(), want_bad)
    got = d.cpu().numpy().reshape(nb, R, S)
    for b in range(nb):
        if b == rb:
            continue  # rebuilt from a rotted survivor: garbage by design (re-issued by the caller)
        for i in range(R):
            if pats[b, i] or i < k or heal:
                assert np.array_equal(got[b, i], sh[b, i]), (b, i)
            if heal and not pats[b, i]:
                assert np.array_equal(out.cpu().numpy()[b, i], sums[b, i]), (b, i)


@pytest.mark.parametrize("erased,heal", [([0, 5], False), ([0, 5], True), ([3, 13], True), ([1, 2, 3, 4], False),
                                         ([7], True)])
@pytest.mark.parametrize("variant", [0, 423, 429, 434])
def test_verify_reconstruct_rs124_large(oracle, erased, heal, variant):
    """RS(12+4) GET / heal above 1024 stripes on the warp-specialised kernel with
    unaligned rows (S = 1 100: two 512-byte tiles and a 76-byte tail) and the
    diagnostics forms of those instances (423 high
    table dwords from LDS, 429 rebuild role without issue priority, 434 survivor splits
    first); every stripe vs the
    oracle, one corrupt survivor flagged exactly."""
    k, m, nb, S = 12, 4, 1030, 1100
    R = k + m
    mat = oracle.build_matrix(k, m)
    base = np.stack([oracle.encode_data(k, m, oracle.fill(9, b, k * S), mat).reshape(R, S) for b in range(32)])
    sh = np.concatenate([base] * (-(-nb // 32)))[:nb]
    sums = np.stack([oracle.hh256_rows(KEY, s) for s in base])
    sums = np.concatenate([sums] * (-(-nb // 32)))[:nb]
    d = torch.from_numpy(sh.copy()).to(DEV)
    for e in erased:
        d[:, e, :] = 0x5A
    survivors = [i for i in range(R) if i not in erased][:k]
    bad_blk, bad_row = 1027, survivors[2]
    d[bad_blk, bad_row, 1099] ^= 0x80
    exp = torch.from_numpy(sums).to(DEV)
    bad = torch.full((nb, R), 7, dtype=torch.int32, device=DEV)
    out = torch.zeros((nb, R, 32), dtype=torch.uint8, device=DEV) if heal else None
    with variant_ctx(variant):
        z.Codec(k, m).verify_reconstruct_batch(d, R * S, S, nb, [i not in erased for i in range(R)], not heal, exp,
                                               bad, sums_out=out)
        torch.cuda.synchronize()
        assert z.last_path() == 2, f"kernel family {z.last_path()} ran"
    want = np.zeros((nb, R), np.int32)
    want[bad_blk, bad_row] = 1
    assert np.array_equal(bad.cpu().numpy(), want)
    got = d.cpu().numpy()
    rebuilt = [i for i in erased if i < k or heal]
    ok = np.ones(nb, bool)
    ok[bad_blk] = False
    for i in range(R):
        if i in erased and i not in rebuilt:
            assert (got[:, i] == 0x5A).all()
        else:
            assert np.array_equal(got[ok, i], sh[ok, i]), f"shard {i}"
    if heal:
        o = out.cpu().numpy()
        for i in rebuilt:
            assert np.array_equal(o[ok, i], sums[ok, i]), f"heal sum of shard {i}"
