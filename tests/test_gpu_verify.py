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
@pytest.mark.parametrize("variant", [0, 200])
def test_verify_reconstruct(oracle, k, m, blen, erased, data_only, heal, variant):
    """variant 0 = default dispatch (k_vr_ws for RS(8+4)-shaped verify / rebuild-2),
    200 = k_verify_reconstruct for every shape."""
    z.set_variant(variant)
    try:
        run_verify_case(oracle, k, m, blen, erased, data_only, heal)
    finally:
        z.set_variant(0)


# warp-specialised GET / heal kernel (fused_v2.hip k_vr_ws, RS(8+4)-shaped, e = 0 or 2):
# tile edges (no full tile, one tile, ragged tails) and dead stripes of the 16-stripe
# workgroup
WS_CASES = [(8, 4, 1 << 16, []), (8, 4, 1 << 16, [0, 5]), (8, 4, 1 << 16, [3, 9]), (8, 4, 8 * 48, [2, 11]),
            (8, 4, 8 * 256, [1, 4]), (8, 4, 8 * (256 * 3 + 16), [0, 7]), (8, 4, 8 * (256 * 2 + 48), [])]


@pytest.mark.parametrize("k,m,blen,erased", WS_CASES)
@pytest.mark.parametrize("data_only", [True, False])
@pytest.mark.parametrize("heal", [False, True])
@pytest.mark.parametrize("variant", [210, 211, 212, 213])
def test_verify_reconstruct_ws(oracle, k, m, blen, erased, data_only, heal, variant):
    z.set_variant(variant)
    try:
        run_verify_case(oracle, k, m, blen, erased, data_only, heal, nb=17)
    finally:
        z.set_variant(0)


WS4_CASES = [(4, 2, 1 << 16, []), (4, 2, 1 << 16, [1]), (4, 2, 1 << 16, [0, 5]), (4, 2, 4 * 48, [2, 3]),
             (4, 2, 4 * (256 * 3 + 16), [1, 4]), (4, 2, 4 * 256, [0])]


@pytest.mark.parametrize("k,m,blen,erased", WS4_CASES)
@pytest.mark.parametrize("data_only", [True, False])
@pytest.mark.parametrize("heal", [False, True])
@pytest.mark.parametrize("variant", [0, 210])
def test_verify_reconstruct_ws_rs42(oracle, k, m, blen, erased, data_only, heal, variant):
    """RS(4+2)-shaped GET / heal on k_vr_ws: quad-form (default) and pair-form (210)
    hash waves, tile edges and dead stripes."""
    z.set_variant(variant)
    try:
        run_verify_case(oracle, k, m, blen, erased, data_only, heal, nb=11)
    finally:
        z.set_variant(0)


WS16_HEAL_CASES = [(16, 4, 1 << 16, [0, 5]), (16, 4, 1 << 16, [3, 17]), (16, 4, 16 * 48, [2, 19]),
                   (16, 4, 16 * (256 * 3 + 16), [0, 1, 16, 19]), (16, 4, 16 * 256, [4, 5, 6, 7]),
                   (16, 4, 16 * (256 * 2 + 48), [15, 18])]


@pytest.mark.parametrize("k,m,blen,erased", WS16_HEAL_CASES)
@pytest.mark.parametrize("variant", [0, 215])
def test_heal_ws_rs164(oracle, k, m, blen, erased, variant):
    """RS(16+4) heal (rebuild 2 or 4 shards and hash them) on k_vr_ws with quad-form
    hash waves: tile edges, ragged tails and dead stripes of the 8-stripe workgroup."""
    z.set_variant(variant)
    try:
        run_verify_case(oracle, k, m, blen, erased, False, True, nb=11)
    finally:
        z.set_variant(0)


def run_verify_case(oracle, k, m, blen, erased, data_only, heal, nb=3):
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
    assert z.last_path() == 1


@pytest.mark.parametrize("k,m,blen,erased,heal", [(8, 4, 8 * 640, [], False), (8, 4, 8 * 640, [0, 5], False),
                                                  (8, 4, 8 * 640, [2, 10], True), (4, 2, 4 * 512, [1], True),
                                                  (16, 4, 16 * 256, [3, 17], False),
                                                  (16, 4, 16 * 256, [3, 17], True)])
@pytest.mark.parametrize("variant", [0, 200, 201, 210, 211, 212])
def test_verify_reconstruct_large_batch(oracle, k, m, blen, erased, heal, variant):
    """4096 stripes through the default launch (k_vr_ws where it applies), the
    first-generation kernel (200), its one-workgroup-per-CU launch (201) and k_vr_ws
    with one tile of prefetch (211); every stripe checked against the oracle, one
    corrupt survivor flagged."""
    nb = 4096
    R = k + m
    S = -(-blen // k)
    mat = oracle.build_matrix(k, m)
    base = np.stack([oracle.encode_data(k, m, oracle.fill(5, b, blen), mat).reshape(R, S) for b in range(64)])
    sh = np.concatenate([base] * (nb // 64))  # 64 distinct stripes, repeated
    sums = np.stack([oracle.hh256_rows(KEY, s) for s in base])
    sums = np.concatenate([sums] * (nb // 64))
    codec = z.Codec(k, m)
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
    z.set_variant(variant)
    try:
        codec.verify_reconstruct_batch(d, R * S, S, nb, present, not heal, exp, bad, sums_out=out)
        torch.cuda.synchronize()
    finally:
        z.set_variant(0)
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
