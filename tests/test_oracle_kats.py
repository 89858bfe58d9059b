"""Pin the CPU oracles against the reference's own known-answer tests.

KAT sources (all non-test code in the reference):
  * cmd/erasure-coding.go:158-216 erasureSelfTest — xxhash64 over byte(i)||shard_i
    for EncodeData(bytes(range(256))) at 60 (k, m) configs, then delete shard 0 and
    DecodeDataBlocks must restore it (:201-209).
  * cmd/bitrot.go:218-249 bitrotSelfTest — chained HighwayHash256(S) digest.
  * cmd/bitrot.go:36-37 — magic key = HH-256 (zero key) of the first 100 decimals of pi.
Plus the first public HighwayHash-64 vectors (key = bytes 0..31, msg = bytes 0..n-1)
published with Google's HighwayHash.
"""
import numpy as np
import pytest
import xxhash

from oracle import pyoracle

# cmd/erasure-coding.go:169 — the golden table, (data, parity) -> xxhash64
ERASURE_SELFTEST_WANT = {
    (2, 2): 0x23fb21be2496f5d3, (2, 3): 0xa5cd5600ba0d8e7c, (3, 1): 0x60ab052148b010b4,
    (3, 2): 0xe64927daef76435a, (3, 3): 0x672f6f242b227b21, (3, 4): 0x571e41ba23a6dc6,
    (4, 1): 0x524eaa814d5d86e2, (4, 2): 0x62b9552945504fef, (4, 3): 0xcbf9065ee053e518,
    (4, 4): 0x9a07581dcd03da8, (4, 5): 0xbf2d27b55370113f, (5, 1): 0xf71031a01d70daf,
    (5, 2): 0x8e5845859939d0f4, (5, 3): 0x7ad9161acbb4c325, (5, 4): 0xc446b88830b4f800,
    (5, 5): 0xabf1573cc6f76165, (5, 6): 0x7b5598a85045bfb8, (6, 1): 0xe2fc1e677cc7d872,
    (6, 2): 0x7ed133de5ca6a58e, (6, 3): 0x39ef92d0a74cc3c0, (6, 4): 0xcfc90052bc25d20,
    (6, 5): 0x71c96f6baeef9c58, (6, 6): 0x4b79056484883e4c, (6, 7): 0xb1a0e2427ac2dc1a,
    (7, 1): 0x937ba2b7af467a22, (7, 2): 0x5fd13a734d27d37a, (7, 3): 0x3be2722d9b66912f,
    (7, 4): 0x14c628e59011be3d, (7, 5): 0xcc3b39ad4c083b9f, (7, 6): 0x45af361b7de7a4ff,
    (7, 7): 0x456cc320cec8a6e6, (7, 8): 0x1867a9f4db315b5c, (8, 1): 0xbc5756b9a9ade030,
    (8, 2): 0xdfd7d9d0b3e36503, (8, 3): 0x72bb72c2cdbcf99d, (8, 4): 0x3ba5e9b41bf07f0,
    (8, 5): 0xd7dabc15800f9d41, (8, 6): 0xb482a6169fd270f, (8, 7): 0x50748e0099d657e8,
    (9, 1): 0xc77ae0144fcaeb6e, (9, 2): 0x8a86c7dbebf27b68, (9, 3): 0xa64e3be6d6fe7e92,
    (9, 4): 0x239b71c41745d207, (9, 5): 0x2d0803094c5a86ce, (9, 6): 0xa3c2539b3af84874,
    (10, 1): 0x7d30d91b89fcec21, (10, 2): 0xfa5af9aa9f1857a3, (10, 3): 0x84bc4bda8af81f90,
    (10, 4): 0x6c1cba8631de994a, (10, 5): 0x4383e58a086cc1ac, (11, 1): 0x4ed2929a2df690b,
    (11, 2): 0xecd6f1b1399775c0, (11, 3): 0xc78cfbfc0dc64d01, (11, 4): 0xb2643390973702d6,
    (12, 1): 0x3b2a88686122d082, (12, 2): 0xfd2f30a48a8e2e9, (12, 3): 0xd5ce58368ae90b13,
    (13, 1): 0x9c88e2a9d1b8fff8, (13, 2): 0xcb8460aa4cf6613, (14, 1): 0x78a28bbaec57996e,
}

# cmd/bitrot.go:222
BITROT_SELFTEST_HH256 = "39c0407ed3f01b18d22c85db4aeff11e060ca5f43131b0126731ca197cd42313"
PI_100 = ("1415926535897932384626433832795028841971693993751058209749"
          "445923078164062862089986280348253421170679")


def selftest_configs():
    """for total in 4..15, data in total/2 .. total-1 (cmd/erasure-coding.go:161-166)."""
    out = []
    for total in range(4, 16):
        for data in range(total // 2, total):
            out.append((data, total - data))
    return out


def _xx(shards):
    h = xxhash.xxh64()
    for i, s in enumerate(shards):
        h.update(bytes([i]))
        h.update(np.asarray(s, dtype=np.uint8).tobytes())
    return h.intdigest()


def test_selftest_config_list_matches_table():
    assert sorted(selftest_configs()) == sorted(ERASURE_SELFTEST_WANT)
    assert len(ERASURE_SELFTEST_WANT) == 60


@pytest.mark.parametrize("k,m", selftest_configs())
def test_erasure_selftest_c_oracle(oracle, k, m):
    data = bytes(range(256))
    shards = oracle.encode_data(k, m, data)
    assert _xx(shards) == ERASURE_SELFTEST_WANT[(k, m)]
    # delete first shard and DecodeDataBlocks (cmd/erasure-coding.go:201-209)
    first = shards[0].copy()
    shards[0] = 0
    pres = [i != 0 for i in range(k + m)]
    assert oracle.reconstruct(k, m, shards, pres, True) == 0
    assert np.array_equal(shards[0], first)


@pytest.mark.parametrize("k,m", selftest_configs())
def test_erasure_selftest_py_oracle(k, m):
    data = bytes(range(256))
    shards = pyoracle.encode_data(k, m, data)
    assert _xx(shards) == ERASURE_SELFTEST_WANT[(k, m)]
    lst = [None] + [shards[i] for i in range(1, k + m)]
    rec = pyoracle.reconstruct(k, m, lst, data_only=True)
    assert np.array_equal(rec[0], shards[0])


def test_matrices_agree_c_vs_py(oracle):
    for k, m in selftest_configs() + [(16, 4), (4, 2), (8, 4), (1, 1), (20, 12)]:
        assert np.array_equal(oracle.build_matrix(k, m), pyoracle.build_matrix(k, m)), (k, m)


def test_derived_parity_rows_survey(oracle):
    # SURVEY.md §8c derived parity rows (from the KAT-pinned restatement)
    assert oracle.build_matrix(4, 2)[4:].tolist() == [[27, 28, 18, 20], [28, 27, 20, 18]]
    assert oracle.build_matrix(8, 4)[8:].tolist()[0] == [26, 132, 186, 51, 231, 16, 198, 39]
    assert oracle.build_matrix(16, 4)[16:].tolist()[3][:4] == [133, 246, 181, 33]


def _bitrot_selftest(hfun):
    # cmd/bitrot.go:233-245: msg grows by the previous sum; Size*BlockSize = 32*32
    msg = b""
    s = b""
    for _ in range(0, 32 * 32, 32):
        s = hfun(pyoracle.MAGIC_HH256_KEY, msg)
        msg = msg + s
    return s.hex()


def test_bitrot_selftest_c(oracle):
    assert _bitrot_selftest(oracle.hh256) == BITROT_SELFTEST_HH256


def test_bitrot_selftest_py():
    assert _bitrot_selftest(pyoracle.hh256) == BITROT_SELFTEST_HH256


def test_magic_key_derivation(oracle):
    zero = bytes(32)
    assert len(PI_100) == 100
    assert oracle.hh256(zero, PI_100.encode()) == pyoracle.MAGIC_HH256_KEY
    assert pyoracle.hh256(zero, PI_100.encode()) == pyoracle.MAGIC_HH256_KEY


def test_hh64_public_vectors(oracle):
    key = bytes(range(32))
    want = [0x907a56de22c26e53, 0x7eab43aac7cddd78, 0xb8d0569ab0b53d62, 0x5c6befab8a463d80]
    for n, w in enumerate(want):
        assert oracle.hh64(key, bytes(range(n))) == w
        assert pyoracle.hh64(key, bytes(range(n))) == w


def test_hh256_remainder_branches_cross_check(oracle):
    """Two independent restatements agree on every length 0..160 (covers all
    size_mod32 branches the KATs do not reach)."""
    rng = np.random.default_rng(7)
    for key in (pyoracle.MAGIC_HH256_KEY, bytes(range(32))):
        for n in range(0, 161):
            msg = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert oracle.hh256(key, msg) == pyoracle.hh256(key, msg), n


def test_encode_reconstruct_c_vs_py(oracle):
    rng = np.random.default_rng(3)
    for (k, m, n) in [(4, 2, 1000), (8, 4, 4097), (5, 3, 1), (16, 4, 333), (3, 3, 17), (12, 4, 2049)]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        a = oracle.encode_data(k, m, data)
        b = pyoracle.encode_data(k, m, data)
        assert np.array_equal(a, b)
        # erase m shards spread across data and parity, full reconstruct
        erased = list(range(0, k + m, max(1, (k + m) // m)))[:m]
        c = a.copy()
        for e in erased:
            c[e] = 0xAA
        pres = [i not in erased for i in range(k + m)]
        assert oracle.reconstruct(k, m, c, pres, False) == 0
        assert np.array_equal(c, a)


def test_fill_c_vs_py(oracle):
    for seed, obj, n in [(0, 0, 64), (1, 5, 1001), (123, 4095, 17)]:
        assert oracle.fill(seed, obj, n).tobytes() == pyoracle.fill(seed, obj, n)


def test_reconstruct_errors(oracle):
    k, m = 4, 2
    a = oracle.encode_data(k, m, bytes(range(256)))
    # fewer than k present -> ErrTooFewShards (-3)
    assert oracle.reconstruct(k, m, a.copy(), [0, 0, 1, 1, 1, 0], True) == -3
    # all present -> no-op
    assert oracle.reconstruct(k, m, a.copy(), [1] * 6, False) == 0
