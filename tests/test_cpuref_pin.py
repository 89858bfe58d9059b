"""Pin oracle/cpu_ref.cpp (the SIMD + threaded CPU baseline, and the fast whole-batch
checker of the full-size GPU tests) to the scalar, KAT-pinned oracle (zs3_oracle.c).

cpu_ref restates the reference's per-block encode structure (cmd/erasure-encode.go:83-111:
Split -> Encode -> k+m bitrot sums, cmd/bitrot-streaming.go:47-49) with GFNI / AVX2 GF
kernels and an AVX2 HighwayHash; this checks its parity rows and sums byte for byte
against the scalar restatement at the BASELINE shapes RS(4+2) (config 1), RS(8+4) and
RS(16+4), full 1 MiB blocks and ragged blocks (Split zero padding and every HighwayHash
remainder branch), all-zero and all-0xFF input, at T = 1 and T = every thread this
process may use.
"""
import numpy as np
import pytest

from oracle import cpuref

KEY = bytes.fromhex("4be734fa8e238acd263e83e6bb968552040f935da39f441497e09d1322de36a0")
MiB = 1 << 20


def _blocks(kind, seed, nb, blen, oracle):
    if kind == "zero":
        return np.zeros(nb * blen, np.uint8)
    if kind == "ff":
        return np.full(nb * blen, 0xFF, np.uint8)
    return np.concatenate([oracle.fill(seed, b, blen) for b in range(nb)])


def _check(oracle, k, m, blen, nb, kind, threads):
    R = k + m
    S = -(-blen // k)
    mat = oracle.build_matrix(k, m)
    data = _blocks(kind, 1000 + blen, nb, blen, oracle)
    par = np.full(nb * m * S, 0xA5, np.uint8)
    sums = np.full(nb * R * 32, 0xA5, np.uint8)
    assert cpuref.encode_hash(k, m, mat, data, blen, nb, blen, par, m * S, sums, KEY, threads) == S
    for b in range(nb):
        want = oracle.encode_data(k, m, data[b * blen:(b + 1) * blen], mat)
        assert want.shape == (R, S)
        assert np.array_equal(par[b * m * S:(b + 1) * m * S].reshape(m, S), want[k:]), (k, m, blen, b)
        assert np.array_equal(sums[b * R * 32:(b + 1) * R * 32].reshape(R, 32), oracle.hh256_rows(KEY, want)), \
            (k, m, blen, b)


@pytest.mark.parametrize("threads", [1, "all"])
@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (16, 4)])
def test_cpuref_full_blocks_vs_oracle(oracle, k, m, threads):
    t = cpuref.threads_available() if threads == "all" else 1
    _check(oracle, k, m, MiB, 3, "random", t)


@pytest.mark.parametrize("threads", [1, "all"])
@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (16, 4)])
@pytest.mark.parametrize("blen", [MiB + 1, MiB - 13, 17, 84, 4 * 21 + 2, 1])
def test_cpuref_ragged_blocks_vs_oracle(oracle, k, m, blen, threads):
    """Ragged last blocks: S' = ceil(n/k) with Split's zero padding; lengths chosen so
    the sums hit size_mod32 & 16 (S = 21), size_mod4 != 0 and 1-byte shards."""
    t = cpuref.threads_available() if threads == "all" else 1
    _check(oracle, k, m, blen, 2, "random", t)


@pytest.mark.parametrize("kind", ["zero", "ff"])
@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (16, 4)])
def test_cpuref_constant_inputs_vs_oracle(oracle, k, m, kind):
    _check(oracle, k, m, MiB, 2, kind, cpuref.threads_available())


def test_cpuref_hh256_vs_oracle(oracle):
    rng = np.random.default_rng(5)
    for n in list(range(0, 70)) + [131072, 131072 + 17, 262144 - 5]:
        msg = rng.integers(0, 256, max(n, 1), dtype=np.uint8)[:n]
        out = np.zeros(32, np.uint8)
        buf = msg if n else np.zeros(1, np.uint8)
        cpuref.lib().cpuref_hh256(KEY, buf.ctypes.data, n, out.ctypes.data)
        assert out.tobytes() == oracle.hh256(KEY, msg.tobytes()), n
