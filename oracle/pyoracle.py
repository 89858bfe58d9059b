"""Independent Python/numpy restatement of the reference's erasure + bitrot path.

TEST INFRASTRUCTURE ONLY — imported by tests/ and tests/golden/make_golden.py
as a second, independent oracle next to the C restatement in zs3_oracle.c.
The product path never imports this module.

Parity status: PINNED by the reference KATs (see tests/test_oracle_kats.py):
cmd/erasure-coding.go:169 (60 xxhash64 configs), cmd/bitrot.go:222-223
(chained HH256 digest) and cmd/bitrot.go:36-37 (magic key = HH256 of pi).

Restated algorithms (not vendored in /root/reference):
  * github.com/klauspost/reedsolomon v1.11.8 (go.mod:48): GF(2^8)/0x11D,
    buildMatrix = Vandermonde * inverse(top), Split, Encode, reconstruct.
  * github.com/minio/highwayhash v1.0.2 (go.mod:54): HighwayHash-256.
HighwayHash here is written lane-by-lane with Python ints (no shared code
with the C file), so the HH remainder branches the KATs do not reach are
cross-checked by two independent restatements.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1

# ---------------------------------------------------------------------------
# GF(2^8) — klauspost galois.go: poly 0x11D, generator 2.
EXP = np.zeros(512, dtype=np.uint8)
LOG = np.zeros(256, dtype=np.int32)
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
EXP[255:510] = EXP[0:255]

# full 256x256 multiplication table (row a = a * b for all b)
MUL = np.zeros((256, 256), dtype=np.uint8)
for _a in range(1, 256):
    _b = np.arange(1, 256)
    MUL[_a, 1:] = EXP[LOG[_a] + LOG[_b]]


def gf_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gf_div(a: int, b: int) -> int:
    if a == 0:
        return 0
    return int(EXP[(LOG[a] - LOG[b]) % 255])


def gal_exp(a: int, n: int) -> int:
    """galExp (klauspost galois.go)."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP[(int(LOG[a]) * n) % 255])


def gf_invert(mat: np.ndarray) -> np.ndarray:
    """Gauss-Jordan inversion over GF(2^8) (klauspost matrix.go Invert)."""
    n = mat.shape[0]
    w = np.zeros((n, 2 * n), dtype=np.uint8)
    w[:, :n] = mat
    w[:, n:] = np.eye(n, dtype=np.uint8)
    for r in range(n):
        if w[r, r] == 0:
            for rb in range(r + 1, n):
                if w[rb, r] != 0:
                    w[[r, rb]] = w[[rb, r]]
                    break
        if w[r, r] == 0:
            raise ValueError("matrix is singular")
        if w[r, r] != 1:
            s = gf_div(1, int(w[r, r]))
            w[r] = MUL[s][w[r]]
        for rb in range(n):
            if rb != r and w[rb, r] != 0:
                w[rb] ^= MUL[int(w[rb, r])][w[r]]
    return w[:, n:].copy()


def gf_matmul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = np.zeros((a.shape[0], b.shape[1]), dtype=np.uint8)
    for i in range(a.shape[0]):
        for t in range(a.shape[1]):
            if a[i, t]:
                out[i] ^= MUL[int(a[i, t])][b[t]]
    return out


def build_matrix(k: int, m: int) -> np.ndarray:
    """buildMatrix: Vandermonde(k+m, k) * inverse(top k x k); NewErasure checks
    mirror cmd/erasure-coding.go:44-50."""
    if k <= 0 or m <= 0:
        raise ValueError("ErrInvShardNum")
    if k + m > 256:
        raise ValueError("ErrMaxShardNum")
    v = np.array([[gal_exp(r & 0xFF, c) for c in range(k)] for r in range(k + m)], dtype=np.uint8)
    return gf_matmul(v, gf_invert(v[:k]))


def shard_size(length: int, k: int) -> int:
    """ceilFrac(length, k) — cmd/erasure-coding.go:122, cmd/utils.go:691."""
    return -(-length // k) if length > 0 else 0


def encode_data(k: int, m: int, data: bytes, matrix: np.ndarray | None = None) -> np.ndarray:
    """Erasure.EncodeData (cmd/erasure-coding.go:77-91): Split (ceil, zero pad) +
    Encode.  Returns a (k+m, per) uint8 array; len 0 -> shape (k+m, 0)."""
    if matrix is None:
        matrix = build_matrix(k, m)
    n = len(data)
    if n == 0:
        return np.zeros((k + m, 0), dtype=np.uint8)
    per = shard_size(n, k)
    buf = np.zeros((k + m) * per, dtype=np.uint8)
    buf[:n] = np.frombuffer(bytes(data), dtype=np.uint8)
    shards = buf.reshape(k + m, per)
    for r in range(m):
        acc = np.zeros(per, dtype=np.uint8)
        for j in range(k):
            acc ^= MUL[int(matrix[k + r, j])][shards[j]]
        shards[k + r] = acc
    return shards


def reconstruct(k: int, m: int, shards: list, data_only: bool, matrix: np.ndarray | None = None) -> list:
    """reedsolomon ReconstructData / Reconstruct as used by
    Erasure.DecodeDataBlocks (cmd/erasure-coding.go:96) and
    DecodeDataAndParityBlocks (:113).  `shards` is a list of k+m numpy arrays
    or None (missing).  Returns the filled list; raises on too few shards."""
    if matrix is None:
        matrix = build_matrix(k, m)
    n = k + m
    if len(shards) != n:
        raise ValueError("ErrTooFewShards")
    sizes = {len(s) for s in shards if s is not None and len(s)}
    if not sizes:
        raise ValueError("ErrShardNoData")
    if len(sizes) > 1:
        raise ValueError("ErrShardSize")
    per = sizes.pop()
    present = [s is not None and len(s) > 0 for s in shards]
    if all(present) or (data_only and all(present[:k])):
        return shards
    if sum(present) < k:
        raise ValueError("ErrTooFewShards")
    valid = [i for i in range(n) if present[i]][:k]
    dec = gf_invert(matrix[valid])
    out = list(shards)
    for d in range(k):
        if not present[d]:
            acc = np.zeros(per, dtype=np.uint8)
            for t in range(k):
                acc ^= MUL[int(dec[d, t])][np.asarray(shards[valid[t]], dtype=np.uint8)]
            out[d] = acc
    if not data_only:
        for p in range(k, n):
            if not present[p]:
                acc = np.zeros(per, dtype=np.uint8)
                for j in range(k):
                    acc ^= MUL[int(matrix[p, j])][out[j]]
                out[p] = acc
    return out


# ---------------------------------------------------------------------------
# HighwayHash-256 (minio/highwayhash v1.0.2 == Google C reference).
_MUL0 = [0xdbe6d5d5fe4cce2f, 0xa4093822299f31d0, 0x13198a2e03707344, 0x243f6a8885a308d3]
_MUL1 = [0x3bd39e10cb0ef593, 0xc0acf169b5f18a8c, 0xbe5466cf34e90c6c, 0x452821e638d01377]


def _rot32(x: int) -> int:
    return ((x >> 32) | (x << 32)) & M64


def _bytes_of(x: int) -> list:
    return [(x >> (8 * i)) & 0xFF for i in range(8)]


def _from_bytes(bs: list) -> int:
    return sum(b << (8 * i) for i, b in enumerate(bs))


def _zipper(hi: int, lo: int) -> tuple[int, int]:
    """ZipperMergeAndAdd as byte permutations of the lane pair (hi = lane 2i+1,
    lo = lane 2i).  Returns (add_for_lo, add_for_hi)."""
    a = _bytes_of(hi)
    b = _bytes_of(lo)
    add_lo = _from_bytes([b[3], a[4], b[2], b[5], a[6], b[1], a[7], b[0]])
    add_hi = _from_bytes([a[3], b[4], a[2], a[5], a[1], b[6], a[0], b[7]])
    return add_lo, add_hi


class HighwayHash:
    def __init__(self, key: bytes):
        assert len(key) == 32
        kw = [int.from_bytes(key[8 * i: 8 * i + 8], "little") for i in range(4)]
        self.mul0 = list(_MUL0)
        self.mul1 = list(_MUL1)
        self.v0 = [(self.mul0[i] ^ kw[i]) & M64 for i in range(4)]
        self.v1 = [(self.mul1[i] ^ _rot32(kw[i])) & M64 for i in range(4)]

    def _update(self, lanes):
        v0, v1, mul0, mul1 = self.v0, self.v1, self.mul0, self.mul1
        for i in range(4):
            v1[i] = (v1[i] + mul0[i] + lanes[i]) & M64
            mul0[i] ^= ((v1[i] & M32) * (v0[i] >> 32)) & M64
            v0[i] = (v0[i] + mul1[i]) & M64
            mul1[i] ^= ((v0[i] & M32) * (v1[i] >> 32)) & M64
        for lo, hi in ((0, 1), (2, 3)):
            add_lo, add_hi = _zipper(v1[hi], v1[lo])
            v0[lo] = (v0[lo] + add_lo) & M64
            v0[hi] = (v0[hi] + add_hi) & M64
        for lo, hi in ((0, 1), (2, 3)):
            add_lo, add_hi = _zipper(v0[hi], v0[lo])
            v1[lo] = (v1[lo] + add_lo) & M64
            v1[hi] = (v1[hi] + add_hi) & M64

    def _packet(self, p: bytes):
        self._update([int.from_bytes(p[8 * i: 8 * i + 8], "little") for i in range(4)])

    def _remainder(self, tail: bytes):
        n = len(tail)
        for i in range(4):
            self.v0[i] = (self.v0[i] + (n << 32) + n) & M64
            lo, hi = self.v1[i] & M32, self.v1[i] >> 32
            lo = ((lo << n) | (lo >> (32 - n))) & M32
            hi = ((hi << n) | (hi >> (32 - n))) & M32
            self.v1[i] = (hi << 32) | lo
        mod4 = n & 3
        remain = n - mod4
        pkt = bytearray(32)
        pkt[:remain] = tail[:remain]
        if n >= 16:
            pkt[28:32] = tail[n - 4: n]
        elif mod4:
            pkt[16] = tail[remain]
            pkt[17] = tail[remain + (mod4 >> 1)]
            pkt[18] = tail[n - 1]
        self._packet(bytes(pkt))

    def digest_rounds(self, msg: bytes, rounds: int):
        full = len(msg) - (len(msg) % 32)
        for i in range(0, full, 32):
            self._packet(msg[i: i + 32])
        if len(msg) % 32:
            self._remainder(msg[full:])
        for _ in range(rounds):
            v0 = self.v0
            self._update([_rot32(v0[2]), _rot32(v0[3]), _rot32(v0[0]), _rot32(v0[1])])


def _reduce(a3: int, a2: int, a1: int, a0: int) -> tuple[int, int]:
    a3 &= 0x3FFFFFFFFFFFFFFF
    m1 = a1 ^ (((a3 << 1) | (a2 >> 63)) & M64) ^ (((a3 << 2) | (a2 >> 62)) & M64)
    m0 = a0 ^ ((a2 << 1) & M64) ^ ((a2 << 2) & M64)
    return m1 & M64, m0 & M64


def hh256(key: bytes, msg: bytes) -> bytes:
    h = HighwayHash(key)
    h.digest_rounds(bytes(msg), 10)
    v0, v1, m0, m1 = h.v0, h.v1, h.mul0, h.mul1
    h1, h0 = _reduce((v1[1] + m1[1]) & M64, (v1[0] + m1[0]) & M64, (v0[1] + m0[1]) & M64, (v0[0] + m0[0]) & M64)
    h3, h2 = _reduce((v1[3] + m1[3]) & M64, (v1[2] + m1[2]) & M64, (v0[3] + m0[3]) & M64, (v0[2] + m0[2]) & M64)
    return b"".join(x.to_bytes(8, "little") for x in (h0, h1, h2, h3))


def hh64(key: bytes, msg: bytes) -> int:
    h = HighwayHash(key)
    h.digest_rounds(bytes(msg), 4)
    return (h.v0[0] + h.v1[0] + h.mul0[0] + h.mul1[0]) & M64


# cmd/bitrot.go:37
MAGIC_HH256_KEY = bytes.fromhex("4be734fa8e238acd263e83e6bb968552040f935da39f441497e09d1322de36a0")

# ---------------------------------------------------------------------------
# Synthetic input (identical to oracle_fill in zs3_oracle.c and the device
# fill kernel): word i of object obj = splitmix64_mix(seed + obj*2^40 + (i+1)*GAMMA)
_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def fill(seed: int, obj: int, nbytes: int) -> bytes:
    nw = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        s0 = np.uint64((seed + (obj << 40)) & M64)
        z = s0 + (np.arange(1, nw + 1, dtype=np.uint64) * _GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:nbytes]
