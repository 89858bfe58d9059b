// digest.hip — batched MD5 (S3 ETag) and SHA-256 (x-amz-content-sha256) on gfx950.
//
// once the encode is on the device, the PUT stream's per-object CPU
// digests are the next serial cost.  Replaces the arithmetic of:
//   internal/etag/reader.go:106-144   etag.NewReader / Reader.ETag: crypto/md5 over the
//                                     object bytes = the object's ETag
//   internal/etag/etag.go:211-226     etag.Multipart: MD5 over the parts' ETags ‖ "-N"
//                                     (zs3_etag_multipart runs that MD5 here too)
//   internal/hash/reader.go:123-153   content SHA-256 (sha256-simd, FIPS 180-4), compared
//                                     at EOF -> SHA256Mismatch
// Both digests are Merkle–Damgård chains over 64-byte blocks, so one message's blocks
// are processed in order by one lane; messages are independent (one lane each).
//
// Latency roof (round 4).  A wave issues at most one VALU instruction per 4 cycles
// (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'), and one message's blocks are a
// serial chain, so a message cannot go faster than (VALU instructions per block on its
// wave) x 4 cycles per block, whatever the batch size; a batch of n messages runs n/64
// such chains side by side.  The round-3 kernels ran the whole block on one wave: MD5
// 364 and SHA-256 1733 instructions per block in the compiled loop, and one block of
// load prefetch, so MD5 also waited on HBM (4096 x 1 MiB: 15.5 / 55.0 ms).  Here two
// waves share each group of 64 messages:
//   feeder wave      loads the blocks 4 ahead (compiler-tracked 16-byte loads), builds
//                    the padded final block(s), and writes per block the 64 words the
//                    rounds consume, constants folded in: MD5 m[g(t)] + K[t], SHA-256
//                    the message schedule W[t] + K[t] (byte-swapped, sigma functions)
//                    into a two-slot LDS ring ([slot][word quad][lane], 16-byte lanes:
//                    conflict-free ds_read_b128 / ds_write_b128);
//   compression wave 16 ds_read_b128 + the rounds only: MD5 4 instructions per step
//                    (bitop3, add3, alignbit, add), SHA-256 14 per round (two xor3-folded
//                    Sigma functions, bitop3 ch / maj, three adds).
// One workgroup barrier per block hands the slot over.  The roof is the compression
// wave's instruction count per block x 4 cycles (DESIGN.md §4 lists the counts and the
// measured per-block time).
#include "kernels.hpp"

#include <stdint.h>

namespace zs3k {

namespace {

__constant__ uint32_t kMd5K[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
    0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
    0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
    0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
    0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
    0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
    0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u,
};
__constant__ uint32_t kShaK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u,
};

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, s); }

// RFC 1321 compression of one 64-byte block (little-endian words m[0..15]).
__device__ __forceinline__ void md5_compress(uint32_t (&h)[4], const uint32_t (&m)[16]) {
    constexpr int R[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) & 15;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) & 15;
        }
        const uint32_t t = a + f + kMd5K[i] + m[g];
        a = d;
        d = c;
        c = b;
        b = b + rotl32(t, R[i >> 4][i & 3]);
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

// FIPS 180-4 SHA-256 compression (big-endian words already swapped into w[0..15]).
__device__ __forceinline__ void sha256_compress(uint32_t (&h)[8], uint32_t (&w)[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
            const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
        }
        const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = hh + S1 + ch + kShaK[i] + wi;
        const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
        const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        const uint32_t t2 = S0 + mj;
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += hh;
}

__device__ __forceinline__ void load_block(uint32_t (&m)[16], const uint8_t* p) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 v;
        __builtin_memcpy(&v, p + 16 * q, 16);
        m[4 * q + 0] = v.x;
        m[4 * q + 1] = v.y;
        m[4 * q + 2] = v.z;
        m[4 * q + 3] = v.w;
    }
}

// The final 1 or 2 blocks: tail bytes, 0x80, zeros, 64-bit bit length (little-endian
// for MD5, big-endian for SHA-256).  Returns the number of blocks written to m0/m1.
template <bool BE>
__device__ __forceinline__ int pad_tail(uint32_t (&m0)[16], uint32_t (&m1)[16], const uint8_t* tail, int nt,
                                        uint64_t total) {
    // Fully unrolled over the 64 byte positions so every word index is a constant
    // (a runtime-indexed register array would go to scratch).
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * w + j;
            const uint32_t byte = i < nt ? (uint32_t)tail[i] : (i == nt ? 0x80u : 0u);
            v |= BE ? byte << (8 * (3 - j)) : byte << (8 * j);
        }
        m0[w] = v;
        m1[w] = 0;
    }
    const uint64_t bits = total * 8;
    const uint32_t lo = (uint32_t)bits, hi = (uint32_t)(bits >> 32);
    const uint32_t w14 = BE ? hi : lo, w15 = BE ? lo : hi;
    if (nt < 56) {
        m0[14] = w14;
        m0[15] = w15;
        return 1;
    }
    m1[14] = w14;
    m1[15] = w15;
    return 2;
}

__device__ __forceinline__ void bswap16w(uint32_t (&m)[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = __builtin_bswap32(m[i]);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One SHA-256 round from the scheduled word + constant wk (FIPS 180-4 §6.2.2 step 3).
__device__ __forceinline__ void sha_round(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                          uint32_t& f, uint32_t& g, uint32_t& h, uint32_t wk) {
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);   // e ? f : g
    const uint32_t t1 = h + S1 + ch + wk;
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);   // majority
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
}

// MD5 step t from mk = m[g(t)] + K[t] (RFC 1321 §3.4).
template <int T>
__device__ __forceinline__ void md5_step(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t mk) {
    constexpr int R[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
    uint32_t f;
    if constexpr (T < 16)
        f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);  // b ? c : d
    else if constexpr (T < 32)
        f = __builtin_amdgcn_bitop3_b32(d, b, c, 0xCA);  // d ? b : c
    else if constexpr (T < 48)
        f = xor3(b, c, d);
    else
        f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x39);  // c ^ (b | ~d)
    const uint32_t t = a + f + mk;
    a = d;
    d = c;
    c = b;
    b = b + rotl32(t, R[T >> 4][T & 3]);
}

// the 64 round words of one block in a two-slot ring: ring[slot][q][lane], word t of the
// lane in component t % 4 of quad t / 4
typedef uint4 DgRing[2][16][64];

// Feeder wave: block b of this lane's message -> the 64 round words.
template <bool SHA>
__device__ __forceinline__ void dg_produce(uint4 (&slot)[16][64], int lane, int64_t b, int64_t nfull, int64_t nblk,
                                           const uint4 (&raw)[4], const uint8_t* msg, int nt, int64_t len) {
    uint32_t m[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        m[4 * q + 0] = raw[q].x;
        m[4 * q + 1] = raw[q].y;
        m[4 * q + 2] = raw[q].z;
        m[4 * q + 3] = raw[q].w;
    }
    if constexpr (SHA) bswap16w(m);
    if (b >= nfull && b < nblk) {
        // the padded final block(s): tail bytes, 0x80, zeros, bit length
        uint32_t m0[16], m1[16];
        pad_tail<SHA>(m0, m1, msg + (nfull << 6), nt, (uint64_t)len);
        const bool first = b == nfull;
#pragma unroll
        for (int w = 0; w < 16; ++w) m[w] = first ? m0[w] : m1[w];
    }
    uint32_t wk[64];
    if constexpr (SHA) {
#pragma unroll
        for (int t = 0; t < 64; ++t) {
            if (t >= 16) {
                const uint32_t w15 = m[(t - 15) & 15], w2 = m[(t - 2) & 15];
                const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
                m[t & 15] = m[t & 15] + s0 + m[(t - 7) & 15] + s1;
            }
            wk[t] = m[t & 15] + kShaK[t];
        }
    } else {
#pragma unroll
        for (int t = 0; t < 64; ++t) {
            const int g = t < 16 ? t : t < 32 ? (5 * t + 1) & 15 : t < 48 ? (3 * t + 5) & 15 : (7 * t) & 15;
            wk[t] = m[g] + kMd5K[t];
        }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) slot[q][lane] = make_uint4(wk[4 * q], wk[4 * q + 1], wk[4 * q + 2], wk[4 * q + 3]);
}

template <int T>
__device__ __forceinline__ void md5_rounds(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, const uint32_t (&wk)[64]) {
    if constexpr (T < 64) {
        md5_step<T>(a, b, c, d, wk[T]);
        md5_rounds<T + 1>(a, b, c, d, wk);
    }
}

}  // namespace

// Two-wave digest pipeline (see the header): 128 threads = compression wave (0) +
// feeder wave (1) over the same 64 messages.  Message i: bytes at msgs + offs[i] (or
// i*stride), length lens[i] (or len).
template <bool SHA>
__global__ void __launch_bounds__(128) k_digest_ws(DigestArgs a) {
    __shared__ DgRing ring;
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t i0 = (int64_t)blockIdx.x * 64 + lane;
    const bool live = i0 < a.n;
    const int64_t i = live ? i0 : a.n - 1;  // dead lanes repeat the last message
    const uint8_t* msg = a.msgs + (a.offs ? a.offs[i] : i * a.stride);
    const int64_t len = a.lens ? a.lens[i] : a.len;
    const int64_t nfull = len >> 6;
    const int nt = (int)(len & 63);
    const int64_t nblk = nfull + (nt < 56 ? 1 : 2);
    // blocks of the wave's longest message (both waves compute the same value: the
    // number of barriers below must agree)
    int nbw = (int)nblk;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nbw = max(nbw, __shfl_xor(nbw, off));
    if (__builtin_amdgcn_readfirstlane(tid) >= 64) {
        // ---- feeder: loads 4 blocks ahead
        constexpr int P = 4;
        uint4 raw[P][4];
        auto issue = [&](uint4 (&r)[4], int64_t b) {
            if (b < nfull) {
                const uint8_t* p = msg + (b << 6);
#pragma unroll
                for (int q = 0; q < 4; ++q) __builtin_memcpy(&r[q], p + 16 * q, 16);
            }
        };
#pragma unroll
        for (int p = 0; p < P; ++p) issue(raw[p], p);
        for (int s0 = 0; s0 <= nbw; s0 += P) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const int s = s0 + p;
                if (s > nbw) break;
                if (s < nbw) dg_produce<SHA>(ring[s & 1], lane, s, nfull, nblk, raw[p], msg, nt, len);
                issue(raw[p], s + P);
                __syncthreads();
            }
        }
        return;
    }
    // ---- compression
    uint32_t h[8];
    if constexpr (SHA) {
        h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
        h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
    } else {
        h[0] = 0x67452301u; h[1] = 0xefcdab89u; h[2] = 0x98badcfeu; h[3] = 0x10325476u;
        h[4] = h[5] = h[6] = h[7] = 0;
    }
    for (int s = 0; s <= nbw; ++s) {
        if (s >= 1) {
            const int b = s - 1;
            uint32_t wk[64];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint4 v = ring[b & 1][q][lane];
                wk[4 * q] = v.x;
                wk[4 * q + 1] = v.y;
                wk[4 * q + 2] = v.z;
                wk[4 * q + 3] = v.w;
            }
            const bool upd = b < nblk;
            if constexpr (SHA) {
                uint32_t A = h[0], B = h[1], C = h[2], D = h[3], E = h[4], F = h[5], G = h[6], H = h[7];
#pragma unroll
                for (int t = 0; t < 64; ++t) sha_round(A, B, C, D, E, F, G, H, wk[t]);
                h[0] = upd ? h[0] + A : h[0];
                h[1] = upd ? h[1] + B : h[1];
                h[2] = upd ? h[2] + C : h[2];
                h[3] = upd ? h[3] + D : h[3];
                h[4] = upd ? h[4] + E : h[4];
                h[5] = upd ? h[5] + F : h[5];
                h[6] = upd ? h[6] + G : h[6];
                h[7] = upd ? h[7] + H : h[7];
            } else {
                uint32_t A = h[0], B = h[1], C = h[2], D = h[3];
                md5_rounds<0>(A, B, C, D, wk);
                h[0] = upd ? h[0] + A : h[0];
                h[1] = upd ? h[1] + B : h[1];
                h[2] = upd ? h[2] + C : h[2];
                h[3] = upd ? h[3] + D : h[3];
            }
        }
        __syncthreads();
    }
    if (!live) return;
    if constexpr (SHA) {
        uint32_t* out = reinterpret_cast<uint32_t*>(a.out + i * 32);
#pragma unroll
        for (int w = 0; w < 8; ++w) out[w] = __builtin_bswap32(h[w]);  // big-endian digest
    } else {
        uint32_t* out = reinterpret_cast<uint32_t*>(a.out + i * 16);
#pragma unroll
        for (int w = 0; w < 4; ++w) out[w] = h[w];  // digest = h0..h3 little-endian
    }
}

// Round-3 kernels (diagnostics variant 1): the whole block on one wave, one block of
// load prefetch.
__global__ void __launch_bounds__(64) k_md5_batch(DigestArgs a) {
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    const uint8_t* msg = a.msgs + (a.offs ? a.offs[i] : i * a.stride);
    const int64_t len = a.lens ? a.lens[i] : a.len;
    const int64_t nfull = len >> 6;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    uint32_t cur[16], nxt[16];
    if (nfull > 0) load_block(cur, msg);
    for (int64_t blk = 0; blk < nfull; ++blk) {
        if (blk + 1 < nfull) load_block(nxt, msg + ((blk + 1) << 6));
        md5_compress(h, cur);
#pragma unroll
        for (int w = 0; w < 16; ++w) cur[w] = nxt[w];
    }
    uint32_t m0[16], m1[16];
    const int nb = pad_tail<false>(m0, m1, msg + (nfull << 6), (int)(len & 63), (uint64_t)len);
    md5_compress(h, m0);
    if (nb == 2) md5_compress(h, m1);
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out + i * 16);
#pragma unroll
    for (int w = 0; w < 4; ++w) out[w] = h[w];  // digest = h0..h3 little-endian
}

__global__ void __launch_bounds__(64) k_sha256_batch(DigestArgs a) {
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    const uint8_t* msg = a.msgs + (a.offs ? a.offs[i] : i * a.stride);
    const int64_t len = a.lens ? a.lens[i] : a.len;
    const int64_t nfull = len >> 6;
    uint32_t h[8] = {
        0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u
    };
    uint32_t cur[16], nxt[16];
    if (nfull > 0) load_block(cur, msg);
    for (int64_t blk = 0; blk < nfull; ++blk) {
        if (blk + 1 < nfull) load_block(nxt, msg + ((blk + 1) << 6));
        bswap16w(cur);
        sha256_compress(h, cur);
#pragma unroll
        for (int w = 0; w < 16; ++w) cur[w] = nxt[w];
    }
    uint32_t m0[16], m1[16];
    const int nb = pad_tail<true>(m0, m1, msg + (nfull << 6), (int)(len & 63), (uint64_t)len);
    sha256_compress(h, m0);
    if (nb == 2) sha256_compress(h, m1);
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out + i * 32);
#pragma unroll
    for (int w = 0; w < 8; ++w) out[w] = __builtin_bswap32(h[w]);  // big-endian digest
}

hipError_t launch_md5(const DigestArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    if (ZS3_DIAG && a.variant == 1)
        hipLaunchKernelGGL(k_md5_batch, dim3((unsigned)((a.n + 63) / 64)), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL(k_digest_ws<false>, dim3((unsigned)((a.n + 63) / 64)), dim3(128), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_sha256(const DigestArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    if (ZS3_DIAG && a.variant == 1)
        hipLaunchKernelGGL(k_sha256_batch, dim3((unsigned)((a.n + 63) / 64)), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL(k_digest_ws<true>, dim3((unsigned)((a.n + 63) / 64)), dim3(128), 0, s, a);
    return hipGetLastError();
}

}  // namespace zs3k
