// gf_dev.hpp — GF(2^8) multiply-accumulate on packed bytes for gfx950.
//
// Arithmetic of klauspost/reedsolomon v1.11.8 (poly 0x11D) as called by
// Erasure.EncodeData (cmd/erasure-coding.go:86) and the decoders (:108, :114),
// restated for the VALU: no MFMA (GF(256) bytes, not a float contraction).
//
// c*x is GF(2)-linear in x, so with x = a | b<<3 | c<<6 (3+3+2 bits):
//   c*x = Ta[a] ^ Tb[b] ^ Tc[c]
// Each table has <= 8 byte entries and is applied to four packed bytes at once by
// one v_perm_b32 (byte select from an 8-byte {hi:lo} pair).  The lookups fold into
// the accumulator with v_bitop3_b32 (XOR3, truth table 0x96): two coefficients =
// six lookups = three XOR3.
// Per data dword: 5 VALU to split nibbles (shared by all parity rows), then per
// coefficient 3 x v_perm_b32 + 1.5 x XOR3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zs3dev {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct Nib {
    uint32_t a, b, c;
};

__device__ __forceinline__ Nib split_nibbles(uint32_t x) {
    Nib n;
    n.a = x & 0x07070707u;
    n.b = (x >> 3) & 0x07070707u;
    n.c = (x >> 6) & 0x03030303u;
    return n;
}

// Coefficient tables as held in LDS: 8 dwords per coefficient (32 B aligned),
// Ta.lo Ta.hi Tb.lo Tb.hi | Tc 0 0 0.
struct CoefTab {
    uint4 ab;
    uint32_t c;
};

__device__ __forceinline__ CoefTab load_coef(const uint32_t* lds_tab, int idx) {
    CoefTab t;
    t.ab = *reinterpret_cast<const uint4*>(lds_tab + 8 * idx);
    t.c = lds_tab[8 * idx + 4];
    return t;
}

// The three partial products of c*x (XOR of the three = c*x).
struct Prod3 {
    uint32_t a, b, c;
};

__device__ __forceinline__ Prod3 gf_lookup(const Nib& n, const CoefTab& t) {
    Prod3 p;
    p.a = __builtin_amdgcn_perm(t.ab.y, t.ab.x, n.a);
    p.b = __builtin_amdgcn_perm(t.ab.w, t.ab.z, n.b);
    p.c = __builtin_amdgcn_perm(t.c, t.c, n.c);
    return p;
}

// Accumulator with one pending term so that lookups fold two at a time.
struct GfAcc {
    uint32_t acc, pend;
    bool has;
};

__device__ __forceinline__ void acc_init(GfAcc& s) {
    s.acc = 0;
    s.pend = 0;
    s.has = false;
}

// Unrolled call sites make `has` a compile-time constant per step.
__device__ __forceinline__ void acc_add(GfAcc& s, const Prod3& p) {
    if (!s.has) {
        s.acc = xor3(s.acc, p.a, p.b);
        s.pend = p.c;
        s.has = true;
    } else {
        s.acc = xor3(s.acc, s.pend, p.a);
        s.acc = xor3(s.acc, p.b, p.c);
        s.has = false;
    }
}

__device__ __forceinline__ uint32_t acc_done(const GfAcc& s) {
    return s.has ? (s.acc ^ s.pend) : s.acc;
}

// A column of NWd packed data dwords (4 * NWd bytes of one shard row).
template <int NWd>
struct Col {
    uint32_t w[NWd];
};

__device__ __forceinline__ Nib nib_xor(const Nib& x, const Nib& y) {
    Nib r;
    r.a = x.a ^ y.a;
    r.b = x.b ^ y.b;
    r.c = x.c ^ y.c;
    return r;
}

__device__ __forceinline__ uint32_t fold3(const Prod3& p) { return xor3(p.a, p.b, p.c); }

// An SGPR zero the compiler cannot see through: indexing the LDS coefficient
// tables with it keeps their loads where they are used instead of hoisting every
// table into VGPRs (which would cap occupancy).
__device__ __forceinline__ int opaque_zero() {
    int z = 0;
    asm volatile("" : "+s"(z));
    return z;
}

// Dyadic encode (parity block = K/M blocks [[A,B],[B,A]]; see zs3gpu.hip).
// M = 4, per block with generator (a,b,c,d) and inputs x0..x3:
//   T = a.x0 + b.x1 + c.x2 + d.x3,  R = (a+b)(x0+x1) + (c+d)(x2+x3)
//   UV = (a+c)(x0+x2) + (b+d)(x1+x3),  W = (a+b+c+d)(x0+x1+x2+x3)
//   y0 = T, y1 = T+R, y2 = T+UV, y3 = T+R+UV+W          (9 multiplies, not 16)
// M = 2: y0 = a.x0 + b.x1, y1 = y0 + (a+b)(x0+x1)      (3 multiplies, not 4)
// Nibble splits are GF(2)-linear, so the split of a sum is the XOR of splits.
template <int NWd, int K, int M>
__device__ __forceinline__ void encode_dyadic(const Col<NWd> (&x)[K], Col<NWd> (&out)[M], const uint32_t* dtabs) {
    static_assert(M == 2 || M == 4, "dyadic block");
    constexpr int PER = M == 4 ? 9 : 3;
    uint32_t acc[M][NWd];
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
        for (int w = 0; w < NWd; ++w) acc[r][w] = 0;
#pragma unroll
    for (int q = 0; q < K / M; ++q) {
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t* tq = dtabs + opaque_zero() + q * PER * 8;
        CoefTab t[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) t[i] = load_coef(tq, i);
#pragma unroll
        for (int w = 0; w < NWd; ++w) {
            if constexpr (M == 4) {
                const Nib n0 = split_nibbles(x[4 * q + 0].w[w]), n1 = split_nibbles(x[4 * q + 1].w[w]);
                const Nib n2 = split_nibbles(x[4 * q + 2].w[w]), n3 = split_nibbles(x[4 * q + 3].w[w]);
                const Nib d01 = nib_xor(n0, n1), d23 = nib_xor(n2, n3);
                const Nib s0 = nib_xor(n0, n2), s1 = nib_xor(n1, n3), s01 = nib_xor(s0, s1);
                const Prod3 P = gf_lookup(n0, t[0]), Q = gf_lookup(n1, t[1]);
                const Prod3 P2 = gf_lookup(n2, t[3]), Q2 = gf_lookup(n3, t[4]);
                const Prod3 R1 = gf_lookup(d01, t[2]), R2 = gf_lookup(d23, t[5]);
                const Prod3 U = gf_lookup(s0, t[6]), V = gf_lookup(s1, t[7]);
                const Prod3 W = gf_lookup(s01, t[8]);
                uint32_t T = xor3(P.a, P.b, P.c);
                T = xor3(T, Q.a, Q.b);
                T = xor3(T, Q.c, P2.a);
                T = xor3(T, P2.b, P2.c);
                T = xor3(T, Q2.a, Q2.b);
                T = T ^ Q2.c;
                const uint32_t R = xor3(fold3(R1), R2.a, R2.b) ^ R2.c;
                const uint32_t UV = xor3(fold3(U), V.a, V.b) ^ V.c;
                const uint32_t Wv = fold3(W);
                acc[0][w] ^= T;
                acc[1][w] = xor3(acc[1][w], T, R);
                acc[2][w] = xor3(acc[2][w], T, UV);
                acc[3][w] = xor3(acc[3][w], xor3(T, R, UV), Wv);
            } else {
                const Nib n0 = split_nibbles(x[2 * q + 0].w[w]), n1 = split_nibbles(x[2 * q + 1].w[w]);
                const Nib d01 = nib_xor(n0, n1);
                const Prod3 P = gf_lookup(n0, t[0]), Q = gf_lookup(n1, t[1]), R = gf_lookup(d01, t[2]);
                const uint32_t PQ = xor3(fold3(P), Q.a, Q.b) ^ Q.c;
                acc[0][w] ^= PQ;
                acc[1][w] = xor3(acc[1][w], PQ, fold3(R));
            }
        }
    }
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
        for (int w = 0; w < NWd; ++w) out[r].w[w] = acc[r][w];
}

// Scalar GF multiply with log/exp tables (generic byte path).
__device__ __forceinline__ uint8_t gf_mul_log(const uint8_t* lg, const uint8_t* ex, uint8_t a, uint8_t b) {
    return (a && b) ? ex[(int)lg[a] + (int)lg[b]] : (uint8_t)0;
}

}  // namespace zs3dev
