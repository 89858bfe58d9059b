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

// Scalar GF multiply with log/exp tables (generic byte path).
__device__ __forceinline__ uint8_t gf_mul_log(const uint8_t* lg, const uint8_t* ex, uint8_t a, uint8_t b) {
    return (a && b) ? ex[(int)lg[a] + (int)lg[b]] : (uint8_t)0;
}

}  // namespace zs3dev
