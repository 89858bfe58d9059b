// hh256_dev.hpp — HighwayHash-256 on CDNA4 (gfx950), one chain per quad.
//
// Restates minio/highwayhash v1.0.2 (== Google's C reference) as used by the
// streaming bitrot writer/reader: cmd/bitrot.go:47-64 (hash factory, magic key
// cmd/bitrot.go:37) and cmd/bitrot-streaming.go:47-49 / :171-182.
//
// Mapping: HighwayHash keeps 4 independent 64-bit lanes (v0, v1, mul0, mul1)
// that only interact in ZipperMergeAndAdd, which mixes lane pairs (0,1) and
// (2,3).  Each thread of a quad owns ONE HH lane; the zipper needs only the
// partner's high dword, fetched with one DPP quad_perm [1,0,3,2] move.  A
// 64-lane wavefront therefore advances 16 independent hash chains in lockstep.
// Per packet and thread: 2 x v_lshl_add_u64, 2 x v_mad_u64_u32, 4 x xor,
// 2 x DPP, 6 x v_perm_b32, 2 x 64-bit add.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zs3dev {

struct HHLane {
    uint64_t v0, v1, mul0, mul1;
};

__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v) {  // lane ^ 1 within the quad
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t v) {  // lane ^ 2 within the quad
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
}

// Zipper-merge term for this thread's lane from its own 64-bit value and the
// partner lane's high dword.  Byte maps (C reference ZipperMergeAndAdd):
//   even lane: [o3 p4 o2 o5 | p6 o1 p7 o0]   odd lane: [o3 p4 o2 o5 | o1 p6 o0 p7]
// (oN = own byte N, pN = partner byte N); v_perm_b32 selects byte i of {S0:S1}.
__device__ __forceinline__ uint64_t zipper(uint64_t own, uint32_t partner_hi, uint32_t sel_hi) {
    const uint32_t olo = (uint32_t)own, ohi = (uint32_t)(own >> 32);
    const uint32_t t = __builtin_amdgcn_perm(partner_hi, olo, 0x0c020403u);
    const uint32_t lo = __builtin_amdgcn_perm(t, ohi, 0x01060504u);
    const uint32_t hi = __builtin_amdgcn_perm(partner_hi, olo, sel_hi);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t zipper_sel(int lane) {
    return (lane & 1) ? 0x07000601u : 0x00070106u;
}

// 64-bit add as ONE v_lshl_add_u64.  Written in asm because hipcc otherwise
// splits `x + ((hi << 32) | lo)` into two adds plus two v_mov (disjoint-or -> add).
__device__ __forceinline__ uint64_t add64(uint64_t a, uint64_t b) {
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ uint64_t zipper_add(uint64_t acc, uint64_t own, uint32_t partner_hi,
                                               uint32_t sel_hi) {
    const uint32_t olo = (uint32_t)own, ohi = (uint32_t)(own >> 32);
    const uint32_t t = __builtin_amdgcn_perm(partner_hi, olo, 0x0c020403u);
    const uint32_t lo = __builtin_amdgcn_perm(t, ohi, 0x01060504u);
    const uint32_t hi = __builtin_amdgcn_perm(partner_hi, olo, sel_hi);
    return add64(acc, ((uint64_t)hi << 32) | lo);
}

// One HighwayHash Update() step for this thread's lane (C reference Update).
__device__ __forceinline__ void hh_update(HHLane& s, uint64_t w, uint32_t sel_hi) {
    s.v1 = add64(s.v1, add64(s.mul0, w));
    s.mul0 ^= (uint64_t)(uint32_t)s.v1 * (s.v0 >> 32);
    s.v0 = add64(s.v0, s.mul1);
    s.mul1 ^= (uint64_t)(uint32_t)s.v0 * (s.v1 >> 32);
    s.v0 = zipper_add(s.v0, s.v1, dpp_xor1((uint32_t)(s.v1 >> 32)), sel_hi);
    s.v1 = zipper_add(s.v1, s.v0, dpp_xor1((uint32_t)(s.v0 >> 32)), sel_hi);
}

// N consecutive Update() steps (round 6): the same arithmetic as N x hh_update with a
// shorter dependent chain.  Update's last add (v1 += zipper(v0)) and the next packet's
// first (v1 += mul0 + w) both land on v1; 64-bit adds commute, so the next packet's
// mul0 + w is added to v1 while the zipper of v0 is still being formed, and the zipper
// result is added once: per packet the chain v1 -> DPP -> 2 v_perm -> add -> DPP -> 2
// v_perm -> add -> v1 is 8 dependent instructions instead of 9, with no extra VALU.
// Between the first and last packet v1 carries the next packet's mul0 + w (V1 below);
// the state on return is the standard one.
template <int N>
__device__ __forceinline__ void hh_update_n(HHLane& s, const uint64_t (&w)[N], uint32_t sel_hi) {
    uint64_t V1 = add64(s.v1, add64(s.mul0, w[0]));
#pragma unroll
    for (int i = 0; i < N; ++i) {
        s.mul0 ^= (uint64_t)(uint32_t)V1 * (s.v0 >> 32);
        s.v0 = add64(s.v0, s.mul1);
        s.mul1 ^= (uint64_t)(uint32_t)s.v0 * (V1 >> 32);
        s.v0 = zipper_add(s.v0, V1, dpp_xor1((uint32_t)(V1 >> 32)), sel_hi);
        const uint64_t base = i + 1 < N ? add64(V1, add64(s.mul0, w[i + 1])) : V1;
        V1 = zipper_add(base, s.v0, dpp_xor1((uint32_t)(s.v0 >> 32)), sel_hi);
    }
    s.v1 = V1;
}

// Initial state for lane `lane` under key words key[0..3] (C reference Reset).
__device__ __forceinline__ HHLane hh_init(int lane, uint64_t k0, uint64_t k1, uint64_t k2, uint64_t k3) {
    const uint64_t key = lane == 0 ? k0 : lane == 1 ? k1 : lane == 2 ? k2 : k3;
    const uint64_t i0 = lane == 0 ? 0xdbe6d5d5fe4cce2fULL
                      : lane == 1 ? 0xa4093822299f31d0ULL
                      : lane == 2 ? 0x13198a2e03707344ULL
                                  : 0x243f6a8885a308d3ULL;
    const uint64_t i1 = lane == 0 ? 0x3bd39e10cb0ef593ULL
                      : lane == 1 ? 0xc0acf169b5f18a8cULL
                      : lane == 2 ? 0xbe5466cf34e90c6cULL
                                  : 0x452821e638d01377ULL;
    HHLane s;
    s.mul0 = i0;
    s.mul1 = i1;
    s.v0 = i0 ^ key;
    s.v1 = i1 ^ ((key >> 32) | (key << 32));
    return s;
}

// Hash `npk` full 32-byte packets of a row staged in LDS (8-byte aligned).
__device__ __forceinline__ void hh_packets(HHLane& s, const uint8_t* row, int npk, int lane,
                                           uint32_t sel_hi) {
    const uint64_t* p = reinterpret_cast<const uint64_t*>(row) + lane;
    if (npk <= 0) return;
    // Software-pipelined: the next packet's ds_read_b64 is in flight while the
    // current packet runs the serial HighwayHash chain.
    uint64_t w = p[0];
    for (int i = 1; i < npk; ++i) {
        const uint64_t nxt = p[4 * i];
        hh_update(s, w, sel_hi);
        w = nxt;
    }
    hh_update(s, w, sel_hi);
}

// Full-tile form: NPK (compile-time) packets, fully unrolled so every ds_read_b64
// uses an immediate offset and the register rotation of the loop disappears.
// Next-packet prefetch as above.
// Round 6: runs of up to 8 packets through hh_update_n (the next run's reads are issued
// before the current run's arithmetic).
template <int NPK>
__device__ __forceinline__ void hh_packets_n(HHLane& s, const uint8_t* row, int lane, uint32_t sel_hi) {
    const uint64_t* p = reinterpret_cast<const uint64_t*>(row) + lane;
    // the longest run of at most 8 packets that divides NPK
    constexpr int RUN = NPK <= 8 ? NPK : NPK % 8 == 0 ? 8 : NPK % 6 == 0 ? 6 : NPK % 4 == 0 ? 4 : NPK % 2 == 0 ? 2 : 1;
    static_assert(NPK % RUN == 0, "whole runs");
    uint64_t w[RUN];
#pragma unroll
    for (int i = 0; i < RUN; ++i) w[i] = p[4 * i];
#pragma unroll
    for (int r = 0; r < NPK / RUN; ++r) {
        uint64_t nx[RUN];
        if (r + 1 < NPK / RUN) {
#pragma unroll
            for (int i = 0; i < RUN; ++i) nx[i] = p[4 * ((r + 1) * RUN + i)];
        }
        hh_update_n<RUN>(s, w, sel_hi);
        if (r + 1 < NPK / RUN) {
#pragma unroll
            for (int i = 0; i < RUN; ++i) w[i] = nx[i];
        }
    }
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, 32u - n);  // n in 1..31
}

// HighwayHashUpdateRemainder for the final size_mod32 = n (1..31) bytes at `tail`
// (LDS).  The packet is zero-filled, holds tail[0 .. n&~3), and then either
// packet[28..31] = last 4 bytes (n & 16) or packet[16..18] = the 1-3 trailing bytes.
__device__ __forceinline__ void hh_remainder(HHLane& s, const uint8_t* tail, uint32_t n, int lane,
                                             uint32_t sel_hi) {
    s.v0 += ((uint64_t)n << 32) + n;
    s.v1 = ((uint64_t)rotl32((uint32_t)(s.v1 >> 32), n) << 32) | rotl32((uint32_t)s.v1, n);
    const uint32_t remain = n & ~3u, mod4 = n & 3u;
    uint8_t b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t idx = 8u * lane + i;
        b[i] = idx < remain ? tail[idx] : 0;
    }
    if (n & 16u) {
        if (lane == 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) b[4 + i] = tail[n - 4 + i];
        }
    } else if (mod4) {
        if (lane == 2) {
            b[0] = tail[remain];
            b[1] = tail[remain + (mod4 >> 1)];
            b[2] = tail[n - 1];
        }
    }
    uint64_t w = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) w = (w << 8) | b[i];
    hh_update(s, w, sel_hi);
}

// 10 PermuteAndUpdate rounds + ModularReduction.  Returns this lane's 64-bit
// digest word h[lane] (digest = h0||h1||h2||h3 little-endian).
__device__ __forceinline__ uint64_t hh_finalize256(HHLane& s, int lane, uint32_t sel_hi) {
    for (int r = 0; r < 10; ++r) {
        // permuted[l] = rot32(v0[(l + 2) & 3])
        const uint32_t plo = dpp_xor2((uint32_t)s.v0);
        const uint32_t phi = dpp_xor2((uint32_t)(s.v0 >> 32));
        hh_update(s, ((uint64_t)plo << 32) | phi, sel_hi);
    }
    const uint64_t a_hi = s.v1 + s.mul1;  // a3 (odd lane) / a2 (even lane)
    const uint64_t a_lo = s.v0 + s.mul0;  // a1 (odd lane) / a0 (even lane)
    const uint32_t q_lo = dpp_xor1((uint32_t)a_hi);
    const uint32_t q_hi = dpp_xor1((uint32_t)(a_hi >> 32));
    if (lane & 1) {
        const uint64_t a2 = ((uint64_t)q_hi << 32) | q_lo;
        const uint64_t a3 = a_hi & 0x3FFFFFFFFFFFFFFFULL;
        return a_lo ^ ((a3 << 1) | (a2 >> 63)) ^ ((a3 << 2) | (a2 >> 62));
    }
    return a_lo ^ (a_hi << 1) ^ (a_hi << 2);
}

// ---------------------------------------------------------------------------
// Pair form: one chain per PAIR of threads, each thread owning the HH lane pair
// (2h, 2h+1) that ZipperMergeAndAdd mixes, so an Update needs no cross-lane move.
// With A = lane 2h+1 and B = lane 2h (C reference ZipperMergeAndAdd(v1=A, v0=B)):
//   addB = [B3 A4 B2 B5 | A6 B1 A7 B0],  addA = [A3 B4 A2 A5 | A1 B6 A0 B7]
// X = [A4 B5 B4 A5] (one v_perm of A.hi, B.hi) feeds both low dwords: 5 v_perm per
// zipper for two lanes instead of 6.
struct HHPair {
    uint64_t v0[2], v1[2], mul0[2], mul1[2];  // [0] = lane 2h (B), [1] = lane 2h+1 (A)
};

__device__ __forceinline__ void zipper_pair(uint64_t A, uint64_t B, uint64_t& addA, uint64_t& addB) {
    const uint32_t alo = (uint32_t)A, ahi = (uint32_t)(A >> 32);
    const uint32_t blo = (uint32_t)B, bhi = (uint32_t)(B >> 32);
    const uint32_t X = __builtin_amdgcn_perm(ahi, bhi, 0x05000104u);
    const uint32_t b_lo = __builtin_amdgcn_perm(X, blo, 0x05020403u);
    const uint32_t a_lo = __builtin_amdgcn_perm(X, alo, 0x07020603u);
    const uint32_t b_hi = __builtin_amdgcn_perm(ahi, blo, 0x00070106u);
    const uint32_t a_hi = __builtin_amdgcn_perm(bhi, alo, 0x07000601u);
    addA = ((uint64_t)a_hi << 32) | a_lo;
    addB = ((uint64_t)b_hi << 32) | b_lo;
}

__device__ __forceinline__ void hh2_update(HHPair& s, uint64_t w0, uint64_t w1) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint64_t w = i ? w1 : w0;
        s.v1[i] = add64(s.v1[i], add64(s.mul0[i], w));
        s.mul0[i] ^= (uint64_t)(uint32_t)s.v1[i] * (s.v0[i] >> 32);
        s.v0[i] = add64(s.v0[i], s.mul1[i]);
        s.mul1[i] ^= (uint64_t)(uint32_t)s.v0[i] * (s.v1[i] >> 32);
    }
    uint64_t aA, aB;
    zipper_pair(s.v1[1], s.v1[0], aA, aB);
    s.v0[1] = add64(s.v0[1], aA);
    s.v0[0] = add64(s.v0[0], aB);
    zipper_pair(s.v0[1], s.v0[0], aA, aB);
    s.v1[1] = add64(s.v1[1], aA);
    s.v1[0] = add64(s.v1[0], aB);
}

// N consecutive pair-form updates with the next packet's mul0 + w folded into v1 before
// the second zipper lands (as hh_update_n): the same VALU, one dependent add less per packet.
template <int N>
__device__ __forceinline__ void hh2_update_n(HHPair& s, const uint4 (&w)[N]) {
    uint64_t V1[2];
    V1[0] = add64(s.v1[0], add64(s.mul0[0], ((uint64_t)w[0].y << 32) | w[0].x));
    V1[1] = add64(s.v1[1], add64(s.mul0[1], ((uint64_t)w[0].w << 32) | w[0].z));
#pragma unroll
    for (int p = 0; p < N; ++p) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            s.mul0[i] ^= (uint64_t)(uint32_t)V1[i] * (s.v0[i] >> 32);
            s.v0[i] = add64(s.v0[i], s.mul1[i]);
            s.mul1[i] ^= (uint64_t)(uint32_t)s.v0[i] * (V1[i] >> 32);
        }
        uint64_t aA, aB;
        zipper_pair(V1[1], V1[0], aA, aB);
        s.v0[1] = add64(s.v0[1], aA);
        s.v0[0] = add64(s.v0[0], aB);
        zipper_pair(s.v0[1], s.v0[0], aA, aB);
        uint64_t b0 = V1[0], b1 = V1[1];
        if (p + 1 < N) {
            b0 = add64(b0, add64(s.mul0[0], ((uint64_t)w[p + 1].y << 32) | w[p + 1].x));
            b1 = add64(b1, add64(s.mul0[1], ((uint64_t)w[p + 1].w << 32) | w[p + 1].z));
        }
        V1[1] = add64(b1, aA);
        V1[0] = add64(b0, aB);
    }
    s.v1[0] = V1[0];
    s.v1[1] = V1[1];
}

__device__ __forceinline__ HHPair hh2_init(int h, uint64_t k0, uint64_t k1, uint64_t k2, uint64_t k3) {
    HHPair s;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const HHLane l = hh_init(2 * h + i, k0, k1, k2, k3);
        s.v0[i] = l.v0;
        s.v1[i] = l.v1;
        s.mul0[i] = l.mul0;
        s.mul1[i] = l.mul1;
    }
    return s;
}

// Full packets of a row in LDS (16-byte aligned); this thread reads its 16 bytes.
__device__ __forceinline__ void hh2_packets(HHPair& s, const uint8_t* row, int npk, int h) {
    const uint4* p = reinterpret_cast<const uint4*>(row) + h;
    if (npk <= 0) return;
    uint4 w = p[0];
    for (int i = 1; i < npk; ++i) {
        const uint4 nxt = p[2 * i];
        hh2_update(s, ((uint64_t)w.y << 32) | w.x, ((uint64_t)w.w << 32) | w.z);
        w = nxt;
    }
    hh2_update(s, ((uint64_t)w.y << 32) | w.x, ((uint64_t)w.w << 32) | w.z);
}

template <int NPK>
__device__ __forceinline__ void hh2_packets_n(HHPair& s, const uint8_t* row, int h) {
    const uint4* p = reinterpret_cast<const uint4*>(row) + h;
    uint4 w = p[0];
#pragma unroll
    for (int i = 1; i < NPK; ++i) {
        const uint4 nxt = p[2 * i];
        hh2_update(s, ((uint64_t)w.y << 32) | w.x, ((uint64_t)w.w << 32) | w.z);
        w = nxt;
    }
    hh2_update(s, ((uint64_t)w.y << 32) | w.x, ((uint64_t)w.w << 32) | w.z);
}

// HighwayHashUpdateRemainder (n = 1..31 bytes at tail) for the lanes 2h, 2h+1.
__device__ __forceinline__ void hh2_remainder(HHPair& s, const uint8_t* tail, uint32_t n, int h) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        s.v0[i] += ((uint64_t)n << 32) + n;
        s.v1[i] = ((uint64_t)rotl32((uint32_t)(s.v1[i] >> 32), n) << 32) | rotl32((uint32_t)s.v1[i], n);
    }
    const uint32_t remain = n & ~3u, mod4 = n & 3u;
    uint8_t b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t idx = 16u * h + i;
        b[i] = idx < remain ? tail[idx] : 0;
    }
    if (n & 16u) {
        if (h == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) b[12 + i] = tail[n - 4 + i];
        }
    } else if (mod4) {
        if (h == 1) {
            b[0] = tail[remain];
            b[1] = tail[remain + (mod4 >> 1)];
            b[2] = tail[n - 1];
        }
    }
    uint64_t w0 = 0, w1 = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
        w0 = (w0 << 8) | b[i];
        w1 = (w1 << 8) | b[8 + i];
    }
    hh2_update(s, w0, w1);
}

// Finalize-256.  Returns this thread's 16 digest bytes (h[2h], h[2h+1]).
__device__ __forceinline__ void hh2_finalize256(HHPair& s, uint64_t& d0, uint64_t& d1) {
    for (int r = 0; r < 10; ++r) {
        // permuted[l] = rot32(v0[(l + 2) & 3]): lanes 2h, 2h+1 take the partner's v0
        const uint32_t p0lo = dpp_xor1((uint32_t)s.v0[0]), p0hi = dpp_xor1((uint32_t)(s.v0[0] >> 32));
        const uint32_t p1lo = dpp_xor1((uint32_t)s.v0[1]), p1hi = dpp_xor1((uint32_t)(s.v0[1] >> 32));
        hh2_update(s, ((uint64_t)p0lo << 32) | p0hi, ((uint64_t)p1lo << 32) | p1hi);
    }
    const uint64_t a3 = (s.v1[1] + s.mul1[1]) & 0x3FFFFFFFFFFFFFFFULL;
    const uint64_t a2 = s.v1[0] + s.mul1[0];
    const uint64_t a1 = s.v0[1] + s.mul0[1];
    const uint64_t a0 = s.v0[0] + s.mul0[0];
    d1 = a1 ^ ((a3 << 1) | (a2 >> 63)) ^ ((a3 << 2) | (a2 >> 62));
    d0 = a0 ^ (a2 << 1) ^ (a2 << 2);
}

}  // namespace zs3dev
