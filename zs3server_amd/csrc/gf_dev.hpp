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

#include <type_traits>

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

// Two dwords split with 64-bit shifts (round 6): v_lshrrev_b64 issues in ~4.5 cycles
// where two v_lshrrev_b32 take ~5.5 (profiles/r06/opcost.txt); the high dword's bits that
// the shift moves into the low one land above every kept field.
// SMK (diagnostics): the two masks from SGPRs instead of 32-bit literals (4-byte instead of
// 8-byte VALU encodings).
template <bool SMK = false>
__device__ __forceinline__ void split_nibbles2(uint32_t xlo, uint32_t xhi, Nib& lo, Nib& hi) {
    const uint64_t x = ((uint64_t)xhi << 32) | xlo;
    uint64_t t3, t6;  // (the compiler lowers a 64-bit shift to 32-bit ones: stated here)
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(t3) : "v"(x));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(t6) : "v"(x));
    uint32_t m7 = 0x07070707u, m3 = 0x03030303u;
    if constexpr (SMK) {
        asm("s_mov_b32 %0, 0x7070707" : "=s"(m7));
        asm("s_mov_b32 %0, 0x3030303" : "=s"(m3));
    }
    lo.a = xlo & m7;
    hi.a = xhi & m7;
    lo.b = (uint32_t)t3 & m7;
    hi.b = (uint32_t)(t3 >> 32) & m7;
    lo.c = (uint32_t)t6 & m3;
    hi.c = (uint32_t)(t6 >> 32) & m3;
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

// Coefficient tables read with SCALAR loads: the plan / codec tables are uniform across
// the wave, so a constant-address-space pointer with compile-time offsets compiles to
// s_load and the tables live in SGPRs instead of being re-read from LDS (ds_read_b128 +
// ds_read_b32 per coefficient per column) by every lane.  gfx950 VOP3 instructions read
// at most one SGPR (constant bus), so each v_perm takes the low table dword as its SGPR
// operand and the high dword from a VGPR (one v_mov, shared by the column's dwords).
typedef const __attribute__((address_space(4))) uint32_t* ctab_ptr;

__device__ __forceinline__ ctab_ptr const_tables(const uint32_t* p) { return (ctab_ptr)p; }

__device__ __forceinline__ CoefTab load_coef_s(ctab_ptr t, int idx) {
    CoefTab c;
    c.ab.x = t[8 * idx + 0];
    c.ab.y = t[8 * idx + 1];
    c.ab.z = t[8 * idx + 2];
    c.ab.w = t[8 * idx + 3];
    c.c = t[8 * idx + 4];
    return c;
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

// gf_lookup for SGPR tables: the 2-bit chunk selects bytes 0-3 only (src1), so src0 can
// be any VGPR (the selector itself): one SGPR operand per v_perm.
__device__ __forceinline__ Prod3 gf_lookup_s(const Nib& n, const CoefTab& t) {
    Prod3 p;
    p.a = __builtin_amdgcn_perm(t.ab.y, t.ab.x, n.a);
    p.b = __builtin_amdgcn_perm(t.ab.w, t.ab.z, n.b);
    p.c = __builtin_amdgcn_perm(n.c, t.c, n.c);
    return p;
}

// gf_lookup with the low table dwords in SGPRs and the high ones in VGPRs (hx = Ta.hi,
// hz = Tb.hi): no v_mov per coefficient to satisfy the one-SGPR operand limit.
__device__ __forceinline__ Prod3 gf_lookup_sh(const Nib& n, const CoefTab& t, uint32_t hx, uint32_t hz) {
    Prod3 p;
    p.a = __builtin_amdgcn_perm(hx, t.ab.x, n.a);
    p.b = __builtin_amdgcn_perm(hz, t.ab.z, n.b);
    p.c = __builtin_amdgcn_perm(n.c, t.c, n.c);
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

// XOR of N terms with ceil((N-1)/2) v_bitop3 (the last one a plain XOR if N is even).
template <int N>
__device__ __forceinline__ uint32_t fold_terms(const uint32_t (&t)[N]) {
    uint32_t acc = t[0];
    int i = 1;
#pragma unroll
    for (; i + 1 < N; i += 2) acc = xor3(acc, t[i], t[i + 1]);
    if (i < N) acc ^= t[i];
    return acc;
}

// An SGPR zero the compiler cannot see through: indexing the LDS coefficient
// tables with it keeps their loads where they are used instead of hoisting every
// table into VGPRs (which would cap occupancy).
__device__ __forceinline__ int opaque_zero() {
    int z = 0;
    asm volatile("" : "+s"(z));
    return z;
}

// Dyadic encode.  The parity block is K/M blocks D_q[r ^ t] (see zs3gpu.hip), i.e.
// y = sum_q A_q * x_q in the group algebra GF(256)[Z2^2] (M = 4) or GF(256)[Z2]
// (M = 2).  In characteristic 2 that algebra is the local ring F[s,t]/(s^2,t^2)
// with s = 1+g1, t = 1+g2; in the basis {1, s, t, st} a product is
//   Y0 = A0 X0,  Y1 = A0 X1 + A1 X0,  Y2 = A0 X2 + A2 X0,
//   Y3 = A0 X3 + A1 X2 + A2 X1 + A3 X0                       (9 multiplies)
// with X = (x0+x1+x2+x3, x1+x3, x2+x3, x3) and, per block generator (a,b,c,d),
// A = (a+b+c+d, b+d, c+d, d).  Only the 4 transformed inputs are nibble-split (the
// Karatsuba form needed 9 split combinations) and each block has 4 coefficient
// tables, not 9.  The Y accumulate over blocks and convert back once:
//   y0 = Y0+Y1+Y2+Y3, y1 = Y1+Y3, y2 = Y2+Y3, y3 = Y3.
// M = 2: X = (x0+x1, x1), A = (a+b, b), Y0 = A0 X0, Y1 = A0 X1 + A1 X0,
// y0 = Y0+Y1, y1 = Y1.
// SB: a scheduling barrier per block keeps each block's table reads local (fewer
// VGPRs); without it the scheduler may interleave the encode with other work.
// PRS: lower the wave's issue priority by one after each block (progress-equalising
// priority, fused_v2.hip PM = 4; the caller sets the starting priority).
// ST: tables by scalar loads (ctabs, SGPR operands) instead of LDS (dtabs).
// XF: getx(j) returns data column j; called for a block's M columns at the start of the
// block (a register array, or reads from LDS placed per block so that only one block's
// columns are live).
// H0: called once, after the first block's coefficient-table reads are issued and before
// its arithmetic (scheduling barriers on both sides): LDS writes placed there do not sit
// in front of the table reads in the in-order LDS counter.
struct NoHook {
    __device__ void operator()() const {}
};
// PRE: the K coefficient tables were read once into registers (pre[0..K-1]) before the
// tile loop: no LDS reads (and no LDS-counter waits) inside the encode.
template <int NWd, int K, int M, bool SB = true, bool PRS = false, bool ST = false, bool PRE = false,
          bool S64 = false, bool SMK = false, typename XF, typename H0 = NoHook>
__device__ __forceinline__ void encode_dyadic_f(XF&& getx, Col<NWd> (&out)[M], const uint32_t* dtabs,
                                                ctab_ptr ctabs = nullptr, H0&& hook0 = NoHook{},
                                                const CoefTab* pre = nullptr) {
    static_assert(M == 2 || M == 4, "dyadic block");
    uint32_t Y[M][NWd];
#pragma unroll
    for (int q = 0; q < K / M; ++q) {
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
        Col<NWd> xb[M];
#pragma unroll
        for (int i = 0; i < M; ++i) xb[i] = getx(q * M + i);
        if constexpr (PRS) {
            if (q == 1) __builtin_amdgcn_s_setprio(2);
            if (q == 2) __builtin_amdgcn_s_setprio(1);
            if (q > 0) __builtin_amdgcn_sched_barrier(0);
        }
        CoefTab t[M];
        if constexpr (PRE) {
#pragma unroll
            for (int i = 0; i < M; ++i) t[i] = pre[q * M + i];
        } else if constexpr (ST) {
#pragma unroll
            for (int i = 0; i < M; ++i) t[i] = load_coef_s(ctabs, q * M + i);
        } else {
            const uint32_t* tq = dtabs + opaque_zero() + q * M * 8;
#pragma unroll
            for (int i = 0; i < M; ++i) t[i] = load_coef(tq, i);
        }
        if constexpr (!std::is_same<std::decay_t<H0>, NoHook>::value) {
            if (q == 0) {
                __builtin_amdgcn_sched_barrier(0);
                hook0();
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        auto gf_lookup = [](const Nib& n, const CoefTab& c) { return ST ? gf_lookup_s(n, c) : zs3dev::gf_lookup(n, c); };
        // S64: the four transformed inputs of dwords w and w+1 split together (split_nibbles2)
        // when w is even; dword w+1 takes the split that w left in np[]
        constexpr bool P64 = S64 && M == 4 && NWd % 2 == 0;
        Nib np[4];
#pragma unroll
        for (int w = 0; w < NWd; ++w) {
            if constexpr (M == 4) {
                Nib n0, n1, n2, n3;
                if constexpr (P64) {
                    if (w % 2 == 0) {
                        uint32_t Xs[2][4];
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const uint32_t x3 = xb[3].w[w + h];
                            Xs[h][1] = xb[1].w[w + h] ^ x3;
                            Xs[h][2] = xb[2].w[w + h] ^ x3;
                            Xs[h][0] = xor3(xb[0].w[w + h], Xs[h][1], xb[2].w[w + h]);
                            Xs[h][3] = x3;
                        }
                        Nib nl[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) split_nibbles2<SMK>(Xs[0][i], Xs[1][i], nl[i], np[i]);
                        n0 = nl[0];
                        n1 = nl[1];
                        n2 = nl[2];
                        n3 = nl[3];
                    } else {
                        n0 = np[0];
                        n1 = np[1];
                        n2 = np[2];
                        n3 = np[3];
                    }
                } else {
                    const uint32_t x3 = xb[3].w[w];
                    const uint32_t X1 = xb[1].w[w] ^ x3, X2 = xb[2].w[w] ^ x3;
                    const uint32_t X0 = xor3(xb[0].w[w], X1, xb[2].w[w]);
                    n0 = split_nibbles(X0);
                    n1 = split_nibbles(X1);
                    n2 = split_nibbles(X2);
                    n3 = split_nibbles(x3);
                }
                const Prod3 P00 = gf_lookup(n0, t[0]), P01 = gf_lookup(n1, t[0]);
                const Prod3 P02 = gf_lookup(n2, t[0]), P03 = gf_lookup(n3, t[0]);
                const Prod3 P10 = gf_lookup(n0, t[1]), P12 = gf_lookup(n2, t[1]);
                const Prod3 P20 = gf_lookup(n0, t[2]), P21 = gf_lookup(n1, t[2]);
                const Prod3 P30 = gf_lookup(n0, t[3]);
                if (q == 0) {
                    Y[0][w] = fold_terms<3>({P00.a, P00.b, P00.c});
                    Y[1][w] = fold_terms<6>({P01.a, P01.b, P01.c, P10.a, P10.b, P10.c});
                    Y[2][w] = fold_terms<6>({P02.a, P02.b, P02.c, P20.a, P20.b, P20.c});
                    Y[3][w] = fold_terms<12>({P03.a, P03.b, P03.c, P12.a, P12.b, P12.c,
                                              P21.a, P21.b, P21.c, P30.a, P30.b, P30.c});
                } else {
                    Y[0][w] = fold_terms<4>({Y[0][w], P00.a, P00.b, P00.c});
                    Y[1][w] = fold_terms<7>({Y[1][w], P01.a, P01.b, P01.c, P10.a, P10.b, P10.c});
                    Y[2][w] = fold_terms<7>({Y[2][w], P02.a, P02.b, P02.c, P20.a, P20.b, P20.c});
                    Y[3][w] = fold_terms<13>({Y[3][w], P03.a, P03.b, P03.c, P12.a, P12.b, P12.c,
                                              P21.a, P21.b, P21.c, P30.a, P30.b, P30.c});
                }
            } else {
                const uint32_t x1 = xb[1].w[w];
                const uint32_t X0 = xb[0].w[w] ^ x1;
                const Nib n0 = split_nibbles(X0), n1 = split_nibbles(x1);
                const Prod3 P00 = gf_lookup(n0, t[0]), P01 = gf_lookup(n1, t[0]), P10 = gf_lookup(n0, t[1]);
                if (q == 0) {
                    Y[0][w] = fold_terms<3>({P00.a, P00.b, P00.c});
                    Y[1][w] = fold_terms<6>({P01.a, P01.b, P01.c, P10.a, P10.b, P10.c});
                } else {
                    Y[0][w] = fold_terms<4>({Y[0][w], P00.a, P00.b, P00.c});
                    Y[1][w] = fold_terms<7>({Y[1][w], P01.a, P01.b, P01.c, P10.a, P10.b, P10.c});
                }
            }
        }
    }
#pragma unroll
    for (int w = 0; w < NWd; ++w) {
        if constexpr (M == 4) {
            out[0].w[w] = xor3(Y[0][w], Y[1][w], Y[2][w]) ^ Y[3][w];
            out[1].w[w] = Y[1][w] ^ Y[3][w];
            out[2].w[w] = Y[2][w] ^ Y[3][w];
            out[3].w[w] = Y[3][w];
        } else {
            out[0].w[w] = Y[0][w] ^ Y[1][w];
            out[1].w[w] = Y[1][w];
        }
    }
}

template <int NWd, int K, int M, bool SB = true, bool PRS = false, bool ST = false, bool S64 = false, bool SMK = false>
__device__ __forceinline__ void encode_dyadic(const Col<NWd> (&x)[K], Col<NWd> (&out)[M], const uint32_t* dtabs,
                                              ctab_ptr ctabs = nullptr) {
    encode_dyadic_f<NWd, K, M, SB, PRS, ST, false, S64, SMK>([&](int j) { return x[j]; }, out, dtabs, ctabs);
}

// General (non-dyadic) encode of one column: out[r] = sum_j M[r][j] * x[j] over GF(2^8),
// the coefficient tables of parity row r, data row j at tabs[(r*K + j)*8] (LDS, read with
// wave-uniform addresses: broadcast, no bank conflicts).  Each data dword is nibble-split
// once and multiplied into all M rows (3 v_perm per product, folded with XOR3); the
// server's non-power-of-two geometries (RS(6+4), RS(10+4), RS(3+3), ...) are not dyadic,
// so every parity row needs its K products.
// An SGPR zero that depends on `v`: table reads addressed with it cannot be issued before
// v is computed (an opaque base alone does not stop the compiler from clustering every
// table read of a long unrolled sequence at its start).
__device__ __forceinline__ int opaque_zero_after(uint32_t v) {
    int z = 0;
    asm volatile("" : "+s"(z) : "v"(v));
    return z;
}

template <int NWd, int K, int M>
__device__ __forceinline__ void encode_general(const Col<NWd> (&x)[K], Col<NWd> (&out)[M], const uint32_t* tabs) {
    GfAcc acc[M][NWd];
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
        for (int w = 0; w < NWd; ++w) acc_init(acc[r][w]);
    // the M tables of data row j+1 are read while row j's products run (issued right after
    // row j's nibble split, which their opaque base depends on): two rows of tables live,
    // where letting the compiler cluster all M*K reads spilled 338 VGPRs for RS(10+4)
    CoefTab tn[M];
    {
        const uint32_t* tb = tabs + opaque_zero();
#pragma unroll
        for (int r = 0; r < M; ++r) tn[r] = load_coef(tb, r * K);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        CoefTab t[M];
#pragma unroll
        for (int r = 0; r < M; ++r) t[r] = tn[r];
        Nib n[NWd];
#pragma unroll
        for (int w = 0; w < NWd; ++w) n[w] = split_nibbles(x[j].w[w]);
        if (j + 1 < K) {
            const uint32_t* tb = tabs + opaque_zero_after(n[0].a);
#pragma unroll
            for (int r = 0; r < M; ++r) tn[r] = load_coef(tb, r * K + j + 1);
        }
#pragma unroll
        for (int r = 0; r < M; ++r)
#pragma unroll
            for (int w = 0; w < NWd; ++w) acc_add(acc[r][w], gf_lookup(n[w], t[r]));
    }
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
        for (int w = 0; w < NWd; ++w) out[r].w[w] = acc_done(acc[r][w]);
}

// Scalar GF multiply with log/exp tables (generic byte path).
__device__ __forceinline__ uint8_t gf_mul_log(const uint8_t* lg, const uint8_t* ex, uint8_t a, uint8_t b) {
    return (a && b) ? ex[(int)lg[a] + (int)lg[b]] : (uint8_t)0;
}

}  // namespace zs3dev
