// vr_quad.hpp — RS(16+4) GET rebuild 4 / heal 4 with the rebuild split over survivor
// quads (round 5).  Same contract as k_vr_ws (fused_v2.hpp): verify the k survivors of
// every stripe against their stored HighwayHash-256 sums (errFileCorrupt per shard,
// cmd/bitrot-streaming.go:171-186), rebuild the e = 4 lost rows
// (Erasure.DecodeDataBlocks / DecodeDataAndParityBlocks, cmd/erasure-coding.go:96-119)
// and, for heal, hash them (Erasure.Heal, cmd/erasure-decode.go:287-332).
//
// Why a second kernel: k_vr_ws gives every rebuild thread a column of all 16 survivors and
// all 4 rebuilt rows, i.e. 64 GF(2^8) coefficient tables per tile, which do not fit a
// wave's registers (5 dwords each) and are re-read with scalar loads every tile; with
// every product on one batch of tables the same instance runs 16-28 % faster
// (diagnostics 431, profiles/r05/abl_get.jsonl).  Here the rebuild waves are split into
// four quads: quad q owns survivors 4q .. 4q+3 and multiplies them into all four rebuilt
// rows, so a wave needs only 16 tables, held for the whole launch (the three low dwords
// of each in SGPRs, the two high dwords in VGPRs: a v_perm reads one SGPR).  Each quad
// writes its four partial rows to LDS; one step later quad q XORs the four partials of
// rebuilt row q, stores it and (heal) places it in LDS for the hash waves, which
// therefore hash the rebuilt rows one tile behind the survivors.
//
// Per step s (one barrier):
//   rebuild quads: survivors of tile s (loaded one step ahead) -> LDS SV[s&1];
//                  partials of tile s -> LDS PB[s&1]; loads of tile s+1;
//                  row q of tile s-1 = XOR of PB[(s-1)&1][0..3][q] -> global, LDS RB[(s-1)&1]
//   hash waves:    survivor chains hash tile s-1 from SV, rebuilt chains tile s-2 from RB
// Requires S % T == 0, S / T >= 2, no block-id list, buffer-addressable stripe groups
// (launch_vr_quad); other batches take k_vr_ws.  Measured against the k_vr_ws instances
// (K16Rebuild34 / K16Heal with SPL; diagnostics 440), with the rebuild quads at issue
// priority 1 and the partials read at the start of each step (profiles/r05/
// ab_quad3.jsonl): RS(16+4) 2 048 x 1 MiB rebuild 4 0.595 -> 0.551 ms, heal 4 0.668 ->
// 0.616; 8 192 x 1 MiB 2.34 -> 2.27 / 2.61 -> 2.47 ms.
#pragma once
#include "fused_v2.hpp"

namespace zs3k {

namespace shape {
// 8 stripes of 256-byte tiles, 16-byte columns: 4 quads x 2 waves of rebuild, 4-5
// pair-form hash waves, conflict-free LDS rows.  (4 stripes of 512-byte tiles, half the
// steps per byte: 4-12 % slower, profiles/r05/ab_quad.jsonl; 4 stripes of 256-byte tiles,
// two workgroups per CU: 5-19 % slower, ab_quad5.jsonl.)
struct Quad16 {
    static constexpr int G = 8, T = 256, CW = 16, TSP = 1, XMAP = 0, PRIO = 1;
    static constexpr bool RR = true;  // partials read at the start of the step
    static constexpr bool UL = false;  // survivors and rebuilt rows in one LDS row array
    // heal: each stripe's survivor rows 128 bytes further apart (below k_vr_quad)
    static constexpr bool SWZ = true;
};
// Diagnostics: heal without the survivor-stripe pad (the round-5 layout: 8.4 M bank
// conflicts per 2 048-stripe launch, profiles/r05/pmc_compute.json).
struct Quad16NoSwz : Quad16 {
    static constexpr bool SWZ = false;
};
// Diagnostics: survivors and rebuilt rows in one LDS row array (the heal hash waves' rows
// at consecutive strides: SQ_LDS_BANK_CONFLICT 8.4 M -> 0 per launch, but heal 4 3-4 %
// slower, profiles/r05/ab_quad4.jsonl).
struct Quad16OneArray : Quad16 {
    static constexpr bool UL = true;
};
// Diagnostics: the partials read at the end of the step, just before they are combined.
struct Quad16LateRead : Quad16 {
    static constexpr bool RR = false;
};
// Diagnostics: the rebuild quads without issue priority.
struct Quad16Prio0 : Quad16 {
    static constexpr int PRIO = 0;
};
// The heal instance with the XCD-region workgroup order over 8 regions (round 6: heal 4
// 1-4 % faster at 2 048 / 8 192 x 1 MiB, rebuild 4 within noise either way, diagnostics
// 446 = without; profiles/r06/ab_quad_x8.jsonl).
struct Quad16Heal : Quad16 {
    static constexpr int XMAP = 8;
};
// Diagnostics (round 6): issue priority 2 for the rebuild quads.
struct Quad16P2 : Quad16 {
    static constexpr int PRIO = 2;
};
}  // namespace shape

template <bool HOUT, class C>
__global__ void __launch_bounds__((vr_nh<C::G, 16 + (HOUT ? 4 : 0), false>() + 4 * C::G * (C::T / C::CW)))
__attribute__((amdgpu_waves_per_eu(4))) k_vr_quad(VrArgs a) {
    constexpr int K = 16, EX = 4, NQ = 4, SQ = K / NQ;
    constexpr int G = C::G, T = C::T, CW = C::CW, NWd = CW / 4;
    constexpr int RH = K + (HOUT ? EX : 0);
    constexpr int NH = vr_nh<G, RH, false>();
    constexpr int CPS = T / CW;  // columns per stripe
    constexpr int NQT = G * CPS;  // threads per quad
    constexpr int NT = NH + NQ * NQT;
    constexpr int TS = ws_ts<T, false, C::TSP>();
    constexpr int NPK = T / 32;
    // UL: survivors and rebuilt rows of a stripe in one row array ([2][G*RH][TS]: the
    // hash waves' rows at consecutive strides, conflict-free); else two arrays
    constexpr bool UL = C::UL;
    // SWZ (heal, two arrays; round 6): a wave's 32 hash chains run across stripes, so a
    // ds_read_b128 lane group reads survivor rows of one stripe next to rebuilt rows of the
    // previous one.  Rows at TS = T + 32 apart are conflict-free only while the group's 8
    // rows start at 8 distinct 32-byte slots mod 256, which the one-array layout gives
    // (row j of stripe g at (20 g + j) * 32 mod 256) and two arrays did not (survivor rows
    // at (16 g + j) * 32 = j * 32: odd stripes collided with the rebuilt rows of the even
    // ones: SQ_LDS_BANK_CONFLICT 12.9 % of SQ_LDS_IDX_ACTIVE).  128 bytes more
    // between survivor stripes put row j of stripe g at g * 128 + j * 32 mod 256, the
    // one-array slots, while the rebuilt rows keep their own array.
    constexpr int SSTR = UL ? RH * TS : K * TS + (HOUT && C::SWZ ? 128 : 0);  // survivor stripe stride
    constexpr int SVB = G * SSTR, RBB = UL ? SVB : G * EX * TS, PBB = G * T;
    constexpr int RBR = UL ? RH : EX, RB0 = UL ? K : 0;  // rebuilt rows per stripe, first rebuilt
    static_assert(NH % 64 == 0 && NQT % 64 == 0 && NWd == 4 && T % 32 == 0, "whole waves, 16-byte columns");
    typedef typename VecOf<NWd>::type VT;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_dyn[];
    uint8_t* const SV = smem_dyn;                            // [2][G][SSTR] survivors
    uint8_t* const RB = UL ? SV : SV + 2 * SVB;              // [2][G*RBR][TS] rebuilt rows (heal)
    uint8_t* const PB = SV + 2 * SVB + (HOUT && !UL ? 2 * RBB : 0);  // [2][NQ][EX][G*T] partials
    __shared__ int32_t srows[K + EX];

    const int tid = threadIdx.x;
    const int64_t blk0 = (int64_t)ws_group<C::XMAP>() * G;
    const int64_t S = a.S;
    const int R = a.k + a.m;
    const int64_t nfull = S / T;
    for (int i = tid; i < K + EX; i += NT) srows[i] = a.rows[i];
    lds_barrier2();

    if (__builtin_amdgcn_readfirstlane(tid) < NH) {
        // ---- hash role, pair form: row cj of stripe g (pad pairs hash a real row again)
        const int chain0 = tid >> 1, hh = tid & 1;
        const bool pad = chain0 >= G * RH;
        const int chain = pad ? chain0 - G * RH : chain0;
        const int g = chain / RH, cj = chain % RH;
        const bool reb = cj >= K;
        const uint8_t* const base = reb ? RB + (g * RBR + RB0 + (cj - K)) * TS : SV + g * SSTR + cj * TS;
        const int bufb = reb ? RBB : SVB;
        const int lag = reb ? 2 : 1;
        HHPair st = hh2_init(hh, a.key[0], a.key[1], a.key[2], a.key[3]);
        for (int64_t s = 0; s <= nfull + 1; ++s) {
            const int64_t t = s - lag;
            if (t >= 0 && t < nfull) {
                const uint4* p = reinterpret_cast<const uint4*>(base + (t & 1) * bufb) + hh;
                uint4 w[NPK];
#pragma unroll
                for (int i = 0; i < NPK; ++i) w[i] = p[2 * i];
#pragma unroll
                for (int i = 0; i < NPK; ++i)
                    hh2_update(st, ((uint64_t)w[i].y << 32) | w[i].x, ((uint64_t)w[i].w << 32) | w[i].z);
            }
            lds_barrier2();
        }
        uint64_t d0, d1;
        hh2_finalize256(st, d0, d1);
        const bool live = !pad && blk0 + g < a.n_blocks;
        const int64_t b = blk0 + g;
        const int srow = srows[cj];
        if (cj < K) {
            bool mis = false;
            if (live) {
                uint64_t e0, e1;
                __builtin_memcpy(&e0, a.expect + (b * R + srow) * 32 + 16 * hh, 8);
                __builtin_memcpy(&e1, a.expect + (b * R + srow) * 32 + 16 * hh + 8, 8);
                mis = e0 != d0 || e1 != d1;
            }
            const unsigned long long m = __ballot(mis);
            const bool bad = ((m >> (tid & 62)) & 3ull) != 0;
            if (live && hh == 0) a.bad[b * R + srow] = bad ? 1 : 0;
        } else if (HOUT && live && a.sums_out) {
            uint64_t* out = reinterpret_cast<uint64_t*>(a.sums_out + (b * R + srow) * 32 + 16 * hh);
            out[0] = d0;
            out[1] = d1;
        }
        return;
    }

    // ---- rebuild role: quad q (wave-uniform), column o of stripe g; issue priority over
    // the hash waves as in k_vr_ws (GetShape PRIO)
    if constexpr (C::PRIO > 0) __builtin_amdgcn_s_setprio(C::PRIO);
    const int e = tid - NH;
    const int q = __builtin_amdgcn_readfirstlane(e / NQT);
    const int eq = e % NQT;
    const int g = eq / CPS, o = (eq % CPS) * CW;
    const int64_t bl = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.shards + blk0 * a.block_stride), 0, 0x7FFFFFFF, 0x00020000);
    const uint32_t vo = (uint32_t)((bl - blk0) * a.block_stride + o);
    uint32_t roff[SQ];
#pragma unroll
    for (int jj = 0; jj < SQ; ++jj) roff[jj] = (uint32_t)__builtin_amdgcn_readfirstlane(srows[SQ * q + jj]) * (uint32_t)S;
    const uint32_t ooff = (uint32_t)__builtin_amdgcn_readfirstlane(srows[K + q]) * (uint32_t)S;

    // the quad's 16 coefficient tables (rebuilt row r, survivor 4q + jj), held for the launch
    const ctab_ptr tg = const_tables(a.tables);
    CoefTab tq[EX][SQ];
    uint32_t hy[EX][SQ], hw[EX][SQ];
#pragma unroll
    for (int r = 0; r < EX; ++r)
#pragma unroll
        for (int jj = 0; jj < SQ; ++jj) {
            tq[r][jj] = load_coef_s(tg, r * K + SQ * q + jj);
            asm volatile("v_mov_b32 %0, %1" : "=v"(hy[r][jj]) : "s"(tq[r][jj].ab.y));
            asm volatile("v_mov_b32 %0, %1" : "=v"(hw[r][jj]) : "s"(tq[r][jj].ab.w));
        }

    VT x[SQ];
    auto load = [&](int64_t tile) {
#pragma unroll
        for (int jj = 0; jj < SQ; ++jj) {
            // (s_nop: the SGPR offset may come from a v_readfirstlane, 5 wait states before
            // a VMEM instruction reads it; the compiler does not pad inline asm)
            const uint32_t so = __builtin_amdgcn_readfirstlane(roff[jj] + (uint32_t)(tile * T));
            asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, %3 offen nt"
                         : "=v"(x[jj])
                         : "v"(vo), "s"(rs), "s"(so)
                         : "memory");
        }
    };
    // tile s: survivors to LDS (hash waves), the quad's partials of the four rebuilt rows
    auto compute = [&](int64_t s) {
        uint8_t* const sv = SV + (s & 1) * SVB + g * SSTR + SQ * q * TS + o;
        Col<NWd> xs[SQ];
#pragma unroll
        for (int jj = 0; jj < SQ; ++jj) {
            xs[jj] = to_col<NWd>(x[jj]);
            st_col<NWd>(sv + jj * TS, xs[jj]);
        }
        GfAcc acc[EX][NWd];
#pragma unroll
        for (int r = 0; r < EX; ++r)
#pragma unroll
            for (int w = 0; w < NWd; ++w) acc_init(acc[r][w]);
#pragma unroll
        for (int jj = 0; jj < SQ; ++jj) {
            Nib sp[NWd];
#pragma unroll
            for (int w = 0; w < NWd; ++w) sp[w] = split_nibbles(xs[jj].w[w]);
#pragma unroll
            for (int r = 0; r < EX; ++r)
#pragma unroll
                for (int w = 0; w < NWd; ++w)
                    acc_add(acc[r][w], gf_lookup_sh(sp[w], tq[r][jj], hy[r][jj], hw[r][jj]));
        }
        uint8_t* const pb = PB + ((s & 1) * NQ + q) * EX * PBB + g * T + o;
#pragma unroll
        for (int r = 0; r < EX; ++r) {
            Col<NWd> y;
#pragma unroll
            for (int w = 0; w < NWd; ++w) y.w[w] = acc_done(acc[r][w]);
            st_col<NWd>(pb + r * PBB, y);
        }
    };
    // rebuilt row q of tile t: the XOR of the four quads' partials -> global (and LDS for
    // the hash waves when healing).  The partials are read at the start of the step
    // (reduce_read) and combined at its end (reduce_store), so the LDS latency hides
    // behind the step's products instead of sitting in front of its barrier.
    Col<NWd> part[NQ];
    auto reduce_read = [&](int64_t t) {
        const uint8_t* const pr = PB + (t & 1) * NQ * EX * PBB + q * PBB + g * T + o;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) part[qq] = ld_col<NWd>(pr + qq * EX * PBB);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto reduce_store = [&](int64_t t) {
        Col<NWd> y = part[0];
#pragma unroll
        for (int qq = 1; qq < NQ; ++qq)
#pragma unroll
            for (int w = 0; w < NWd; ++w) y.w[w] ^= part[qq].w[w];
        const int so = (int)__builtin_amdgcn_readfirstlane(ooff + (uint32_t)(t * T));
        const VT v = {y.w[0], y.w[1], y.w[2], y.w[3]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)vo, so, 2);
        if constexpr (HOUT) st_col<NWd>(RB + (t & 1) * RBB + (g * RBR + RB0 + q) * TS + o, y);
    };
    // The next tile's loads are issued unconditionally (the last step reloads its own tile)
    // and before the step's row store, so every wait below retires exactly the loads: the
    // asm-load destinations stay allocated from issue to wait (scripts/check_async_loads.py).
    load(0);
    vm_wait<0>(x);  // step 0
    compute(0);
    load(1);
    lds_barrier2();
    if constexpr (C::RR) reduce_read(0);  // step 1
    vm_wait<0>(x);  // (no store issued yet)
    compute(1);
    load(nfull > 2 ? 2 : 1);
    if constexpr (!C::RR) reduce_read(0);
    reduce_store(0);
    lds_barrier2();
    for (int64_t s = 2; s < nfull; ++s) {
        if constexpr (C::RR) reduce_read(s - 1);
        vm_wait<1>(x);  // outstanding: this tile's loads, then step s-1's row store
        compute(s);
        load(s + 1 < nfull ? s + 1 : s);
        if constexpr (!C::RR) reduce_read(s - 1);
        reduce_store(s - 1);
        lds_barrier2();
    }
    vm_wait<0>(x);  // the last step's reload: its registers are reused from here on
    reduce_read(nfull - 1);  // step nfull
    reduce_store(nfull - 1);
    lds_barrier2();
    lds_barrier2();  // step nfull + 1: the hash waves' last rebuilt tile
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The launch: RS(16+4) with e = 4, S a multiple of T with at least two tiles, no block-id
// list, and a stripe group addressable by one buffer resource; false otherwise.
template <bool HOUT, class C = shape::Quad16>
static bool launch_vr_quad_t(const VrArgs& a, hipStream_t s) {
    constexpr int G = C::G, T = C::T, CW = C::CW;
    constexpr int RH = 16 + (HOUT ? 4 : 0);
    constexpr int NT = vr_nh<G, RH, false>() + 4 * G * (T / CW);
    constexpr int TS = ws_ts<T, false, C::TSP>();
    // either layout, plus the heal survivor stripes' pad (SWZ)
    constexpr size_t dyn = (size_t)2 * G * RH * TS + (HOUT && C::SWZ && !C::UL ? (size_t)2 * G * 128 : 0) +
                           (size_t)2 * 4 * 4 * G * T;
    static_assert(dyn + 4 * 20 <= 163840 && NT <= 1024, "one workgroup's LDS and threads");
    if (a.k != 16 || a.e != 4 || a.ids || HOUT != (a.sums_out != nullptr)) return false;
    if (a.S % T != 0 || a.S / T < 2 || a.block_stride <= 0) return false;
    if ((int64_t)(a.k + a.m) * a.S >= ((int64_t)1 << 31) || (int64_t)G * a.block_stride >= ((int64_t)1 << 31))
        return false;
    auto kern = k_vr_quad<HOUT, C>;
    if (ensure_dyn_lds((const void*)kern, dyn) != hipSuccess) return false;
    const int64_t grid = (a.n_blocks + G - 1) / G;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), dyn, s, a);
    return true;
}

template <class C = shape::Quad16>
static bool launch_vr_quad(const VrArgs& a, hipStream_t s) {
    return a.sums_out ? launch_vr_quad_t<true, C>(a, s) : launch_vr_quad_t<false, C>(a, s);
}

// The product instances: rebuild 4 on Quad16, heal 4 on Quad16Heal.
static bool launch_vr_quad_product(const VrArgs& a, hipStream_t s) {
    return a.sums_out ? launch_vr_quad_t<true, shape::Quad16Heal>(a, s) : launch_vr_quad_t<false, shape::Quad16>(a, s);
}

}  // namespace zs3k
