// ehx_mx.hpp — balanced fused Split + Encode + HighwayHash-256 kernel (round 6).
//
// Replaces the arithmetic of Erasure.EncodeData (cmd/erasure-coding.go:77-91) plus the
// k+m streamingBitrotWriter sums (cmd/bitrot-streaming.go:43-65), as k_ehx_ws does, for
// the dyadic shapes.
//
// Why a second form.  k_ehx_ws gives each wave ONE role: 2*G*R/64 pair-form hash waves
// beside G*T/1024 encode waves.  For RS(8+4) (R = 12, G = 16, T = 384) that is 6 + 6
// waves, and a workgroup's waves share SIMDs as {w, w+4, w+8}: two SIMDs carry 2 hash + 1
// encode wave, two carry 1 hash + 2 encode (6 is not a multiple of 4).  Per 384-byte step
// a hash wave issues ~384 VALU instructions and an encode wave ~542, so the "1H+2E" SIMDs
// issue 1 468 against 1 310, and per-wave stamps of the product (diagnostics 313,
// profiles/r06/stamps_enc.jsonl) show exactly those SIMDs pacing the step: their hash wave
// waits 3.7 % of its cycles at the barrier, every other wave 12-39 %.  No role placement
// fixes it (a wave's issue cost does not depend on how many of its lanes have work, and
// 3*G/8 hash waves are never a multiple of 4).
//
// Here every thread has BOTH roles: it is one lane of a pair-form HighwayHash chain (2*G*R
// threads = G*R chains) and it encodes one 16-byte column (G*T/16 threads), so T = 32*R
// (RS(8+4): 384).  Every wave then issues the same ~926 instructions per step and every
// SIMD the same ~1 389 (5.4 % under the pacing SIMD of k_ehx_ws) — provided the CU's
// waves spread evenly over its SIMDs: G = 32 (12 waves, one workgroup per CU) or several
// smaller workgroups per CU (G = 16: 6 waves, two per CU; G = 8: 3 waves, four per CU),
// whose placement the stamps (WT) record.
//
// One LDS tile per workgroup (G*R rows of T bytes at the conflict-free stride ws_ts), two
// barriers per step:
//   [B] wait for tile s's loads, encode it into registers (GF lookups: LDS tables)
//   [A] issue this thread's hash reads of tile s-1 (12 ds_read_b128, pair form)
//   [C] barrier: every read of tile s-1 done, the tile may be overwritten
//   [D] write tile s (data + parity rows) into LDS, [E] issue the loads of tile s+1,
//   [F] store tile s's parity, [G] HighwayHash tile s-1 from registers (under the LDS
//       writes' drain), [H] barrier: tile s visible.
// Loads of tile s+1 are issued before the parity stores of tile s, so the wait at step
// s+1 leaves those stores in flight (vm_wait<M>), as in k_ehx_ws.
#pragma once
#include "fused_v2.hpp"

namespace zs3k {

struct MixShape {
    static constexpr int G = 0;          // stripes per workgroup
    static constexpr int NTM = 3;        // non-temporal policy: bit 0 data loads, bit 1 parity stores
    static constexpr int TSP = 1;        // LDS row stride rule (ws_ts)
    static constexpr int XMAP = 8;       // workgroup -> stripe-group order (ws_group)
    static constexpr bool WT = false;    // diagnostics: per-wave barrier / load-wait stamps
    static constexpr int RD = 0;         // where the hash reads go: 0 after the encode, 1 before
    static constexpr int WPE = 3;        // waves per SIMD the register budget is sized for
};

template <int K, int M, class C>
constexpr int mx_nt() {
    return 2 * C::G * (K + M);
}

template <int K, int M, class C>
__global__ void __launch_bounds__((mx_nt<K, M, C>())) __attribute__((amdgpu_waves_per_eu(C::WPE)))
k_ehx_mx(EncArgs a) {
    constexpr int G = C::G, R = K + M, NTM = C::NTM;
    constexpr int T = 32 * R;            // bytes of each row per step
    constexpr int NT = mx_nt<K, M, C>();
    constexpr int CPS = T / 16;          // encode columns per stripe row
    constexpr int TS = ws_ts<T, false, C::TSP>();
    constexpr int NPK = T / 32;          // packets per row per step
    constexpr int NWd = 4;
    typedef typename VecOf<NWd>::type VT;
    static_assert(M == 2 || M == 4, "dyadic shapes");
    static_assert(NT % 64 == 0 && G * CPS == NT, "one hash lane and one encode column per thread");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_dyn[];
    uint8_t* tile = smem_dyn;
    __shared__ __attribute__((aligned(16))) uint32_t tabs[K * 8];

    const int tid = threadIdx.x;
    const int64_t blk0 = (int64_t)ws_group<C::XMAP>() * G;
    const int64_t S = a.S;
    for (int i = tid; i < K * 8; i += NT) tabs[i] = a.dtables[i];
    const int64_t nfull = S / T;
    const int tail = (int)(S - nfull * T);  // multiple of 16

    uint64_t rt0 = 0, ct0 = 0, wsum = 0, vwsum = 0;
    if (a.dbg) {
        rt0 = __builtin_amdgcn_s_memrealtime();
        ct0 = __builtin_amdgcn_s_memtime();
    }
    auto bar = [&]() {
        if constexpr (C::WT) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            lds_barrier2();
            wsum += __builtin_amdgcn_s_memtime() - t;
        } else {
            lds_barrier2();
        }
    };

    // ---- hash lane: lanes (2hh, 2hh+1) of chain `chain` = row chain % R of stripe chain / R
    const int chain = tid >> 1, hh = tid & 1;
    const int row_off = chain * TS;
    HHPair st = hh2_init(hh, a.key[0], a.key[1], a.key[2], a.key[3]);

    // ---- encode column: 16 bytes at o of every row of stripe g (dead stripes of the last
    // workgroup alias the last live block and store byte-identical parity)
    const int g = tid / CPS, o = (tid % CPS) * 16;
    const int64_t b = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
    const int col_off = g * R * TS + o;
    const __amdgpu_buffer_rsrc_t rs_d =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.data + blk0 * a.data_stride), 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_p =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.parity + blk0 * a.parity_stride), 0, 0x7FFFFFFF, 0x00020000);
    const uint32_t vo_d = (uint32_t)((b - blk0) * a.data_stride + o);
    const uint32_t vo_p = (uint32_t)((b - blk0) * a.parity_stride + o);

    VT x[K];
    auto load = [&](int64_t tn) {
        // tile tn of every data row (the tail tile only in the columns below `tail`;
        // anything else re-reads offset 0 and is discarded)
        const bool ok = tn < nfull || (tn == nfull && o < tail);
        const uint32_t vo = vo_d + (ok ? (uint32_t)(tn * T) : 0u);
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(j * S));
            if constexpr (NTM & 1)
                asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen nt"
                             : "=v"(x[j])
                             : "v"(vo), "s"(rs_d), "s"(so)
                             : "memory");
            else
                asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                             : "=v"(x[j])
                             : "v"(vo), "s"(rs_d), "s"(so)
                             : "memory");
        }
    };
    auto store_par = [&](const Col<NWd> (&par)[M], int64_t t0) {
#pragma unroll
        for (int r = 0; r < M; ++r) {
            const int so = (int)__builtin_amdgcn_readfirstlane((uint32_t)(r * S + t0));
            const VT v = {par[r].w[0], par[r].w[1], par[r].w[2], par[r].w[3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, rs_p, (int)vo_p, so, (NTM & 2) ? 2 : 0);
        }
    };
    uint4 w[NPK];
    auto read_tile = [&]() {
        const uint4* p = reinterpret_cast<const uint4*>(tile + row_off) + hh;
#pragma unroll
        for (int i = 0; i < NPK; ++i) w[i] = p[2 * i];
    };
    auto hash_words = [&]() {
#pragma unroll
        for (int i = 0; i < NPK; ++i)
            hh2_update(st, ((uint64_t)w[i].y << 32) | w[i].x, ((uint64_t)w[i].w << 32) | w[i].z);
    };
    // one step: encode tile ti (live: it is a full tile, or the tail tile and this column
    // is below `tail`), hash tile ti-1 (hash_prev), and with MORE issue the loads of tile
    // ti+1 (the last step issues none, so no load is in flight past the loop)
    auto step = [&](int64_t ti, bool hash_prev, bool full, auto more) {
        constexpr bool MORE = decltype(more)::value;
        Col<NWd> par[M];
        const bool live = full || o < tail;
        if (hash_prev && C::RD == 1) read_tile();
        if constexpr (C::WT) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            vm_wait<M, K>(x);
            vwsum += __builtin_amdgcn_s_memtime() - t;
        } else {
            vm_wait<M, K>(x);
        }
        Col<NWd> xs[K];
#pragma unroll
        for (int j = 0; j < K; ++j) xs[j] = to_col<NWd>(x[j]);
        encode_dyadic<NWd, K, M, true, false, false>(xs, par, tabs);
        if (hash_prev && C::RD == 0) read_tile();
        bar();  // [C] tile ti-1 read by every thread
        if (live) {
#pragma unroll
            for (int j = 0; j < K; ++j) st_col<NWd>(tile + col_off + j * TS, xs[j]);
#pragma unroll
            for (int r = 0; r < M; ++r) st_col<NWd>(tile + col_off + (K + r) * TS, par[r]);
        }
        if constexpr (MORE) load(ti + 1);
        if (live) store_par(par, ti * T);
        if (hash_prev) hash_words();
        bar();  // [H] tile ti written
    };
    using More = std::true_type;
    using Last = std::false_type;

    // tiles 0 .. L (the tail tile is tile nfull)
    const int64_t L = tail ? nfull : nfull - 1;
    load(0);
    vm_wait<0, K>(x);
    bar();  // tables visible
    if (L >= 1) {
        step(0, false, true, More{});
        for (int64_t s = 1; s < L; ++s) step(s, true, true, More{});
        step(L, true, L < nfull, Last{});
    } else if (L == 0) {
        step(0, false, L < nfull, Last{});
    }
    if (tail) {
        // the tail tile itself
        const uint8_t* row = tile + row_off;
        hh2_packets(st, row, tail >> 5, hh);
        if (tail & 31) hh2_remainder(st, row + (tail & ~31), (uint32_t)(tail & 31), hh);
    } else if (L >= 0) {
        read_tile();
        hash_words();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint64_t d0, d1;
    hh2_finalize256(st, d0, d1);
    if (blk0 + chain / R < a.n_blocks) {
        const int64_t bb = blk0 + chain / R;
        uint64_t* out = reinterpret_cast<uint64_t*>(a.sums + (bb * R + chain % R) * 32 + 16 * hh);
        out[0] = d0;
        out[1] = d1;
    }
    if (a.dbg && (tid & 63) == 0) {
        const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
        const uint64_t ct1 = __builtin_amdgcn_s_memtime();
        uint64_t* d = a.dbg + ((int64_t)blockIdx.x * (NT / 64) + (tid >> 6)) * 5;
        d[0] = rt0;
        d[1] = rt1;
        d[2] = ct1 - ct0;
        d[3] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
        d[4] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) | ((wsum & 0xFFFFFFF) << 8) | (vwsum << 36);
    }
}

template <int K, int M, class C>
static bool launch_mx(const EncArgs& a, hipStream_t s) {
    constexpr int R = K + M, T = 32 * R, G = C::G;
    constexpr int NT = mx_nt<K, M, C>();
    constexpr size_t dyn = (size_t)G * R * ws_ts<T, false, C::TSP>();
    if constexpr (dyn + K * 32 > 163840 || NT > 1024) {
        return false;
    } else {
        if (a.k != K || a.m != M || a.dyb != M || !a.sums) return false;
        if ((a.S % 16) != 0 || a.n != (int64_t)K * a.S) return false;
        if ((G - 1) * a.data_stride + K * a.S > 0x7FFFFFFF || (G - 1) * a.parity_stride + M * a.S > 0x7FFFFFFF ||
            a.data_stride < 0 || a.parity_stride < 0)
            return false;
        auto kern = k_ehx_mx<K, M, C>;
        if (ensure_dyn_lds((const void*)kern, dyn) != hipSuccess) return false;
        const int64_t grid = (a.n_blocks + G - 1) / G;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), dyn, s, a);
        return true;
    }
}

namespace shape {
template <int G_>
struct Mix : MixShape {
    static constexpr int G = G_;
};
template <class S>
struct MixWT : S {
    static constexpr bool WT = true;
};
template <class S>
struct MixRd1 : S {
    static constexpr int RD = 1;
};

}  // namespace shape

}  // namespace zs3k
