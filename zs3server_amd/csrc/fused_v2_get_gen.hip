// fused_v2_get_gen.hip — GET / heal (rebuild e = 1..4 rows, optionally hashing the
// rebuilt rows) on the warp-specialised k_vr_ws for the server-default geometries whose
// data-shard count is not 4, 8, 12 or 16 (RS(2+2), (3+2), (3+3), (5+4), (6+4), (7+4),
// (9+4), (10+4), (11+4); cmd/erasure-sets.go's default parity for 4-15 drive sets).
// Before round 4 these ran as a stripe-mode verify hash launch + the reconstruct kernel
// + a heal hash launch (13-34 % of HBM on 4096 x 1 MiB, profiles/r04/geom_gen_ws.jsonl).
// Replaces the same reference arithmetic as fused_v2_get.hip: parallelReader +
// streamingBitrotReader.ReadAt (cmd/erasure-decode.go:165-179,
// cmd/bitrot-streaming.go:171-186), Erasure.DecodeDataBlocks
// (cmd/erasure-coding.go:96-109) and Erasure.Heal (cmd/erasure-decode.go:287-332).
//
// Shapes (one workgroup per CU): the hashed rows are few and long (RS(3+2): 3-5 rows of
// 341 KiB per stripe), so the hash chains per CU, not the bytes, bound the hash role
// for small k —
//   k = 2, 3: 8 stripes, quad-form hash waves (one HH lane per thread), 16-byte rebuild
//             columns of 1 KiB tiles, 2 of prefetch;
//   k = 5-7:  16 stripes, pair-form hash waves, 8-byte rebuild columns of 256-byte tiles;
//   k = 9-11: the RS(12+4) shape (fused_v2_get.hip): 8 stripes, 8-byte columns of
//             512-byte tiles (16 stripes at k = 10, 11 spill at the 128-VGPR budget of
//             a 1024-thread workgroup).
// Coefficient tables are scalar loads in double-buffered batches of 4 (a batch may
// straddle two rebuilt rows).  1 MiB blocks give unaligned rows for every k here but 2
// (S = ceil(2^20 / k)): UA mode, temporal survivor loads (launch_vr_ws_t).
#include "fused_v2.hpp"

namespace zs3k {

template <int K, int EX, bool HOUT>
static bool launch_gget_e(const VrArgs& a, hipStream_t s) {
    constexpr bool UA = K != 2;
    // k <= 3 (round 4, diagnostics 350): 8 stripes of 1 KiB tiles, 2 of prefetch:
    // 4096 x 1 MiB RS(2+2) rebuild / heal 2 2.30 / 2.38 -> 1.96 / 1.97 ms, RS(3+2)
    // 1.75 / 1.80 -> 1.53 / 1.51, RS(3+3) 1.83 / 1.87 -> 1.65 / 1.65 (16 stripes of
    // 256-byte tiles before; profiles/r04/get_ab_gen.jsonl)
    if constexpr (K <= 3)
        return launch_vr_ws_t<K, EX, HOUT, shape::GenGetQuad1K<UA>>(a, s);
    else if constexpr (K <= 7)
        return launch_vr_ws_t<K, EX, HOUT, shape::GenGet16x256<UA>>(a, s);
    else
        return launch_vr_ws_t<K, EX, HOUT, shape::Wide512<UA>>(a, s);
}

template <int K, int MAXE>
static bool launch_gget_k(const VrArgs& a, hipStream_t s) {
    const bool heal = a.sums_out != nullptr;
    switch (a.e) {
        case 1: return heal ? launch_gget_e<K, 1, true>(a, s) : launch_gget_e<K, 1, false>(a, s);
        case 2: return heal ? launch_gget_e<K, 2, true>(a, s) : launch_gget_e<K, 2, false>(a, s);
        case 3:
            if constexpr (MAXE >= 3) return heal ? launch_gget_e<K, 3, true>(a, s) : launch_gget_e<K, 3, false>(a, s);
            return false;
        case 4:
            if constexpr (MAXE >= 4) return heal ? launch_gget_e<K, 4, true>(a, s) : launch_gget_e<K, 4, false>(a, s);
            return false;
        default: return false;
    }
}

// true = launched on a warp-specialised instance (PATH_WS); false = no instance for
// this (k, e) (the caller falls back to the generic launches).
bool launch_vr_ws_gen(const VrArgs& a, hipStream_t s) {
    if (a.e < 1 || a.e > a.m) return false;
    switch (a.k) {
        case 2: return launch_gget_k<2, 2>(a, s);
        case 3: return launch_gget_k<3, 3>(a, s);
        case 5: return launch_gget_k<5, 4>(a, s);
        case 6: return launch_gget_k<6, 4>(a, s);
        case 7: return launch_gget_k<7, 4>(a, s);
        case 9: return launch_gget_k<9, 4>(a, s);
        case 10: return launch_gget_k<10, 4>(a, s);
        case 11: return launch_gget_k<11, 4>(a, s);
        default: return false;
    }
}

}  // namespace zs3k
