// fused_v2_gen.hip — the warp-specialised fused Split + Encode + HighwayHash-256 kernel
// (k_ehx_ws, fused_v2.hpp) for the server's default geometries that are NOT dyadic:
// getDefaultParityBlocks (cmd/format-erasure.go:870-881) gives RS(2+2), (3+2), (3+3),
// (4+3) for 4-7-drive sets and RS(5+4), (6+4), (7+4), (9+4), (10+4), (11+4) for 9-15-drive
// sets (RS(4+4), (8+4), (12+4) are dyadic and take fused_v2.hip's shapes).  Replaces
// Erasure.EncodeData (cmd/erasure-coding.go:77-91) + the k+m streamingBitrotWriter sums
// (cmd/bitrot-streaming.go:43-65) for those geometries.
//
// Before round 4 these ran the any-geometry encode (8-byte columns) + a separate
// stripe-mode hash launch: 23-26 % of 8 TB/s at 4096 x 1 MiB encode + sums
// (profiles/r04/geom_before.jsonl); RS(2+2) / (4+3) the first-generation fused kernel (44 / 51 %).
// Here the encode role multiplies every data row into every parity row (GEN: the general
// M x K matrix, encode_general) with the coefficient tables in LDS; the rest is the
// RS(12+4) unaligned-row recipe: buffer-addressed columns, non-temporal loads and stores,
// the hash waves touching the data lines two tiles ahead (PFD = 2), UA mode (S = ceil(B/k)
// is not a multiple of 16 for any k here but 2 and 4), bank-conflict-free LDS rows (TSP 1).
// Shapes: k <= 3: 8 stripes, 16-byte columns of 1 KiB tiles (8 encode waves beside 1-2
// pair-form hash waves); RS(4+3): 16 stripes, 16-byte columns of 512-byte tiles; K+M > 8:
// 8 stripes, 8-byte columns of 512-byte tiles (K rows of
// 16-byte columns do not fit the 168-VGPR budget beside the general encode's
// accumulators).
#include "fused_v2.hpp"

namespace zs3k {

// Round 4 shape sweep (diagnostics 340-344, profiles/r04/sweep_gen.jsonl, 4096 x 1 MiB):
// k <= 3 gains from 8 stripes of 1 KiB tiles (each chain hashes 32 packets between
// barriers; the rows are long: RS(3+3) S = 341 KiB): RS(3+2) 1.91 -> 1.75 ms, RS(3+3)
// 2.79 -> 2.23, RS(2+2) 2.01 -> 1.90 (geom_r9.jsonl); RS(5+4) / RS(6+4) gain 2 % from temporal data loads without the L2
// prefetch (2.09 -> 2.04, 1.93 -> 1.89); RS(10+4) keeps the first shape (1 KiB tiles:
// 1.70 -> 2.90 ms at 8-byte columns).  Later in round 4 RS(5+4) / RS(6+4) moved to the
// RS(12+4) product shape (4 stripes of 1 KiB tiles, quad-form hash waves issuing the L2
// prefetch, 16-byte columns on the 256-VGPR budget; diagnostics 345): 2.04-2.05 -> 1.95-1.97
// and 1.89-1.90 -> 1.88-1.89 ms (sweep_gen_1k.jsonl, one box, three runs); K >= 7 spills
// there (RS(10+4): 231 VGPRs).
template <int K, int M, int XM = 0>
static bool launch_gen_t(const EncArgs& a, hipStream_t s) {
    if constexpr (K <= 3)
        return launch_ws<K, M, WithXMap<shape::GenLong1K, XM>>(a, s);
    else if constexpr (K + M <= 8)  // RS(4+3): 1 KiB tiles measured 1.54 -> 1.64 ms (geom_r9.jsonl)
        return launch_ws<K, M, WithXMap<shape::Gen16x512, XM>>(a, s);
    else if constexpr (K <= 6)  // RS(5+4) / (6+4): diagnostics 345 (profiles/r04/sweep_gen_1k.jsonl)
        return launch_ws<K, M, WithXMap<shape::GenQuad1K, XM>>(a, s);
    else
        return launch_ws<K, M, WithXMap<shape::Gen8x512, XM>>(a, s);
}

#define ZS3_GEN_KM(X) X(2, 2) X(3, 2) X(3, 3) X(4, 3) X(5, 4) X(6, 4) X(7, 4) X(9, 4) X(10, 4) X(11, 4)

bool has_gen_encode(int k, int m) {
#define X(K, M) if (k == K && m == M) return true;
    ZS3_GEN_KM(X)
#undef X
    return false;
}

#if ZS3_DIAG
// diagnostics 419: every general-matrix shape with the region-interleaved workgroup order
bool launch_ehx_gen_xmap(const EncArgs& a, hipStream_t s) {
    if (!a.sums) return false;
#define X(K, M) \
    if (a.k == K && a.m == M) return launch_gen_t<K, M, 8>(a, s);
    ZS3_GEN_KM(X)
#undef X
    return false;
}
#endif

int launch_ehx_gen(const EncArgs& a, hipStream_t s) {
    if (!a.sums) return PATH_NONE;
#define X(K, M) \
    if (a.k == K && a.m == M) return launch_gen_t<K, M>(a, s) ? PATH_WS : PATH_NONE;
    ZS3_GEN_KM(X)
#undef X
    return PATH_NONE;
}

}  // namespace zs3k
