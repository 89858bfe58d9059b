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
// Shapes: K+M <= 8: 16 stripes, 16-byte columns of 512-byte tiles (8 encode waves beside
// 2-4 pair-form hash waves); K+M > 8: 8 stripes, 8-byte columns (K rows of 16-byte columns
// do not fit the 168-VGPR budget beside the general encode's accumulators).
#include "fused_v2.hpp"

namespace zs3k {

template <int K, int M>
static bool launch_gen_t(const EncArgs& a, hipStream_t s) {
    if constexpr (K + M <= 8)
        return launch_ws_t<K, M, 16, 512, 1, true, false, 0, false, 0, 16, false, 3, false, 0, 2, true, 3, 1, 0, true>(a, s);
    else
        return launch_ws_t<K, M, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 0, 2, true, 3, 1, 0, true>(a, s);
}

#define ZS3_GEN_KM(X) X(2, 2) X(3, 2) X(3, 3) X(4, 3) X(5, 4) X(6, 4) X(7, 4) X(9, 4) X(10, 4) X(11, 4)

bool has_gen_encode(int k, int m) {
#define X(K, M) if (k == K && m == M) return true;
    ZS3_GEN_KM(X)
#undef X
    return false;
}

int launch_ehx_gen(const EncArgs& a, hipStream_t s) {
    if (!a.sums) return PATH_NONE;
#define X(K, M) \
    if (a.k == K && a.m == M) return launch_gen_t<K, M>(a, s) ? PATH_WS : PATH_NONE;
    ZS3_GEN_KM(X)
#undef X
    return PATH_NONE;
}

}  // namespace zs3k
