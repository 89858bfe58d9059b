// fused_v2_km124.hip — RS(12+4) encode variants on 1 MiB blocks (diagnostics build only).
// RS(12+4) is the server's default for 16-drive sets (cmd/format-erasure.go:870-881);
// 1 MiB blocks give S = 87 382 (rows 2-byte aligned), so every instance runs k_ehx_ws in
// UA mode with buffer-addressed rows.  The product instance (launch_ehx_ua: 8 stripes,
// 8-byte columns of 384-byte tiles) has 4 hash + 6 encode waves, i.e. two SIMDs with
// two encode waves and two with one; these shapes put the same work on every SIMD:
//  195: 16 stripes, 8-byte columns of 256-byte tiles: 8 hash + 8 encode waves (16 waves,
//       2 + 2 per SIMD, 128 VGPRs)
//  196: 8 stripes, 8-byte columns of 512-byte tiles: 4 hash + 8 encode waves (1 + 2 per
//       SIMD), data rows written to LDS before the encode
//  197: 196 without the early data write
//  198 / 199: 8 stripes, 16-byte columns of 512-byte tiles: 4 hash + 4 encode waves (one
//       of each per SIMD), with / without the early data write; 165 / 166 the same with
//       the 2-waves-per-SIMD register budget (256 VGPRs)
//  (195-199 / 165-166 first ran in session 3 of round 3: before that, launch_encode sent
//  every non-zero variant with unaligned rows to the any-geometry kernels)
//  175 / 176: the product instance + L2 prefetch by the hash waves, 2 / 3 tiles ahead
//  177: the product instance with two tiles of register prefetch
//  179 / 180 / 181: 196 + L2 prefetch by the hash waves, 2 / 3 / 1 tiles ahead
//  178: 16 stripes, 16-byte columns of 256-byte tiles: 8 hash + 4 encode waves (2 + 1 per SIMD)
//  330 / 331 (round 4): the product instance (179) with the conflict-free LDS row stride
//  (TSP = 1), L2 prefetch 2 / 3 tiles ahead (no gain: profiles/r04/sweep_rs124_tsp.jsonl)
//  332 / 333: the product instance with temporal data loads (nt stores only) / no nt at
//  all: unaligned rows share each tile's edge lines with the neighbouring tiles
//  335: 4 stripes of 1 KiB tiles; 337: 16-byte columns (4 encode waves) with the
//  256-VGPR budget, L2 prefetch, conflict-free LDS stride
//  334 / 336 / 338 (timing ablations of the product instance, output differs): no
//  HighwayHash arithmetic or LDS reads in the hash waves / no GF arithmetic in the encode
//  waves / neither (the memory pattern alone, L2 prefetch kept)
//  380-387: the memory pattern alone (ABL 7, no GF) of other shapes: 380 no L2 prefetch,
//  381 16 stripes of 256-byte tiles, 382 4 stripes of 1 KiB tiles, 383 16-byte columns
//  (256-VGPR budget), 384 temporal data loads, 385 L2 prefetch 4 tiles ahead, 386 4 stripes
//  of 1 KiB tiles with 16-byte columns, 387 8 stripes of 256-byte tiles (two workgroups
//  per CU, 128-VGPR budget)
//  390-392: 4 stripes of 1 KiB tiles (the best memory pattern above, 386) with the L2
//  prefetch two tiles ahead: 390 pair-form hash waves, 16-byte columns (256-VGPR budget);
//  391 quad-form hash waves (4 instead of 2), 16-byte columns; 392 quad-form, 8-byte columns;
//  391 with two tiles of register prefetch (393), without the early data write (394), with
//  the L2 prefetch three tiles ahead (395)
#include "fused_v2.hpp"

namespace zs3k {

#if ZS3_DIAG
bool launch_ehx_km_12_4(int v, const EncArgs& a, hipStream_t s) {
    switch (v) {
        case 175: return launch_ws_t<12, 4, 8, 384, 1, true, false, 0, false, 0, 0, false, 3, false, 2, 2, true>(a, s);
        case 176: return launch_ws_t<12, 4, 8, 384, 1, true, false, 0, false, 0, 0, false, 3, false, 2, 3, true>(a, s);
        case 177: return launch_ws_t<12, 4, 8, 384, 2, true, false, 0, false, 0, 0, false, 3, false, 2, 0, true>(a, s);
        case 178: return launch_ws_t<12, 4, 16, 256, 1, true, false, 0, false, 0, 16, false, 3, false, 2, 0, true>(a, s);
        case 179: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 2, 2, true>(a, s);
        case 180: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 2, 3, true>(a, s);
        case 181: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 2, 1, true>(a, s);
        case 195: return launch_ws_t<12, 4, 16, 256, 1, true, false, 0, false, 0, 8, false, 3, false, 0, 0, true>(a, s);
        case 196: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 2, 0, true>(a, s);
        case 197: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 0, 0, true>(a, s);
        case 198: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 16, false, 3, false, 2, 0, true>(a, s);
        case 199: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 16, false, 3, false, 0, 0, true>(a, s);
        case 165: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 16, false, 3, false, 2, 0, true, 2>(a, s);
        case 166: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 16, false, 3, false, 0, 0, true, 2>(a, s);
        case 330: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 2, 2, true, 3, 1>(a, s);
        case 331: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 2, 3, true, 3, 1>(a, s);
        case 332: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 2, false, 2, 2, true>(a, s);
        case 333: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 0, false, 2, 2, true>(a, s);
        case 335: return launch_ws_t<12, 4, 4, 1024, 1, true, false, 0, false, 0, 8, false, 3, false, 2, 2, true, 3, 1>(a, s);
        case 337: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 16, false, 3, false, 2, 2, true, 2, 1>(a, s);
        case 334: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 2, 2, true, 3, 0, 3>(a, s);
        case 336: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 9, 2, true>(a, s);
        case 380: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 9, 0, true, 3, 0, 7>(a, s);
        case 381: return launch_ws_t<12, 4, 16, 256, 1, true, false, 0, false, 0, 8, false, 3, false, 9, 2, true, 3, 1, 7>(a, s);
        case 382: return launch_ws_t<12, 4, 4, 1024, 1, true, false, 0, false, 0, 8, false, 3, false, 9, 2, true, 3, 1, 7>(a, s);
        case 383: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 16, false, 3, false, 9, 2, true, 2, 1, 7>(a, s);
        case 384: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 2, false, 9, 2, true, 3, 0, 7>(a, s);
        case 385: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 9, 4, true, 3, 0, 7>(a, s);
        case 386: return launch_ws_t<12, 4, 4, 1024, 1, true, false, 0, false, 0, 16, false, 3, false, 9, 2, true, 3, 1, 7>(a, s);
        case 387: return launch_ws_t<12, 4, 8, 256, 1, true, false, 0, false, 0, 8, false, 3, false, 9, 2, true, 4, 1, 7>(a, s);
        case 390: return launch_ws_t<12, 4, 4, 1024, 1, true, false, 0, false, 0, 16, false, 3, false, 2, 2, true, 2, 1>(a, s);
        case 391: return launch_ws_t<12, 4, 4, 1024, 1, true, true, 0, false, 0, 16, false, 3, false, 2, 2, true, 2, 1>(a, s);
        case 392: return launch_ws_t<12, 4, 4, 1024, 1, true, true, 0, false, 0, 8, false, 3, false, 2, 2, true, 3, 1>(a, s);
        case 393: return launch_ws_t<12, 4, 4, 1024, 2, true, true, 0, false, 0, 16, false, 3, false, 2, 2, true, 2, 1>(a, s);
        case 394: return launch_ws_t<12, 4, 4, 1024, 1, true, true, 0, false, 0, 16, false, 3, false, 0, 2, true, 2, 1>(a, s);
        case 395: return launch_ws_t<12, 4, 4, 1024, 1, true, true, 0, false, 0, 16, false, 3, false, 2, 3, true, 2, 1>(a, s);
        case 338: return launch_ws_t<12, 4, 8, 512, 1, true, false, 0, false, 0, 8, false, 3, false, 9, 2, true, 3, 0, 7>(a, s);
        default: return false;
    }
}
#endif

}  // namespace zs3k
