// fused_v2_get_diag.hip — diagnostics variants of the GET / heal pass (diagnostics build
// only): earlier product instances and A/B shapes of k_vr_ws, selected by variant number
// through zs3server_amd.diag(v).  The product defaults are in fused_v2_get.hip.
#include "fused_v2.hpp"

namespace zs3k {

#if ZS3_DIAG
// Diagnostics variants of the GET / heal pass (v != 0), one translation unit per data
// shard count (compiled in parallel): A/B instances measured against the product
// defaults (fused_v2_get.hip) in profiles/r02 and profiles/r03.
bool launch_vr_ws_diag_k4(int v, const VrArgs& a, hipStream_t s);   // fused_v2_get_diag4.hip
bool launch_vr_ws_diag_k8(int v, const VrArgs& a, hipStream_t s);   // fused_v2_get_diag8.hip
bool launch_vr_ws_diag_k16(int v, const VrArgs& a, hipStream_t s);  // fused_v2_get_diag16.hip

// RS(12+4) on unaligned rows (UA), round 3: shape candidates against the product
// instances (the RS(16+4) shapes; fused_v2_get.hip)
//  264: the first product instances (the RS(16+4) shapes); 8-byte columns of 512-byte
//       tiles for every e measured fastest and became the product (get_ab_rs124.jsonl)
//  (16 stripes with 16-byte columns, the RS(8+4) GET shape, spill 90-4 000 VGPRs at
//  K = 12 and are not compiled; 16 stripes of 8-byte columns spill 19-24 in heal)
//  267: 8 stripes, 8-byte columns of 256-byte tiles, two tiles of prefetch, batched tables
template <int EX, bool H>
static bool vr12_ua(int v, const VrArgs& a, hipStream_t s) {
    switch (v) {
        case 264:  // round-3 RS(16+4)-shaped instances (4-byte rebuild-1/2 columns, 384-byte heal tiles)
            if constexpr (H) return launch_vr_ws_t<12, EX, H, 8, 384, 1, 8, false, true, 4, true>(a, s);
            else if constexpr (EX <= 2) return launch_vr_ws_t<12, EX, H, 8, 256, 2, 4, false, true, 0, true>(a, s);
            else return launch_vr_ws_t<12, EX, H, 8, 512, 1, 8, false, true, 4, true>(a, s);
        case 267: return launch_vr_ws_t<12, EX, H, 8, 256, 2, 8, false, true, 4, true>(a, s);
        // round 4: 4 stripes of 1 KiB tiles (269); two tiles of survivor prefetch at 512
        // bytes spill in-flight load registers (scripts/check_async_loads.py) and are not
        // compiled
        case 269: return launch_vr_ws_t<12, EX, H, 4, 1024, 1, 8, false, true, 4, true>(a, s);
        // the L2 prefetch by the hash waves (PFD, as in the encode): product + prefetch 2
        // tiles ahead (265; 3 tiles ahead measured slower still, profiles/r04/
        // get_ab_k12_pfd.jsonl); 4 stripes of 1 KiB tiles, quad-form hash waves issuing it
        // 2 tiles ahead (268); 266: 4 stripes of 1 KiB tiles, quad-form hash waves, 16-byte
        // rebuild columns, no prefetch
        case 265: return launch_vr_ws_t<12, EX, H, 8, 512, 1, 8, false, true, 4, true, false, 2>(a, s);
        case 266: return launch_vr_ws_t<12, EX, H, 4, 1024, 1, 16, true, true, 4, true>(a, s);
        case 268: return launch_vr_ws_t<12, EX, H, 4, 1024, 1, 8, true, true, 4, true, false, 2>(a, s);
        default: return false;
    }
}

bool launch_vr_ws_diag(int v, const VrArgs& a, hipStream_t s) {
    if (a.k == 12 && v >= 264 && v <= 269) {
        const bool h = a.sums_out != nullptr;
        switch (a.e) {
            case 1: return h ? vr12_ua<1, true>(v, a, s) : vr12_ua<1, false>(v, a, s);
            case 2: return h ? vr12_ua<2, true>(v, a, s) : vr12_ua<2, false>(v, a, s);
            case 3: return h ? vr12_ua<3, true>(v, a, s) : vr12_ua<3, false>(v, a, s);
            case 4: return h ? vr12_ua<4, true>(v, a, s) : vr12_ua<4, false>(v, a, s);
            default: return false;
        }
    }
    if (a.k == 4) return launch_vr_ws_diag_k4(v, a, s);
    if (a.k == 8) return launch_vr_ws_diag_k8(v, a, s);
    if (a.k == 16) return launch_vr_ws_diag_k16(v, a, s);
    return false;
}
#endif

}  // namespace zs3k
