// fused_v2_get_diag4.hip — diagnostics variants of the RS(4+m)-shaped GET / heal pass (diagnostics build
// only): earlier product instances and A/B shapes of k_vr_ws, selected by variant number
// through zs3server_amd.diag(v).  The product defaults are in fused_v2_get.hip.
#include "fused_v2.hpp"

#include <type_traits>

namespace zs3k {

#if ZS3_DIAG
bool launch_vr_ws_diag_k4(int v, const VrArgs& a, hipStream_t s) {
    if (a.k == 4 && v == 214) {
        // the RS(4+2)-shaped product instances (quad-form hash waves, 8 stripes)
        if (a.sums_out != nullptr)
            return a.e == 2 && launch_vr_ws_t<4, 2, true, 8, 256, 4, 16, true>(a, s);
        if (a.e == 0) return launch_vr_ws_t<4, 0, false, 8, 256, 4, 16, true>(a, s);
        if (a.e == 1) return launch_vr_ws_t<4, 1, false, 8, 256, 4, 16, true>(a, s);
        if (a.e == 2) return launch_vr_ws_t<4, 2, false, 8, 256, 4, 16, true>(a, s);
        return false;
    }
    if (a.k == 4 && v == 210) {
        // RS(4+2)-shaped GET / heal, pair-form hash waves: 16 stripes, 256-byte tiles
        if (a.sums_out != nullptr)
            return a.e == 2 && launch_vr_ws_t<4, 2, true, 16, 256, 2>(a, s);
        if (a.e == 0) return launch_vr_ws_t<4, 0, false, 16, 256, 2>(a, s);
        if (a.e == 1) return launch_vr_ws_t<4, 1, false, 16, 256, 2>(a, s);
        if (a.e == 2) return launch_vr_ws_t<4, 2, false, 16, 256, 2>(a, s);
        return false;
    }
    if (a.k == 4 && v >= 270 && v <= 272) {
        // round 4: longer tiles for the chain-latency-bound RS(4+2) / RS(4+4) GET / heal
        // (fewer barriers per hashed byte, as config 2's encode; 8 stripes, quad form)
        //  270: 512-byte tiles, 4 of prefetch; 271: 1 KiB tiles, 2 of prefetch;
        //  272: 1 KiB tiles, 4 of prefetch
        const bool h = a.sums_out != nullptr;
        auto go = [&](auto ex) -> bool {
            constexpr int EX = decltype(ex)::value;
            if (v == 270) return h ? launch_vr_ws_t<4, EX, true, 8, 512, 4, 16, true>(a, s)
                                   : launch_vr_ws_t<4, EX, false, 8, 512, 4, 16, true>(a, s);
            if (v == 271) return h ? launch_vr_ws_t<4, EX, true, 8, 1024, 2, 16, true>(a, s)
                                   : launch_vr_ws_t<4, EX, false, 8, 1024, 2, 16, true>(a, s);
            return h ? launch_vr_ws_t<4, EX, true, 8, 1024, 4, 16, true>(a, s)
                     : launch_vr_ws_t<4, EX, false, 8, 1024, 4, 16, true>(a, s);
        };
        switch (a.e) {
            case 0: return !h && go(std::integral_constant<int, 0>{});
            case 1: return go(std::integral_constant<int, 1>{});
            case 2: return go(std::integral_constant<int, 2>{});
            case 3: return go(std::integral_constant<int, 3>{});
            case 4: return go(std::integral_constant<int, 4>{});
            default: return false;
        }
    }
    return false;
}
#endif

}  // namespace zs3k
