// fused_v2_get_diag4.hip — diagnostics variants of the RS(4+m)-shaped GET / heal pass (diagnostics build
// only): earlier product instances and A/B shapes of k_vr_ws, selected by variant number
// through zs3server_amd.diag(v).  The product defaults are in fused_v2_get.hip.
#include "fused_v2.hpp"

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
    return false;
}
#endif

}  // namespace zs3k
