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

bool launch_vr_ws_diag(int v, const VrArgs& a, hipStream_t s) {
    if (a.k == 4) return launch_vr_ws_diag_k4(v, a, s);
    if (a.k == 8) return launch_vr_ws_diag_k8(v, a, s);
    if (a.k == 16) return launch_vr_ws_diag_k16(v, a, s);
    return false;
}
#endif

}  // namespace zs3k
