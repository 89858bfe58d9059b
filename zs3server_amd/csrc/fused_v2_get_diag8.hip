// fused_v2_get_diag8.hip — diagnostics variants of the RS(8+m)-shaped GET / heal pass (diagnostics build
// only): earlier product instances and A/B shapes of k_vr_ws, selected by variant number
// through zs3server_amd.diag(v).  The product defaults are in fused_v2_get.hip.
#include "fused_v2.hpp"

namespace zs3k {

#if ZS3_DIAG
bool launch_vr_ws_diag_k8(int v, const VrArgs& a, hipStream_t s) {
    if (a.k == 8 && v >= 260 && v <= 263 && a.e >= 1) {
        // RS(8+4) GET / heal with longer tiles (round 3): 260 / 261 heal on 8 stripes with
        // 8-byte columns of 384 / 256-byte tiles; 262 heal on 16 stripes, 16-byte columns
        // of 256-byte tiles; 263 rebuild on 8 stripes, 8-byte columns of 384-byte tiles
        const bool h = a.sums_out != nullptr;
        switch (v * 8 + a.e) {
            case 260 * 8 + 1: return h && launch_vr_ws_t<8, 1, true, 8, 384, 1, 8, false, true, 4>(a, s);
            case 260 * 8 + 2: return h && launch_vr_ws_t<8, 2, true, 8, 384, 1, 8, false, true, 4>(a, s);
            case 260 * 8 + 3: return h && launch_vr_ws_t<8, 3, true, 8, 384, 1, 8, false, true, 4>(a, s);
            case 260 * 8 + 4: return h && launch_vr_ws_t<8, 4, true, 8, 384, 1, 8, false, true, 4>(a, s);
            case 261 * 8 + 1: return h && launch_vr_ws_t<8, 1, true, 8, 256, 1, 8, false, true, 4>(a, s);
            case 261 * 8 + 2: return h && launch_vr_ws_t<8, 2, true, 8, 256, 1, 8, false, true, 4>(a, s);
            case 261 * 8 + 3: return h && launch_vr_ws_t<8, 3, true, 8, 256, 1, 8, false, true, 4>(a, s);
            case 261 * 8 + 4: return h && launch_vr_ws_t<8, 4, true, 8, 256, 1, 8, false, true, 4>(a, s);
            case 262 * 8 + 1: return h && launch_vr_ws_t<8, 1, true, 16, 256, 1, 16, false, true, 4>(a, s);
            case 262 * 8 + 2: return h && launch_vr_ws_t<8, 2, true, 16, 256, 1, 16, false, true, 4>(a, s);
            case 262 * 8 + 3: return h && launch_vr_ws_t<8, 3, true, 16, 256, 1, 16, false, true, 4>(a, s);
            case 262 * 8 + 4: return h && launch_vr_ws_t<8, 4, true, 16, 256, 1, 16, false, true, 4>(a, s);
            case 263 * 8 + 1: return !h && launch_vr_ws_t<8, 1, false, 8, 384, 1, 8, false, true, 4>(a, s);
            case 263 * 8 + 2: return !h && launch_vr_ws_t<8, 2, false, 8, 384, 1, 8, false, true, 4>(a, s);
            case 263 * 8 + 3: return !h && launch_vr_ws_t<8, 3, false, 8, 384, 1, 8, false, true, 4>(a, s);
            case 263 * 8 + 4: return !h && launch_vr_ws_t<8, 4, false, 8, 384, 1, 8, false, true, 4>(a, s);
            default: return false;
        }
    }
    if (v == 232 && a.k == 8 && a.sums_out != nullptr && a.e >= 3) {
        // round-2 RS(8+4) heal 3-4 instances: 8-byte columns of 128-byte tiles, two tiles
        // of survivor prefetch (1.41 / 1.61 ms vs 1.49 / 1.79 unbatched and 2.01 / 2.32 for
        // the first-generation kernel; profiles/r02/get_ab_bt.jsonl, get_ab_waves.jsonl)
        if (a.e == 3) return launch_vr_ws_t<8, 3, true, 16, 128, 2, 8, false, true, 4>(a, s);
        if (a.e == 4) return launch_vr_ws_t<8, 4, true, 16, 128, 2, 8, false, true, 4>(a, s);
        return false;
    }
    if (a.sums_out != nullptr) {
        // heal (10 hashed rows): 8-byte rebuild columns and 128-byte tiles keep the
        // 9-wave workgroup inside 168 VGPRs (1.50 -> 1.25 ms, 1 data + 1 parity)
        // (scalar coefficient tables, variant 216: 1.28 -> 1.18 ms on 4096 x 1 MiB,
        // profiles/r02/get_ab.txt)
        if (v == 216 && a.e == 1) return launch_vr_ws_t<8, 1, true, 16, 128, 2, 8, false, true, 4>(a, s);
        if (a.e != 2) return false;
        if (v == 216) return launch_vr_ws_t<8, 2, true, 16, 128, 2, 8, false, true, 4>(a, s);
        if (v == 212) return launch_vr_ws_t<8, 2, true, 16, 128, 2, 8>(a, s);
        if (v == 213) return launch_vr_ws_t<8, 2, true, 16, 256, 1, 8>(a, s);
        return false;
    }
    switch (v) {
        case 210:
            if (a.e == 0) return launch_vr_ws_t<8, 0, false, 16, 256, 2>(a, s);
            if (a.e == 1) return launch_vr_ws_t<8, 1, false, 16, 256, 2>(a, s);
            if (a.e == 2) return launch_vr_ws_t<8, 2, false, 16, 256, 2>(a, s);
            // rebuild 3/4: 8-byte columns (8 rebuild waves, scalar tables): 4096 x 1 MiB
            // 1.27 / 1.42 ms vs 1.35 / 1.58 with 16-byte columns (get_ab_waves.jsonl);
            // batched scalar tables: 1.34 vs 1.40 ms for rebuild 4
            if (a.e == 3) return launch_vr_ws_t<8, 3, false, 16, 256, 1>(a, s);
            if (a.e == 4) return launch_vr_ws_t<8, 4, false, 16, 256, 1>(a, s);
            return false;
        case 211:
            if (a.e == 0) return launch_vr_ws_t<8, 0, false, 16, 256, 1>(a, s);
            if (a.e == 2) return launch_vr_ws_t<8, 2, false, 16, 256, 1>(a, s);
            return false;
        case 214:  // twice the rebuild waves: 8-byte columns (12 waves, 3 per SIMD);
                   // e >= 2 with scalar coefficient tables (VGPR tables spill at 168)
            if (a.e == 1) return launch_vr_ws_t<8, 1, false, 16, 256, 1, 8>(a, s);
            if (a.e == 2) return launch_vr_ws_t<8, 2, false, 16, 256, 1, 8, false, true>(a, s);
            if (a.e == 3) return launch_vr_ws_t<8, 3, false, 16, 256, 1, 8, false, true>(a, s);
            if (a.e == 4) return launch_vr_ws_t<8, 4, false, 16, 256, 1, 8, false, true>(a, s);
            return false;
        case 216:
            if (a.e == 1) return launch_vr_ws_t<8, 1, false, 16, 256, 2, 16, false, true>(a, s);
            if (a.e == 2) return launch_vr_ws_t<8, 2, false, 16, 256, 2, 16, false, true>(a, s);
            if (a.e == 3) return launch_vr_ws_t<8, 3, false, 16, 256, 1, 16, false, true>(a, s);
            if (a.e == 4) return launch_vr_ws_t<8, 4, false, 16, 256, 1, 16, false, true>(a, s);
            return false;
        default:
            return false;
    }
    return false;
}
#endif

}  // namespace zs3k
