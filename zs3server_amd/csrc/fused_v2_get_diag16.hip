// fused_v2_get_diag16.hip — diagnostics variants of the RS(16+m)-shaped GET / heal pass (diagnostics build
// only): earlier product instances and A/B shapes of k_vr_ws, selected by variant number
// through zs3server_amd.diag(v).  The product defaults are in fused_v2_get.hip.
#include "fused_v2.hpp"

namespace zs3k {

#if ZS3_DIAG
// Round 4 candidates for the RS(16+4) rebuild / heal of 3-4 rows, measured and dropped
// (profiles/r04/get_ab_k16.jsonl, 2048 x 1 MiB; their instances are no longer compiled):
//  273: 4 stripes, 768-byte tiles          heal 4 0.88 vs 0.78 ms, rebuild 4 0.73 vs 0.76
//  274: 8 stripes, 512-byte tiles          = the product rebuild shape; heal 1.05-1.35 ms
//  275: quad-form hash waves               1.3-2.8 ms (spills 100-190 VGPRs)
//  276 / 277: 16-byte rebuild columns      spill 100-570 VGPRs at compile time
// The product RS(16+4) rebuild 3-4 / heal 2-4 instances spill 44-58 VGPRs at the 168-VGPR
// budget of their 11-wave workgroups.
bool launch_vr_ws_diag_k16(int v, const VrArgs& a, hipStream_t s) {
    // survivor prefetch depth / tile length / column width candidates (round 3); the
    // rejected ones (251-255, 257: 8-45 % slower, profiles/r03/get_ab_rs164_vr16.jsonl)
    // are no longer compiled; 250 / 256 / 259 became the product instances
    if (a.k == 16 && v >= 250 && v <= 259 && a.e >= 1) {
        const bool h = a.sums_out != nullptr;
        switch (v) {
            case 250: return h ? vr16<128, 2, true, 4>(a, s) : vr16<256, 2, false, 0>(a, s);
            case 256: return h ? vr16<256, 1, true, 4, 8>(a, s) : vr16<512, 1, false, 4, 8>(a, s);
            case 259: return h ? vr16<384, 1, true, 4, 8>(a, s) : vr16<384, 1, false, 4, 8>(a, s);
            default: return false;
        }
    }
    if (a.k == 16 && (v == 242 || v == 219) && a.sums_out == nullptr && a.e >= 1) {
        // round-2 RS(16+4) rebuild instances (4-byte columns, one table per scalar wait)
        if (a.e == 1) return launch_vr_ws_t<16, 1, false, 8, 256, 1, 4, false, true>(a, s);
        if (a.e == 2) return launch_vr_ws_t<16, 2, false, 8, 256, 1, 4, false, true>(a, s);
        if (a.e == 3) return launch_vr_ws_t<16, 3, false, 8, 256, 1, 4, false, true>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, false, 8, 256, 1, 4, false, true>(a, s);
        return false;
    }
    if ((v == 242 || v == 232) && a.k == 16 && a.sums_out != nullptr && a.e >= 1) {
        // round-2 RS(16+4) heal instances: heal 1 with 8-byte columns, heal 2-4 with
        // 4-byte columns of 128-byte tiles
        if (a.e == 1) return launch_vr_ws_t<16, 1, true, 8, 256, 1, 8, false, false>(a, s);
        if (a.e == 2) return launch_vr_ws_t<16, 2, true, 8, 128, 1, 4, false, true, 4>(a, s);
        if (a.e == 3) return launch_vr_ws_t<16, 3, true, 8, 128, 1, 4, false, true, 4>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, true, 8, 128, 1, 4, false, true, 4>(a, s);
        return false;
    }
    if (a.k == 16 && v == 217 && a.sums_out == nullptr) {
        // twice the rebuild waves (12 waves, 3 per SIMD): 4-byte columns of 256-byte
        // tiles (8-byte columns of 512-byte tiles spill in the hash role)
        if (a.e == 1) return launch_vr_ws_t<16, 1, false, 8, 256, 1, 4>(a, s);
        if (a.e == 2) return launch_vr_ws_t<16, 2, false, 8, 256, 1, 4>(a, s);
        if (a.e == 3) return launch_vr_ws_t<16, 3, false, 8, 256, 1, 4>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, false, 8, 256, 1, 4>(a, s);
        return false;
    }
    if (a.k == 16 && (v == 210 || v == 215 || v == 216)) {
        // RS(16+4)-shaped GET: 8 stripes, 256-byte tiles; rebuilds with 8-byte columns
        // (16-byte columns spill: 16 survivors x 2 tiles beside 32-64 generic products).
        if (a.sums_out != nullptr && v == 216) {
            // Heal (17..20 hashed rows): 8 stripes per workgroup, pair-form hash waves
            // padded to whole waves (e.g. heal 2: 288 -> 320 threads) beside 2-4 rebuild
            // waves with 8-byte columns; e >= 2 reads the rebuild tables with scalar loads
            // (the VGPR copy spills).  Product default for heal 1 only: 0.535 vs 0.785 ms
            // (first generation) on 2048 x 1 MiB; heal 2/3/4 measured 0.967/1.31/1.58 vs
            // 0.946/1.13/1.31 ms (2 rebuild waves are the bound), diagnostics 216
            // (profiles/r02/get_ab.txt)
            if (a.e == 1) return launch_vr_ws_t<16, 1, true, 8, 256, 1, 8, false, false>(a, s);
            if (a.e == 2) return launch_vr_ws_t<16, 2, true, 8, 128, 1, 8, false, false>(a, s);
            if (a.e == 3) return launch_vr_ws_t<16, 3, true, 8, 128, 1, 8, false, true>(a, s);
            if (a.e == 4) return launch_vr_ws_t<16, 4, true, 8, 128, 1, 8, false, true>(a, s);
            return false;
        }
        if (a.sums_out != nullptr) {
            // Heal (18 / 20 hashed rows): 2*8*18 pair-form threads are not whole waves,
            // so the hash role runs in quad form (padded to 9 / 10 waves) beside 4
            // rebuild waves.  Measured slower than the first-generation kernel on
            // 2048 x 1 MiB (heal 2: 1.29 vs 0.95 ms, heal 4: 2.86 vs 1.31 ms; 13 waves
            // leave 128 VGPRs), so opt-in only (variant 215).
            if (v == 215) {
                if (a.e == 2) return launch_vr_ws_t<16, 2, true, 8, 256, 1, 8, true>(a, s);
                if (a.e == 4) return launch_vr_ws_t<16, 4, true, 8, 256, 1, 8, true>(a, s);
            }
            return false;
        }
        if (v == 215) return false;
        if (v == 210) {  // 8-byte rebuild columns (4 rebuild waves), the round-2 first cut
            if (a.e == 1) return launch_vr_ws_t<16, 1, false, 8, 256, 1, 8>(a, s);
            if (a.e == 3) return launch_vr_ws_t<16, 3, false, 8, 256, 1, 8>(a, s);
        }
        if (v == 216) {  // scalar coefficient tables in the rebuild role
            if (a.e == 1) return launch_vr_ws_t<16, 1, false, 8, 256, 1, 8, false, true>(a, s);
            if (a.e == 3) return launch_vr_ws_t<16, 3, false, 8, 256, 1, 8, false, true>(a, s);
            if (a.e == 2) return launch_vr_ws_t<16, 2, false, 8, 256, 1, 8, false, true>(a, s);
            if (a.e == 4) return launch_vr_ws_t<16, 4, false, 8, 256, 1, 8, false, true>(a, s);
            return false;
        }
        if (a.e == 0) return launch_vr_ws_t<16, 0, false, 8, 256, 2>(a, s);
        if (a.e == 2) return launch_vr_ws_t<16, 2, false, 8, 256, 1, 8>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, false, 8, 256, 1, 8>(a, s);
        return false;
    }
    return false;
}
#endif

}  // namespace zs3k
