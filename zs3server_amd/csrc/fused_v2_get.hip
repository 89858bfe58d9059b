// fused_v2_get.hip — GET / heal dispatch onto the warp-specialised k_vr_ws instances
// (templates in fused_v2.hpp): the product defaults and the diagnostics variants.
// Replaces the arithmetic of parallelReader + streamingBitrotReader.ReadAt
// (cmd/erasure-decode.go:165-179, cmd/bitrot-streaming.go:171-186),
// Erasure.DecodeDataBlocks (cmd/erasure-coding.go:96-109) and Erasure.Heal
// (cmd/erasure-decode.go:287-332) for one batch of stripes.
#include "fused_v2.hpp"

namespace zs3k {

// GET / heal defaults (variant 0) and diagnostics variants 210-215.
// RS(8+4)-shaped GET: 16 stripes, 256-byte tiles, verify-only or rebuild 2; heal with
// 8-byte columns (16-byte columns spill at the heal's 168-VGPR budget: 4.7 ms).
bool launch_vr_ws(int v, const VrArgs& a, hipStream_t s) {
    if (!ZS3_DIAG && v != 0) return false;
#if ZS3_DIAG
    if (a.k == 16 && v >= 250 && v <= 259 && a.e >= 1) {
        const bool h = a.sums_out != nullptr;
        switch (v) {
            case 250: return h ? vr16<128, 2, true, 4>(a, s) : vr16<256, 2, false, 0>(a, s);
            case 251: return h ? vr16<128, 3, true, 0>(a, s) : vr16<128, 3, false, 4>(a, s);
            case 252: return h ? vr16<256, 2, true, 4>(a, s) : vr16<256, 3, false, 0>(a, s);
            case 253: return h ? vr16<256, 1, true, 4>(a, s) : vr16<512, 1, false, 0>(a, s);
            case 254: return h ? vr16<128, 3, true, 4>(a, s) : vr16<128, 2, false, 0>(a, s);
            case 255: return h ? vr16<256, 2, true, 0>(a, s) : vr16<256, 2, false, 4>(a, s);
            case 256: return h ? vr16<256, 1, true, 4, 8>(a, s) : vr16<512, 1, false, 4, 8>(a, s);
            case 257: return h ? vr16<512, 1, true, 4, 8>(a, s) : vr16<256, 2, false, 4, 8>(a, s);
            case 259: return h ? vr16<384, 1, true, 4, 8>(a, s) : vr16<384, 1, false, 4, 8>(a, s);
            default: return false;
        }
    }
#endif
    if (a.k == 4 && (v == 0 || v == 214)) {
        // RS(4+2)-shaped GET / heal default: quad-form hash waves, 8 stripes, one wave
        // of each kind per SIMD (the 8 192 chains of a 2048-object batch are
        // latency-bound: verify 0.63 -> 0.44 ms over the pair form)
        if (a.sums_out != nullptr)
            return a.e == 2 && launch_vr_ws_t<4, 2, true, 8, 256, 4, 16, true>(a, s);
        if (a.e == 0) return launch_vr_ws_t<4, 0, false, 8, 256, 4, 16, true>(a, s);
        if (a.e == 1) return launch_vr_ws_t<4, 1, false, 8, 256, 4, 16, true>(a, s);
        if (a.e == 2) return launch_vr_ws_t<4, 2, false, 8, 256, 4, 16, true>(a, s);
        return false;
    }
#if ZS3_DIAG
    if (a.k == 4 && v == 210) {
        // RS(4+2)-shaped GET / heal, pair-form hash waves: 16 stripes, 256-byte tiles
        if (a.sums_out != nullptr)
            return a.e == 2 && launch_vr_ws_t<4, 2, true, 16, 256, 2>(a, s);
        if (a.e == 0) return launch_vr_ws_t<4, 0, false, 16, 256, 2>(a, s);
        if (a.e == 1) return launch_vr_ws_t<4, 1, false, 16, 256, 2>(a, s);
        if (a.e == 2) return launch_vr_ws_t<4, 2, false, 16, 256, 2>(a, s);
        return false;
    }
#endif
    if (a.k == 16 && (v == 0 || v == 219) && a.sums_out == nullptr && a.e >= 1) {
        // RS(16+4) GET rebuild 1-4: 4-byte rebuild columns (8 rebuild waves beside the 4
        // hash waves, 3 waves per SIMD) with scalar coefficient tables.  2048 x 1 MiB:
        // rebuild 1/2/3/4 0.50/0.55/0.66/0.75 ms vs 0.52/0.62/0.75/0.85 with 8-byte
        // columns (4 rebuild waves); profiles/r02/get_ab_waves.jsonl.  Batched scalar tables
        // (diagnostics 240) measured 2-4 % slower here (get_ab_bt.jsonl)
        if (a.e == 1) return launch_vr_ws_t<16, 1, false, 8, 256, 1, 4, false, true>(a, s);
        if (a.e == 2) return launch_vr_ws_t<16, 2, false, 8, 256, 1, 4, false, true>(a, s);
        if (a.e == 3) return launch_vr_ws_t<16, 3, false, 8, 256, 1, 4, false, true>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, false, 8, 256, 1, 4, false, true>(a, s);
        return false;
    }
    if ((v == 0 || v == 232) && a.k == 16 && a.sums_out != nullptr && a.e >= 2) {
        // RS(16+4) heal 2-4: 4-byte rebuild columns of 128-byte tiles (4 rebuild waves
        // beside 5 pair-form hash waves, scalar tables read in double-buffered batches).
        // 2048 x 1 MiB: heal 2/3/4 0.81/0.93/1.06 ms vs 0.82/0.99/1.17 with one table
        // per scalar wait and 0.95/1.13/1.31 for the first-generation kernel
        // (profiles/r02/get_ab_bt.jsonl, get_ab_waves.jsonl)
        if (a.e == 2) return launch_vr_ws_t<16, 2, true, 8, 128, 1, 4, false, true, 4>(a, s);
        if (a.e == 3) return launch_vr_ws_t<16, 3, true, 8, 128, 1, 4, false, true, 4>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, true, 8, 128, 1, 4, false, true, 4>(a, s);
        return false;
    }
    if ((v == 0 || v == 232) && a.k == 8 && a.sums_out != nullptr && a.e >= 3) {
        // RS(8+4) heal 3-4: padded pair-form hash waves (11 / 12 hashed rows x 16 stripes)
        // beside 4 rebuild waves, batched scalar tables; 4096 x 1 MiB: 1.41 / 1.61 ms vs
        // 1.49 / 1.79 unbatched and 2.01 / 2.32 for the first-generation kernel
        // (profiles/r02/get_ab_bt.jsonl, get_ab_waves.jsonl)
        if (a.e == 3) return launch_vr_ws_t<8, 3, true, 16, 128, 2, 8, false, true, 4>(a, s);
        if (a.e == 4) return launch_vr_ws_t<8, 4, true, 16, 128, 2, 8, false, true, 4>(a, s);
        return false;
    }
#if ZS3_DIAG
    if (a.k == 16 && v == 217 && a.sums_out == nullptr) {
        // twice the rebuild waves (12 waves, 3 per SIMD): 4-byte columns of 256-byte
        // tiles (8-byte columns of 512-byte tiles spill in the hash role)
        if (a.e == 1) return launch_vr_ws_t<16, 1, false, 8, 256, 1, 4>(a, s);
        if (a.e == 2) return launch_vr_ws_t<16, 2, false, 8, 256, 1, 4>(a, s);
        if (a.e == 3) return launch_vr_ws_t<16, 3, false, 8, 256, 1, 4>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, false, 8, 256, 1, 4>(a, s);
        return false;
    }
#endif
    if (a.k == 16 && (v == 0 || v == 210 || v == 215 || v == 216)) {
        // RS(16+4)-shaped GET: 8 stripes, 256-byte tiles; rebuilds with 8-byte columns
        // (16-byte columns spill: 16 survivors x 2 tiles beside 32-64 generic products).
        if (a.sums_out != nullptr && ((v == 0 && a.e == 1) || v == 216)) {
            // Heal (17..20 hashed rows): 8 stripes per workgroup, pair-form hash waves
            // padded to whole waves (e.g. heal 2: 288 -> 320 threads) beside 2-4 rebuild
            // waves with 8-byte columns; e >= 2 reads the rebuild tables with scalar loads
            // (the VGPR copy spills).  Product default for heal 1 only: 0.535 vs 0.785 ms
            // (first generation) on 2048 x 1 MiB; heal 2/3/4 measured 0.967/1.31/1.58 vs
            // 0.946/1.13/1.31 ms (2 rebuild waves are the bound), diagnostics 216
            // (profiles/r02/get_ab.txt)
            if (a.e == 1) return launch_vr_ws_t<16, 1, true, 8, 256, 1, 8, false, false>(a, s);
#if ZS3_DIAG
            if (a.e == 2) return launch_vr_ws_t<16, 2, true, 8, 128, 1, 8, false, false>(a, s);
            if (a.e == 3) return launch_vr_ws_t<16, 3, true, 8, 128, 1, 8, false, true>(a, s);
            if (a.e == 4) return launch_vr_ws_t<16, 4, true, 8, 128, 1, 8, false, true>(a, s);
#endif
            return false;
        }
        if (a.sums_out != nullptr) {
#if ZS3_DIAG
            // Heal (18 / 20 hashed rows): 2*8*18 pair-form threads are not whole waves,
            // so the hash role runs in quad form (padded to 9 / 10 waves) beside 4
            // rebuild waves.  Measured slower than the first-generation kernel on
            // 2048 x 1 MiB (heal 2: 1.29 vs 0.95 ms, heal 4: 2.86 vs 1.31 ms; 13 waves
            // leave 128 VGPRs), so opt-in only (variant 215).
            if (v == 215) {
                if (a.e == 2) return launch_vr_ws_t<16, 2, true, 8, 256, 1, 8, true>(a, s);
                if (a.e == 4) return launch_vr_ws_t<16, 4, true, 8, 256, 1, 8, true>(a, s);
            }
#endif
            return false;
        }
        if (v == 215) return false;
#if ZS3_DIAG
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
#endif
        if (a.e == 0) return launch_vr_ws_t<16, 0, false, 8, 256, 2>(a, s);
#if ZS3_DIAG
        if (a.e == 2) return launch_vr_ws_t<16, 2, false, 8, 256, 1, 8>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, false, 8, 256, 1, 8>(a, s);
#endif
        return false;
    }
    if (a.k != 8) return false;
    if (a.sums_out != nullptr) {
        // heal (10 hashed rows): 8-byte rebuild columns and 128-byte tiles keep the
        // 9-wave workgroup inside 168 VGPRs (1.50 -> 1.25 ms, 1 data + 1 parity)
        // (scalar coefficient tables, variant 216: 1.28 -> 1.18 ms on 4096 x 1 MiB,
        // profiles/r02/get_ab.txt)
        if ((v == 0 || v == 216) && a.e == 1) return launch_vr_ws_t<8, 1, true, 16, 128, 2, 8, false, true, 4>(a, s);
        if (a.e != 2) return false;
        if (v == 0 || v == 216) return launch_vr_ws_t<8, 2, true, 16, 128, 2, 8, false, true, 4>(a, s);
#if ZS3_DIAG
        if (v == 212) return launch_vr_ws_t<8, 2, true, 16, 128, 2, 8>(a, s);
#endif
#if ZS3_DIAG
        if (v == 213) return launch_vr_ws_t<8, 2, true, 16, 256, 1, 8>(a, s);
#endif
        return false;
    }
    switch (v) {
        case 0:
        case 210:
            if (a.e == 0) return launch_vr_ws_t<8, 0, false, 16, 256, 2>(a, s);
            if (a.e == 1) return launch_vr_ws_t<8, 1, false, 16, 256, 2>(a, s);
            if (a.e == 2) return launch_vr_ws_t<8, 2, false, 16, 256, 2>(a, s);
            // rebuild 3/4: 8-byte columns (8 rebuild waves, scalar tables): 4096 x 1 MiB
            // 1.27 / 1.42 ms vs 1.35 / 1.58 with 16-byte columns (get_ab_waves.jsonl);
            // batched scalar tables: 1.34 vs 1.40 ms for rebuild 4
            if (v == 0 && a.e == 3) return launch_vr_ws_t<8, 3, false, 16, 256, 1, 8, false, true, 4>(a, s);
            if (v == 0 && a.e == 4) return launch_vr_ws_t<8, 4, false, 16, 256, 1, 8, false, true, 4>(a, s);
#if ZS3_DIAG
            if (a.e == 3) return launch_vr_ws_t<8, 3, false, 16, 256, 1>(a, s);
            if (a.e == 4) return launch_vr_ws_t<8, 4, false, 16, 256, 1>(a, s);
#endif
            return false;
#if ZS3_DIAG
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
#endif
        default:
            return false;
    }
}

}  // namespace zs3k
