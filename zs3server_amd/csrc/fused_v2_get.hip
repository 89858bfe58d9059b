// fused_v2_get.hip — GET / heal dispatch onto the warp-specialised k_vr_ws instances
// (templates and named shapes in fused_v2.hpp): the product defaults.
// Replaces the arithmetic of parallelReader + streamingBitrotReader.ReadAt
// (cmd/erasure-decode.go:165-179, cmd/bitrot-streaming.go:171-186),
// Erasure.DecodeDataBlocks (cmd/erasure-coding.go:96-109) and Erasure.Heal
// (cmd/erasure-decode.go:287-332) for one batch of stripes.
#include "fused_v2.hpp"
#include "vr_quad.hpp"

namespace zs3k {

// Product GET / heal instances by shape, erasure count e and heal (sums of the rebuilt
// rows); false = no warp-specialised instance (the caller falls back).
static bool launch_vr_ws_default(const VrArgs& a, hipStream_t s) {
    const bool heal = a.sums_out != nullptr;
    if (a.k == 4) {
        // RS(4+2)- / RS(4+4)-shaped: quad-form hash waves, 8 stripes, one wave of each kind
        // per SIMD (the 8 192 chains of a 2048-object batch are latency-bound: verify 0.63 ->
        // 0.44 ms over the pair form).  Verify only: 256-byte tiles, 4 of prefetch.
        // Rebuild / heal (round 4, diagnostics 270-272): 1 KiB tiles, so each chain runs 32
        // packets between barriers instead of 8, as config 2's encode: RS(4+2) 2048 x 1 MiB
        // heal 2 0.85 -> 0.63-0.70 ms, RS(4+4) 4096 x 1 MiB rebuild 2 / 4 1.45 / 2.27 ->
        // 1.21 / 1.78, heal 2 / 3 1.68 / 2.27 -> 1.24 / 1.65 (4 of prefetch), heal 4 2.69
        // -> 1.92 (2 of prefetch: the 4-deep instance measured 2.19)
        // (profiles/r04/get_ab_k4.jsonl, mean of two rounds)
        if (heal) {
            if (a.e == 1) return launch_vr_ws_t<4, 1, true, shape::K4Quad<1024, 4>>(a, s);
            if (a.e == 2) return launch_vr_ws_t<4, 2, true, shape::K4Quad<1024, 4>>(a, s);
            if (a.e == 3) return launch_vr_ws_t<4, 3, true, shape::K4Quad<1024, 4>>(a, s);
            if (a.e == 4) return launch_vr_ws_t<4, 4, true, shape::K4Quad<1024, 2>>(a, s);
            return false;
        }
        if (a.e == 0) return launch_vr_ws_t<4, 0, false, shape::K4Quad<256, 4>>(a, s);
        if (a.e == 1) return launch_vr_ws_t<4, 1, false, shape::K4Quad<1024, 4>>(a, s);
        if (a.e == 2) return launch_vr_ws_t<4, 2, false, shape::K4Quad<1024, 4>>(a, s);
        if (a.e == 3) return launch_vr_ws_t<4, 3, false, shape::K4Quad<1024, 4>>(a, s);
        if (a.e == 4) return launch_vr_ws_t<4, 4, false, shape::K4Quad<1024, 4>>(a, s);
        return false;
    }
    if (a.k == 16) {
        // rebuild 4 / heal 4 (round 5): the rebuild split over survivor quads, each wave's
        // 16 coefficient tables held for the launch (vr_quad.hpp; 4-5 % over the k_vr_ws
        // instances below, which serve every other batch; diagnostics 440 = those instead)
        if (a.e == 4 && !(ZS3_DIAG && (a.variant == 440 || (a.variant >= 442 && a.variant <= 447))) &&
            launch_vr_quad_product(a, s)) {
            note_kernel(KERNEL_VR_QUAD);
            return true;
        }
#if ZS3_DIAG
        if (a.variant == 442 && a.e == 4 && launch_vr_quad<shape::Quad16Prio0>(a, s)) return note_kernel(KERNEL_VR_QUAD), true;
        if (a.variant == 443 && a.e == 4 && launch_vr_quad<shape::Quad16LateRead>(a, s)) return note_kernel(KERNEL_VR_QUAD), true;
        if (a.variant == 444 && a.e == 4 && launch_vr_quad<shape::Quad16OneArray>(a, s)) return note_kernel(KERNEL_VR_QUAD), true;
        if (a.variant == 445 && a.e == 4 && launch_vr_quad<shape::Quad16NoSwz>(a, s)) return note_kernel(KERNEL_VR_QUAD), true;
        // 446: both instances on Quad16 (heal in the linear workgroup order of round 5)
        if (a.variant == 446 && a.e == 4 && launch_vr_quad<shape::Quad16>(a, s)) return note_kernel(KERNEL_VR_QUAD), true;
        if (a.variant == 447 && a.e == 4 && launch_vr_quad<shape::Quad16P2>(a, s)) return note_kernel(KERNEL_VR_QUAD), true;
#endif
        if (!heal) {
            // verify only: 8 stripes, 256-byte tiles, two tiles of survivor prefetch.
            // Rebuild, scalar coefficient tables: e = 1, 2 with 4-byte rebuild columns
            // (8 rebuild waves beside 4 hash waves), survivors two tiles ahead; e = 3, 4
            // with 8-byte columns of 512-byte tiles (8 rebuild waves), tables in
            // double-buffered batches.  2048 x 1 MiB: rebuild 1/2/3/4
            // 0.463/0.525/0.620/0.699 ms vs 0.492/0.544/0.622/0.741 for the round-2
            // instances (diagnostics 242; profiles/r03/get_ab_rs164_vr16*.jsonl, variants
            // 250 / 256)
            if (a.e == 0) return launch_vr_ws_t<16, 0, false, shape::K16Verify>(a, s);
            if (a.e == 1) return launch_vr_ws_t<16, 1, false, shape::K16Rebuild12>(a, s);
            if (a.e == 2) return launch_vr_ws_t<16, 2, false, shape::K16Rebuild12>(a, s);
            if (a.e == 3) return launch_vr_ws_t<16, 3, false, shape::K16Rebuild34>(a, s);
            if (a.e == 4) return launch_vr_ws_t<16, 4, false, shape::K16Rebuild34>(a, s);
            return false;
        }
        // heal 1-4: 8-byte rebuild columns of 384-byte tiles (6 rebuild waves beside 5
        // pair-form hash waves padded to whole waves), batched scalar tables.  2048 x
        // 1 MiB: heal 1/2/3/4 0.501/0.573/0.652/0.759 ms vs 0.525/0.816/0.945/1.073 for
        // the round-2 instances (128-byte tiles, 4-byte columns; diagnostics 242)
        // (variant 259, profiles/r03/get_ab_rs164_vr16*.jsonl)
        if (a.e == 1) return launch_vr_ws_t<16, 1, true, shape::K16Heal>(a, s);
        if (a.e == 2) return launch_vr_ws_t<16, 2, true, shape::K16Heal>(a, s);
        if (a.e == 3) return launch_vr_ws_t<16, 3, true, shape::K16Heal>(a, s);
        if (a.e == 4) return launch_vr_ws_t<16, 4, true, shape::K16Heal>(a, s);
        return false;
    }
    if (a.k == 12) {
        // (UA instances serve 16-byte-aligned rows too: RS(12+4) blocks of 12 * 16 * j
        // bytes, round 4; before, those fell back to the first-generation kernel)
        // RS(12+4) on 1 MiB blocks (the 16-drive default; S = 87 382, unaligned rows):
        // the RS(16+4) shapes in UA mode (round 3) instead of a survivor-verify hash launch
        // + the reconstruct kernel + a heal hash launch: 4096 x 1 MiB rebuild 2 1.77 ->
        // 1.48 ms, heal 2 2.09 -> 1.44 ms (profiles/r03/bench_paths_get_ua.jsonl).  Verify
        // only stays on the stripe-mode hash launch (0.77 vs 0.87 ms).
        // Every e: 8-byte rebuild columns of 512-byte tiles with batched scalar tables
        // (diagnostics 264): 4096 x 1 MiB rebuild 1/2/3 1.35/1.46/1.51 -> 1.21/1.30/1.31 ms,
        // heal 1/2/3/4 1.28/1.43/1.61/1.78 -> 1.25/1.37/1.50/1.63 (rebuild 4 1.55 vs 1.58);
        // the RS(16+4) shapes they replace (4-byte columns for rebuild 1-2, 384-byte heal
        // tiles) and 267 (256-byte tiles) are in profiles/r03/get_ab_rs124.jsonl.  Survivor
        // loads are temporal in UA mode (launch_vr_ws_t): rebuild 1/2/3/4 -> 1.17/1.18/
        // 1.15/1.43 ms, heal 1/2/3/4 -> 1.14/1.26/1.43/1.60 (get_ab_rs124_temporal.jsonl)
        if (a.e < 1 || a.e > 4) return false;
        if (!heal) {
            if (a.e == 1) return launch_vr_ws_t<12, 1, false, shape::Wide512<true>>(a, s);
            if (a.e == 2) return launch_vr_ws_t<12, 2, false, shape::Wide512<true>>(a, s);
            if (a.e == 3) return launch_vr_ws_t<12, 3, false, shape::Wide512<true>>(a, s);
            return launch_vr_ws_t<12, 4, false, shape::Wide512<true>>(a, s);
        }
        if (a.e == 1) return launch_vr_ws_t<12, 1, true, shape::Wide512<true>>(a, s);
        if (a.e == 2) return launch_vr_ws_t<12, 2, true, shape::Wide512<true>>(a, s);
        if (a.e == 3) return launch_vr_ws_t<12, 3, true, shape::Wide512<true>>(a, s);
        return launch_vr_ws_t<12, 4, true, shape::Wide512<true>>(a, s);
    }
    if (a.k != 8) return false;
    if (heal) {
        // RS(8+4) heal 1-2 (9-10 hashed rows): 8-byte rebuild columns and 128-byte tiles
        // keep the 9-wave workgroup inside 168 VGPRs (1.50 -> 1.25 ms, 1 data + 1 parity);
        // scalar coefficient tables in batches (1.28 -> 1.18 ms on 4096 x 1 MiB,
        // profiles/r02/get_ab.txt, get_ab_bt.jsonl).
        // Heal 3-4: padded pair-form hash waves (11 / 12 hashed rows x 16 stripes) beside
        // 4 rebuild waves with 16-byte columns of 256-byte tiles, batched scalar tables;
        // 4096 x 1 MiB: 1.34 / 1.51 ms vs 1.40 / 1.61 for the round-2 instances (8-byte
        // columns of 128-byte tiles, diagnostics 232) (variant 262,
        // profiles/r03/get_ab_r03_84.jsonl)
        if (a.e == 1) return launch_vr_ws_t<8, 1, true, shape::K8Heal12>(a, s);
        if (a.e == 2) return launch_vr_ws_t<8, 2, true, shape::K8Heal12>(a, s);
        if (a.e == 3) return launch_vr_ws_t<8, 3, true, shape::K8Heal34>(a, s);
        if (a.e == 4) return launch_vr_ws_t<8, 4, true, shape::K8Heal34>(a, s);
        return false;
    }
    // RS(8+4) GET: 16 stripes, 256-byte tiles, verify-only or rebuild 1-2 with 16-byte
    // columns and two tiles of prefetch; rebuild 3/4 with 8-byte columns (8 rebuild
    // waves, batched scalar tables): 4096 x 1 MiB 1.27 / 1.42 ms vs 1.35 / 1.58 with
    // 16-byte columns (profiles/r02/get_ab_waves.jsonl), batching 1.34 vs 1.40 ms for
    // rebuild 4
    if (a.e == 0) return launch_vr_ws_t<8, 0, false, shape::K8Get>(a, s);
    if (a.e == 1) return launch_vr_ws_t<8, 1, false, shape::K8Get>(a, s);
    if (a.e == 2) return launch_vr_ws_t<8, 2, false, shape::K8Get>(a, s);
    if (a.e == 3) return launch_vr_ws_t<8, 3, false, shape::K8Rebuild34>(a, s);
    if (a.e == 4) return launch_vr_ws_t<8, 4, false, shape::K8Rebuild34>(a, s);
    return false;
}

// v: 0 = the product shapes (the diagnostics build's GET variants change a product
// shape's memory policy or layout inside launch_vr_ws_t, with a.variant set)
bool launch_vr_ws(int v, const VrArgs& a, hipStream_t s) {
    return v == 0 && launch_vr_ws_default(a, s);
}

}  // namespace zs3k
