// fused_v2.hip — second-generation fused Split + Encode + HighwayHash-256 kernel.
//
// Replaces the arithmetic of Erasure.EncodeData (cmd/erasure-coding.go:77-91) plus
// the k+m streamingBitrotWriter sums (cmd/bitrot-streaming.go:43-65) for the
// dyadic RS shapes (m in {2,4}, m | k: RS(8+4), RS(4+2), RS(16+4), ...).
//
// Same work decomposition as k_encode_hash (kernels.hip): G whole stripes per
// workgroup, one HighwayHash lane per thread (a quad per shard row), one CW-byte
// column per thread for the encode, tiles of T bytes per shard row staged in LDS.
// What changes is the memory pipeline, measured on MI355X (scripts/sweep_variants.py):
//  * vmcnt is one in-order counter for loads AND stores, so the old order
//    (store parity(i), then load tile i+1) made the wait for tile i+1's data also
//    wait for tile i's store acknowledgements.  Here the loads of tile i+PF are
//    issued BEFORE the parity stores of tile i, so the wait at step i+1 leaves the
//    stores in flight.
//  * every LDS read of a tile's hash words is issued before the first HighwayHash
//    update (one lgkmcnt wait per tile instead of one per two packets).
//  * NBUF = 2 LDS tiles: one barrier per step.
//  * full tiles run a branch-free body; the ragged tail tile (S % T) is peeled.
#include "fused_v2.hpp"

namespace zs3k {

// Only instances that scripts/check_async_loads.py proves clean are compiled (wider
// columns and deeper prefetch on the other shapes make hipcc copy or re-use
// registers of in-flight loads).
//
// Product defaults (variant 0), by shape and batch size n (scripts/sweep_sizes.py,
// profiles/r02/sweep_sizes_*.txt: the fastest launch at each n, so throughput grows
// monotonically with the batch).  Data loads and parity stores of the 16-stripe
// kernels carry the non-temporal cache policy (NTM = 3: each byte is touched once;
// +2-3 % over the default policy at 4096-65536 stripes, profiles/r02/sweep_sizes_nt*.txt).
// The grid is one workgroup per CU: the stripes per workgroup G are the smallest that
// keep ceil(n / G) <= 256 (a second, partial round of workgroups costs a whole
// workgroup time: profiles/r02/sweep_cliffs.jsonl).
//  RS(8+4)  n > 2048:  k_ehx_ws G = 16 (variant 151: 6 pair-form hash waves + 6 encode
//                      waves with 16-byte columns, encode waves at s_setprio 1, nt policy;
//                      one workgroup of 12 waves per CU)
//           128 < n <= 2048: G = 4 with quad-form hash waves, 1 KiB tiles, two tiles
//                      of prefetch, 256-VGPR budget (variant 199, round 3; replaced the
//                      8-stripe kernel above 1024 and the first-generation kernel
//                      below); n <= 128: the small-batch latency path (kernels.hip)
//  RS(16+4) n > 1024:  k_ehx_ws G = 8 (variant 162: 5 pair-form hash waves + 6 encode
//                      waves with 8-byte buffer-addressed columns, nt policy, data rows
//                      written to LDS before the encode (EP = 2): 0.577 -> 0.590 of HBM
//                      spec at 8192 stripes, profiles/r02/ab_encode_ep.jsonl)
//           n <= 1024: G = 4 with quad-form hash waves, nt loads and stores (variant
//                      125; 1-2 % over 121)
//  RS(4+2)  n <= 2048: k_ehx_ws G = 4, quad-form hash waves, nt stores (variant 116;
//                      BASELINE config 2: the hash chains' latency sets the pace); nt loads
//                      too from 1024 stripes (variant 117: config 2 0.410 -> 0.400 ms)
//           n >  2048: k_ehx_ws G = 16, pair-form hash waves, nt policy (variant 115)
template <int K, int M>
static int launch_ehx_default(const EncArgs& a, hipStream_t s) {
    const int64_t n = a.n_blocks;
    if constexpr (K == 8 && M == 4) {
        // n > 2048: 16 stripes, 384-byte tiles, 4 pair-form hash + 6 encode waves, nt policy;
        // round 4: buffer-addressed loads and stores (BUF) and the conflict-free LDS row
        // stride (TSP = 1: SQ_LDS_BANK_CONFLICT 20 % -> 0 % of LDS cycles), diagnostics 302:
        // 4.98 / 4.84 -> 4.79 ms on 16384 x 1 MiB pairs of runs (profiles/r04/r04_ab1.jsonl)
        if (n > 2048)
            return launch_ws<K, M, shape::Rs84Bulk>(a, s) ? PATH_WS : PATH_NONE;
        // up to 2048 stripes (round 3, variant 199): 4 stripes per workgroup, quad-form
        // hash waves (3) beside 4 encode waves, 1 KiB tiles, two tiles of prefetch, and
        // the 2-waves-per-SIMD register budget (7-wave workgroups: no spills, where the
        // 168-VGPR budget spilled 26): 256 / 512 / 640 / 1024 / 1536 / 2048 stripes
        // 0.275 / 0.285 / 0.281 / 0.336 / 0.611 / 0.676 ms vs 0.32 / 0.42 / 0.47 / 0.555 /
        // 0.684 / 0.73-0.78 for the latency path, first-generation and 8-stripe kernels
        // (profiles/r03/ab_rs84_mid_batches.jsonl, sweep_rs84_sizes199.jsonl)
        return launch_ws<K, M, shape::Rs84Mid>(a, s) ? PATH_WS : PATH_NONE;
    } else if constexpr (K == 16 && M == 4) {
        if (n > 4 * 256)
            return launch_ws<K, M, shape::Rs164Bulk>(a, s) ? PATH_WS : PATH_NONE;
        return launch_ws<K, M, shape::Quad512>(a, s) ? PATH_WS : PATH_NONE;
    } else if constexpr (K == 12 && M == 4) {
        // RS(12+4), the 16-drive default (cmd/format-erasure.go:870-881), at shard sizes
        // that are multiples of 16; 1 MiB blocks (S = 87 382) take launch_ehx_ua.  Above
        // 1024 stripes the unaligned-row product shape (8 stripes of 8-byte columns of
        // 512-byte tiles, L2 prefetch two tiles ahead) with the conflict-free LDS stride
        // (diagnostics 330): 4 096 x (12 x 87 392 bytes) 1.42-1.51 -> 1.23 ms over the
        // RS(16+4) shape it had (profiles/r04/abl_rs124_al.jsonl); 4 stripes with
        // quad-form hash waves up to 1024.
        if (n > 4 * 256)
            return launch_ws<K, M, shape::Rs124AlignedBulk>(a, s) ? PATH_WS : PATH_NONE;
        return launch_ws<K, M, shape::Quad512>(a, s) ? PATH_WS : PATH_NONE;
    } else if constexpr (K == 4 && M == 4) {
        // RS(4+4), the 8-drive default: the RS(8+4) shape (16 stripes, 16-byte columns,
        // pair-form hash waves) for large batches, the RS(4+2) config-2 shape (4 stripes,
        // quad-form hash waves, 4 tiles of prefetch) below.  Round 5: with the conflict-free
        // LDS row stride (SQ_LDS_BANK_CONFLICT 33.5 M per launch -> 0 at equal time,
        // diagnostics 400 = the round-4 instance, profiles/r05/ab_enc.jsonl)
        if (n > 8 * 256)
            return launch_ws<K, M, shape::Rs44Bulk>(a, s) ? PATH_WS : PATH_NONE;
        return launch_ws<K, M, shape::QuadSmall<3>>(a, s) ? PATH_WS : PATH_NONE;
    } else if constexpr (K == 4 && M == 2) {
        // config 2 (1024 objects, 6 144 chains: the chain latency sets the pace): 2 KiB
        // tiles, so each chain runs 64 packets between barriers (0.397 -> 0.364 ms over
        // 512-byte tiles, profiles/r03/ab_config2_tiles.jsonl)
        if (n >= 1024 && n <= 8 * 256)
            return launch_ws<K, M, shape::Config2>(a, s) ? PATH_WS : PATH_NONE;
        if (n <= 8 * 256)
            return launch_ws<K, M, shape::QuadSmall<2>>(a, s) ? PATH_WS : PATH_NONE;
        return launch_ws<K, M, shape::PairG16>(a, s) ? PATH_WS : PATH_NONE;
    }
    return PATH_NONE;
}

int launch_ehx_ua(const EncArgs& a, hipStream_t s) {
    if (a.k == 12 && a.m == 4) {
        // n > 1024 (round 3, diagnostics 179): 8 stripes of 8-byte columns of 512-byte
        // tiles (4 hash + 8 encode waves: one hash and two encode waves on every SIMD,
        // where 384-byte tiles left two SIMDs with one encode wave), data rows written to
        // LDS before the encode, and the hash waves touching every line of the data rows
        // two tiles ahead (PFD = 2) so the unaligned row loads of the encode waves hit L2:
        // 4096 / 16384 x 1 MiB 1.72-1.79 / 6.72 -> 1.41 / 5.48 ms
        // (profiles/r03/ab_rs124_pfd.jsonl; 196 = no prefetch 1.54-1.59 / 5.98-6.01).
        // Round 4 (diagnostics 391): 4 stripes of 1 KiB tiles, whose memory pattern alone
        // is 7 % faster (386 vs 338, profiles/r04/mem_rs124.jsonl), with 4 quad-form hash
        // waves doing the L2 prefetch and 4 encode waves of 16-byte columns (256-VGPR
        // budget): 1.41 -> 1.40 ms / 5.59 -> 5.56 ms at 4096 / 16384 x 1 MiB on the same
        // box, 1-2 % over two boxes (sweep_rs124_1k.jsonl, sweep_rs124_1k_b.jsonl)
        if (a.n_blocks > 4 * 256)
            return launch_ws<12, 4, shape::Rs124Ua1K>(a, s) ? PATH_WS : PATH_NONE;
        return launch_ws<12, 4, shape::Rs124UaSmall>(a, s) ? PATH_WS : PATH_NONE;
    }
    return PATH_NONE;
}

int launch_ehx(int v, const EncArgs& a, hipStream_t s) {
    if (v == 0) {
        if (a.k == 8 && a.m == 4) return launch_ehx_default<8, 4>(a, s);
        if (a.k == 4 && a.m == 2) return launch_ehx_default<4, 2>(a, s);
        if (a.k == 16 && a.m == 4) return launch_ehx_default<16, 4>(a, s);
        if (a.k == 12 && a.m == 4) return launch_ehx_default<12, 4>(a, s);
        if (a.k == 4 && a.m == 4) return launch_ehx_default<4, 4>(a, s);
        return PATH_NONE;
    }
#if ZS3_DIAG
    if (launch_ehx_diag(v, a, s)) return PATH_WS;
#endif
    return PATH_NONE;
}

}  // namespace zs3k
