// fused_v2_km.hpp — encode variants of the diagnostics build (A/B and ablation
// instances of k_ehx / k_ehx_ws, measured in profiles/r0*/ and tests/test_gpu_variants.py),
// instantiated once per shape by fused_v2_km{84,42,164}.hip.
#pragma once
#include "fused_v2.hpp"

namespace zs3k {

#if ZS3_DIAG
template <int K, int M>
static bool launch_ehx_km(int v, const EncArgs& a, hipStream_t s) {
    constexpr bool deep = K == 8 && M == 4;
    constexpr bool few = K == 4 && M == 2;  // BASELINE config 2: 1024 objects, latency-bound
    switch (v) {
        case 90: if constexpr (few) return launch_ehx_t<K, M, 8, 4, 2, false, 0, false, 1, false, 83968>(a, s); else return false;
        case 91: if constexpr (few) return launch_ehx_t<K, M, 8, 4, 2, false, 0, true, 1, false, 83968>(a, s); else return false;
        case 92: if constexpr (few) return launch_ehx_t<K, M, 8, 2, 2, false, 0, false, 1, false, 83968>(a, s); else return false;
        case 93: if constexpr (few) return launch_ehx_t<K, M, 8, 4, 2>(a, s); else return false;
        case 94: if constexpr (few) return launch_ehx_t<K, M, 8, 8, 2, false, 0, false, 1, false, 83968>(a, s); else return false;
        case 50: return launch_ehx_t<K, M, 8, 1, 2>(a, s);
        case 51: return launch_ehx_t<K, M, 8, 1, 1>(a, s);
        case 52: if constexpr (deep) return launch_ehx_t<K, M, 8, 2, 2>(a, s); else return false;
        case 53: if constexpr (deep) return launch_ehx_t<K, M, 8, 2, 1>(a, s); else return false;
        case 55: return launch_ehx_t<K, M, 8, 1, 2, true>(a, s);
        case 70: return launch_ehx_t<K, M, 8, 1, 2, false, 0, true>(a, s);
        case 71: if constexpr (deep) return launch_ehx_t<K, M, 8, 2, 2, false, 0, true>(a, s); else return false;
        case 80: if constexpr (deep) return launch_ehx_t<K, M, 8, 1, 2, false, 0, false, 4>(a, s); else return false;
        case 81: if constexpr (deep) return launch_ehx_t<K, M, 8, 1, 1, false, 0, false, 4, false, 83968>(a, s); else return false;
        case 82: return launch_ehx_t<K, M, 8, 1, 2, false, 0, false, 1, true>(a, s);
        case 83: if constexpr (deep) return launch_ehx_t<K, M, 8, 2, 2, false, 0, false, 4>(a, s); else return false;
        case 84: if constexpr (deep) return launch_ehx_t<K, M, 8, 1, 2, false, 0, false, 2>(a, s); else return false;
        case 85: if constexpr (deep) return launch_ehx_t<K, M, 8, 1, 2, false, 0, true, 4>(a, s); else return false;
        case 86: if constexpr (deep) return launch_ehx_t<K, M, 8, 1, 2, false, 1, false, 4>(a, s); else return false;
        case 87: if constexpr (deep) return launch_ehx_t<K, M, 8, 1, 2, false, 2, false, 4>(a, s); else return false;
        case 88: if constexpr (deep) return launch_ehx_t<K, M, 8, 1, 2, false, 3, false, 4>(a, s); else return false;
        case 100: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1>(a, s); else return false;
        case 103: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, true>(a, s); else return false;
        case 102: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true>(a, s); else return false;
        case 109: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1>(a, s); else return false;
        case 108: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 4>(a, s); else return false;
        case 105: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1>(a, s); else return false;
        case 106: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 2>(a, s); else return false;
        case 107: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 3>(a, s); else return false;
        case 104: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, true>(a, s); else return false;
        case 150: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 1>(a, s); else return false;
        case 151: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3>(a, s); else return false;
        case 155: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, true>(a, s); else return false;
        case 153: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 2>(a, s); else return false;
        case 154: if constexpr (deep) return launch_ws_t<K, M, 8, 384, 1, false, false, 0, false, 1, 0, false, 2>(a, s); else return false;
        case 117: if constexpr (few) return launch_ws_t<K, M, 4, 512, 4, false, true, 83968, false, 0, 0, false, 3>(a, s); else return false;
        case 133: if constexpr (deep) return launch_ws_t<K, M, 8, 384, 1, false, false, 0, false, 1, 0, false, 3>(a, s); else return false;
        case 125: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 4, 512, 1, true, true, 0, false, 0, 0, false, 3>(a, s); else return false;
        // RS(16+4) small batches with 16-byte columns on 7-wave workgroups (2 waves per
        // SIMD's register budget), two / one tile of prefetch
        case 126: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 4, 512, 2, true, true, 83968, false, 0, 16, false, 3, false, 0, 0, false, 2>(a, s); else return false;
        case 127: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 4, 512, 1, true, true, 83968, false, 0, 16, false, 3, false, 0, 0, false, 2>(a, s); else return false;
        case 156: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 1>(a, s); else return false;
        case 157: if constexpr (few) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 1>(a, s); else return false;
        case 160: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 2>(a, s); else return false;
        case 161: if constexpr (few) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 2>(a, s); else return false;
        case 163: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 3>(a, s); else return false;
        case 164: if constexpr (few) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 3>(a, s); else return false;
        // L2 prefetch of the data rows PFD tiles ahead by the hash waves (product 151 + PFD)
        case 170: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 0, 2>(a, s); else return false;
        case 171: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 0, 3>(a, s); else return false;
        case 172: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 0, 4>(a, s); else return false;
        case 173: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 0, 6>(a, s); else return false;
        case 174: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 2, false, 0, 3>(a, s); else return false;
        case 175: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 8, 384, 1, true, false, 0, false, 0, 0, false, 3, false, 2, 3>(a, s); else return false;
        // tile / wave-count shapes for RS(8+4) at the product's memory policy (r03)
        case 180: if constexpr (deep) return launch_ws_t<K, M, 8, 768, 1, false, false, 0, false, 1, 0, false, 3>(a, s); else return false;
        case 182: if constexpr (deep) return launch_ws_t<K, M, 8, 768, 1, false, false, 0, false, 1, 8, false, 3>(a, s); else return false;
        case 183: if constexpr (deep) return launch_ws_t<K, M, 8, 512, 2, false, false, 0, false, 1, 0, false, 3>(a, s); else return false;
        case 184: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, true, 1, 0, false, 3>(a, s); else return false;
        case 185: if constexpr (deep) return launch_ws_t<K, M, 16, 256, 1, false, false, 0, false, 1, 0, false, 3>(a, s); else return false;
        case 186: if constexpr (deep) return launch_ws_t<K, M, 8, 512, 1, false, false, 0, false, 1, 0, false, 3>(a, s); else return false;
        // issue priority on the product shape (r03 stamps: the SIMDs holding one hash and
        // two encode waves are the critical path): 191 younger encode wave of each pair at
        // 2 (PM = 2), 192 hash waves at 1 (PM = 3), 193 no priorities, 194 = 191 + WT stamps
        case 191: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 2, 0, false, 3>(a, s); else return false;
        case 192: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 3, 0, false, 3>(a, s); else return false;
        case 193: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 0, 0, false, 3>(a, s); else return false;
        case 194: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, true, 2, 0, false, 3>(a, s); else return false;
        // RS(8+4) mid batches (641-1024 stripes run the first-generation kernel): 4 stripes
        // per workgroup with quad-form hash waves, as config 2 / RS(16+4) <= 1024
        case 187: if constexpr (deep) return launch_ws_t<K, M, 4, 512, 1, false, true, 0, false, 0, 0, false, 3>(a, s); else return false;
        case 188: if constexpr (deep) return launch_ws_t<K, M, 4, 512, 2, false, true, 83968, false, 0, 0, false, 3>(a, s); else return false;
        case 189: if constexpr (deep) return launch_ws_t<K, M, 4, 1024, 2, false, true, 83968, false, 0, 0, false, 3>(a, s); else return false;
        // the same with the register budget of 2 waves per SIMD (7-waves workgroups)
        case 197: if constexpr (deep) return launch_ws_t<K, M, 4, 512, 1, false, true, 83968, false, 0, 0, false, 3, false, 0, 0, false, 2>(a, s); else return false;
        case 198: if constexpr (deep) return launch_ws_t<K, M, 4, 512, 2, false, true, 83968, false, 0, 0, false, 3, false, 0, 0, false, 2>(a, s); else return false;
        case 199: if constexpr (deep) return launch_ws_t<K, M, 4, 1024, 2, false, true, 83968, false, 0, 0, false, 3, false, 0, 0, false, 2>(a, s); else return false;
        // config 2 (latency-bound chains): longer tiles = fewer per-step barriers and LDS
        // read latencies on the chain's critical path
        case 177: if constexpr (few) return launch_ws_t<K, M, 4, 1024, 4, false, true, 83968, false, 0, 0, false, 3>(a, s); else return false;
        case 178: if constexpr (few) return launch_ws_t<K, M, 4, 1024, 2, false, true, 83968, false, 0, 0, false, 3>(a, s); else return false;
        case 179: if constexpr (few) return launch_ws_t<K, M, 4, 2048, 2, false, true, 83968, false, 0, 0, false, 3>(a, s); else return false;
        case 176: if constexpr (few) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 0, 3>(a, s); else return false;
        case 168: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 8>(a, s); else return false;
        case 169: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 9>(a, s); else return false;
        // RS(16+4) product 162 + L2 prefetch by the hash waves 2 / 3 tiles ahead (round 3)
        case 158: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 8, 384, 1, true, false, 0, false, 0, 0, false, 3, false, 2, 2>(a, s); else return false;
        case 159: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 8, 384, 1, true, false, 0, false, 0, 0, false, 3, false, 2, 3>(a, s); else return false;
        case 162: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 8, 384, 1, true, false, 0, false, 0, 0, false, 3, false, 2>(a, s); else return false;
        case 152: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, false, false, 0, false, 1>(a, s); else return false;
        case 140: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, true>(a, s); else return false;
        case 141: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 0, 0, true>(a, s); else return false;
        case 130: if constexpr (deep) return launch_ws_t<K, M, 8, 384, 1, false, false, 0, false, 1>(a, s); else return false;
        case 131: if constexpr (deep) return launch_ws_t<K, M, 4, 512, 2, false, true>(a, s); else return false;
        case 132: if constexpr (deep) return launch_ws_t<K, M, 2, 512, 2, false, true>(a, s); else return false;
        case 120: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 8, 384, 1, true>(a, s); else return false;
        case 122: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 8, 384, 1, true, false, 0, false, 0, 0, false, 3>(a, s); else return false;
        case 123: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 8, 384, 1, true, false, 0, false, 0, 0, false, 2>(a, s); else return false;
        case 124: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 4, 512, 1, true, true, 0, false, 0, 0, false, 3>(a, s); else return false;
        case 121: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 4, 512, 1, true, true>(a, s); else return false;
        case 110: if constexpr (few) return launch_ws_t<K, M, 4, 512, 2, false, true, 83968>(a, s); else return false;
        case 111: if constexpr (few) return launch_ws_t<K, M, 4, 512, 4, false, true, 83968>(a, s); else return false;
        case 112: if constexpr (few) return launch_ws_t<K, M, 4, 256, 4, false, true, 83968>(a, s); else return false;
        case 113: if constexpr (few) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1>(a, s); else return false;
        case 114: if constexpr (few) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 2>(a, s); else return false;
        case 115: if constexpr (few) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3>(a, s); else return false;
        case 116: if constexpr (few) return launch_ws_t<K, M, 4, 512, 4, false, true, 83968, false, 0, 0, false, 2>(a, s); else return false;
        case 61: if constexpr (deep) return launch_ehx_t<K, M, 8, 1, 2, false, 1>(a, s); else return false;
        case 64: if constexpr (deep) return launch_ehx_t<K, M, 8, 2, 2, false, 1>(a, s); else return false;
        // round 4: conflict-free LDS rows (TSP = 1), buffer-addressed
        // encode columns (no VGPR spills) with one / two tiles of register prefetch
        case 300: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, false, 1, 0, false, 3, false, 0, 0, false, 3, 1>(a, s); else return false;
        case 301: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, true, false, 0, false, 1, 0, false, 3, false, 0, 0, false, 3, 1>(a, s); else return false;
        case 302: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 3, false, 0, 0, false, 3, 1>(a, s); else return false;
        case 303: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, true, false, 0, false, 0, 0, false, 3, false, 0, 0, false, 3, 1>(a, s); else return false;
        case 304: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, true, false, 0, false, 1, 0, false, 3, false, 2, 0, false, 3, 1>(a, s); else return false;
        case 305: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, true, false, 0, false, 1, 0, false, 3, false, 0, 0, false, 3, 0>(a, s); else return false;
        case 306: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, true, false, 0, true, 1, 0, false, 3, false, 0, 0, false, 3, 1>(a, s); else return false;
        case 307: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, false, false, 0, true, 1, 0, false, 3, false, 0, 0, false, 3, 1>(a, s); else return false;
        // energy / pipeline ablations of 302 (timing only): no hash arithmetic, no GF
        // arithmetic, neither
        case 310: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 3, false, 0, 0, false, 3, 1, 1>(a, s); else return false;
        case 311: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 0>(a, s); else return false;
        case 312: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 1>(a, s); else return false;
        // pure-memory ablations (no GF, no hash arithmetic) of other shapes / policies
        case 320: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 1>(a, s); else return false;
        case 321: if constexpr (deep) return launch_ws_t<K, M, 16, 256, 1, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 1>(a, s); else return false;
        case 322: if constexpr (deep) return launch_ws_t<K, M, 8, 768, 1, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 1>(a, s); else return false;
        case 323: if constexpr (deep) return launch_ws_t<K, M, 8, 512, 1, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 1>(a, s); else return false;
        case 324: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 0, false, 9, 0, false, 3, 1, 1>(a, s); else return false;
        case 325: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 1, false, 9, 0, false, 3, 1, 1>(a, s); else return false;
        case 326: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 2, false, 9, 0, false, 3, 1, 1>(a, s); else return false;
        case 327: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 3>(a, s); else return false;
        case 328: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 1, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 7>(a, s); else return false;
        case 329: if constexpr (deep) return launch_ws_t<K, M, 16, 384, 2, true, false, 0, false, 1, 0, false, 3, false, 9, 0, false, 3, 1, 7>(a, s); else return false;
        // 1 KiB tiles (the RS(12+4) memory-pattern finding, profiles/r04/mem_rs124.jsonl):
        // 360 / 361 / 362 the memory pattern alone of 4 stripes of 1 KiB tiles with / without
        // the L2 prefetch, 2 stripes of 2 KiB tiles; 363 / 364 the real roles on 4 stripes of
        // 1 KiB tiles with quad-form hash waves issuing the L2 prefetch, 16-byte columns, with /
        // without encode priority; 365 = 363 with 8 stripes of 512-byte tiles
        case 360: if constexpr (deep) return launch_ws_t<K, M, 4, 1024, 1, true, false, 0, false, 1, 16, false, 3, false, 9, 2, false, 3, 1, 7>(a, s); else return false;
        case 361: if constexpr (deep) return launch_ws_t<K, M, 4, 1024, 1, true, false, 0, false, 1, 16, false, 3, false, 9, 0, false, 3, 1, 7>(a, s); else return false;
        case 362: if constexpr (deep) return launch_ws_t<K, M, 2, 2048, 1, true, false, 0, false, 1, 16, false, 3, false, 9, 2, false, 3, 1, 7>(a, s); else return false;
        case 363: if constexpr (deep) return launch_ws_t<K, M, 4, 1024, 1, true, true, 0, false, 1, 16, false, 3, false, 0, 2, false, 2, 1>(a, s); else return false;
        case 364: if constexpr (deep) return launch_ws_t<K, M, 4, 1024, 1, true, true, 0, false, 0, 16, false, 3, false, 0, 2, false, 2, 1>(a, s); else return false;
        case 365: if constexpr (deep) return launch_ws_t<K, M, 8, 512, 1, true, true, 0, false, 1, 16, false, 3, false, 0, 2, false, 2, 1>(a, s); else return false;
        // RS(16+4) encode + sums with the RS(12+4) round-4 recipe: 4 stripes of 768-byte
        // tiles (1 KiB does not fit the LDS), quad-form hash waves issuing the L2 prefetch,
        // 16-byte (366) / 8-byte (367) columns; 368 the product + L2 prefetch + TSP 1
        case 366: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 4, 768, 1, true, true, 0, false, 0, 16, false, 3, false, 2, 2, false, 2, 1>(a, s); else return false;
        case 367: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 4, 768, 1, true, true, 0, false, 0, 8, false, 3, false, 2, 2, false, 3, 1>(a, s); else return false;
        case 368: if constexpr (K == 16 && M == 4) return launch_ws_t<K, M, 8, 384, 1, true, false, 0, false, 0, 0, false, 3, false, 2, 2, false, 3, 1>(a, s); else return false;
        default: return false;
    }
}
#endif  // ZS3_DIAG

}  // namespace zs3k
