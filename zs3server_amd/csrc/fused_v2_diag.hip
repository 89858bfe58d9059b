// fused_v2_diag.hip — encode variants of the diagnostics build (libzs3gpu_diag.so only),
// selected per thread by zs3server_amd.diag(v) / zs3_debug_set_variant.  Each variant is
// a product shape (fused_v2.hpp, namespace shape) with one knob changed, named here; the
// product dispatch is fused_v2.hip.  (Round 5 pruned the ~140 earlier-round candidates:
// their numbers and measurements stay in profiles/r02-r04 and DESIGN.md §4-§12.)
//
//  310 / 311 / 312  RS(8+4) Rs84Bulk timing ablations (output differs): no HighwayHash
//                   arithmetic / no GF arithmetic / neither — the memory pattern alone,
//                   the headline's pattern roof
//  313              Rs84Bulk with per-wave barrier / load-wait stamps (scripts/stamps3.py)
//  400 / 401        the RS(4+4) bulk shape without the conflict-free LDS row stride (PairG16,
//                   the round-4 product) / the RS(16+4) bulk shape without XMAP
//  402              RS(4+4) on the RS(8+4) headline shape (Rs84Bulk)
//  409-414          Rs84Bulk with the region-interleaved workgroup order (ws_group) over 1
//                   (none: the round-4 product) / 2 / 4 / 8 (the product) / 16 / 32 regions
//  401 / 415 / 417  the RS(16+4) bulk shape without XMAP / without TSP / without either
//                   (417 = the round-4 product)
//  416              the RS(12+4) 1 KiB UA shape without XMAP (the round-4 product)
//  418              XMAP 8 on PairG16 (RS(4+4) / RS(4+2) bulk); 419 XMAP 8 on every GEN shape
//  403              the RS(16+4) bulk shape with PM 0 (the encode waves without issue
//                   priority, as before round 5's adoption)
//  (Measured this round and removed: PM 2 / PM 0 on Rs84Bulk, PM 2 on the RS(16+4) bulk
//  shape, PM 1 / temporal loads or stores / L2 prefetch 1 or 3 tiles ahead / XMAP 16 on the
//  RS(12+4) UA shape, the pair-form 8 x 512 UA shape on 1 MiB RS(12+4) with or without
//  XMAP, the LDS-counter hand-off and the L2 prefetch on Rs84Bulk: profiles/r05/
//  ab_prio_enc*.jsonl, ab_ntm124.jsonl, ab_enc3.jsonl, ab_rs124pair.jsonl)
#include "fused_v2.hpp"
#include "ehx_mx.hpp"

namespace zs3k {

#if ZS3_DIAG
namespace shape {
struct Rs84NoHash : Rs84Bulk {
    static constexpr int ABL = 1;
};
struct Rs84NoGf : Rs84Bulk {
    static constexpr int EP = 9;
};
struct Rs84MemOnly : Rs84Bulk {
    static constexpr int EP = 9, ABL = 1;
};
struct Rs84Stamped : Rs84Bulk {
    static constexpr bool WT = true;
};
struct Rs84Pf2 : Rs84Bulk {
    static constexpr int PF = 2;
    static constexpr bool S64 = false;  // (two tiles of registers + S64 spill)
};
struct Rs84Ep1 : Rs84Bulk {
    static constexpr int EP = 1;
};
// round 6: the quad-form hash role without the fused packet runs (hh_update_n)
template <class S>
struct Hf0 : S {
    static constexpr bool HF = false;
};
template <class S>
struct Hf2 : S {
    static constexpr bool HF2 = true;
};
// round 6: RS(12+4) on 1 MiB blocks (S % 16 = 6) with aligned data-row loads realigned
// in registers (ALN, fused_v2.hpp)
struct Rs124Aln : Rs124Ua1K {
    static constexpr int ALN = 6;
};
template <class S>
struct Stamp : S {
    static constexpr bool WT = true;
};
// round 6: 32 stripes of 128-byte tiles: 12 pair-form hash waves + 4 encode waves, so
// every SIMD of the 16-wave workgroup holds three hash waves and one encode wave (the
// 12-wave product puts 2 hash + 1 encode on two SIMDs and 1 + 2 on the others, §14.1)
struct Rs84G32 : Rs84Bulk {
    static constexpr int G = 32, T = 128, WPE = 4;
};
template <class S, int N>
struct Ntm : S {
    static constexpr int NTM = N;
};
template <class S, int N>
struct Pfd : S {
    static constexpr int PFD = N;
};
template <class S>
struct Split64 : S {
    static constexpr bool S64 = true;
};
template <class S>
struct Smk : S {
    static constexpr bool SMK = true;
};
// the product shapes without the 64-bit nibble splits (round 6 adopted S64 for them)
template <class S>
struct Split32 : S {
    static constexpr bool S64 = false;
};
struct Rs124Pfe : Rs124Ua1K {
    static constexpr bool PFE = true;
};
struct Rs124Ua1K8 : Rs124Ua1K {
    static constexpr int CWX = 8, WPE = 3;
};
// round 6: start stagger of the workgroups (STG phases of SLP * 64 cycles)
template <class S, int STG_, int SLP_>
struct Stg : S {
    static constexpr int STG = STG_, SLP = SLP_;
};
}  // namespace shape

bool launch_ehx_diag(int v, const EncArgs& a, hipStream_t s) {
    using namespace shape;
    if (a.k == 8 && a.m == 4) {
        switch (v) {
            case 310: return launch_ws<8, 4, Rs84NoHash>(a, s);
            case 311: return launch_ws<8, 4, Rs84NoGf>(a, s);
            case 312: return launch_ws<8, 4, Rs84MemOnly>(a, s);
            case 313: return launch_ws<8, 4, Rs84Stamped>(a, s);
            case 409: return launch_ws<8, 4, XMap<Rs84Bulk, 0>>(a, s);
            case 410: return launch_ws<8, 4, XMap<Rs84Bulk, 2>>(a, s);
            case 411: return launch_ws<8, 4, XMap<Rs84Bulk, 4>>(a, s);
            case 412: return launch_ws<8, 4, XMap<Rs84Bulk, 8>>(a, s);
            case 413: return launch_ws<8, 4, XMap<Rs84Bulk, 16>>(a, s);
            case 414: return launch_ws<8, 4, XMap<Rs84Bulk, 32>>(a, s);
            // round 6: the balanced mixed-role kernel (ehx_mx.hpp), G = 16 / 8 / 32, stamped,
            // hash reads before the encode
            case 450: return launch_mx<8, 4, Mix<16>>(a, s);
            case 451: return launch_mx<8, 4, Mix<8>>(a, s);
            case 452: return launch_mx<8, 4, Mix<32>>(a, s);
            case 453: return launch_mx<8, 4, MixWT<Mix<16>>>(a, s);
            case 454: return launch_mx<8, 4, MixWT<Mix<8>>>(a, s);
            case 455: return launch_mx<8, 4, MixWT<Mix<32>>>(a, s);
            case 456: return launch_mx<8, 4, MixRd1<Mix<16>>>(a, s);
            case 457: return launch_mx<8, 4, MixRd1<Mix<32>>>(a, s);
            // round 6: issue priority by SIMD mix (fused_v2.hpp PM 5-8) and PM 3 retested
            // under the XCD-region order
            case 460: return launch_ws<8, 4, Pm<Rs84Bulk, 3>>(a, s);
            case 461: return launch_ws<8, 4, Pm<Rs84Bulk, 5>>(a, s);
            case 462: return launch_ws<8, 4, Pm<Rs84Bulk, 6>>(a, s);
            case 463: return launch_ws<8, 4, Pm<Rs84Bulk, 7>>(a, s);
            case 464: return launch_ws<8, 4, Pm<Rs84Bulk, 8>>(a, s);
            case 465: return launch_ws<8, 4, Stamp<Pm<Rs84Bulk, 5>>>(a, s);
            case 466: return launch_ws<8, 4, Stamp<Pm<Rs84Bulk, 6>>>(a, s);
            // two tiles of register prefetch / the data columns to LDS before the encode
            // and the next tile's loads issued right after (the youngest encode waves wait
            // 17-22 % of their cycles for their tile's loads)
            case 467: return launch_ws<8, 4, Rs84Pf2>(a, s);
            case 468: return launch_ws<8, 4, Rs84Ep1>(a, s);
            case 469: return launch_ws<8, 4, Pm<Rs84Pf2, 5>>(a, s);
            case 470: return launch_ws<8, 4, Pm<Rs84Ep1, 5>>(a, s);
            case 471: return launch_ws<8, 4, Stamp<Rs84Pf2>>(a, s);
            case 472: return launch_ws<8, 4, Stamp<Rs84Ep1>>(a, s);
            case 482: return launch_ws<8, 4, Hf0<Rs84Mid>>(a, s);
            case 483: return launch_ws<8, 4, Hf2<Rs84Bulk>>(a, s);  // pair-form fused packet runs
            case 474: return launch_ws<8, 4, Pm<Rs84Bulk, 4>>(a, s);  // progress-equalising priority
            case 494: return launch_ws<8, 4, Rs84Mid>(a, s);               // the <= 2048-stripe shape
            case 495: return launch_ws<8, 4, XMap<Rs84Mid, 8>>(a, s);
            case 504: return launch_ws<8, 4, Split32<Rs84Bulk>>(a, s);  // without the 64-bit nibble splits
            case 507: return launch_ws<8, 4, Split64<Rs84Mid>>(a, s);
            case 509: return launch_ws<8, 4, Smk<Rs84Bulk>>(a, s);  // split masks from SGPRs
            case 490: return launch_ws<8, 4, Rs84G32>(a, s);
            case 491: return launch_ws<8, 4, Pm<Rs84G32, 0>>(a, s);
            case 492: return launch_ws<8, 4, Stamp<Rs84G32>>(a, s);
            case 487: return launch_ws<8, 4, Stg<Rs84Bulk, 8, 17>>(a, s);   // 8 phases, ~1/8 step apart
            case 488: return launch_ws<8, 4, Stg<Rs84Bulk, 4, 34>>(a, s);   // 4 phases, ~1/4 step apart
            case 489: return launch_ws<8, 4, Stg<Rs84Bulk, 16, 120>>(a, s); // 16 phases, ~0.9 step apart
            default: return false;
        }
    }
    if (a.k == 4 && (a.m == 4 || a.m == 2)) {
        switch (v) {
            case 400: return a.m == 4 && launch_ws<4, 4, PairG16>(a, s);
            case 402: return a.m == 4 && launch_ws<4, 4, Rs84Bulk>(a, s);
            case 508: return a.m == 4 && launch_ws<4, 4, Split32<Rs44Bulk>>(a, s);
            case 418: return a.m == 4 ? launch_ws<4, 4, XMap<PairG16, 8>>(a, s) : launch_ws<4, 2, XMap<PairG16, 8>>(a, s);
            case 480: return a.m == 2 && launch_ws<4, 2, Hf0<Config2>>(a, s);  // config 2 without hh_update_n
            default: return false;
        }
    }
    if (a.k == 16 && a.m == 4) {
        switch (v) {
            case 401: return launch_ws<16, 4, XMap<Rs164Bulk, 0>>(a, s);
            case 499: return launch_ws<16, 4, Stamp<Rs164Bulk>>(a, s);  // per-wave stamps
            case 505: return launch_ws<16, 4, Split64<Rs164Bulk>>(a, s);
            case 415: return launch_ws<16, 4, Tsp0<Rs164Bulk>>(a, s);
            case 417: return launch_ws<16, 4, XMap<Tsp0<Rs164Bulk>, 0>>(a, s);
            case 403: return launch_ws<16, 4, Pm<Rs164Bulk, 0>>(a, s);
            default: return false;
        }
    }
    if (a.k == 12 && a.m == 4 && v == 416) return launch_ws<12, 4, XMap<Rs124Ua1K, 0>>(a, s);
    if (a.k == 12 && a.m == 4 && v == 481) return launch_ws<12, 4, Hf0<Rs124Ua1K>>(a, s);
    if (a.k == 12 && a.m == 4 && v == 484) return launch_ws<12, 4, Stamp<Rs124Ua1K>>(a, s);  // per-wave stamps
    if (a.k == 12 && a.m == 4 && v == 485) return launch_ws<12, 4, Rs124Aln>(a, s);
    if (a.k == 12 && a.m == 4 && v == 486) return launch_ws<12, 4, Stamp<Rs124Aln>>(a, s);
    // two encode waves per SIMD (8-byte columns: 8 encode + 4 hash waves, the 168-VGPR
    // budget) instead of one; and the aligned-row shape (8 stripes of 512) on these rows
    if (a.k == 12 && a.m == 4 && v == 496) return launch_ws<12, 4, Rs124Ua1K8>(a, s);
    if (a.k == 12 && a.m == 4 && v == 497) return launch_ws<12, 4, Stamp<Rs124Ua1K8>>(a, s);
    if (a.k == 12 && a.m == 4 && v == 498) return launch_ws<12, 4, XMap<Rs124AlignedBulk, 8>>(a, s);
    // memory policy: temporal data loads (NTM 2: only the parity stores non-temporal), all
    // temporal (0): do the non-temporal data loads evict the tiles' shared edge lines?
    if (a.k == 12 && a.m == 4 && v == 500) return launch_ws<12, 4, Ntm<Rs124Ua1K, 2>>(a, s);
    if (a.k == 12 && a.m == 4 && v == 501) return launch_ws<12, 4, Ntm<Rs124Ua1K, 0>>(a, s);
    // L2 prefetch one tile ahead (in flight per XCD: 32 CUs x 2 tiles x 48 KiB = 3 MiB of its
    // 4 MiB L2, against 4.5 MiB at two tiles ahead)
    if (a.k == 12 && a.m == 4 && v == 502) return launch_ws<12, 4, Pfd<Rs124Ua1K, 1>>(a, s);
    if (a.k == 12 && a.m == 4 && v == 503) return launch_ws<12, 4, Rs124Pfe>(a, s);   // edge-line re-touch
    if (a.k == 12 && a.m == 4 && v == 506) return launch_ws<12, 4, Split32<Rs124Ua1K>>(a, s);
    if (v == 419) return launch_ehx_gen_xmap(a, s);
    return false;
}
#endif

}  // namespace zs3k
