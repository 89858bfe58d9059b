// fused_v2.hpp — kernel templates of the second-generation fused kernels (k_ehx, k_ehx_ws,
// k_vr_ws) and their template launchers, shared by the translation units that
// instantiate them: fused_v2.hip (encode defaults), fused_v2_get.hip (GET / heal) and,
// in the diagnostics build only, fused_v2_km{84,42,164}.hip (encode variants).
//
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
#pragma once
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "hh256_dev.hpp"

#include <type_traits>

using namespace zs3dev;

namespace zs3k {

namespace {

__device__ __forceinline__ void lds_barrier2() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int NWd>
__device__ __forceinline__ Col<NWd> ld_col(const uint8_t* p) {
    Col<NWd> v;
    __builtin_memcpy(&v, p, 4 * NWd);
    return v;
}
template <int NWd>
__device__ __forceinline__ void st_col(uint8_t* p, const Col<NWd>& v) {
    __builtin_memcpy(p, &v, 4 * NWd);
}
template <int NWd>
__device__ __forceinline__ void st_col_nt(uint8_t* p, const Col<NWd>& v) {
    if constexpr (NWd == 4) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 t = {v.w[0], v.w[1], v.w[2], v.w[3]};
        __builtin_nontemporal_store(t, reinterpret_cast<u4*>(p));
    } else if constexpr (NWd == 2) {
        typedef uint32_t u2 __attribute__((ext_vector_type(2)));
        u2 t = {v.w[0], v.w[1]};
        __builtin_nontemporal_store(t, reinterpret_cast<u2*>(p));
    } else {
        __builtin_nontemporal_store(v.w[0], reinterpret_cast<uint32_t*>(p));
    }
}

// Raw 4/8/16-byte register types for the in-flight columns.
template <int NWd> struct VecOf;
template <> struct VecOf<1> { typedef uint32_t type; };
template <> struct VecOf<2> { typedef uint32_t type __attribute__((ext_vector_type(2))); };
template <> struct VecOf<4> { typedef uint32_t type __attribute__((ext_vector_type(4))); };

// Global load whose completion the compiler does not track: LLVM's waitcnt pass waits
// vmcnt(0) before the first use of a load that has stores issued after it, which
// serialises the parity stores with the next tile's data (and defeats any deeper
// prefetch).  The hardware retires vector-memory ops in issue order, so the kernel
// waits for exactly the loads it needs with vm_wait<N>().  The destination is the
// long-lived prefetch variable itself (no temporary), so its register stays
// allocated until the wait; scripts/check_async_loads.py verifies in the ISA that no
// instruction reads a load's destination before the next s_waitcnt vmcnt.
template <int NWd>
__device__ __forceinline__ void ld_async(typename VecOf<NWd>::type& dst, const uint8_t* p) {
    if constexpr (NWd == 4)
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(p) : "memory");
    else if constexpr (NWd == 2)
        asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(dst) : "v"(p) : "memory");
    else
        asm volatile("global_load_dword %0, %1, off" : "=v"(dst) : "v"(p) : "memory");
}

// s_waitcnt vmcnt(N), then an empty asm that "redefines" each column, so no use of a
// column can be scheduled above the wait.
// Non-temporal form (streamed data read once: nt cache policy).
template <int NWd>
__device__ __forceinline__ void ld_async_nt(typename VecOf<NWd>::type& dst, const uint8_t* p) {
    if constexpr (NWd == 4)
        asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(dst) : "v"(p) : "memory");
    else if constexpr (NWd == 2)
        asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(dst) : "v"(p) : "memory");
    else
        asm volatile("global_load_dword %0, %1, off nt" : "=v"(dst) : "v"(p) : "memory");
}

template <int N, int K, typename V>
__device__ __forceinline__ void vm_wait(V (&xs)[K]) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
    for (int j = 0; j < K; ++j) asm volatile("" : "+v"(xs[j]));
}

// LDS hand-off counters (k_ehx_ws RING).  Signal: this wave's LDS accesses have
// completed (lgkmcnt(0)), then one lane adds 1.  Wait: poll until the count reaches
// `target`, sleeping between polls; the spin is bounded so that a protocol error can
// only produce wrong output, never a wave that does not finish.
__device__ __forceinline__ void ring_signal(uint32_t* ctr) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (__lane_id() == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ring_wait(const uint32_t* ctr, uint32_t target) {
    for (int spin = 0; spin < (1 << 22); ++spin) {
        const uint32_t v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane(v) >= target) break;
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
}

template <int NWd>
__device__ __forceinline__ Col<NWd> to_col(const typename VecOf<NWd>::type& v) {
    Col<NWd> c;
    if constexpr (NWd == 1) {
        c.w[0] = v;
    } else {
#pragma unroll
        for (int w = 0; w < NWd; ++w) c.w[w] = v[w];
    }
    return c;
}

}  // namespace

// Warp-specialised form (one workgroup per CU, G stripes): the first NH = 2*G*R threads
// only hash, one HighwayHash chain per thread PAIR (hh256_dev.hpp pair form: no DPP and
// a shared zipper v_perm, 16 instead of 19 VALU per lane-packet); the other NE threads
// only encode, one 16-byte column each (dwordx4 loads/stores, half the memory
// instructions per byte of the 8-byte form).  Step s: encode waves encode tile s into
// LDS buffer s&1 and store its parity; hash waves hash tile s-1 from buffer (s-1)&1;
// one barrier.  Both roles run the same number of steps, so barriers stay matched.
// With 6 + 6 waves on 4 SIMDs the busiest SIMD carries one hash and two encode waves:
// ~6 % less issue than three mixed waves (asm_loops.py + scripts/ubench/opcost.hip).
// BUF: the encode role addresses rows through buffer resources (workgroup base in
// SGPRs, row/tile offset in an SGPR soffset, one constant per-lane voffset) instead
// of 64-bit per-lane pointers: no VALU address arithmetic per load/store.
// HQ: the hash waves use the quad form (one HH lane per thread, as k_ehx; 19 VALU per
// lane-packet but the shortest dependent chain per packet) — for small batches, where a
// hash wave has its SIMD to itself and the chain latency, not issue, bounds the launch
// (RS(4+2) config 2: 6 144 chains); the hash thread count is padded to whole waves, the
// pad quads hash a real row and discard the digest.
template <int K, int M, int G, int T, bool HQ>
constexpr int ws_nh() {
    // whole wavefronts; pad pairs / quads past G*(K+M) chains hash a real row and discard it
    return HQ ? ((4 * G * (K + M) + 63) / 64) * 64 : ((2 * G * (K + M) + 63) / 64) * 64;
}
// Encode column width: 16 bytes, 8 for K > 8 (16 rows of 16-byte columns do not fit
// the 168-VGPR budget beside the encode's working set).
template <int K, int CWX = 0>
constexpr int ws_cwe() {
    return CWX ? CWX : (K > 8 ? 8 : 16);
}
// LDS row stride of the hash tiles.  TSP = 0: the round-1 padding (T + 16 pair form,
// T + 32 quad form).  TSP = 1: bank-conflict-free for both read forms: the pair form's
// ds_read_b128 serves 16 lanes = 8 chains per LDS cycle from lane groups
// {0-3,12-15,20-27} / {4-11,16-19,28-31} (MI355X_MICROARCH.md §LDS), the quad form's
// ds_read_b64 8 chains per 32-lane half; both are conflict-free iff consecutive rows
// start 32 mod 64 bytes apart (row r's 16-byte slot pair then lands on a distinct pair
// of the 256-byte bank row for every group).  T + 16 put every group 2-way
// (SQ_LDS_BANK_CONFLICT = 20 % of SQ_LDS_IDX_ACTIVE on the RS(8+4) bench launch).
template <int T, bool HQ, int TSP>
constexpr int ws_ts() {
    return TSP ? T + (T % 64 == 0 ? 32 : 0) : (HQ ? T + 32 : T + 16);
}

// ---- Named kernel shapes ------------------------------------------------------------
// Every compile-time knob of k_ehx_ws with its default.  A shape derives from EncShape
// and overrides what it changes, so a launch site names its shape
// (launch_ws<8, 4, shape::Rs84Bulk>) instead of passing 19 positional template
// arguments, and rocprof reports the kernel by that name.  The knobs are described below.
struct EncShape {
    static constexpr int G = 0;          // stripes per workgroup (every shape sets it)
    static constexpr int T = 0;          // tile: bytes of each shard row per step (every shape sets it)
    static constexpr int PF = 1;         // tiles of register prefetch in the encode role
    static constexpr bool BUF = false;   // buffer-resource addressing of the encode columns
    static constexpr bool HQ = false;    // quad-form hash waves (else pair form)
    static constexpr int LDSMIN = 0;     // dynamic-LDS floor (bounds workgroups per CU)
    static constexpr bool WT = false;    // diagnostics: barrier / load-wait cycle stamps
    static constexpr int PM = 0;         // issue-priority scheme
    static constexpr int CWX = 0;        // encode column width (0 = ws_cwe's default)
    static constexpr bool RING = false;  // LDS counters instead of the per-step barrier
    static constexpr int NTM = 0;        // non-temporal policy: bit 0 data loads, bit 1 parity stores
    static constexpr bool STB = false;   // scalar coefficient tables in the encode role
    static constexpr int EP = 0;         // encode-role order (2 = data rows to LDS first)
    static constexpr int PFD = 0;        // L2 prefetch distance of the hash waves, in tiles
    static constexpr bool UA = false;    // unaligned shard sizes
    static constexpr int WPE = 3;        // waves per SIMD the register budget is sized for
    static constexpr int TSP = 0;        // LDS row stride rule (ws_ts)
    static constexpr int ABL = 0;        // diagnostics timing ablations (output differs)
    static constexpr bool GEN = false;   // general M x K coding matrix (not dyadic)
    static constexpr int XMAP = 0;       // workgroup -> stripe-group order (ws_group)
    static constexpr bool DIAGMOD = false;  // a diagnostics modifier of a product shape
    static constexpr bool HF = true;     // quad-form hash role: fused packet runs (hh_update_n)
    static constexpr bool HF2 = false;   // pair-form hash role: fused packet runs (hh2_update_n)
    static constexpr int ALN = 0;        // UA: realign in registers for S % 16 == ALN (below)
    static constexpr int STG = 0;        // start stagger: workgroup w waits (w % STG) * SLP * 64 cycles
    static constexpr int SLP = 0;
    static constexpr bool PFE = false;   // quad-form PFD: re-touch each data row's next-tile edge line
    static constexpr bool S64 = false;   // dyadic encode: nibble splits of dword pairs by 64-bit shifts
    static constexpr bool SMK = false;   // with S64: the split masks from SGPRs (diagnostics)
};

// workgroup -> stripe group (XMAP above k_ehx_ws); a bijection on [0, gridDim.x)
template <int P>
__device__ __forceinline__ int64_t ws_group() {
    if constexpr (P <= 1) {
        return blockIdx.x;
    } else {
        const uint32_t w = blockIdx.x, q = gridDim.x / P;
        if (w >= q * P) return w;  // the last gridDim.x % P workgroups keep their place
        return (int64_t)(w % P) * q + w / P;
    }
}

// WT (diagnostic): per-wave shader cycles spent waiting at barriers, into the dbg stamps.
// PM (issue-priority experiments): 1 = encode waves s_setprio 1 over hash waves; 2 = as 1
// plus the younger encode wave of each SIMD-sharing pair (waves w, w+4) at 2; 3 = hash
// waves at 1.
// CWX: encode column width override (0 = ws_cwe's default).
// RING: the two roles hand tiles over through per-slot LDS counters instead of one
// workgroup barrier per step (pair-form hash role only).  An encode wave waits only
// until every hash wave has read the slot it is about to overwrite (tile s-2), a hash
// wave only until every encode wave has written tile s; a hash wave releases the slot
// as soon as its 12 reads have landed, before hashing them.  So the older encode wave
// of a SIMD goes straight on to the next tile instead of idling at a barrier while its
// younger partner finishes alone.
// NTM (memory policy, bit mask): 1 = data loads non-temporal, 2 = parity stores non-temporal.
// STB: encode role reads the coefficient tables with scalar loads (SGPRs) instead of LDS.
// EP = 1 (early prefetch): the encode wave first copies its data columns into the LDS
// tile, issues the next tile's loads into the freed registers, and then encodes from the
// LDS copy (one block of M rows at a time): the loads get a whole step to land instead of
// the parity stores + barrier.  EP = 2 (early data write): the data columns go to LDS
// before the encode instead of after it, so the LDS drains the tile's data rows while
// the VALU encodes and only the parity rows are written between encode and barrier.
// PFD (L2 prefetch distance, pair-form hash role): while hashing tile s-1 the hash waves
// touch every 128-byte line of the data rows of tile s+PFD with one untracked
// global_load_dword each (result discarded), so the HBM fetch of a tile starts PFD-1
// steps before the encode waves load it and their own loads hit L2: the HBM stream
// keeps ~PFD tiles of reads in flight per CU instead of the one tile the encode waves'
// registers hold.  The hash waves never wait on these loads (they have no other vector
// loads in the loop); the sink register stays allocated until the final vmcnt(0).
// UA (unaligned shard size): S need not be a multiple of 16 (RS(12+4) on 1 MiB blocks:
// S = 87 382, every row 2-byte aligned; k*S - n = 8 bytes of Split padding).  Full tiles
// use the same vector loads and stores at the rows' byte offsets (the GPU runs global
// memory in unaligned mode); the ragged tail tile is never prefetched: each lane reads
// its columns of it byte by byte, with the Split padding of the last data row (n..k*S)
// and everything past the row read as zero, and stores only the parity bytes below S.
// WPE: minimum waves per SIMD the register allocation is sized for (3 = 168 VGPRs; 2 =
// 256, for workgroups of at most 8 waves, one per CU).
// GEN: any M x K coding matrix (the server's non-power-of-two geometries, not dyadic): the
// encode role multiplies every data row into every parity row (encode_general, a.tables).
// TSP: LDS row stride rule (ws_ts).  ABL (timing-only diagnostics, output differs):
// bit 0 = the pair-form hash waves XOR the words instead of running HighwayHash; bit 1 =
// they skip their LDS reads; bit 2 = the encode waves skip their LDS writes.
// XMAP (round 5): workgroup -> stripe-group order.  0: workgroup w encodes stripes
// [w*G, w*G+G).  P > 1: the grid is cut into P equal regions and consecutive workgroups
// alternate between them (w -> region w % P, position w / P), so the workgroups resident
// at one time stream from P places of the batch at once instead of one contiguous window
// (with P = 8 = XCDs and the round-robin dispatch, each XCD walks its own eighth).
template <int K, int M, class C>
__global__ void __launch_bounds__((ws_nh<K, M, C::G, C::T, C::HQ>() + C::G * (C::T / ws_cwe<K, C::CWX>())))
__attribute__((amdgpu_waves_per_eu(C::WPE))) k_ehx_ws(EncArgs a) {
    constexpr int G = C::G, T = C::T, PF = C::PF, PM = C::PM, CWX = C::CWX, NTM = C::NTM, EP = C::EP, PFD = C::PFD,
                  TSP = C::TSP, ABL = C::ABL, ALN = C::ALN;
    constexpr bool BUF = C::BUF, HQ = C::HQ, WT = C::WT, RING = C::RING, STB = C::STB, UA = C::UA, GEN = C::GEN;
    constexpr int R = K + M;
    constexpr int NH = ws_nh<K, M, G, T, HQ>();  // hash threads
    constexpr int CWE = ws_cwe<K, CWX>();
    constexpr int CPS = T / CWE;    // encode columns per stripe row
    constexpr int NE = G * CPS;     // encode threads
    constexpr int NT = NH + NE;
    constexpr int TS = ws_ts<T, HQ, TSP>();
    constexpr int NPK = T / 32;
    constexpr int NTAB = GEN ? M * K * 8 : K * 8;
    static_assert(GEN || M == 2 || M == 4, "dyadic shapes only (GEN: any M x K matrix)");
    static_assert(NH % 64 == 0 && NE % 64 == 0 && T % 32 == 0, "whole wavefronts per role");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_dyn[];
    uint8_t(*tile)[G * R * TS] = reinterpret_cast<uint8_t(*)[G * R * TS]>(smem_dyn);
    __shared__ __attribute__((aligned(16))) uint32_t tabs[NTAB];
    // RING: [0..1] encode-wave completions per slot, [2..3] hash-wave releases per slot
    __shared__ uint32_t ring[4];
    static_assert(!RING || !HQ, "ring hand-off: pair-form hash role");
    constexpr uint32_t NEW = (uint32_t)(NT - NH) / 64, NHW = (uint32_t)NH / 64;

    const int tid = threadIdx.x;
    const int64_t blk0 = (int64_t)ws_group<C::XMAP>() * G;
    const int64_t S = a.S;
    if constexpr (C::STG > 1) {
        // start stagger (round 6, diagnostics): the workgroups of one launch wave otherwise
        // walk the same row offsets of their stripes in lockstep
        const int ph = (int)(blockIdx.x % C::STG);
        for (int i = 0; i < ph; ++i) __builtin_amdgcn_s_sleep(C::SLP);
    }
    for (int i = tid; i < NTAB; i += NT) tabs[i] = GEN ? a.tables[i] : a.dtables[i];
    if (RING && tid < 4) ring[tid] = 0;
    const int64_t nfull = S / T;
    const int tail = (int)(S - nfull * T);  // multiple of 16 unless UA
    // Step schedule shared by both roles: PF edge steps, the steady loop in units of PF
    // while i + 2*PF <= nfull, 2*PF edge steps, one step that only hashes.
    int64_t iend = PF;
    if (nfull >= 3 * PF) iend = PF + ((nfull - 3 * PF) / PF + 1) * PF;
    const int64_t total = iend + 2 * PF + 1;

    // Diagnostics (a.dbg set): per-wave real time, shader clocks, HW_ID, XCC_ID, as in
    // k_ehx (waves 0..NH/64-1 of a workgroup hash, the rest encode).
    uint64_t rt0 = 0, ct0 = 0;
    if (a.dbg) {
        rt0 = __builtin_amdgcn_s_memrealtime();
        ct0 = __builtin_amdgcn_s_memtime();
    }
    uint64_t wsum = 0, vwsum = 0;  // WT: shader cycles in barriers / in the encode's load wait
    auto bar = [&]() {
        if constexpr (WT) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            lds_barrier2();
            wsum += __builtin_amdgcn_s_memtime() - t;
        } else {
            lds_barrier2();
        }
    };
    auto stamp = [&]() {
        if (a.dbg && (tid & 63) == 0) {
            const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
            const uint64_t ct1 = __builtin_amdgcn_s_memtime();
            uint64_t* d = a.dbg + ((int64_t)blockIdx.x * (NT / 64) + (tid >> 6)) * 5;
            d[0] = rt0;
            d[1] = rt1;
            d[2] = ct1 - ct0;
            d[3] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
            // XCC_ID | barrier-wait cycles (bits 8-35) | load-wait cycles (bits 36-63)
            d[4] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) | ((wsum & 0xFFFFFFF) << 8) | (vwsum << 36);
        }
    };

    if (HQ && __builtin_amdgcn_readfirstlane(tid) < NH) {
        // ---- hash role, quad form: lane `lane` of chain `chain`
        const int chain = tid >> 2, lane = tid & 3;
        const bool live = chain < G * R && blk0 + chain / R < a.n_blocks;
        const int crow = chain < G * R ? chain : chain - G * R;
        const int row_off = crow * TS + 8 * lane;
        const uint32_t sel = zipper_sel(lane);
        HHLane st = hh_init(lane, a.key[0], a.key[1], a.key[2], a.key[3]);
        // PFD: the same L2 prefetch of the data rows as the pair-form role below
        constexpr int LPR = T / 128, NLN = G * K * LPR, NPL = PFD ? (NLN + NH - 1) / NH : 1;
        const uint8_t* pfa[NPL];
        uint32_t sink = 0;
        if constexpr (PFD > 0) {
            static_assert(T % 128 == 0, "prefetch whole 128-byte lines");
#pragma unroll
            for (int q = 0; q < NPL; ++q) {
                const int li = tid + q * NH < NLN ? tid + q * NH : NLN - 1;
                const int r = li / LPR, g = r / K, j = r % K;
                const int64_t b = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
                pfa[q] = a.data + b * a.data_stride + (int64_t)j * S + (li % LPR) * 128;
            }
        }
        // PFE (round 6, diagnostics): thread r < G*K re-touches the first byte of data row r's
        // next tile (the line it shares with the current tile when rows are unaligned) with a
        // temporal load in each step, after the encode's non-temporal load of the current
        // tile has marked that line for early eviction
        const uint8_t* pfe = nullptr;
        if constexpr (PFD > 0 && C::PFE) {
            const int r = tid < G * K ? tid : 0, g = r / K, j = r % K;
            const int64_t b = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
            pfe = a.data + b * a.data_stride + (int64_t)j * S;
        }
        bar();  // tables (matches the encode role)
        bar();  // step 0: tile 0 being encoded
        for (int64_t s = 1; s <= nfull; ++s) {
            if constexpr (PFD > 0) {
                if (s + PFD < nfull) {
#pragma unroll
                    for (int q = 0; q < NPL; ++q)
                        asm volatile("global_load_dword %0, %1, off" : "+v"(sink) : "v"(pfa[q] + (s + PFD) * T));
                }
                if constexpr (C::PFE) {
                    if (tid < G * K && s + 1 < nfull)
                        asm volatile("global_load_dword %0, %1, off" : "+v"(sink) : "v"(pfe + (s + 1) * T));
                }
            }
            const uint64_t* p = reinterpret_cast<const uint64_t*>(tile[(s - 1) & 1] + row_off);
            uint64_t w[NPK];
#pragma unroll
            for (int i = 0; i < NPK; ++i) w[i] = p[4 * i];
            if constexpr (C::HF) {
                hh_update_n<NPK>(st, w, sel);
            } else {
#pragma unroll
                for (int i = 0; i < NPK; ++i) hh_update(st, w[i], sel);
            }
            bar();
        }
        if constexpr (PFD > 0) asm volatile("s_waitcnt vmcnt(0)" : "+v"(sink)::"memory");
        if (tail) {
            const uint8_t* row = tile[nfull & 1] + crow * TS;
            hh_packets(st, row, tail >> 5, lane, sel);
            if (tail & 31) hh_remainder(st, row + (tail & ~31), (uint32_t)(tail & 31), lane, sel);
        }
        for (int64_t s = nfull + 1; s < total; ++s) bar();
        const uint64_t h = hh_finalize256(st, lane, sel);
        if (live) {
            const int64_t bb = blk0 + chain / R;
            *reinterpret_cast<uint64_t*>(a.sums + (bb * R + chain % R) * 32 + 8 * lane) = h;
        }
        stamp();
        return;
    }
    if constexpr (PM == 3) {
        if (__builtin_amdgcn_readfirstlane(tid) < NH) __builtin_amdgcn_s_setprio(1);
    } else if constexpr (PM >= 5 && PM <= 8) {
        // round 6 (per-wave stamps, profiles/r06/stamps_enc.jsonl): a 12-wave workgroup's
        // waves share SIMDs as {w, w+4, w+8}, so the pair-form hash waves 2 and 3 are the
        // ones beside two encode waves ("1H+2E") and pace the step.  5: encode waves 1,
        // those two hash waves 2; 6: encode waves 1, every hash wave 2; 7: encode waves and
        // hash waves 2-3 at 1; 8: only hash waves 2-3 at 1.
        const int wv = (int)__builtin_amdgcn_readfirstlane(tid) >> 6;
        const bool enc = wv >= NH / 64, hb = !enc && (wv & 3) >= 2 && wv < 4;
        int pr = 0;
        if (PM == 5) pr = enc ? 1 : hb ? 2 : 0;
        if (PM == 6) pr = enc ? 1 : 2;
        if (PM == 7) pr = enc || hb ? 1 : 0;
        if (PM == 8) pr = hb ? 1 : 0;
        if (pr == 1) __builtin_amdgcn_s_setprio(1);
        if (pr == 2) __builtin_amdgcn_s_setprio(2);
    } else if constexpr (PM == 1 || PM == 2) {
        if (__builtin_amdgcn_readfirstlane(tid) >= NH) {
            if (PM == 2 && __builtin_amdgcn_readfirstlane(tid) >= NH + 256)
                __builtin_amdgcn_s_setprio(2);
            else
                __builtin_amdgcn_s_setprio(1);
        }
    }
    if (!HQ && __builtin_amdgcn_readfirstlane(tid) < NH) {
        // ---- hash role: lanes (2hh, 2hh+1) of chain `chain` = shard row s of stripe g
        // (pad pairs past the G*R chains of a workgroup hash chain - G*R and discard it)
        const int chain0 = tid >> 1, hh = tid & 1;
        const bool hpad = chain0 >= G * R;
        const int chain = hpad ? chain0 - G * R : chain0;
        const int row_off = chain * TS;
        HHPair st = hh2_init(hh, a.key[0], a.key[1], a.key[2], a.key[3]);
        bar();  // tables (matches the encode role)
        if constexpr (RING) {
            for (int64_t s = 0; s <= nfull; ++s) {
                if (s == nfull && !tail) break;
                ring_wait(&ring[s & 1], NEW * (uint32_t)((s >> 1) + 1));  // tile s written
                if (s == nfull) {
                    const uint8_t* row = tile[nfull & 1] + row_off;
                    hh2_packets(st, row, tail >> 5, hh);
                    if (tail & 31) hh2_remainder(st, row + (tail & ~31), (uint32_t)(tail & 31), hh);
                    break;
                }
                const uint4* p = reinterpret_cast<const uint4*>(tile[s & 1] + row_off) + hh;
                uint4 w[NPK];
#pragma unroll
                for (int i = 0; i < NPK; ++i) w[i] = p[2 * i];
                ring_signal(&ring[2 + (s & 1)]);  // reads landed: the slot may be refilled
#pragma unroll
                for (int i = 0; i < NPK; ++i)
                    hh2_update(st, ((uint64_t)w[i].y << 32) | w[i].x, ((uint64_t)w[i].w << 32) | w[i].z);
            }
            uint64_t d0, d1;
            hh2_finalize256(st, d0, d1);
            if (!hpad && blk0 + chain / R < a.n_blocks) {
                const int64_t bb = blk0 + chain / R;
                uint64_t* out = reinterpret_cast<uint64_t*>(a.sums + (bb * R + chain % R) * 32 + 16 * hh);
                out[0] = d0;
                out[1] = d1;
            }
            stamp();
            return;
        }
        // PFD: this thread's prefetch lines (line li = tid + q*NH of the tile's data rows)
        constexpr int LPR = T / 128, NLN = G * K * LPR, NPL = PFD ? (NLN + NH - 1) / NH : 1;
        const uint8_t* pfa[NPL];
        uint32_t sink = 0;
        if constexpr (PFD > 0) {
            static_assert(T % 128 == 0, "prefetch whole 128-byte lines");
#pragma unroll
            for (int q = 0; q < NPL; ++q) {
                const int li = tid + q * NH < NLN ? tid + q * NH : NLN - 1;
                const int r = li / LPR, g = r / K, j = r % K;
                const int64_t b = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
                pfa[q] = a.data + b * a.data_stride + (int64_t)j * S + (li % LPR) * 128;
            }
        }
        bar();  // step 0: tile 0 being encoded
        for (int64_t s = 1; s <= nfull; ++s) {
            if constexpr (PFD > 0) {
                if (s + PFD < nfull) {
#pragma unroll
                    for (int q = 0; q < NPL; ++q)
                        asm volatile("global_load_dword %0, %1, off" : "+v"(sink) : "v"(pfa[q] + (s + PFD) * T));
                }
            }
            const uint4* p = reinterpret_cast<const uint4*>(tile[(s - 1) & 1] + row_off) + hh;
            uint4 w[NPK];
            if constexpr (ABL & 2) {
                // timing ablation: no LDS reads (the words are the step number)
#pragma unroll
                for (int i = 0; i < NPK; ++i) w[i] = make_uint4((uint32_t)s, (uint32_t)i, 0u, 0u);
            } else {
#pragma unroll
                for (int i = 0; i < NPK; ++i) w[i] = p[2 * i];
            }
            if constexpr (PM == 4) __builtin_amdgcn_s_setprio(3);
            if constexpr (C::HF2 && ABL == 0 && PM != 4) {
                hh2_update_n<NPK>(st, w);
            } else
#pragma unroll
            for (int i = 0; i < NPK; ++i) {
                if constexpr (PM == 4) {
                    // progress-equalising priority: 3, 2, 1, 0 over the quarters of the tile
                    if (i > 0 && (4 * i) % NPK == 0) {
                        __builtin_amdgcn_sched_barrier(0);
                        if (4 * i / NPK == 1) __builtin_amdgcn_s_setprio(2);
                        if (4 * i / NPK == 2) __builtin_amdgcn_s_setprio(1);
                        if (4 * i / NPK == 3) __builtin_amdgcn_s_setprio(0);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                if constexpr (ABL & 1) {
                    // timing ablation (diagnostics only; sums differ): no HighwayHash arithmetic
                    st.v0[0] ^= ((uint64_t)w[i].y << 32) | w[i].x;
                    st.v0[1] ^= ((uint64_t)w[i].w << 32) | w[i].z;
                } else {
                    hh2_update(st, ((uint64_t)w[i].y << 32) | w[i].x, ((uint64_t)w[i].w << 32) | w[i].z);
                }
            }
            bar();
        }
        // the L2 prefetches have all retired before the tail code may reuse the sink register
        if constexpr (PFD > 0) asm volatile("s_waitcnt vmcnt(0)" : "+v"(sink)::"memory");
        if (tail) {
            const uint8_t* row = tile[nfull & 1] + row_off;
            hh2_packets(st, row, tail >> 5, hh);
            if (tail & 31) hh2_remainder(st, row + (tail & ~31), (uint32_t)(tail & 31), hh);
        }
        for (int64_t s = nfull + 1; s < total; ++s) bar();
        uint64_t d0, d1;
        hh2_finalize256(st, d0, d1);
        if (!hpad && blk0 + chain / R < a.n_blocks) {
            const int64_t bb = blk0 + chain / R;
            uint64_t* out = reinterpret_cast<uint64_t*>(a.sums + (bb * R + chain % R) * 32 + 16 * hh);
            out[0] = d0;
            out[1] = d1;
        }
        stamp();
        return;
    }

    // ---- encode role: 16-byte column o of stripe g (dead stripes of the last
    // workgroup alias the last live block and store byte-identical parity)
    constexpr int NWd = CWE / 4;
    typedef typename VecOf<NWd>::type VT;
    const int e = tid - NH;
    const int g = e / CPS, o = (e % CPS) * CWE;
    const int64_t b = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
    const uint8_t* src = a.data + b * a.data_stride + o;
    uint8_t* pdst = a.parity + b * a.parity_stride + o;
    const int col_off = g * R * TS + o;
    // buffer form (launch checks that every offset fits in 31 bits)
    const __amdgpu_buffer_rsrc_t rs_d =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.data + blk0 * a.data_stride), 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_p =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.parity + blk0 * a.parity_stride), 0, 0x7FFFFFFF, 0x00020000);
    const uint32_t vo_d = (uint32_t)((b - blk0) * a.data_stride + o);
    const uint32_t vo_p = (uint32_t)((b - blk0) * a.parity_stride + o);

    VT x[PF][K];
    CoefTab ptab[EP == 3 ? K : 1];  // EP = 3: coefficient tables held in registers
    // ALN (round 6, unaligned rows, 16-byte buffer-addressed columns, one wave per stripe,
    // PF 1): row j starts r_j = (j*S) mod 16 bytes past a 16-byte boundary, so the column
    // loads of the round-3 UA form are unaligned and each tile's last line is fetched again
    // by the next tile (RS(12+4) on 1 MiB blocks: 1.055 x the data rows' bytes, profiles/
    // r05/traffic_req_rs124.json).  Here lane l loads the ALIGNED 16-byte chunk l+1 of the
    // row's tile (for r_j != 0), takes chunk l from lane l-1 (DPP wave_shr) — lane 0 from
    // a carry, the previous tile's last chunk, handed over by DPP wave_ror — and shifts
    // the pair into place (v_alignbyte); every chunk is loaded once.
    VT pc[ALN ? K : 1];
    static_assert(!ALN || (UA && BUF && NWd == 4 && PF == 1 && T == 1024), "ALN: one 16-byte column per lane, one wave per stripe");
    // rows j of tile offset t0u (wave-uniform) at per-lane byte offset vo within the row
    auto load_buf = [&](VT (&xs)[K], uint32_t vo_in, int64_t t0u) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            // ALN: chunk l+1 of the aligned tile, i.e. 16 - r_j bytes past the lane's column
            // (in the voffset, so the rows keep the product's SGPR offsets)
            const int rj = ALN ? (int)((j * ALN) & 15) : 0;
            const uint32_t vo = vo_in + (rj ? (uint32_t)(16 - rj) : 0u);
            const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(j * S + t0u));
            if constexpr (NWd == 4 && (NTM & 1))
                asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen nt"
                             : "=v"(xs[j])
                             : "v"(vo), "s"(rs_d), "s"(so)
                             : "memory");
            else if constexpr (NWd == 4)
                asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                             : "=v"(xs[j])
                             : "v"(vo), "s"(rs_d), "s"(so)
                             : "memory");
            else if constexpr (NTM & 1)
                asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen nt"
                             : "=v"(xs[j])
                             : "v"(vo), "s"(rs_d), "s"(so)
                             : "memory");
            else
                asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen"
                             : "=v"(xs[j])
                             : "v"(vo), "s"(rs_d), "s"(so)
                             : "memory");
        }
    };
    auto load = [&](VT (&xs)[K], int64_t t0) {
        if constexpr (BUF) {
            load_buf(xs, vo_d, t0);
        } else if constexpr ((NTM & 1) != 0) {
#pragma unroll
            for (int j = 0; j < K; ++j) ld_async_nt<NWd>(xs[j], src + (int64_t)j * S + t0);
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j) ld_async<NWd>(xs[j], src + (int64_t)j * S + t0);
        }
    };
    auto prefetch_any = [&](VT (&xs)[K], int64_t tn) {
        // UA: the tail tile is read byte by byte in its step (tail_cols), never prefetched
        const bool ok = tn < nfull || (!UA && tn == nfull && o < tail);
        if constexpr (BUF)
            load_buf(xs, vo_d + (ok ? (uint32_t)(tn * T) : 0u), 0);  // per-lane part in voffset
        else
            load(xs, ok ? tn * T : 0);
    };
    // UA tail tile: bytes [o, o + CWE) of every data row, zero past the row's valid length
    // (tail, or for the last data row the end of the block: Split padding reads as zero)
    auto tail_cols = [&](VT (&xs)[K]) {
        const uint8_t* t0p = src + nfull * T;
        const int64_t last_valid = a.n - (int64_t)(K - 1) * S - nfull * T;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int64_t valid = j == K - 1 ? (last_valid < tail ? last_valid : tail) : tail;
            uint32_t w[NWd];
#pragma unroll
            for (int q = 0; q < NWd; ++q) {
                uint32_t v = 0;
#pragma unroll
                for (int bb = 0; bb < 4; ++bb) {
                    const int pos = o + 4 * q + bb;
                    if (pos < valid) v |= (uint32_t)t0p[(int64_t)j * S + 4 * q + bb] << (8 * bb);
                }
                w[q] = v;
            }
            if constexpr (NWd == 1) {
                xs[j] = w[0];
            } else {
#pragma unroll
                for (int q = 0; q < NWd; ++q) xs[j][q] = w[q];
            }
        }
    };
    auto store_tail = [&](const Col<NWd> (&par)[M]) {
        uint8_t* t0p = pdst + nfull * T;
#pragma unroll
        for (int r = 0; r < M; ++r)
#pragma unroll
            for (int q = 0; q < NWd; ++q)
#pragma unroll
                for (int bb = 0; bb < 4; ++bb)
                    if (o + 4 * q + bb < tail) t0p[(int64_t)r * S + 4 * q + bb] = (uint8_t)(par[r].w[q] >> (8 * bb));
    };
    auto encode = [&](VT (&xr)[K], uint8_t* tl, Col<NWd> (&par)[M]) {
        Col<NWd> xs[K];
#pragma unroll
        for (int j = 0; j < K; ++j) xs[j] = to_col<NWd>(xr[j]);
        if constexpr (GEN) {
            // general M x K matrix: the data rows go to LDS first (they drain under the
            // products), then every parity row from all K data rows
#pragma unroll
            for (int j = 0; j < K; ++j) st_col<NWd>(tl + col_off + j * TS, xs[j]);
            encode_general<NWd, K, M>(xs, par, tabs);
        } else if constexpr (EP == 9) {
            // timing ablation (diagnostics only; output differs): no GF arithmetic
#pragma unroll
            for (int r = 0; r < M; ++r)
#pragma unroll
                for (int w = 0; w < NWd; ++w) par[r].w[w] = xs[r].w[w] ^ xs[r + M].w[w];
        } else if constexpr (EP == 8) {
            // timing ablation: only the first half of the data rows enter the parity
            Col<NWd> xh[K];
#pragma unroll
            for (int j = 0; j < K; ++j) xh[j] = xs[j % (K / 2)];
            encode_dyadic<NWd, K / 2, M, true, false, STB>(*reinterpret_cast<const Col<NWd>(*)[K / 2]>(xh), par, tabs,
                                                            const_tables(a.dtables));
        } else if constexpr (EP == 3) {
            // tables held in registers: the data rows go to LDS first and drain under the encode
#pragma unroll
            for (int j = 0; j < K; ++j) st_col<NWd>(tl + col_off + j * TS, xs[j]);
            encode_dyadic_f<NWd, K, M, true, false, false, true>(
                [&](int j) { return xs[j]; }, par, tabs, nullptr, NoHook{}, ptab);
        } else if constexpr (EP == 2) {
            // data rows written right after the first block's table reads
            encode_dyadic_f<NWd, K, M, true, false, STB, false, C::S64, C::SMK>(
                [&](int j) { return xs[j]; }, par, tabs, const_tables(a.dtables), [&]() {
#pragma unroll
                    for (int j = 0; j < K; ++j) st_col<NWd>(tl + col_off + j * TS, xs[j]);
                });
        } else if constexpr (PM == 4) {
            __builtin_amdgcn_s_setprio(3);
            encode_dyadic<NWd, K, M, true, true>(xs, par, tabs);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(K / M >= 3 ? 0 : 1);
        } else {
            encode_dyadic<NWd, K, M, true, false, STB, C::S64, C::SMK>(xs, par, tabs, const_tables(a.dtables));
        }
        if constexpr (ABL & 4) {
            // timing ablation: no LDS writes (the hash waves read stale tiles)
        } else {
            if constexpr (EP != 2 && EP != 3 && !GEN) {
#pragma unroll
                for (int j = 0; j < K; ++j) st_col<NWd>(tl + col_off + j * TS, xs[j]);
            }
#pragma unroll
            for (int r = 0; r < M; ++r) st_col<NWd>(tl + col_off + (K + r) * TS, par[r]);
        }
    };
    auto store_par = [&](const Col<NWd> (&par)[M], int64_t t0) {
#pragma unroll
        for (int r = 0; r < M; ++r) {
            if constexpr (BUF) {
                const int so = (int)__builtin_amdgcn_readfirstlane((uint32_t)(r * S + t0));
                constexpr int aux = (NTM & 2) ? 2 : 0;  // cache policy: 2 = nt (gfx940 family)
                if constexpr (NWd == 4) {
                    const VT v = {par[r].w[0], par[r].w[1], par[r].w[2], par[r].w[3]};
                    __builtin_amdgcn_raw_buffer_store_b128(v, rs_p, (int)vo_p, so, aux);
                } else {
                    const VT v = {par[r].w[0], par[r].w[1]};
                    __builtin_amdgcn_raw_buffer_store_b64(v, rs_p, (int)vo_p, so, aux);
                }
            } else if constexpr ((NTM & 2) != 0) {
                st_col_nt<NWd>(pdst + (int64_t)r * S + t0, par[r]);
            } else {
                st_col<NWd>(pdst + (int64_t)r * S + t0, par[r]);
            }
        }
    };
    // RING: slot of tile ti free = every hash wave has read tile ti-2 out of it
    auto slot_free = [&](int64_t ti) {
        if (RING && ti >= 2) ring_wait(&ring[2 + (ti & 1)], NHW * (uint32_t)(ti >> 1));
    };
    // ALN: tile ti's loaded chunks (lane l: chunk l+1 of each unaligned row) -> the row's
    // bytes [ti*T + 16 l, +16); lane 0's carry becomes the tile's last chunk (for ti+1)
    auto realign = [&](VT (&xs)[K]) {
        if constexpr (ALN != 0) {
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const int r = (j * ALN) & 15;
                if (r == 0) continue;
                const int q = r >> 2, sh = r & 3;
                uint32_t cc[8];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    cc[d] = 0;
                    cc[4 + d] = xs[j][d];
                }
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    if (d < q) continue;
                    // wave_shr:1 (lane l <- lane l-1; lane 0 keeps `old`, the carry), then
                    // wave_ror:1 (lane 0 <- lane 63: the next tile's carry)
                    cc[d] = (uint32_t)__builtin_amdgcn_update_dpp((int)pc[j][d], (int)xs[j][d], 0x138, 0xF, 0xF, false);
                    pc[j][d] = (uint32_t)__builtin_amdgcn_update_dpp((int)pc[j][d], (int)xs[j][d], 0x13C, 0xF, 0xF, false);
                }
                VT out;
#pragma unroll
                for (int d = 0; d < 4; ++d)
                    out[d] = sh ? __builtin_amdgcn_alignbyte(cc[q + d + 1], cc[q + d], (uint32_t)sh) : cc[q + d];
                xs[j] = out;
            }
        }
    };
    // steady step (see k_ehx): wait for loads(ti) only
    auto step = [&](VT (&xs)[K], int64_t ti) {
        Col<NWd> par[M];
        slot_free(ti);
        if constexpr (WT) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            vm_wait<M + (PF - 1) * (K + M)>(xs);
            vwsum += __builtin_amdgcn_s_memtime() - t;
        } else {
            vm_wait<M + (PF - 1) * (K + M)>(xs);
        }
        realign(xs);
        if constexpr (EP == 1) {
            static_assert(PF == 1 && !RING && PM != 4, "early prefetch: PF = 1, barrier hand-off");
            uint8_t* tl = tile[ti & 1];
#pragma unroll
            for (int j = 0; j < K; ++j) st_col<NWd>(tl + col_off + j * TS, to_col<NWd>(xs[j]));
            load(xs, (ti + PF) * T);
            // read back this wave's own columns (LDS keeps one wave's accesses in order)
            encode_dyadic_f<NWd, K, M, true, false, STB>(
                [&](int j) { return ld_col<NWd>(tl + col_off + j * TS); }, par, tabs, const_tables(a.dtables));
#pragma unroll
            for (int r = 0; r < M; ++r) st_col<NWd>(tl + col_off + (K + r) * TS, par[r]);
        } else {
            encode(xs, tile[ti & 1], par);
            if constexpr (RING) ring_signal(&ring[ti & 1]);
            load(xs, (ti + PF) * T);
        }
        store_par(par, ti * T);
        if constexpr (!RING) bar();
    };
    auto edge = [&](VT (&xs)[K], int64_t ti) {
        const bool full = ti < nfull, part = ti == nfull && tail;
        if (full || part) slot_free(ti);
        vm_wait<0>(xs);
        Col<NWd> par[M];
        if constexpr (ALN != 0) {
            if (full) realign(xs);
        }
        if constexpr (UA) {
            if (part) tail_cols(xs);
        }
        if (full || part) encode(xs, tile[ti & 1], par);
        if (RING && (full || part)) ring_signal(&ring[ti & 1]);
        prefetch_any(xs, ti + PF);
        if constexpr (UA) {
            if (full) store_par(par, ti * T);
            else if (part && o < tail) store_tail(par);
        } else {
            if (full || (part && o < tail)) store_par(par, ti * T);
        }
        if constexpr (!RING) bar();
    };
    bar();  // tables visible
    if constexpr (EP == 3) {
#pragma unroll
        for (int i = 0; i < K; ++i) ptab[i] = load_coef(tabs, i);
        // consume them here, so the LDS-counter wait for the table reads sits before the
        // loop rather than at the first use inside every step
#pragma unroll
        for (int i = 0; i < K; ++i) asm volatile("" ::"v"(ptab[i].ab.x), "v"(ptab[i].ab.y), "v"(ptab[i].ab.z), "v"(ptab[i].ab.w), "v"(ptab[i].c));
    }
    if constexpr (ALN != 0) {
        // the first tile's carry: chunk 0 of every row (the 16 bytes ending at its start), the
        // same address in every lane of the stripe's wave
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int rj = (int)((j * ALN) & 15);
            const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(j * S - rj));
            asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                         : "=v"(pc[j])
                         : "v"(vo_d - (uint32_t)o), "s"(rs_d), "s"(so)
                         : "memory");
        }
        vm_wait<0>(pc);
    }
#pragma unroll
    for (int p = 0; p < PF; ++p) prefetch_any(x[p], p);
#pragma unroll
    for (int p = 0; p < PF; ++p) edge(x[p], p);
    int64_t i = PF;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; i + 2 * PF <= nfull; i += PF) {
#pragma unroll
        for (int p = 0; p < PF; ++p) step(x[p], i + p);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < 2 * PF; ++p) edge(x[p % PF], i + p);
    if constexpr (!RING) bar();  // the hash-only step
#pragma unroll
    for (int p = 0; p < PF; ++p) vm_wait<0>(x[p]);
    stamp();
}

template <int K, int M, class C>
static bool launch_ws(const EncArgs& a, hipStream_t s) {
    constexpr int G = C::G, T = C::T;
    constexpr int R = K + M;
    constexpr int NT = ws_nh<K, M, G, T, C::HQ>() + G * (T / ws_cwe<K, C::CWX>());
    constexpr size_t tiles = (size_t)2 * G * R * ws_ts<T, C::HQ, C::TSP>();
    constexpr size_t dyn = tiles > (size_t)C::LDSMIN ? tiles : (size_t)C::LDSMIN;
    static_assert(G > 0 && T > 0, "a shape names its stripes per workgroup and tile length");
    if constexpr (dyn + (C::GEN ? M * K : K) * 32 > 163840 || NT > 1024) {
        return false;
    } else {
        if (!C::GEN && a.dyb != M) return false;
        if (a.k != K || a.m != M) return false;
        if constexpr (C::UA) {
            // the Split padding (n .. k*S) must lie in the last data row's tail tile
            const int64_t tail = a.S % T;
            if ((int64_t)K * a.S - a.n > tail || a.n <= (int64_t)(K - 1) * a.S) return false;
            // ALN: the instance's row alignments; the last full tile's chunk 64 must lie inside
            // the row (a tail of at least 16 bytes)
            if (C::ALN && ((a.S % 16) != C::ALN || tail < 16)) return false;
        } else {
            if ((a.S % 16) != 0 || a.n != (int64_t)K * a.S) return false;
        }
        if (C::BUF && ((G - 1) * a.data_stride + K * a.S > 0x7FFFFFFF ||
                       (G - 1) * a.parity_stride + M * a.S > 0x7FFFFFFF || a.data_stride < 0 || a.parity_stride < 0))
            return false;
        auto kern = k_ehx_ws<K, M, C>;
        if (ensure_dyn_lds((const void*)kern, dyn) != hipSuccess) return false;
        const int64_t grid = (a.n_blocks + G - 1) / G;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), dyn, s, a);
        return true;
    }
}

// ---------------------------------------------------------------------------
// GET / heal pass, warp-specialised (replaces the arithmetic of
// streamingBitrotReader.ReadAt's verify, bitrot-streaming.go:171-186, and
// Erasure.DecodeDataBlocks, erasure-coding.go:96-109, for one batch of stripes).
// Same contract as k_verify_reconstruct (kernels.hip) for exactly EX missing rows:
// the k survivor rows are hashed and compared with their stored sums, the EX missing
// rows rebuilt from the same loads (one HBM read per survivor), HOUT also hashes the
// rebuilt rows.  Layout as k_ehx_ws: one workgroup per CU (LDS padded), G stripes;
// the first 2*G*RH threads hash (pair form, RH = hashed rows per stripe), the other
// G*T/16 rebuild (16-byte columns, untracked loads PF tiles ahead, exact vmcnt waits).
template <int G, int RH, bool HQ>
constexpr int vr_nh() {
    // whole wavefronts; the pad chains hash a real row and discard the digest
    return HQ ? ((4 * G * RH + 63) / 64) * 64 : ((2 * G * RH + 63) / 64) * 64;
}

// HQ: quad-form hash waves (one HH lane per thread; pad quads hash a real row and
// discard the digest) for chain-latency-bound shapes (few chains per CU, e.g. RS(4+2)).
// ST: the rebuild role reads its coefficient tables with scalar loads (SGPRs) instead of
// from LDS (gf_dev.hpp load_coef_s): rebuilding e rows from k survivors needs e*k
// tables per column, which from LDS is ~10x the column's own bytes for RS(16+4), e = 4.
// BT (with ST): the scalar tables are read in batches of 4 coefficients, double-buffered
// in SGPRs: batch i+1's s_loads are issued right after the wait for batch i and land
// while batch i's 4 products are computed.  (Scalar loads return out of order, so every
// wait is lgkmcnt(0); one table per wait serialises the rebuild on scalar-cache latency.)
// NTL: non-temporal survivor loads and rebuilt-row stores.
// UA (round 3): S need not be a multiple of 16 (RS(12+4) on 1 MiB blocks: S = 87 382,
// rows 2-byte aligned).  Full tiles use the same vector accesses at the rows' byte
// offsets (unaligned-access mode); the ragged tail tile is never prefetched: each lane
// reads its columns of it byte by byte (zero past the row) and stores only the rebuilt
// bytes below S.
// BUF (round 4; aligned rows, no id list): survivor loads and rebuilt-row stores
// buffer-addressed — one per-lane VGPR offset (the lane's stripe and column inside the
// workgroup's span) and a wave-uniform SGPR offset per row — instead of one 64-bit VGPR
// address per survivor row, which the RS(16+4) 3-4-row instances kept as 16 loop
// invariants and spilled (scratch reloads in the steady loop).
// PFD (round 4): as in k_ehx_ws, the hash waves touch every 128-byte line of the survivor
// rows of tile s+PFD while hashing tile s-1 (one untracked global_load_dword per line,
// result discarded), so the rebuild waves' survivor loads hit L2.
// TSP (round 5): LDS row stride rule, as k_ehx_ws (ws_ts; 0 = the round-1 padding).
// XMAP (round 5): workgroup -> stripe-group order, as k_ehx_ws (ws_group).
// PRIO (round 5): the rebuild role's s_setprio.  The hash waves are the oldest waves of the
// workgroup, so age-ordered VALU arbitration served them first although they wait 60-80 %
// of each step at the barrier (per-wave stamps, diagnostics 424), while the younger
// rebuild wave of each SIMD finished the step alone.  Priority 1 for the rebuild role:
// RS(16+4) rebuild 2-4 / heal 2-4 5-8 % faster, RS(12+4) 3-8 %, RS(8+4) 1-4 %, RS(6+4)
// 1-4 % (profiles/r05/ab_prio_get.jsonl, diagnostics 429 = the other priority).  The
// quad-form shapes keep 0: their hash chains are few and latency-bound, and the priority
// cost RS(4+2) heal 8 % and RS(2+2) 12-20 %.
// SPL (round 5): the survivors' nibble splits are computed before the first coefficient
// batch is waited for, so its scalar loads land behind that work: RS(16+4) rebuild 3-4 /
// heal 4 and RS(8+4) rebuild 4 1.5-4 % faster, the other shapes within noise
// (profiles/r05/ab_spl.jsonl; diagnostics 434 = the other placement).
struct GetShape {
    static constexpr int G = 0;          // stripes per workgroup (every shape sets it)
    static constexpr int T = 0;          // tile: bytes of each row per step (every shape sets it)
    static constexpr int PF = 1;         // tiles of survivor prefetch in the rebuild role
    static constexpr int CW = 16;        // rebuild column width, bytes
    static constexpr bool HQ = false;    // quad-form hash waves
    static constexpr bool ST = false;    // scalar coefficient tables
    static constexpr int BT = 0;         // scalar tables per batch (0 = one per wait)
    static constexpr bool NTL = false;   // non-temporal survivor loads / rebuilt stores (set by the launch)
    static constexpr bool UA = false;    // unaligned shard sizes allowed
    static constexpr bool BUF = false;   // buffer addressing (requested; the launch decides)
    static constexpr int PFD = 0;        // L2 prefetch distance of the hash waves
    static constexpr int TSP = 0;        // LDS row stride rule
    static constexpr int XMAP = 0;       // workgroup -> stripe-group order
    static constexpr bool STH = false;   // with ST + BT: the tables' high dwords from LDS (below)
    static constexpr bool WT = false;    // diagnostics: per-wave barrier / load-wait cycle stamps
    static constexpr int WPE = 2;        // waves per SIMD the register budget is sized for
    static constexpr int LDSMIN = 83968; // dynamic-LDS floor (83 968: one workgroup per CU)
    static constexpr int PRIO = 1;       // s_setprio of the rebuild role
    static constexpr bool HF = true;     // quad-form hash role: fused packet runs (hh_update_n)
    static constexpr int ABL = 0;        // diagnostics timing ablations (output differs)
    static constexpr bool SPL = false;   // with ST + BT: survivor splits before the first table wait
    static constexpr bool DIAGMOD = false;  // a diagnostics modifier of a product shape (Tsp0, XMap, ...)
};
// The instance a launch picks for a requested shape: its memory policy (non-temporal,
// buffer-addressed) fixed by the batch (launch_vr_ws_t).
template <class C, bool NTL_, bool BUF_>
struct VrMem : C {
    static constexpr bool NTL = NTL_;
    static constexpr bool BUF = BUF_;
};

template <int K, int EX, bool HOUT, class C>
__global__ void __launch_bounds__((vr_nh<C::G, K + (HOUT ? EX : 0), C::HQ>() + C::G * (C::T / C::CW)))
__attribute__((amdgpu_waves_per_eu(C::WPE))) k_vr_ws(VrArgs a) {
    constexpr int G = C::G, T = C::T, PF = C::PF, CW = C::CW, BT = C::BT, PFD = C::PFD;
    constexpr bool HQ = C::HQ, ST = C::ST, NTL = C::NTL, UA = C::UA, BUF = C::BUF;
    // STH (round 5): a v_perm reads at most one SGPR, so with scalar tables each
    // coefficient's two high table dwords were copied to VGPRs by two v_mov per step
    // (~15 % of the rebuild role's VALU for RS(16+4) heal 4); with STH they come from an
    // LDS copy instead (one broadcast ds_read_b64 per coefficient, issued with its batch's
    // scalar loads), and the scalar loads fetch only the three dwords used as SGPRs.
    constexpr bool STH = C::STH && ST && BT > 0 && EX > 0;
    constexpr bool SPL = C::SPL && ST && BT > 0 && !STH && EX > 0;
    constexpr int RH = K + (HOUT ? EX : 0);
    constexpr int NH = vr_nh<G, RH, HQ>();
    constexpr int CPS = T / CW;
    constexpr int NE = G * CPS;
    constexpr int NT = NH + NE;
    constexpr int TS = ws_ts<T, HQ, C::TSP>();
    constexpr int NPK = T / 32;
    constexpr int NTAB = (EX > 0 ? EX : 1) * K * 8;
    static_assert(NH % 64 == 0 && NE % 64 == 0 && T % 32 == 0, "whole wavefronts per role");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_dyn[];
    uint8_t(*tile)[G * RH * TS] = reinterpret_cast<uint8_t(*)[G * RH * TS]>(smem_dyn);
    __shared__ __attribute__((aligned(16))) uint32_t tabs[NTAB];
    __shared__ int32_t srows[K + EX];
    __shared__ __attribute__((aligned(8))) uint2 htabs[STH ? EX * K : 1];

    const int tid = threadIdx.x;
    const int64_t blk0 = (int64_t)ws_group<C::XMAP>() * G;
    const int64_t S = a.S;
    const int R = a.k + a.m;
    if (EX > 0)
        for (int i = tid; i < EX * K * 8; i += NT) tabs[i] = a.tables[i];
    if constexpr (STH)
        for (int i = tid; i < EX * K; i += NT) htabs[i] = make_uint2(a.tables[8 * i + 1], a.tables[8 * i + 3]);
    // WT (diagnostics): per-wave real time, shader cycles, HW_ID and the cycles spent in
    // barriers / in the rebuild role's survivor-load waits (k_ehx_ws's stamp format: waves
    // 0..NH/64-1 of a workgroup hash, the rest rebuild)
    uint64_t rt0 = 0, ct0 = 0, wbar = 0, wvm = 0;
    if (C::WT && a.dbg) {
        rt0 = __builtin_amdgcn_s_memrealtime();
        ct0 = __builtin_amdgcn_s_memtime();
    }
    auto bar = [&]() {
        if constexpr (C::WT) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            lds_barrier2();
            wbar += __builtin_amdgcn_s_memtime() - t;
        } else {
            lds_barrier2();
        }
    };
    auto stamp = [&]() {
        if (C::WT && a.dbg && (tid & 63) == 0) {
            const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
            const uint64_t ct1 = __builtin_amdgcn_s_memtime();
            uint64_t* d = a.dbg + ((int64_t)blockIdx.x * (NT / 64) + (tid >> 6)) * 5;
            d[0] = rt0;
            d[1] = rt1;
            d[2] = ct1 - ct0;
            d[3] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
            d[4] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) | ((wbar & 0xFFFFFFF) << 8) | (wvm << 36);
        }
    };
    for (int i = tid; i < K + EX; i += NT) srows[i] = a.rows[i];
    const int64_t nfull = S / T;
    const int tail = (int)(S - nfull * T);
    int64_t iend = PF;
    if (nfull >= 3 * PF) iend = PF + ((nfull - 3 * PF) / PF + 1) * PF;
    const int64_t total = iend + 2 * PF + 1;
    // PFD: this hash thread's prefetch lines (line li = tid + q*NH of the tile's survivor
    // rows); set up after the first barrier (srows)
    constexpr int LPR = T / 128, NLN = G * K * LPR, NPL = PFD ? (NLN + NH - 1) / NH : 1;
    static_assert(PFD == 0 || T % 128 == 0, "prefetch whole 128-byte lines");
    const uint8_t* pfa[NPL];
    uint32_t sink = 0;
    auto pf_setup = [&]() {
        if constexpr (PFD > 0) {
#pragma unroll
            for (int q = 0; q < NPL; ++q) {
                const int li = tid + q * NH < NLN ? tid + q * NH : NLN - 1;
                const int r = li / LPR, gg = r / K, j = r % K;
                const int64_t bl = (blk0 + gg) < a.n_blocks ? (blk0 + gg) : (a.n_blocks - 1);
                const int64_t bb = a.ids ? (int64_t)a.ids[bl] : bl;
                pfa[q] = a.shards + bb * a.block_stride + (int64_t)srows[j] * S + (li % LPR) * 128;
            }
        }
    };
    auto pf_issue = [&](int64_t s) {
        if constexpr (PFD > 0) {
            if (s + PFD < nfull) {
#pragma unroll
                for (int q = 0; q < NPL; ++q)
                    asm volatile("global_load_dword %0, %1, off" : "+v"(sink) : "v"(pfa[q] + (s + PFD) * T));
            }
        }
    };
    auto pf_drain = [&]() {
        if constexpr (PFD > 0) asm volatile("s_waitcnt vmcnt(0)" : "+v"(sink)::"memory");
    };

    if (HQ && __builtin_amdgcn_readfirstlane(tid) < NH) {
        // ---- hash role (quad form): lane `lane` of hashed row cj of stripe g
        const int chain = tid >> 2, lane = tid & 3;
        const int crow = chain < G * RH ? chain : chain - G * RH;
        const int g = crow / RH, cj = crow % RH;
        const int row_off = crow * TS + 8 * lane;
        const uint32_t sel = zipper_sel(lane);
        HHLane st = hh_init(lane, a.key[0], a.key[1], a.key[2], a.key[3]);
        bar();  // tables / rows (matches the rebuild role)
        pf_setup();
        bar();  // step 0
        for (int64_t s = 1; s <= nfull; ++s) {
            pf_issue(s);
            const uint64_t* p = reinterpret_cast<const uint64_t*>(tile[(s - 1) & 1] + row_off);
            uint64_t w[NPK];
#pragma unroll
            for (int i = 0; i < NPK; ++i) w[i] = p[4 * i];
            if constexpr (C::HF) {
                hh_update_n<NPK>(st, w, sel);
            } else {
#pragma unroll
                for (int i = 0; i < NPK; ++i) hh_update(st, w[i], sel);
            }
            bar();
        }
        pf_drain();
        if (tail) {
            const uint8_t* row = tile[nfull & 1] + crow * TS;
            hh_packets(st, row, tail >> 5, lane, sel);
            if (tail & 31) hh_remainder(st, row + (tail & ~31), (uint32_t)(tail & 31), lane, sel);
        }
        for (int64_t s = nfull + 1; s < total; ++s) bar();
        const uint64_t h = hh_finalize256(st, lane, sel);
        const bool live = chain < G * RH && blk0 + g < a.n_blocks;
        const int64_t b = live && a.ids ? (int64_t)a.ids[blk0 + g] : blk0 + g;
        const int srow = srows[cj];
        if (cj < K) {
            bool mis = false;
            if (live) {
                uint64_t want;
                __builtin_memcpy(&want, a.expect + (b * R + srow) * 32 + 8 * lane, 8);
                mis = want != h;
            }
            const unsigned long long m = __ballot(mis);
            const bool bad = ((m >> (tid & 60)) & 0xFull) != 0;
            if (live && lane == 0) a.bad[b * R + srow] = bad ? 1 : 0;
        } else if (HOUT && live && a.sums_out) {
            *reinterpret_cast<uint64_t*>(a.sums_out + (b * R + srow) * 32 + 8 * lane) = h;
        }
        stamp();
        return;
    }
    if (!HQ && __builtin_amdgcn_readfirstlane(tid) < NH) {
        // ---- hash role (pair form): hashed row cj of stripe g (pad pairs past G*RH
        // hash row chain - G*RH again and discard the digest)
        const int chain0 = tid >> 1, hh = tid & 1;
        const bool pad = chain0 >= G * RH;
        const int chain = pad ? chain0 - G * RH : chain0;
        const int g = chain / RH, cj = chain % RH;
        const int row_off = chain * TS;
        HHPair st = hh2_init(hh, a.key[0], a.key[1], a.key[2], a.key[3]);
        bar();  // tables / rows (matches the rebuild role)
        pf_setup();
        bar();  // step 0
        for (int64_t s = 1; s <= nfull; ++s) {
            pf_issue(s);
            const uint4* p = reinterpret_cast<const uint4*>(tile[(s - 1) & 1] + row_off) + hh;
            uint4 w[NPK];
#pragma unroll
            for (int i = 0; i < NPK; ++i) w[i] = p[2 * i];
            if constexpr (C::ABL == 3) {
                // ablation: the tile's LDS reads without the HighwayHash arithmetic
#pragma unroll
                for (int i = 0; i < NPK; ++i) asm volatile("" ::"v"(w[i].x), "v"(w[i].y), "v"(w[i].z), "v"(w[i].w));
            } else {
#pragma unroll
                for (int i = 0; i < NPK; ++i)
                    hh2_update(st, ((uint64_t)w[i].y << 32) | w[i].x, ((uint64_t)w[i].w << 32) | w[i].z);
            }
            bar();
        }
        pf_drain();
        if (tail) {
            const uint8_t* row = tile[nfull & 1] + row_off;
            hh2_packets(st, row, tail >> 5, hh);
            if (tail & 31) hh2_remainder(st, row + (tail & ~31), (uint32_t)(tail & 31), hh);
        }
        for (int64_t s = nfull + 1; s < total; ++s) bar();
        uint64_t d0, d1;
        hh2_finalize256(st, d0, d1);
        const bool live = !pad && blk0 + g < a.n_blocks;
        const int64_t b = live && a.ids ? (int64_t)a.ids[blk0 + g] : blk0 + g;
        const int srow = srows[cj];
        if (cj < K) {
            // errFileCorrupt per (stripe, survivor): either half of the digest differs
            bool mis = false;
            if (live) {
                uint64_t e0, e1;
                __builtin_memcpy(&e0, a.expect + (b * R + srow) * 32 + 16 * hh, 8);
                __builtin_memcpy(&e1, a.expect + (b * R + srow) * 32 + 16 * hh + 8, 8);
                mis = e0 != d0 || e1 != d1;
            }
            const unsigned long long m = __ballot(mis);
            const bool bad = ((m >> (tid & 62)) & 3ull) != 0;
            if (live && hh == 0) a.bad[b * R + srow] = bad ? 1 : 0;
        } else if (HOUT && live && a.sums_out) {
            uint64_t* out = reinterpret_cast<uint64_t*>(a.sums_out + (b * R + srow) * 32 + 16 * hh);
            out[0] = d0;
            out[1] = d1;
        }
        stamp();
        return;
    }

    // ---- rebuild role: CW-byte column o of stripe g
    constexpr int NWd = CW / 4;
    typedef typename VecOf<NWd>::type VT;
    const int e = tid - NH;
    const int g = e / CPS, o = (e % CPS) * CW;
    const int64_t bl = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
    const int64_t b = a.ids ? (int64_t)a.ids[bl] : bl;
    uint8_t* blk = a.shards + b * a.block_stride + o;
    const int col_off = g * RH * TS + o;
    static_assert(!(BUF && UA), "buffer addressing: aligned rows");
    // BUF: the launch guarantees no id list and a span of G stripes below 2^31 bytes
    const __amdgpu_buffer_rsrc_t rs_s =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.shards + blk0 * a.block_stride), 0, 0x7FFFFFFF, 0x00020000);
    const uint32_t vo_s = (uint32_t)((bl - blk0) * a.block_stride + o);
    bar();  // tables / rows visible
    if constexpr (C::PRIO > 0) __builtin_amdgcn_s_setprio(C::PRIO);
    // row offsets in 32 bits (the launch requires (k + m) * S < 2^31): half the SGPRs
    uint32_t roff[K];
#pragma unroll
    for (int j = 0; j < K; ++j) roff[j] = (uint32_t)__builtin_amdgcn_readfirstlane(srows[j]) * (uint32_t)S;
    uint32_t ooff[EX > 0 ? EX : 1];
#pragma unroll
    for (int r = 0; r < EX; ++r) ooff[r] = (uint32_t)__builtin_amdgcn_readfirstlane(srows[K + r]) * (uint32_t)S;

    VT x[PF][K];
    // t0: wave-uniform tile offset; vx (BUF): a per-lane addition to it (the prefetch of
    // the partial last tile: lanes past the row's tail re-read tile 0), carried in the
    // VGPR offset — the SGPR offset is read from lane 0
    auto load = [&](VT (&xs)[K], int64_t t0, uint32_t vx = 0) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if constexpr (BUF) {
                static_assert(NWd == 2 || NWd == 4, "buffer loads: 8- or 16-byte columns");
                const uint32_t vo = vo_s + vx;
                // (the row offset may come out of a v_readfirstlane: an SGPR written by
                // the VALU needs 5 wait states before a VMEM instruction reads it, which
                // the compiler does not insert in front of inline asm — hence the s_nop)
                const uint32_t so = __builtin_amdgcn_readfirstlane(roff[j] + (uint32_t)t0);
                if constexpr (NWd == 4)
                    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, %3 offen nt"
                                 : "=v"(xs[j])
                                 : "v"(vo), "s"(rs_s), "s"(so)
                                 : "memory");
                else
                    asm volatile("s_nop 4\n\tbuffer_load_dwordx2 %0, %1, %2, %3 offen nt"
                                 : "=v"(xs[j])
                                 : "v"(vo), "s"(rs_s), "s"(so)
                                 : "memory");
            } else if constexpr (NTL) {
                ld_async_nt<NWd>(xs[j], blk + roff[j] + t0);
            } else {
                ld_async<NWd>(xs[j], blk + roff[j] + t0);
            }
        }
    };
    auto prefetch_any = [&](VT (&xs)[K], int64_t tn) {
        const bool ok = tn < nfull || (!UA && tn == nfull && o < tail);
        if constexpr (BUF)
            load(xs, 0, ok ? (uint32_t)(tn * T) : 0u);  // per-lane choice: VGPR offset
        else
            load(xs, ok ? tn * T : 0);
    };
    // UA tail tile: bytes [o, o + CW) of every survivor row, zero past the row
    auto tail_cols = [&](VT (&xs)[K]) {
        const uint8_t* t0p = blk + nfull * T;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            uint32_t w[NWd];
#pragma unroll
            for (int q = 0; q < NWd; ++q) {
                uint32_t v = 0;
#pragma unroll
                for (int bb = 0; bb < 4; ++bb)
                    if (o + 4 * q + bb < tail) v |= (uint32_t)t0p[roff[j] + 4 * q + bb] << (8 * bb);
                w[q] = v;
            }
            if constexpr (NWd == 1) {
                xs[j] = w[0];
            } else {
#pragma unroll
                for (int q = 0; q < NWd; ++q) xs[j][q] = w[q];
            }
        }
    };
    // survivors to LDS, rebuilt rows into y (and LDS when hashed)
    auto rebuild = [&](VT (&xr)[K], uint8_t* tl, Col<NWd> (&y)[EX > 0 ? EX : 1]) {
        Col<NWd> xs[K];
#pragma unroll
        for (int j = 0; j < K; ++j) xs[j] = to_col<NWd>(xr[j]);
        if constexpr (EX > 0) {
            const uint32_t* tb = tabs + opaque_zero();
            // opaque offset: the tables are reloaded per tile (scalar cache hits), not
            // hoisted out of the tile loop into e*k*5 SGPRs
            const ctab_ptr tg = const_tables(a.tables) + opaque_zero();
            constexpr int NB = BT > 0 ? BT : 4;  // BT: coefficients per scalar batch
            CoefTab tbat[2][NB];
            uint2 hbat[2][STH ? NB : 1];  // STH: the batch's high table dwords (VGPRs, from LDS)
            const uint2* hb = htabs + opaque_zero();
            // (a batch may straddle two rebuilt rows; the last one re-reads table EX*K-1
            // for its slots past the end)
            auto load_batch = [&](CoefTab (&d)[NB], uint2 (&h)[STH ? NB : 1], int c0) {
#pragma unroll
                for (int i = 0; i < NB; ++i) {
                    const int ci = c0 + i < EX * K ? c0 + i : EX * K - 1;
                    if constexpr (STH) {
                        d[i].ab.x = tg[8 * ci + 0];
                        d[i].ab.z = tg[8 * ci + 2];
                        d[i].c = tg[8 * ci + 4];
                        h[i] = hb[ci];
                    } else {
                        d[i] = load_coef_s(tg, ci);
                    }
                }
            };
            // BT: consume batch d (the wait for its scalar loads sits here), then issue the
            // next batch's loads, then compute; the scheduling barriers keep that order
            auto wait_batch = [&](const CoefTab (&d)[NB], const uint2 (&h)[STH ? NB : 1]) {
#pragma unroll
                for (int i = 0; i < NB; ++i) {
                    if constexpr (STH)
                        asm volatile("" ::"s"(d[i].ab.x), "s"(d[i].ab.z), "s"(d[i].c), "v"(h[i].x), "v"(h[i].y));
                    else
                        asm volatile("" ::"s"(d[i].ab.x), "s"(d[i].ab.y), "s"(d[i].ab.z), "s"(d[i].ab.w), "s"(d[i].c));
                }
                __builtin_amdgcn_sched_barrier(0);
            };
            if constexpr (ST && BT) load_batch(tbat[0], hbat[0], 0);
            // SPL: every survivor's nibble split before the first table wait (they are all
            // live across the rebuilt rows anyway), so the first batch's scalar loads land
            // behind that VALU work instead of stalling the step's first product
            Nib sp[SPL ? K : 1][NWd];
            if constexpr (SPL) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < K; ++j)
#pragma unroll
                    for (int w = 0; w < NWd; ++w) sp[j][w] = split_nibbles(xs[j].w[w]);
                __builtin_amdgcn_sched_barrier(0);
            }
            auto nib = [&](int j, int w) { return SPL ? sp[SPL ? j : 0][w] : split_nibbles(xs[j].w[w]); };
#pragma unroll
            for (int r = 0; r < EX; ++r) {
                GfAcc acc[NWd];
#pragma unroll
                for (int w = 0; w < NWd; ++w) acc_init(acc[w]);
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    if constexpr (ST && BT) {
                        // ABL 1 (ablation): every product uses the first batch's tables, so
                        // the loop issues no scalar loads and waits for none
                        const int c = r * K + j, bi = C::ABL == 1 ? 0 : c / NB, cur = bi & 1;
                        if (c % NB == 0 && (C::ABL != 1 || c == 0)) {
                            wait_batch(tbat[cur], hbat[cur]);
                            if (c + NB < EX * K && C::ABL != 1) load_batch(tbat[cur ^ 1], hbat[cur ^ 1], c + NB);
                            __builtin_amdgcn_sched_barrier(0);
                        }
                        const CoefTab t = tbat[cur][c % NB];
                        if constexpr (STH) {
                            const uint2 hi = hbat[cur][c % NB];
#pragma unroll
                            for (int w = 0; w < NWd; ++w)
                                acc_add(acc[w], gf_lookup_sh(split_nibbles(xs[j].w[w]), t, hi.x, hi.y));
                        } else {
#pragma unroll
                            for (int w = 0; w < NWd; ++w) acc_add(acc[w], gf_lookup_s(nib(j, w), t));
                        }
                    } else if constexpr (ST) {
                        const CoefTab t = load_coef_s(tg, r * K + j);
#pragma unroll
                        for (int w = 0; w < NWd; ++w) acc_add(acc[w], gf_lookup_s(split_nibbles(xs[j].w[w]), t));
                    } else {
                        const CoefTab t = load_coef(tb, r * K + j);
#pragma unroll
                        for (int w = 0; w < NWd; ++w) acc_add(acc[w], gf_lookup(split_nibbles(xs[j].w[w]), t));
                    }
                }
#pragma unroll
                for (int w = 0; w < NWd; ++w) y[r].w[w] = acc_done(acc[w]);
                // one rebuilt row at a time: its K coefficient tables, not all E*K, live
                if constexpr (!(ST && BT)) __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int j = 0; j < K; ++j) st_col<NWd>(tl + col_off + j * TS, xs[j]);
        if constexpr (HOUT) {
#pragma unroll
            for (int r = 0; r < EX; ++r) st_col<NWd>(tl + col_off + (K + r) * TS, y[r]);
        }
    };
    auto store_rows = [&](const Col<NWd> (&y)[EX > 0 ? EX : 1], int64_t t0) {
#pragma unroll
        for (int r = 0; r < EX; ++r) {
            if constexpr (BUF) {
                const int so = (int)__builtin_amdgcn_readfirstlane(ooff[r] + (uint32_t)t0);
                if constexpr (NWd == 4) {
                    const VT v = {y[r].w[0], y[r].w[1], y[r].w[2], y[r].w[3]};
                    __builtin_amdgcn_raw_buffer_store_b128(v, rs_s, (int)vo_s, so, 2);
                } else {
                    const VT v = {y[r].w[0], y[r].w[1]};
                    __builtin_amdgcn_raw_buffer_store_b64(v, rs_s, (int)vo_s, so, 2);
                }
            } else if constexpr (NTL)
                st_col_nt<NWd>(blk + ooff[r] + t0, y[r]);
            else
                st_col<NWd>(blk + ooff[r] + t0, y[r]);
        }
    };
    auto step = [&](VT (&xs)[K], int64_t ti) {
        Col<NWd> y[EX > 0 ? EX : 1];
        if constexpr (C::WT) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            vm_wait<EX + (PF - 1) * (K + EX)>(xs);
            wvm += __builtin_amdgcn_s_memtime() - t;
        } else {
            vm_wait<EX + (PF - 1) * (K + EX)>(xs);
        }
        rebuild(xs, tile[ti & 1], y);
        load(xs, (ti + PF) * T);
        store_rows(y, ti * T);
        bar();
    };
    auto store_tail = [&](const Col<NWd> (&y)[EX > 0 ? EX : 1]) {
        uint8_t* t0p = blk + nfull * T;
#pragma unroll
        for (int r = 0; r < EX; ++r)
#pragma unroll
            for (int q = 0; q < NWd; ++q)
#pragma unroll
                for (int bb = 0; bb < 4; ++bb)
                    if (o + 4 * q + bb < tail) t0p[ooff[r] + 4 * q + bb] = (uint8_t)(y[r].w[q] >> (8 * bb));
    };
    auto edge = [&](VT (&xs)[K], int64_t ti) {
        const bool full = ti < nfull, part = ti == nfull && tail;
        vm_wait<0>(xs);
        Col<NWd> y[EX > 0 ? EX : 1];
        if constexpr (UA) {
            if (part) tail_cols(xs);
        }
        if (full || part) rebuild(xs, tile[ti & 1], y);
        prefetch_any(xs, ti + PF);
        if constexpr (UA) {
            if (full) store_rows(y, ti * T);
            else if (part && o < tail) store_tail(y);
        } else {
            if (full || (part && o < tail)) store_rows(y, ti * T);
        }
        bar();
    };
#pragma unroll
    for (int p = 0; p < PF; ++p) prefetch_any(x[p], p);
    // edge(0) is step 0: its barrier pairs with the hash role's second barrier
#pragma unroll
    for (int p = 0; p < PF; ++p) edge(x[p], p);
    int64_t i = PF;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; i + 2 * PF <= nfull; i += PF) {
#pragma unroll
        for (int p = 0; p < PF; ++p) step(x[p], i + p);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < 2 * PF; ++p) edge(x[p % PF], i + p);
    bar();  // the hash-only step
#pragma unroll
    for (int p = 0; p < PF; ++p) vm_wait<0>(x[p]);
    stamp();
}

template <int K, int EX, bool HOUT, class C>
static bool launch_vr_inst(const VrArgs& a, hipStream_t s);

// Shape modifiers (diagnostics A/B of a product shape): the conflict-free LDS row stride,
// the region-interleaved workgroup order.
template <class C, int P>
struct XMap : C {
    static constexpr int XMAP = P;
    static constexpr bool DIAGMOD = true;
};
template <class C>
struct Tsp0 : C {
    static constexpr int TSP = 0;
    static constexpr bool DIAGMOD = true;
};
template <class C>
struct Stamped : C {
    static constexpr bool WT = true;
    static constexpr bool DIAGMOD = true;
};
template <class C>
struct Sth : C {
    static constexpr bool STH = true;
    static constexpr bool DIAGMOD = true;
};
// The rebuild role's issue priority (PRIO above k_vr_ws).
template <class C, int P>
struct RbPrio : C {
    static constexpr int PRIO = P;
    static constexpr bool DIAGMOD = true;
};
// Survivor splits before the first table wait (SPL above k_vr_ws).
template <class C, bool S>
struct Spl : C {
    static constexpr bool SPL = S;
    static constexpr bool DIAGMOD = true;
};
// Timing ablation of a product shape (output differs).
template <class C, int A>
struct Abl : C {
    static constexpr int ABL = A;
    static constexpr bool DIAGMOD = true;
};
// Encode issue-priority scheme (PM above k_ehx_ws).
template <class C, int P>
struct Pm : C {
    static constexpr int PM = P;
    static constexpr bool DIAGMOD = true;
};
// C itself when P == 0 (product instances keep their shape's name)
template <class C, int P>
using WithXMap = std::conditional_t<P == 0, C, XMap<C, P>>;

// Launch a requested GET shape: the instance's memory policy follows the batch.
template <int K, int EX, bool HOUT, class C>
static bool launch_vr_ws_t(const VrArgs& a, hipStream_t s) {
#if ZS3_DIAG
    // Diagnostics A/B of a product GET shape (one modifier at a time: a modified shape is
    // not modified again): 420 = the round-4 LDS row stride (TSP 0) on the pair-form
    // shapes of k = 8 / 12 / 16; 423 = the tables' high dwords from LDS (STH) on the
    // scalar-table shapes of k = 8 / 12 / 16; 424 = per-wave stamps (WT).  Instantiated for those k only:
    // every modifier multiplies the diagnostics library by the product GET instances.
    // (421, the region-interleaved workgroup order, measured within +-1 % on k = 8 / 12 /
    // 16 twice this round and was removed: profiles/r05/ab_get.jsonl, ab_get12_xmap.jsonl.)
    if constexpr (!C::DIAGMOD) {
        if constexpr (C::TSP == 1 && !C::HQ && (K == 8 || K == 12 || K == 16)) {
            if (a.variant == 420) return launch_vr_ws_t<K, EX, HOUT, Tsp0<C>>(a, s);
        }
        if constexpr (C::ST && C::BT > 0 && EX > 0 && (K == 8 || K == 12 || K == 16)) {
            if (a.variant == 423) return launch_vr_ws_t<K, EX, HOUT, Sth<C>>(a, s);
        }
        // 424: the product shape with per-wave stamps (k = 8 / 12 / 16)
        if constexpr (K == 8 || K == 12 || K == 16) {
            if (a.variant == 424) return launch_vr_ws_t<K, EX, HOUT, Stamped<C>>(a, s);
        }
        // 431 / 433: timing ablations (output differs) of RS(16+4) rebuild / heal 4 and
        // RS(12+4) rebuild / heal 2: every product on the first batch's tables (no scalar
        // table loads in the loop) / no HighwayHash arithmetic
        if constexpr (((K == 16 && EX == 4) || (K == 12 && EX == 2)) && C::ST && C::BT > 0 && !C::HQ) {
            if (a.variant == 431) return launch_vr_ws_t<K, EX, HOUT, Abl<C, 1>>(a, s);
            if (a.variant == 433) return launch_vr_ws_t<K, EX, HOUT, Abl<C, 3>>(a, s);
        }
        // 434: the other survivor-split placement (SPL) on the scalar-table shapes
        if constexpr (C::ST && C::BT > 0 && !C::HQ && EX >= 1 && (K == 8 || K == 12 || K == 16)) {
            if (a.variant == 434) return launch_vr_ws_t<K, EX, HOUT, Spl<C, !C::SPL>>(a, s);
        }
        // 429: the other rebuild-role priority (the pair-form shapes without it, as in round
        // 4; the quad-form shapes with it)
        if constexpr (K == 2 || K == 4 || K == 6 || K == 8 || K == 12 || K == 16) {
            if (a.variant == 429) return launch_vr_ws_t<K, EX, HOUT, RbPrio<C, C::PRIO ? 0 : 1>>(a, s);
        }
    }
#endif
    if constexpr (C::BUF && !C::UA) {
        // buffer addressing needs the G stripes of a workgroup in order (no id list) and
        // their span below 2^31 bytes; otherwise the 64-bit-address instance (diagnostics
        // 247: always that one)
        if (!a.ids && (int64_t)C::G * a.block_stride < ((int64_t)1 << 31) && a.block_stride > 0 &&
            !(ZS3_DIAG && a.variant == 247 && !C::DIAGMOD))
            return launch_vr_inst<K, EX, HOUT, VrMem<C, true, true>>(a, s);
        return launch_vr_inst<K, EX, HOUT, VrMem<C, true, false>>(a, s);
    }
    if constexpr (C::UA) {
        // plain (temporal) survivor loads: with unaligned rows each tile's first and last
        // 128-byte lines are shared with the neighbouring tiles, and non-temporal loads
        // fetched them twice (RS(12+4) rebuild 2: HBM traffic 1.205 x algorithmic,
        // profiles/r03/final_session3/bench_paths_roofline.jsonl)
        return launch_vr_inst<K, EX, HOUT, VrMem<C, false, false>>(a, s);
    } else {
        // Survivor loads and rebuilt-row stores are non-temporal (each byte is touched once):
        // RS(8+4) verify 0.706 -> 0.627 ms, RS(16+4) verify 0.386 -> 0.351, rebuild 1-4 and
        // heals 1-5 % faster (profiles/r02/ab_get_nt.jsonl).  Diagnostics 246: plain loads.
        if constexpr (ZS3_DIAG && (K == 8 || K == 16) && !C::DIAGMOD) {
            if (a.variant == 246) return launch_vr_inst<K, EX, HOUT, VrMem<C, false, false>>(a, s);
        }
        return launch_vr_inst<K, EX, HOUT, VrMem<C, true, false>>(a, s);
    }
}

template <int K, int EX, bool HOUT, class C>
static bool launch_vr_inst(const VrArgs& a, hipStream_t s) {
    constexpr int G = C::G, T = C::T, CW = C::CW;
    constexpr int RH = K + (HOUT ? EX : 0);
    constexpr int NT = vr_nh<G, RH, C::HQ>() + G * (T / CW);
    constexpr size_t tiles = (size_t)2 * G * RH * ws_ts<T, C::HQ, C::TSP>();
    constexpr size_t dyn = tiles > (size_t)C::LDSMIN ? tiles : (size_t)C::LDSMIN;
    static_assert(G > 0 && T > 0, "a shape names its stripes per workgroup and tile length");
    if constexpr (dyn + (size_t)(EX > 0 ? EX : 1) * K * (32 + (C::STH ? 8 : 0)) + 4 * (K + EX) > 163840 || NT > 1024 ||
                  vr_nh<G, RH, C::HQ>() % 64 != 0 || (G * (T / CW)) % 64 != 0) {
        return false;
    } else {
        if (a.e != EX || (!C::UA && (a.S % 16) != 0) || a.k != K || (HOUT != (a.sums_out != nullptr) && EX > 0))
            return false;
        if ((int64_t)(a.k + a.m) * a.S >= ((int64_t)1 << 31)) return false;  // 32-bit row offsets
        auto kern = k_vr_ws<K, EX, HOUT, C>;
        if (ensure_dyn_lds((const void*)kern, dyn) != hipSuccess) return false;
        const int64_t grid = (a.n_blocks + G - 1) / G;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), dyn, s, a);
        return true;
    }
}

// ---- The product shapes (named; the dispatch in fused_v2.hip, fused_v2_gen.hip,
// fused_v2_get.hip and fused_v2_get_gen.hip says which batch takes which, and why) --------
namespace shape {

// Encode + sums (k_ehx_ws).
// Pair-form hash waves, 16 stripes of 384-byte tiles, non-temporal loads and stores,
// encode waves at priority 1: the large-batch shape of the dyadic geometries.
struct PairG16 : EncShape {
    static constexpr int G = 16, T = 384, PM = 1, NTM = 3;
};
// RS(8+4) above 2048 stripes (the BASELINE config-4 bench): PairG16 with buffer-addressed
// columns and the conflict-free LDS row stride (round 4), and the region-interleaved
// workgroup order over 8 regions (round 5: each XCD walks its own eighth of the batch;
// 65 536 x 1 MiB 19.52 -> 18.77 ms, profiles/r05/xmap84.jsonl); round 6: the nibble
// splits of dword pairs by 64-bit shifts (S64: 65 536 x 1 MiB 18.58-18.68 -> 18.20-18.27
// ms, profiles/r06/ab_split64.jsonl).
struct Rs84Bulk : PairG16 {
    static constexpr bool BUF = true, S64 = true;
    static constexpr int TSP = 1, XMAP = 8;
};
// RS(4+4) above 2048 stripes: PairG16 with the conflict-free LDS row stride (round 5:
// 4 096 / 16 384 x 1 MiB 1.78-1.83 / 7.09-7.14 ms either way, bank conflicts 20 % -> 0);
// round 6: S64 (16 384: 7.10-7.14 -> 7.07-7.09 ms, profiles/r06/ab_split64b.jsonl).
struct Rs44Bulk : PairG16 {
    static constexpr int TSP = 1;
    static constexpr bool S64 = true;
};
// RS(8+4) up to 2048 stripes: 4 stripes of 1 KiB tiles, quad-form hash waves, two tiles
// of prefetch, one workgroup per CU (LDSMIN), the 256-VGPR budget.
struct Rs84Mid : EncShape {
    static constexpr int G = 4, T = 1024, PF = 2, LDSMIN = 83968, NTM = 3, WPE = 2;
    static constexpr bool HQ = true;
};
// RS(16+4) above 1024 stripes: 8 stripes of 384-byte tiles, 8-byte buffer-addressed
// columns, data rows to LDS before the encode; round 5: conflict-free LDS rows and the
// region-interleaved workgroup order (8 192 x 1 MiB 2.342-2.370 -> 2.314-2.341 ms,
// diagnostics 417, profiles/r05/ab_enc2.jsonl), then the encode waves at issue priority 1
// (PM 1, as the RS(8+4) shape: 2.37-2.40 -> 2.28-2.29 ms, diagnostics 403 before its
// adoption, profiles/r05/ab_prio_enc.jsonl).
struct Rs164Bulk : EncShape {
    static constexpr int G = 8, T = 384, NTM = 3, EP = 2, TSP = 1, XMAP = 8, PM = 1;
    static constexpr bool BUF = true;
};
// Quad-form hash waves on 4 stripes of 512-byte tiles (RS(16+4) / RS(12+4) small batches).
struct Quad512 : EncShape {
    static constexpr int G = 4, T = 512, NTM = 3;
    static constexpr bool BUF = true, HQ = true;
};
// RS(12+4) at 16-byte-aligned rows above 1024 stripes: the unaligned-row recipe (8-byte
// columns of 512-byte tiles, L2 prefetch two tiles ahead, conflict-free LDS rows).
struct Rs124AlignedBulk : EncShape {
    static constexpr int G = 8, T = 512, CWX = 8, NTM = 3, EP = 2, PFD = 2, TSP = 1;
    static constexpr bool BUF = true, UA = true;
};
// Small batches of the dyadic shapes: 4 stripes of 512-byte tiles, quad-form hash waves,
// 4 tiles of prefetch, one workgroup per CU (NTM: 3 = nt loads and stores, 2 = stores).
template <int NTM_>
struct QuadSmall : EncShape {
    static constexpr int G = 4, T = 512, PF = 4, LDSMIN = 83968, NTM = NTM_;
    static constexpr bool HQ = true;
};
// BASELINE config 2 (RS(4+2), 1024-2048 stripes): 2 KiB tiles so each latency-bound
// chain hashes 64 packets between barriers.
struct Config2 : EncShape {
    static constexpr int G = 4, T = 2048, PF = 2, LDSMIN = 83968, NTM = 3;
    static constexpr bool HQ = true;
};
// RS(12+4) on 1 MiB blocks (unaligned rows), above 1024 stripes: 4 stripes of 1 KiB
// tiles, quad-form hash waves issuing the L2 prefetch, 16-byte columns (round 4).
// Round 5: with the region-interleaved workgroup order (4 096 / 16 384 x 1 MiB
// 1.37-1.39 / 5.46-5.48 -> 1.33-1.34 / 5.37-5.38 ms, profiles/r05/ab_enc.jsonl).
struct Rs124Ua1K : EncShape {
    static constexpr int G = 4, T = 1024, CWX = 16, NTM = 3, EP = 2, PFD = 2, WPE = 2, TSP = 1, XMAP = 8;
    static constexpr bool BUF = true, HQ = true, UA = true;
    static constexpr bool S64 = true;  // round 6: 16 384 x 1 MiB 5.43-5.45 -> 5.37-5.42 ms (ab_split64b.jsonl)
};
struct Rs124UaSmall : EncShape {
    static constexpr int G = 4, T = 512, NTM = 3;
    static constexpr bool BUF = true, HQ = true, UA = true;
};
// General M x K matrix (the non-dyadic server defaults), unaligned rows, L2 prefetch,
// conflict-free LDS rows: k <= 3 on 8 stripes of 1 KiB tiles; RS(4+3) on 16 stripes of
// 512; RS(5+4) / RS(6+4) on the RS(12+4) 1 KiB quad-form shape; the rest 8 stripes of 512
// with 8-byte columns.
struct GenBase : EncShape {
    static constexpr int NTM = 3, PFD = 2, TSP = 1;
    static constexpr bool BUF = true, UA = true, GEN = true;
};
struct GenLong1K : GenBase {
    static constexpr int G = 8, T = 1024, CWX = 16;
};
struct Gen16x512 : GenBase {
    static constexpr int G = 16, T = 512, CWX = 16;
};
struct GenQuad1K : GenBase {
    static constexpr int G = 4, T = 1024, CWX = 16, WPE = 2;
    static constexpr bool HQ = true;
};
struct Gen8x512 : GenBase {
    static constexpr int G = 8, T = 512, CWX = 8;
};

// GET / heal (k_vr_ws), requested shapes (launch_vr_ws_t fixes the memory policy).
// Round 5: every pair-form shape uses the conflict-free LDS row stride (TSP 1):
// SQ_LDS_BANK_CONFLICT 25 % -> 0 % of SQ_LDS_IDX_ACTIVE at equal time (diagnostics 420,
// profiles/r05/pmc_lds_get.json, get_ab.jsonl); the quad-form shapes already had it.
// RS(4+m): 8 stripes, quad-form hash waves; verify on 256-byte tiles, rebuild / heal on
// 1 KiB tiles (PF tiles of prefetch).
template <int T_, int PF_>
struct K4Quad : GetShape {
    static constexpr int G = 8, T = T_, PF = PF_, PRIO = 0;
    static constexpr bool HQ = true;
};
// RS(8+4): 16 stripes of 256-byte tiles (verify, rebuild 1-2); 8-byte columns with
// batched scalar tables for rebuild 3-4; heal 1-2 on 128-byte tiles, heal 3-4 on 256 with
// 16-byte columns.
struct K8Get : GetShape {
    static constexpr int G = 16, T = 256, PF = 2, TSP = 1;
};
struct K8Rebuild34 : GetShape {
    static constexpr int G = 16, T = 256, CW = 8, BT = 4, TSP = 1;
    static constexpr bool ST = true, BUF = true, SPL = true;
};
struct K8Heal12 : GetShape {
    static constexpr int G = 16, T = 128, PF = 2, CW = 8, BT = 4, TSP = 1;
    static constexpr bool ST = true;
};
struct K8Heal34 : GetShape {
    static constexpr int G = 16, T = 256, CW = 16, BT = 4, TSP = 1;
    static constexpr bool ST = true, BUF = true;
};
// RS(16+4): 8 stripes; verify on 256-byte tiles; rebuild 1-2 with 4-byte columns (one
// table per wait); rebuild 3-4 with 8-byte columns of 512; heal with 8-byte columns of 384.
struct K16Verify : GetShape {
    static constexpr int G = 8, T = 256, PF = 2, TSP = 1;
};
struct K16Rebuild12 : GetShape {
    static constexpr int G = 8, T = 256, PF = 2, CW = 4, TSP = 1;
    static constexpr bool ST = true;
};
struct K16Rebuild34 : GetShape {
    static constexpr int G = 8, T = 512, CW = 8, BT = 4, TSP = 1;
    static constexpr bool ST = true, BUF = true, SPL = true;
};
struct K16Heal : GetShape {
    static constexpr int G = 8, T = 384, CW = 8, BT = 4, TSP = 1;
    static constexpr bool ST = true, BUF = true, SPL = true;
};
// RS(12+4) and k = 9-11: 8 stripes of 8-byte columns of 512-byte tiles, unaligned rows.
template <bool UA_>
struct Wide512 : GetShape {
    static constexpr int G = 8, T = 512, CW = 8, BT = 4, TSP = 1;
    static constexpr bool ST = true, UA = UA_;
};
// k = 2, 3: 8 stripes of 1 KiB tiles, quad-form hash waves; k = 5-7: 16 stripes of 256.
template <bool UA_>
struct GenGetQuad1K : GetShape {
    static constexpr int G = 8, T = 1024, PF = 2, BT = 4, PRIO = 0;
    static constexpr bool HQ = true, ST = true, UA = UA_;
};
template <bool UA_>
struct GenGet16x256 : GetShape {
    static constexpr int G = 16, T = 256, CW = 8, BT = 4, TSP = 1;
    static constexpr bool ST = true, UA = UA_;
};

}  // namespace shape

#if ZS3_DIAG
// Encode variants of the diagnostics build (fused_v2_diag.hip, fused_v2_gen.hip)
bool launch_ehx_diag(int v, const EncArgs& a, hipStream_t s);
bool launch_ehx_gen_xmap(const EncArgs& a, hipStream_t s);
#endif

}  // namespace zs3k
