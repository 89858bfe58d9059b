// fused_dma.hip — fused Split + Encode + HighwayHash-256 with the data rows moved by
// LDS-DMA (global_load_lds_dwordx4): the third-generation RS(8+4)-shaped kernel.
//
// Replaces the arithmetic of Erasure.EncodeData (cmd/erasure-coding.go:77-91) plus the
// k+m streamingBitrotWriter sums (cmd/bitrot-streaming.go:43-65), like k_ehx_ws
// (fused_v2.hip), whose roles it keeps: G stripes per workgroup, one workgroup per CU,
// pair-form hash waves (one HighwayHash chain per thread pair) beside encode waves
// (one 16-byte column each).  What changes is how the data rows reach LDS:
//  * k_ehx_ws loads each data column into VGPRs, encodes, then writes all K data rows
//    and the M parity rows to the LDS tile (12 ds_write_b128 per encode lane and tile,
//    13 issue cycles each) so the hash waves can read rows serially; its VGPRs hold one
//    tile of prefetch, issued after the encode, so a load has about half a step to land.
//  * here the encode waves DMA the data rows of tile s+1 straight into a third LDS slot
//    at the START of step s (no VGPR destination, no ds_write), wait for tile s's DMA
//    (issued a full step earlier) with a counted vmcnt, read their own columns back
//    (ds_read_b128, 4 cycles), encode, and write only the M parity rows to LDS.
// Slots: tile s is encoded in step s and hashed in step s+1 (slot s % 3); the DMA of
// tile s+1 overwrites the slot of tile s-2, which the hash waves finished before the
// barrier that ended step s-1.  Barriers are raw s_barrier with lgkmcnt(0) only: an
// LDS-DMA in flight is a pending write on the VM counter that must stay in flight
// across the barrier (cdna_hip_programming.md, "Pipelining across barriers").
//
// LDS layout (one dynamic array; the coefficient tables first): per slot and stripe,
// R/4 groups of 4 rows x T bytes, each group 1 KiB (T = 256: one DMA wave-instruction,
// lane-linear: lane l -> row l/16 of the group, bytes (l%16)*16) plus 32 bytes of pad,
// so that a stripe spans 3 x 1056 B = 792 dwords (24 mod 64) and the 8 chains a
// ds_read_b128 lane group serves (8 stripes of one row, see the chain mapping) land on
// 8 distinct 8-dword bank groups.
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "hh256_dev.hpp"

using namespace zs3dev;

namespace zs3k {

namespace {

__device__ __forceinline__ void dma_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int N>
__device__ __forceinline__ void dma_vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One LDS-DMA wave-instruction: every lane copies 16 bytes from its own global address
// to lds_base + 16 * lane.  M0 carries the LDS base; it is compiler-reserved, so it is
// saved and restored inside the same statement.
__device__ __forceinline__ void dma16(const uint8_t* gsrc, uint32_t lds_base) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_base))
        : "memory");
}

}  // namespace

template <int K, int M, int G, int T>
constexpr size_t dma_slot_bytes() {
    return (size_t)G * ((K + M) / 4) * (4 * T + 32);
}

template <int K, int M, int G, int T>
__global__ void __launch_bounds__(2 * G * (K + M) + G * (T / 16)) __attribute__((amdgpu_waves_per_eu(2)))
k_ehx_dma(EncArgs a) {
    constexpr int R = K + M;
    constexpr int NH = 2 * G * R;        // hash threads (pair form)
    constexpr int CPS = T / 16;          // 16-byte encode columns per stripe row
    constexpr int NE = G * CPS;          // encode threads
    constexpr int GRP = 4 * T + 32;      // 4-row group + pad
    constexpr int SST = (R / 4) * GRP;   // stripe stride in a slot
    constexpr int SLOT = G * SST;
    constexpr int NPK = T / 32;
    constexpr int NTAB = K * 8;
    constexpr int TABB = NTAB * 4;       // table bytes at the front of the array
    static_assert(T == 256 && K % 4 == 0 && M == 4, "4-row DMA groups of 1 KiB (T = 256), RS(4j+4)");
    static_assert(NH % 64 == 0 && NE % 64 == 0 && (CPS * 4) % 64 == 0, "whole wavefronts; 4 stripes per encode wave");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_dma[];
    uint32_t* tabs = reinterpret_cast<uint32_t*>(smem_dma);
    uint8_t* slots = smem_dma + TABB;
    // LDS byte address of slot 0 (generic -> LDS address-space cast: the 32-bit offset)
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)slots;

    const int tid = threadIdx.x;
    const int64_t blk0 = (int64_t)blockIdx.x * G;
    const int64_t S = a.S;
    const int64_t nfull = S / T;  // launch: S % T == 0
    for (int i = tid; i < NTAB; i += NH + NE) tabs[i] = a.dtables[i];

    auto row_off = [](int slot, int g, int j) { return slot * SLOT + g * SST + (j >> 2) * GRP + (j & 3) * T; };

    if (__builtin_amdgcn_readfirstlane(tid) < NH) {
        // ---- hash role: chain (row j, stripe g), pair index pi = tid / 2:
        // 32 pairs per wave = 2 rows x 16 stripes, so a ds_read_b128 lane group (8
        // pairs) reads 8 stripes of one row: 8 distinct bank groups (3g mod 8)
        const int pi = tid >> 1, hh = tid & 1;
        const int j = pi / G, g = pi % G;
        HHPair st = hh2_init(hh, a.key[0], a.key[1], a.key[2], a.key[3]);
        dma_barrier();  // tables
        dma_barrier();  // step 0: tile 0 encoded
        int slot = 0;
        for (int64_t s = 1; s <= nfull; ++s) {
            const uint4* p = reinterpret_cast<const uint4*>(slots + row_off(slot, g, j)) + hh;
            uint4 w[NPK];
#pragma unroll
            for (int i = 0; i < NPK; ++i) w[i] = p[2 * i];
#pragma unroll
            for (int i = 0; i < NPK; ++i)
                hh2_update(st, ((uint64_t)w[i].y << 32) | w[i].x, ((uint64_t)w[i].w << 32) | w[i].z);
            slot = slot == 2 ? 0 : slot + 1;
            dma_barrier();
        }
        uint64_t d0, d1;
        hh2_finalize256(st, d0, d1);
        if (blk0 + g < a.n_blocks) {
            uint64_t* out = reinterpret_cast<uint64_t*>(a.sums + ((blk0 + g) * R + j) * 32 + 16 * hh);
            out[0] = d0;
            out[1] = d1;
        }
        return;
    }

    // ---- encode role: 16-byte column o of stripe g; wave w DMAs the data rows of its
    // own 4 stripes (K/4 groups each), so its column reads wait only for its own DMAs
    const int e = tid - NH;
    const int g = e / CPS, o = (e % CPS) * 16;
    const int w4 = __builtin_amdgcn_readfirstlane((e >> 6) * 4);  // first stripe of this wave
    const int lane = e & 63;
    typedef uint32_t V4 __attribute__((ext_vector_type(4)));
    auto blk_of = [&](int gg) { return (blk0 + gg) < a.n_blocks ? (blk0 + gg) : (a.n_blocks - 1); };
    const int64_t b = blk_of(g);
    uint8_t* pdst = a.parity + b * a.parity_stride + o;
    // this lane's part of every DMA: row l/16 of a 4-row group, bytes (l%16)*16
    const int64_t lane_off = (int64_t)(lane >> 4) * S + (lane & 15) * 16;
    const uint8_t* dsrc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dsrc[q] = a.data + blk_of(w4 + q) * a.data_stride + lane_off;
    auto issue = [&](int64_t t, int slot) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int grp = 0; grp < K / 4; ++grp)
                dma16(dsrc[q] + (int64_t)grp * 4 * S + t * T, lds0 + (uint32_t)row_off(slot, w4 + q, 4 * grp));
    };
    constexpr int NDMA = 4 * (K / 4);  // DMA instructions per wave and tile
    dma_barrier();  // tables visible
    issue(0, 0);
    int slot = 0;
    for (int64_t s = 0; s < nfull; ++s) {
        const int nslot = slot == 2 ? 0 : slot + 1;
        // DMA of tile s+1 first, then wait for tile s's (issued a step earlier); after it
        // only the parity stores of step s-1 and this step's DMAs may still be in flight
        if (s + 1 < nfull) {
            issue(s + 1, nslot);
            if (s > 0) dma_vm_wait<NDMA + M>(); else dma_vm_wait<NDMA>();
        } else {
            if (s > 0) dma_vm_wait<M>(); else dma_vm_wait<0>();
        }
        Col<4> xs[K];
#pragma unroll
        for (int jj = 0; jj < K; ++jj) {
            const V4 v = *reinterpret_cast<const V4*>(slots + row_off(slot, g, jj) + o);
            xs[jj].w[0] = v.x;
            xs[jj].w[1] = v.y;
            xs[jj].w[2] = v.z;
            xs[jj].w[3] = v.w;
        }
        Col<4> par[M];
        encode_dyadic<4, K, M, true, false, false>(xs, par, tabs);
#pragma unroll
        for (int r = 0; r < M; ++r) {
            const V4 v = {par[r].w[0], par[r].w[1], par[r].w[2], par[r].w[3]};
            *reinterpret_cast<V4*>(slots + row_off(slot, g, K + r) + o) = v;
            __builtin_nontemporal_store(v, reinterpret_cast<V4*>(pdst + (int64_t)r * S + s * T));
        }
        slot = nslot;
        dma_barrier();
    }
    dma_barrier();  // the hash-only step
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int K, int M, int G, int T>
static bool launch_dma_t(const EncArgs& a, hipStream_t s) {
    constexpr int NT = 2 * G * (K + M) + G * (T / 16);
    constexpr size_t dyn = (size_t)K * 32 + 3 * dma_slot_bytes<K, M, G, T>();
    if constexpr (dyn > 163840 || NT > 1024) {
        return false;
    } else {
        if (a.dyb != M || a.k != K || a.m != M || (a.S % T) != 0 || a.n != (int64_t)K * a.S || !a.sums) return false;
        if ((((uintptr_t)a.data | (uintptr_t)a.parity | (uint64_t)a.data_stride | (uint64_t)a.parity_stride) & 15) != 0)
            return false;
        auto kern = k_ehx_dma<K, M, G, T>;
        if (ensure_dyn_lds((const void*)kern, dyn) != hipSuccess) return false;
        const int64_t grid = (a.n_blocks + G - 1) / G;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), dyn, s, a);
        return true;
    }
}

int launch_ehx_dma(int v, const EncArgs& a, hipStream_t s) {
    (void)v;
    if (a.k == 8 && a.m == 4) return launch_dma_t<8, 4, 16, 256>(a, s) ? PATH_WS : PATH_NONE;
    return PATH_NONE;
}

}  // namespace zs3k
