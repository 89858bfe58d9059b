// kernels.hip — gfx950 kernels for the erasure-shard + bitrot-hash data path.
//
// Replaces the arithmetic behind:
//   Erasure.EncodeData                cmd/erasure-coding.go:77-91  (Split + Encode)
//   Erasure.DecodeDataBlocks          cmd/erasure-coding.go:96-109 (ReconstructData)
//   Erasure.DecodeDataAndParityBlocks cmd/erasure-coding.go:113-119 (Reconstruct)
//   streamingBitrotWriter.Write       cmd/bitrot-streaming.go:43-65 (HH256 per shard chunk)
//   streamingBitrotReader.ReadAt      cmd/bitrot-streaming.go:142-189 (HH256 verify)
//
// Design: the fused kernel owns G whole (object, block) stripes per
// workgroup and walks them in tiles of T bytes per shard row.  Each tile:
//   1. data columns (16 B per thread per shard) are loaded with coalesced
//      global_load_dwordx4 one tile AHEAD into registers,
//   2. the m parity columns are computed in registers (v_perm nibble tables +
//      v_bitop3 XOR3), data+parity are written to an LDS tile, parity is stored,
//   3. each quad hashes one shard row of the tile from LDS (HighwayHash lane per
//      thread), so every stripe byte is read from HBM once and parity is hashed
//      without being re-read.
// HBM traffic per block = B (data) + B*m/k (parity) + 32*(k+m) (sums).
#include "kernels.hpp"
#include "gf_dev.hpp"
#include "hh256_dev.hpp"

#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <set>
#include <tuple>
#include <type_traits>

using namespace zs3dev;

namespace zs3k {

thread_local uint32_t t_kernel_bits = 0;

void note_kernel(uint32_t bit) { t_kernel_bits |= bit; }

uint32_t kernel_bits(bool reset) {
    const uint32_t b = t_kernel_bits;
    if (reset) t_kernel_bits = 0;
    return b;
}

hipError_t ensure_dyn_lds(const void* kern, size_t bytes) {
    static std::mutex mu;
    static std::set<std::tuple<const void*, int, size_t>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const auto key = std::make_tuple(kern, dev, bytes);
    std::lock_guard<std::mutex> g(mu);
    if (done.count(key)) return hipSuccess;
    e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) done.insert(key);
    return e;
}

// Barrier that only drains LDS traffic: __syncthreads() would also wait for the
// tile prefetch (vmcnt(0)) and serialise HBM latency with the hash phase.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);  // global_load_dwordx4 (unaligned-access mode)
    return v;
}
__device__ __forceinline__ void st16(uint8_t* p, const uint4& v) { __builtin_memcpy(p, &v, 16); }
// Ragged columns of the unaligned-row kernels: nv = valid bytes of the row from the
// column's start.  Shift = 0 (whole column valid), 16 (none: nothing is read) or the
// bytes the 16-byte load must start early so that it ends at the row's valid end.
__device__ __forceinline__ int tail_shift(int64_t nv) { return nv >= 16 ? 0 : (nv <= 0 ? 16 : (int)(16 - nv)); }
// bytes [sh, 16) of v moved to [0, 16 - sh), zero above; sh in [1, 16]
__device__ __forceinline__ uint4 shr_bytes_zero(const uint4& v, int sh) {
    if (sh >= 16) return make_uint4(0, 0, 0, 0);
    const uint32_t w[8] = {v.x, v.y, v.z, v.w, 0u, 0u, 0u, 0u};
    const int q = sh >> 2;
    const uint32_t r = (uint32_t)(sh & 3);
    uint32_t t[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t a = q & 1 ? w[i + 1] : w[i];
        const uint32_t b = q & 1 ? w[i + 3] : w[i + 2];
        t[i] = q & 2 ? b : a;
    }
    return make_uint4(__builtin_amdgcn_alignbyte(t[1], t[0], r), __builtin_amdgcn_alignbyte(t[2], t[1], r),
                      __builtin_amdgcn_alignbyte(t[3], t[2], r), __builtin_amdgcn_alignbyte(t[4], t[3], r));
}
// the first nv (< 16) bytes of v to p (any alignment): whole dwords, then bytes; fully
// unrolled (a byte loop with a run-time trip count kept every parity row of the unrolled
// K x M encode live across it: 343 VGPRs for RS(12+4))
__device__ __forceinline__ void st16_part(uint8_t* p, const uint4& v, int64_t nv) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (4 * i + 4 <= nv) {
            __builtin_memcpy(p + 4 * i, &w[i], 4);
        } else {
#pragma unroll
            for (int b = 0; b < 3; ++b)
                if (4 * i + b < nv) p[4 * i + b] = (uint8_t)(w[i] >> (8 * b));
        }
    }
}
// Non-temporal forms (bytes streamed once: nt cache policy).  p must be 16-byte aligned.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16_nt(const uint8_t* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16_nt(uint8_t* p, const uint4& v) {
    const u32x4 t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(p));
}


constexpr int gcd_c(int a, int b) { return b ? gcd_c(b, a % b) : a; }

// Stripes per workgroup: smallest G making 4*G*(k+m) a multiple of 64 (so every
// hash lane of every wavefront is used), capped at 512 hash threads.
template <int R>
constexpr int pick_G() {
    int g = 16 / gcd_c(R, 16);
    while (g > 1 && 4 * g * R > 512) g /= 2;
    while (4 * g * R < 192) g *= 2;  // at least three wavefronts per workgroup
    return g;
}
constexpr int round64(int x) { return (x + 63) / 64 * 64; }

// Tile bytes per shard row so that NBUF LDS tiles stay under ~40 KiB (3-4
// workgroups resident per CU).
template <int ROWS, int NBUF>
constexpr int pick_T() {
    return (NBUF * ROWS * (1024 + 32) <= 40960) ? 1024
         : (NBUF * ROWS * (512 + 32) <= 40960)  ? 512
                                                 : 256;
}

// ---------------------------------------------------------------------------
// Fused Split + Encode + HighwayHash-256 over G stripes per workgroup.
// CW = bytes per encode column per thread (16 -> dwordx4 loads, 8 -> dwordx2, 4 -> dword).
template <int NWd>
__device__ __forceinline__ Col<NWd> ldcol(const uint8_t* p) {
    Col<NWd> v;
    __builtin_memcpy(&v, p, 4 * NWd);
    return v;
}
// Non-temporal variants: data blocks are read exactly once and parity is not
// re-read by this kernel, so keep both out of the caches' replacement state.
template <int NWd>
__device__ __forceinline__ Col<NWd> ldcol_nt(const uint8_t* p) {
    Col<NWd> v;
    if constexpr (NWd == 4) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4 t = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p));
        v.w[0] = t.x; v.w[1] = t.y; v.w[2] = t.z; v.w[3] = t.w;
    } else if constexpr (NWd == 2) {
        typedef uint32_t u2 __attribute__((ext_vector_type(2)));
        const u2 t = __builtin_nontemporal_load(reinterpret_cast<const u2*>(p));
        v.w[0] = t.x; v.w[1] = t.y;
    } else {
        v.w[0] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
    }
    return v;
}
template <int NWd>
__device__ __forceinline__ void stcol_nt(uint8_t* p, const Col<NWd>& v) {
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
template <int NWd>
__device__ __forceinline__ void stcol(uint8_t* p, const Col<NWd>& v) {
    __builtin_memcpy(p, &v, 4 * NWd);
}

// ABL (diagnostics, timing only): 1 = skip the hash phase, 2 = skip the GF arithmetic
// (parity rows = data row 0; loads, LDS and stores unchanged), 3 = skip hash and the
// parity stores, 4 = skip hash and the LDS tile writes.
template <int K, int M, int G, int T, int NBUF, int NT, int CW, int PF, bool NTL, bool STAMP = false, int DYB = 0,
          bool PAIR = false, int ABL = 0>
__global__ void __launch_bounds__(NT) k_encode_hash(EncArgs a) {
    constexpr int R = K + M;
    constexpr int NWd = CW / 4;
    constexpr int TS = T + 32;  // LDS row stride: +8 banks per row, conflict-free b64 reads
    constexpr int CPB = T / CW;  // columns per stripe per tile
    constexpr int NCOL = G * CPB;
    constexpr int CPT = (NCOL + NT - 1) / NT;

    constexpr int NTAB = DYB ? K * 8 : M * K * 8;
    __shared__ __attribute__((aligned(16))) uint8_t tile[NBUF][G * R * TS];
    __shared__ __attribute__((aligned(16))) uint32_t tabs[NTAB];
    const uint32_t* dtabs = tabs;

    const int tid = threadIdx.x;
    const int64_t blk0 = (int64_t)blockIdx.x * G;
    const int64_t S = a.S;

    for (int i = tid; i < NTAB; i += NT) tabs[i] = DYB ? a.dtables[i] : a.tables[i];

    // ---- hash-chain role: one shard row of one stripe per quad (PAIR: per thread pair)
    const int chain = PAIR ? (tid >> 1) : (tid >> 2), lane = PAIR ? (tid & 1) : (tid & 3);
    const bool chain_live = chain < G * R && (blk0 + chain / R) < a.n_blocks;
    const int crow = chain < G * R ? chain : 0;
    const uint32_t sel = zipper_sel(lane);
    HHLane st = hh_init(lane, a.key[0], a.key[1], a.key[2], a.key[3]);
    HHPair st2 = hh2_init(lane & 1, a.key[0], a.key[1], a.key[2], a.key[3]);

    // ---- encode role: CPT columns per thread.  Dead stripes of the last workgroup
    // alias the last live block and store byte-identical parity (benign), so the
    // encode has no data-dependent branches (those make hipcc split the parity rows
    // and keep every shard's nibbles live).
    Col<NWd> xs[PF][CPT][K] = {};
    auto prefetch = [&](Col<NWd> (&x)[CPT][K], int64_t t0) {
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            const int col = tid + c * NT;
            const int g = col / CPB;
            const int o = (col % CPB) * CW;
            const int64_t b = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
            const bool live = col < NCOL && t0 + o < S;
            const uint8_t* blk = a.data + b * a.data_stride;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (live) x[c][j] = NTL ? ldcol_nt<NWd>(blk + (int64_t)j * S + t0 + o)
                                        : ldcol<NWd>(blk + (int64_t)j * S + t0 + o);
        }
    };

    auto encode_store = [&](Col<NWd> (&x)[CPT][K], int64_t t0, int L, uint8_t* tl) {
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            const int col = tid + c * NT;
            if (col >= NCOL) continue;
            const int g = col / CPB;
            const int o = (col % CPB) * CW;
            const int64_t b = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
            if (o >= L) continue;
            Col<NWd> par[M];
            if constexpr (ABL == 2) {
#pragma unroll
                for (int r = 0; r < M; ++r) par[r] = x[c][r];
#pragma unroll
                for (int j = 0; j < K; ++j) stcol<NWd>(tl + (g * R + j) * TS + o, x[c][j]);
            } else if constexpr (DYB != 0) {
                encode_dyadic<NWd, K, M>(x[c], par, dtabs);
                if constexpr (ABL != 4) {
#pragma unroll
                    for (int j = 0; j < K; ++j) stcol<NWd>(tl + (g * R + j) * TS + o, x[c][j]);
                }
            } else {
                const uint32_t* tb = tabs + opaque_zero();
                GfAcc acc[M][NWd];
#pragma unroll
                for (int r = 0; r < M; ++r)
#pragma unroll
                    for (int w = 0; w < NWd; ++w) acc_init(acc[r][w]);
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    __builtin_amdgcn_sched_barrier(0);  // keep each shard's table reads local
                    Nib nb[NWd];
#pragma unroll
                    for (int w = 0; w < NWd; ++w) nb[w] = split_nibbles(x[c][j].w[w]);
#pragma unroll
                    for (int r = 0; r < M; ++r) {
                        const CoefTab t = load_coef(tb, r * K + j);
#pragma unroll
                        for (int w = 0; w < NWd; ++w) acc_add(acc[r][w], gf_lookup(nb[w], t));
                    }
                    stcol<NWd>(tl + (g * R + j) * TS + o, x[c][j]);
                }
#pragma unroll
                for (int r = 0; r < M; ++r)
#pragma unroll
                    for (int w = 0; w < NWd; ++w) par[r].w[w] = acc_done(acc[r][w]);
            }
            uint8_t* pbase = a.parity + b * a.parity_stride + t0 + o;
#pragma unroll
            for (int r = 0; r < M; ++r) {
                const Col<NWd>& p = par[r];
                if constexpr (ABL != 4) stcol<NWd>(tl + (g * R + K + r) * TS + o, p);
                if constexpr (ABL == 3) {
                    if (p.w[0] == 0x12345678u && p.w[NWd - 1] == 0x9abcdef0u) stcol<NWd>(pbase + (int64_t)r * S, p);
                } else if (NTL)
                    stcol_nt<NWd>(pbase + (int64_t)r * S, p);
                else
                    stcol<NWd>(pbase + (int64_t)r * S, p);
            }
        }
    };

    lds_barrier();  // tables visible
    // Register prefetch PF tiles deep: tile i lives in xs[i % PF]; the loop is
    // unrolled by PF so the slot index is a compile-time constant.
#pragma unroll
    for (int p = 0; p < PF; ++p)
        if ((int64_t)p * T < S) prefetch(xs[p], (int64_t)p * T);
    // Diagnostics build (STAMP): s_memtime around each phase, summed per wave.
    uint64_t ph[5] = {0, 0, 0, 0, 0};
    auto stamp = [&]() -> uint64_t {
        uint64_t t = 0;
        if constexpr (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            __builtin_amdgcn_sched_barrier(0);
        }
        return t;
    };
    auto step = [&](Col<NWd> (&x)[CPT][K], int64_t t0, int it) {
        const int L = (int)((S - t0) < T ? (S - t0) : T);
        uint8_t* tl = tile[NBUF == 1 ? 0 : (it & 1)];
        const uint64_t s0 = stamp();
        encode_store(x, t0, L, tl);
        const uint64_t s1 = stamp();
        if (t0 + (int64_t)PF * T < S) prefetch(x, t0 + (int64_t)PF * T);
        const uint64_t s2 = stamp();
        lds_barrier();
        const uint64_t s3 = stamp();
        const uint8_t* row = tl + crow * TS;
        if constexpr (ABL == 1 || ABL == 3 || ABL == 4) {
        } else if constexpr (PAIR) {
            if (L == T)
                hh2_packets_n<T / 32>(st2, row, lane);
            else
                hh2_packets(st2, row, L >> 5, lane);
            if (t0 + L >= S && (L & 31)) hh2_remainder(st2, row + (L & ~31), (uint32_t)(L & 31), lane);
        } else {
            if (L == T)
                hh_packets_n<T / 32>(st, row, lane, sel);
            else
                hh_packets(st, row, L >> 5, lane, sel);
            if (t0 + L >= S && (L & 31)) hh_remainder(st, row + (L & ~31), (uint32_t)(L & 31), lane, sel);
        }
        const uint64_t s4 = stamp();
        if (NBUF == 1) lds_barrier();
        const uint64_t s5 = stamp();
        if constexpr (STAMP) {
            ph[0] += s1 - s0;
            ph[1] += s2 - s1;
            ph[2] += s3 - s2;
            ph[3] += s4 - s3;
            ph[4] += s5 - s4;
        }
    };
    int it = 0;
    for (int64_t t0 = 0; t0 < S; t0 += (int64_t)PF * T) {
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int64_t tp = t0 + (int64_t)p * T;
            if (tp < S) step(xs[p], tp, it++);
        }
    }
    if constexpr (PAIR) {
        uint64_t d0, d1;
        hh2_finalize256(st2, d0, d1);
        if (chain_live) {
            const int64_t b = blk0 + chain / R;
            const int s = chain % R;
            uint64_t* out = reinterpret_cast<uint64_t*>(a.sums + (b * R + s) * 32 + 16 * lane);
            out[0] = d0;
            out[1] = d1;
        }
    } else {
        const uint64_t h = hh_finalize256(st, lane, sel);
        if (chain_live) {
            const int64_t b = blk0 + chain / R;
            const int s = chain % R;
            uint8_t* out = a.sums + (b * R + s) * 32 + 8 * lane;
            *reinterpret_cast<uint64_t*>(out) = h;
        }
    }
    if constexpr (STAMP) {
        if ((tid & 63) == 0 && a.dbg) {
            uint64_t* d = a.dbg + ((int64_t)blockIdx.x * (NT / 64) + (tid >> 6)) * 5;
            for (int i = 0; i < 5; ++i) d[i] = ph[i];
        }
    }
}


// ---------------------------------------------------------------------------
// Encode only (no hash): one thread per 16-byte column, K loads -> M stores.
// NTP: non-temporal data loads and parity stores (the encode-only call; not the
// latency path, whose hash pass re-reads both from the cache).  Launch: 16-byte aligned.
// UA (round 4): S need not be a multiple of 16 and the data may carry Split padding
// (n < k*S; RS(12+4), RS(6+4), RS(10+4), ... on 1 MiB blocks): full columns use the same
// 16-byte accesses at the rows' byte offsets (unaligned-access mode: 1-2 % below aligned
// rows on the RS(12+4) streaming shape, profiles/r04/r04_mempat6.jsonl), the column that
// crosses the last data row's valid length or the row end is read byte by byte (zero
// past it) and only its parity bytes below S are stored.
template <int K, int M, bool NTP = false, bool UA = false>
__global__ void __launch_bounds__(256) k_encode_only(EncArgs a) {
    static_assert(!(UA && NTP), "unaligned rows: plain accesses");
    __shared__ __attribute__((aligned(16))) uint32_t tabs[M * K * 8];
    for (int i = threadIdx.x; i < M * K * 8; i += 256) tabs[i] = a.tables[i];
    __syncthreads();
    const int64_t S = a.S, n = a.n;
    const int64_t cols = (S + 15) >> 4;
    const int64_t vlast = n - (int64_t)(K - 1) * S;  // valid bytes of the last data row
    for (int64_t b = blockIdx.y; b < a.n_blocks; b += gridDim.y) {
        const uint8_t* blk = a.data + b * a.data_stride;
        uint8_t* pb = a.parity + b * a.parity_stride;
        for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < cols; c += (int64_t)gridDim.x * 256) {
            const int64_t o = c * 16;
            const uint32_t* tb = tabs + opaque_zero();
            uint4 x[K];
            if constexpr (UA) {
                // A column crossing a row's valid end (S, or the last data row's Split
                // padding) loads the 16 bytes ending at that end and shifts them down
                // (zero fill); past the end nothing of the row is read (the block's first
                // 16 bytes are loaded and discarded).  One 16-byte load per row on every
                // path (a separate byte-wise path doubled the VGPRs).  Launch: S >= 16 and
                // n >= 16, so every load lies inside [blk, blk + n).
                const int shS = tail_shift(S - o);
                const int shL = tail_shift((vlast < S ? vlast : S) - o);
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const int sh = j == K - 1 ? shL : shS;
                    x[j] = ld16(sh == 16 ? blk : blk + (int64_t)j * S + o - sh);
                    if (sh) x[j] = shr_bytes_zero(x[j], sh);
                }
            } else {
#pragma unroll
                for (int j = 0; j < K; ++j) x[j] = NTP ? ld16_nt(blk + (int64_t)j * S + o) : ld16(blk + (int64_t)j * S + o);
            }
            GfAcc acc[M][4];
#pragma unroll
            for (int r = 0; r < M; ++r)
#pragma unroll
                for (int w = 0; w < 4; ++w) acc_init(acc[r][w]);
#pragma unroll
            for (int j = 0; j < K; ++j) {
                __builtin_amdgcn_sched_barrier(0);  // keep each shard's table reads local
                const Nib n0 = split_nibbles(x[j].x), n1 = split_nibbles(x[j].y);
                const Nib n2 = split_nibbles(x[j].z), n3 = split_nibbles(x[j].w);
#pragma unroll
                for (int r = 0; r < M; ++r) {
                    const CoefTab t = load_coef(tb, r * K + j);
                    acc_add(acc[r][0], gf_lookup(n0, t));
                    acc_add(acc[r][1], gf_lookup(n1, t));
                    acc_add(acc[r][2], gf_lookup(n2, t));
                    acc_add(acc[r][3], gf_lookup(n3, t));
                }
            }
            uint4 par[M];
#pragma unroll
            for (int r = 0; r < M; ++r)
                par[r] = make_uint4(acc_done(acc[r][0]), acc_done(acc[r][1]), acc_done(acc[r][2]), acc_done(acc[r][3]));
            if (UA && o + 16 > S) {
                // the ragged last column: only the parity bytes below S
#pragma unroll
                for (int r = 0; r < M; ++r) st16_part(pb + (int64_t)r * S + o, par[r], S - o);
            } else {
#pragma unroll
                for (int r = 0; r < M; ++r) {
                    if (NTP)
                        st16_nt(pb + (int64_t)r * S + o, par[r]);
                    else
                        st16(pb + (int64_t)r * S + o, par[r]);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Latency-regime bitrot sums (small batches): a HighwayHash chain over one shard row
// is S/32 dependent packets, so with fewer chains than SIMDs a launch costs one chain's
// latency whatever its size (~0.55 ms for 128 KiB rows through the tiled kernels, whose
// chains wait on one 256-byte tile of prefetch per step).  Here one quad owns one chain
// (hh256_dev.hpp quad form: the shortest dependent path per packet) and reads it
// straight from global memory, NS*D packets of loads in flight per lane, no LDS, no
// barriers, one wave per workgroup so the chains spread over the SIMDs.  The loop has
// no stores, so the compiler's in-order vmcnt waits are exact.  Chain c = (block
// c / (k+m), row c % (k+m)); data rows at data + b*data_stride + r*S, parity rows at
// parity + b*parity_stride + (r-k)*S (EncArgs addressing, no Split padding), sums as
// k_encode_hash.  Runs after k_encode_only on the same stream.
// One chain per quad straight from global memory: this lane's 64-bit digest word of
// HighwayHash-256(row[0..S)).  All 64 lanes of the wave must call it (DPP).
template <int D, int NS>
__device__ __forceinline__ uint64_t hash_chain_lat(const uint8_t* row, int64_t S, int lane, const uint64_t* key) {
    const uint32_t sel = zipper_sel(lane);
    HHLane st = hh_init(lane, key[0], key[1], key[2], key[3]);
    const uint64_t* p = reinterpret_cast<const uint64_t*>(row) + lane;  // packet q: p[4q]
    const int64_t npk = S >> 5;
    uint64_t w[NS][D];
    // A stage wholly inside the row loads through one pointer with immediate offsets
    // (no per-load address VALU on the lone wave's critical path); the last stages clamp
    // (a packet past the end re-reads the last one and is not hashed).
    auto load = [&](uint64_t (&x)[D], int64_t q0) {
        if (q0 + D <= npk) {
            const uint64_t* q = p + 4 * q0;
#pragma unroll
            for (int j = 0; j < D; ++j) x[j] = __builtin_nontemporal_load(q + 4 * j);
        } else {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const int64_t q = q0 + j < npk ? q0 + j : npk - 1;
                x[j] = __builtin_nontemporal_load(p + 4 * q);
            }
        }
    };
    if (npk > 0) {
#pragma unroll
        for (int s = 0; s < NS - 1; ++s) load(w[s], (int64_t)s * D);
        for (int64_t q0 = 0; q0 < npk; q0 += (int64_t)NS * D) {
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int64_t base = q0 + (int64_t)s * D;
                if (base >= npk) break;
                load(w[(s + NS - 1) % NS], base + (int64_t)(NS - 1) * D);
                if (base + D <= npk) {
                    hh_update_n<D>(st, w[s], sel);
                } else {
#pragma unroll
                    for (int j = 0; j < D; ++j)
                        if (base + j < npk) hh_update(st, w[s][j], sel);
                }
            }
        }
    }
    const uint32_t rem = (uint32_t)(S & 31);
    if (rem) hh_remainder(st, row + (npk << 5), rem, lane, sel);
    return hh_finalize256(st, lane, sel);
}

template <int D, int NS>
__global__ void __launch_bounds__(64) k_hash_lat(EncArgs a) {
    const int R = a.k + a.m;
    const int tid = threadIdx.x, lane = tid & 3;
    const int64_t nch = a.n_blocks * R;
    int64_t c = (int64_t)blockIdx.x * 16 + (tid >> 2);
    const bool live = c < nch;
    if (!live) c = nch - 1;  // dead quads re-hash the last chain (all lanes stay active)
    const int64_t b = c / R;
    const int r = (int)(c % R);
    const uint8_t* row = r < a.k ? a.data + b * a.data_stride + (int64_t)r * a.S
                                 : a.parity + b * a.parity_stride + (int64_t)(r - a.k) * a.S;
    const uint64_t h = hash_chain_lat<D, NS>(row, a.S, lane, a.key);
    if (live) *reinterpret_cast<uint64_t*>(a.sums + (b * R + r) * 32 + 8 * lane) = h;
}

// GET / heal in the latency regime, after k_reconstruct has rebuilt the missing rows:
// chain (block b, i) hashes row rows[i] of block slot(b); i < k verifies a survivor
// against its stored sum (bad flag = errFileCorrupt, a quad ballot), i >= k (heal) writes
// the rebuilt row's new sum.  nr = k (GET) or k + e (heal).
template <int D, int NS>
__global__ void __launch_bounds__(64) k_vr_hash_lat(VrArgs a, int nr) {
    const int R = a.k + a.m;
    const int tid = threadIdx.x, lane = tid & 3;
    const int64_t nch = a.n_blocks * nr;
    int64_t c = (int64_t)blockIdx.x * 16 + (tid >> 2);
    const bool live = c < nch;
    if (!live) c = nch - 1;
    const int64_t b = c / nr;
    const int i = (int)(c % nr);
    const int64_t slot = a.ids ? (int64_t)a.ids[b] : b;
    const int row = a.rows[i];
    const uint8_t* rp = a.shards + slot * a.block_stride + (int64_t)row * a.S;
    const uint64_t h = hash_chain_lat<D, NS>(rp, a.S, lane, a.key);
    const int64_t so = (slot * R + row) * 32 + 8 * lane;
    if (i < a.k) {
        const bool mis = h != *reinterpret_cast<const uint64_t*>(a.expect + so);
        const uint64_t bal = __ballot(mis);
        if (live && lane == 0) a.bad[slot * R + row] = ((bal >> (tid & ~3)) & 0xF) ? 1 : 0;
    } else if (live) {
        *reinterpret_cast<uint64_t*>(a.sums_out + so) = h;
    }
}

// Crossover of the split path against the fused kernels (profiles/r02/sweep_sizes_small_v49.txt,
// sweep_cliffs.jsonl): RS(8+4) between 512 and 768 blocks (~1 GB of stripes), RS(16+4)
// at 512 (448: 1516 vs 1463 GiB/s, 512: 1634 vs 1662).
template <int K, int M>
static bool small_batch(int64_t n_blocks, int64_t S) {
    if (K == 4 && M == 2) return false;
    if (K == 16 && M == 4) return n_blocks < 512;
    // RS(8+4): the 4-stripe fused kernel wins from ~256 stripes of 128 KiB shards (round 3:
    // 0.275 vs 0.32 ms at 256, 0.272 vs 0.269 at 128; profiles/r03/sweep_rs84_sizes199.jsonl)
    if (K == 8 && M == 4) return n_blocks * S <= (int64_t)128 * 131072;
    return n_blocks * (K + M) * S <= (int64_t)640 * 12 * 131072;
}

template <int K, int M>
static void launch_encode_lat(const EncArgs& a, hipStream_t s) {
    const int64_t cols = (a.S + 15) >> 4;
    const unsigned gx = (unsigned)((cols + 255) / 256);
    const unsigned gy = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
    hipLaunchKernelGGL((k_encode_only<K, M>), dim3(gx, gy), dim3(256), 0, s, a);
    const int64_t nch = a.n_blocks * (K + M);
    hipLaunchKernelGGL((k_hash_lat<16, 3>), dim3((unsigned)((nch + 15) / 16)), dim3(64), 0, s, a);
}

// ---------------------------------------------------------------------------
// Reconstruct: E_MAX output rows, each a GF combination of the K valid rows.
// NTP: non-temporal survivor loads and rebuilt-row stores (launch: S % 16 == 0 and a
// 16-byte aligned base, so every access is aligned).
// UA (round 3): S need not be a multiple of 16 (RS(12+4) / RS(10+6) / RS(5+4) ... on
// 1 MiB blocks): full columns use the same 16-byte accesses at the rows' byte offsets
// (unaligned-access mode), the ragged last column is read byte by byte (bytes past the
// row read as zero) and only its bytes below S are stored.
template <int K, int EMAX, int NC = 1, bool NTP = false, bool UA = false>
__global__ void __launch_bounds__(256) k_reconstruct(RecArgs a) {
    static_assert(!UA || (NC == 1 && !NTP), "unaligned rows: one column per thread, plain accesses");
    // NC columns per thread (256 apart, so every load instruction stays coalesced): all
    // NC*K survivor loads are issued before the first product (more bytes in flight).
    __shared__ __attribute__((aligned(16))) uint32_t tabs[EMAX * K * 8];
    __shared__ int32_t rows[K + EMAX];
    for (int i = threadIdx.x; i < a.e * K * 8; i += 256) tabs[i] = a.tables[i];
    for (int i = threadIdx.x; i < K + a.e; i += 256) rows[i] = a.rows[i];
    __syncthreads();
    const int64_t S = a.S;
    const int64_t cols = (S + 15) >> 4;
    const int E = a.e;
    for (int64_t b = blockIdx.y; b < a.n_blocks; b += gridDim.y) {
        uint8_t* blk = a.shards + (a.ids ? (int64_t)a.ids[b] : b) * a.block_stride;
        for (int64_t c0 = (int64_t)blockIdx.x * 256 * NC + threadIdx.x; c0 < cols; c0 += (int64_t)gridDim.x * 256 * NC) {
            const uint32_t* tbl = tabs + opaque_zero();
            uint4 x[NC][K];
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                const int64_t c = c0 + 256 * i;
                const int64_t o = (c < cols ? c : c0) * 16;
                if (UA && c == cols - 1 && (S & 15)) {
                    const int nv = (int)(S & 15);
#pragma unroll
                    for (int t = 0; t < K; ++t) {
                        const uint8_t* p = blk + (int64_t)rows[t] * S + o;
                        uint32_t w[4] = {0, 0, 0, 0};
                        for (int q = 0; q < nv; ++q) w[q >> 2] |= (uint32_t)p[q] << (8 * (q & 3));
                        x[i][t] = make_uint4(w[0], w[1], w[2], w[3]);
                    }
                    continue;
                }
#pragma unroll
                for (int t = 0; t < K; ++t)
                    x[i][t] = NTP ? ld16_nt(blk + (int64_t)rows[t] * S + o) : ld16(blk + (int64_t)rows[t] * S + o);
            }
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                const int64_t c = c0 + 256 * i;
                if (c >= cols) continue;
                const int64_t o = c * 16;
                GfAcc acc[EMAX][4];
#pragma unroll
                for (int r = 0; r < EMAX; ++r)
#pragma unroll
                    for (int w = 0; w < 4; ++w) acc_init(acc[r][w]);
#pragma unroll
                for (int t = 0; t < K; ++t) {
                    const Nib n0 = split_nibbles(x[i][t].x), n1 = split_nibbles(x[i][t].y);
                    const Nib n2 = split_nibbles(x[i][t].z), n3 = split_nibbles(x[i][t].w);
#pragma unroll
                    for (int r = 0; r < EMAX; ++r) {
                        if (r < E) {
                            const CoefTab tb = load_coef(tbl, r * K + t);
                            acc_add(acc[r][0], gf_lookup(n0, tb));
                            acc_add(acc[r][1], gf_lookup(n1, tb));
                            acc_add(acc[r][2], gf_lookup(n2, tb));
                            acc_add(acc[r][3], gf_lookup(n3, tb));
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < EMAX; ++r) {
                    if (r < E) {
                        const uint4 p = make_uint4(acc_done(acc[r][0]), acc_done(acc[r][1]),
                                                   acc_done(acc[r][2]), acc_done(acc[r][3]));
                        uint8_t* dst = blk + (int64_t)rows[K + r] * S + o;
                        if (UA && c == cols - 1 && (S & 15)) {
                            const uint32_t w[4] = {p.x, p.y, p.z, p.w};
                            for (int q = 0; q < (int)(S & 15); ++q) dst[q] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
                        } else if (NTP) {
                            st16_nt(dst, p);
                        } else {
                            st16(dst, p);
                        }
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Generic byte path: any k, m (k+m <= 256), any shard size and alignment.
// One stripe per workgroup; tile rows staged in LDS; log/exp GF tables in LDS.
constexpr int GEN_T = 256;
constexpr int GEN_TS = GEN_T + 32;

__global__ void __launch_bounds__(1024) k_encode_hash_generic(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int k = a.k, m = a.m, R = k + m;
    uint8_t* tile = smem;                           // R * GEN_TS
    uint8_t* lg = smem + (size_t)R * GEN_TS;        // 256
    uint8_t* ex = lg + 256;                         // 512
    uint8_t* mat = ex + 512;                        // m * k parity rows
    const int tid = threadIdx.x, NT = blockDim.x;
    // build GF tables
    if (tid == 0) {
        unsigned v = 1;
        for (int i = 0; i < 255; ++i) {
            ex[i] = (uint8_t)v;
            lg[v] = (uint8_t)i;
            v <<= 1;
            if (v & 0x100) v ^= 0x11D;
        }
        for (int i = 255; i < 512; ++i) ex[i] = ex[i - 255];
        lg[0] = 0;
    }
    for (int i = tid; i < m * k; i += NT) mat[i] = a.matrix[(size_t)k * k + i];
    __syncthreads();

    const int64_t S = a.S, n = a.n;
    const bool hash = a.sums != nullptr;
    const int chain = tid >> 2, lane = tid & 3;
    const int crow = chain < R ? chain : 0;
    const uint32_t sel = zipper_sel(lane);
    for (int64_t b = blockIdx.x; b < a.n_blocks; b += gridDim.x) {
        const uint8_t* blk = a.data + b * a.data_stride;
        uint8_t* pb = a.parity + b * a.parity_stride;
        HHLane st = hh_init(lane, a.key[0], a.key[1], a.key[2], a.key[3]);
        for (int64_t t0 = 0; t0 < S; t0 += GEN_T) {
            const int L = (int)((S - t0) < GEN_T ? (S - t0) : GEN_T);
            for (int i = tid; i < k * L; i += NT) {
                const int j = i / L, o = i - j * L;
                const int64_t pos = (int64_t)j * S + t0 + o;
                tile[j * GEN_TS + o] = pos < n ? blk[pos] : (uint8_t)0;
            }
            __syncthreads();
            for (int i = tid; i < m * L; i += NT) {
                const int r = i / L, o = i - r * L;
                uint8_t acc = 0;
                for (int j = 0; j < k; ++j) acc ^= gf_mul_log(lg, ex, mat[r * k + j], tile[j * GEN_TS + o]);
                tile[(k + r) * GEN_TS + o] = acc;
                pb[(int64_t)r * S + t0 + o] = acc;
            }
            __syncthreads();
            if (hash && chain < R) {
                const uint8_t* row = tile + crow * GEN_TS;
                hh_packets(st, row, L >> 5, lane, sel);
                if (t0 + L >= S && (L & 31)) hh_remainder(st, row + (L & ~31), (uint32_t)(L & 31), lane, sel);
            }
            __syncthreads();
        }
        if (hash && chain < R) {
            const uint64_t h = hh_finalize256(st, lane, sel);
            *reinterpret_cast<uint64_t*>(a.sums + (b * R + chain) * 32 + 8 * lane) = h;
        }
    }
}

__global__ void __launch_bounds__(256) k_reconstruct_generic(RecArgs a) {
    __shared__ uint8_t lg[256], ex[512];
    extern __shared__ uint8_t coef[];  // e*k coefficients then rows
    const int k = a.k, E = a.e;
    if (threadIdx.x == 0) {
        unsigned v = 1;
        for (int i = 0; i < 255; ++i) {
            ex[i] = (uint8_t)v;
            lg[v] = (uint8_t)i;
            v <<= 1;
            if (v & 0x100) v ^= 0x11D;
        }
        for (int i = 255; i < 512; ++i) ex[i] = ex[i - 255];
        lg[0] = 0;
    }
    int32_t* rows = reinterpret_cast<int32_t*>(coef + ((E * k + 3) & ~3));
    for (int i = threadIdx.x; i < E * k; i += blockDim.x) coef[i] = a.coef[i];
    for (int i = threadIdx.x; i < k + E; i += blockDim.x) rows[i] = a.rows[i];
    __syncthreads();
    const int64_t S = a.S;
    for (int64_t b = blockIdx.y; b < a.n_blocks; b += gridDim.y) {
        uint8_t* blk = a.shards + (a.ids ? (int64_t)a.ids[b] : b) * a.block_stride;
        for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < S; o += (int64_t)gridDim.x * blockDim.x) {
            for (int r = 0; r < E; ++r) {
                uint8_t acc = 0;
                for (int t = 0; t < k; ++t)
                    acc ^= gf_mul_log(lg, ex, coef[r * k + t], blk[(int64_t)rows[t] * S + o]);
                blk[(int64_t)rows[k + r] * S + o] = acc;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Any-geometry kernels (k <= 64, m / e <= AMAX, any shard size, any alignment): the
// server's other erasure geometries (set sizes 4-16 with parity upgrades,
// cmd/erasure-object.go:724-775, e.g. RS(11+5), RS(10+6), RS(5+4)) and ragged last
// blocks with Split padding.  One 8-byte column of one stripe per thread, 8-byte
// vector loads and stores at the rows' byte offsets (unaligned global access), the
// parity / rebuilt rows accumulated with the per-coefficient permute tables
// (gf_dev.hpp), the partial last column and the Split padding read byte by byte.
// The bitrot sums of these geometries come from the batched hash kernel in stripe mode.
constexpr int AMAX = 8;

typedef uint32_t u2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u2v ld8_any(const uint8_t* p, int64_t o, int64_t vlen) {
    u2v v = {0u, 0u};
    if (o + 8 <= vlen) {
        __builtin_memcpy(&v, p + o, 8);
    } else if (o < vlen) {
        uint32_t w[2] = {0u, 0u};
        for (int z = 0; z < 8; ++z)
            if (o + z < vlen) w[z >> 2] |= (uint32_t)p[o + z] << (8 * (z & 3));
        v.x = w[0];
        v.y = w[1];
    }
    return v;
}

__device__ __forceinline__ void st8_any(uint8_t* p, int64_t o, int64_t len, uint32_t x, uint32_t y) {
    if (o + 8 <= len) {
        const u2v v = {x, y};
        __builtin_memcpy(p + o, &v, 8);
    } else {
        for (int z = 0; z < 8; ++z)
            if (o + z < len) p[o + z] = (uint8_t)((z < 4 ? x : y) >> (8 * (z & 3)));
    }
}

// acc ^= c * x for two packed dwords (x split once per input row).
__device__ __forceinline__ void gf_mac2(uint32_t& a0, uint32_t& a1, const Nib& n0, const Nib& n1, const CoefTab& t) {
    const Prod3 p0 = gf_lookup(n0, t), p1 = gf_lookup(n1, t);
    a0 = xor3(a0, p0.a, p0.b) ^ p0.c;
    a1 = xor3(a1, p1.a, p1.b) ^ p1.c;
}

// Encode only (Erasure.EncodeData's arithmetic, erasure-coding.go:77-91), any k / m <= AMAX.
__global__ void __launch_bounds__(256) k_encode_any(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t etabs[];  // m*k*8 dwords
    const int k = a.k, m = a.m;
    for (int i = threadIdx.x; i < m * k * 8; i += 256) etabs[i] = a.tables[i];
    __syncthreads();
    const int64_t S = a.S;
    const int64_t cols = (S + 7) >> 3;
    for (int64_t b = blockIdx.y; b < a.n_blocks; b += gridDim.y) {
        const uint8_t* blk = a.data + b * a.data_stride;
        uint8_t* pb = a.parity + b * a.parity_stride;
        for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < cols; c += (int64_t)gridDim.x * 256) {
            const int64_t o = c * 8;
            uint32_t acc[AMAX][2];
#pragma unroll
            for (int r = 0; r < AMAX; ++r) acc[r][0] = acc[r][1] = 0;
            for (int j = 0; j < k; ++j) {
                int64_t vlen = a.n - (int64_t)j * S;  // Split padding of the last rows reads as zero
                vlen = vlen < 0 ? 0 : (vlen < S ? vlen : S);
                const u2v x = ld8_any(blk + (int64_t)j * S, o, vlen);
                const Nib n0 = split_nibbles(x.x), n1 = split_nibbles(x.y);
                const uint32_t* tb = etabs + opaque_zero() + j * 8;
#pragma unroll
                for (int r = 0; r < AMAX; ++r)
                    if (r < m) gf_mac2(acc[r][0], acc[r][1], n0, n1, load_coef(tb, r * k));
            }
#pragma unroll
            for (int r = 0; r < AMAX; ++r)
                if (r < m) st8_any(pb + (int64_t)r * S, o, S, acc[r][0], acc[r][1]);
        }
    }
}

// Reconstruct (ReconstructData / Reconstruct, erasure-coding.go:96-119): e <= AMAX rows
// from the k survivors rows[0..k) into rows[k..k+e), any k.
__global__ void __launch_bounds__(256) k_reconstruct_any(RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rtabs[];  // e*k*8 dwords, then rows
    const int k = a.k, E = a.e;
    int32_t* rows = reinterpret_cast<int32_t*>(rtabs + E * k * 8);
    for (int i = threadIdx.x; i < E * k * 8; i += 256) rtabs[i] = a.tables[i];
    for (int i = threadIdx.x; i < k + E; i += 256) rows[i] = a.rows[i];
    __syncthreads();
    const int64_t S = a.S;
    const int64_t cols = (S + 7) >> 3;
    for (int64_t b = blockIdx.y; b < a.n_blocks; b += gridDim.y) {
        uint8_t* blk = a.shards + (a.ids ? (int64_t)a.ids[b] : b) * a.block_stride;
        for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < cols; c += (int64_t)gridDim.x * 256) {
            const int64_t o = c * 8;
            uint32_t acc[AMAX][2];
#pragma unroll
            for (int r = 0; r < AMAX; ++r) acc[r][0] = acc[r][1] = 0;
            for (int t = 0; t < k; ++t) {
                const u2v x = ld8_any(blk + (int64_t)rows[t] * S, o, S);
                const Nib n0 = split_nibbles(x.x), n1 = split_nibbles(x.y);
                const uint32_t* tb = rtabs + opaque_zero() + t * 8;
#pragma unroll
                for (int r = 0; r < AMAX; ++r)
                    if (r < E) gf_mac2(acc[r][0], acc[r][1], n0, n1, load_coef(tb, r * k));
            }
#pragma unroll
            for (int r = 0; r < AMAX; ++r)
                if (r < E) st8_any(blk + (int64_t)rows[k + r] * S, o, S, acc[r][0], acc[r][1]);
        }
    }
}

// Bitrot sums of every shard of a batch in one launch (hash kernel, stripe mode).
static hipError_t hash_stripes(const EncArgs& a, hipStream_t s) {
    HashArgs h{};
    const int R = a.k + a.m;
    h.rps = R;
    h.kd = a.k;
    h.rtot = R;
    h.msgs = a.data;
    h.stride = a.data_stride;
    h.par = a.parity;
    h.par_stride = a.parity_stride;
    h.len = a.S;
    h.vlim = a.n;
    h.n = a.n_blocks * R;
    h.sums = a.sums;
    for (int i = 0; i < R; ++i) h.rowmap[i] = (uint8_t)i;
    for (int q = 0; q < 4; ++q) h.key[q] = a.key[q];
    return launch_hash(h, s);
}

static bool encode_any_ok(const EncArgs& a) {
    return a.k + a.m <= 64 && a.m <= AMAX && (size_t)a.m * a.k * 32 <= 65536;
}

static hipError_t launch_encode_any(const EncArgs& a, hipStream_t s) {
    const size_t lds = (size_t)a.m * a.k * 32;
    hipError_t e = ensure_dyn_lds((const void*)k_encode_any, lds);
    if (e != hipSuccess) return e;
    const int64_t cols = (a.S + 7) >> 3;
    const int64_t gx = (cols + 255) / 256;
    const unsigned gy = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
    hipLaunchKernelGGL(k_encode_any, dim3((unsigned)gx, gy), dim3(256), lds, s, a);
    e = hipGetLastError();
    if (e != hipSuccess || !a.sums) return e;
    return hash_stripes(a, s);
}

// ---------------------------------------------------------------------------
// HighwayHash-256 of n messages (64 chains = 256 threads per workgroup), with
// optional compare against expected digests (streamingBitrotReader.ReadAt,
// cmd/bitrot-streaming.go:180-186, and bitrotVerify, cmd/bitrot.go:158-210: a
// per-chunk errFileCorrupt flag, never a whole-batch failure).
// Double-buffered: the next tile's 16-byte pieces are loaded into registers while
// the current tile is hashed from LDS, so HBM latency overlaps the hash chain.
// Messages may differ in length (ragged mode, chunked-file mode): every chain runs
// its own packets/remainder inside the shared tile loop, which runs to the longest
// message of the workgroup; bytes past a message's end load as zero.
constexpr int HB_CH = 64;
constexpr int HB_T = 256;
constexpr int HB_TS = HB_T + 32;
constexpr int HB_PPT = HB_CH * (HB_T / 16) / 256;  // 16-byte pieces per thread per tile

struct MsgGeom {
    const uint8_t* p;    // message bytes
    const uint8_t* exp;  // expected digest (or nullptr)
    int64_t len;
    int64_t slot;        // index into sums / bad
    int64_t vlen;        // bytes at or past vlen read as zero (<= len)
};

__device__ __forceinline__ MsgGeom msg_geom(const HashArgs& a, int64_t i) {
    MsgGeom g;
    if (a.rps > 0) {
        // stripe mode: shard rowmap[q] of stripe bq
        const int64_t bq = i / a.rps;
        const int q = (int)(i - bq * a.rps);
        const int64_t slot = a.ids ? (int64_t)a.ids[bq] : bq;
        const int idx = a.rowmap[q];
        g.p = idx < a.kd ? a.msgs + slot * a.stride + (int64_t)idx * a.len
                         : a.par + slot * a.par_stride + (int64_t)(idx - a.kd) * a.len;
        g.len = a.len;
        g.slot = slot * a.rtot + idx;
        g.exp = a.expect ? a.expect + g.slot * 32 : nullptr;
        g.vlen = a.len;
        if (a.vlim > 0 && idx < a.kd) {
            const int64_t v = a.vlim - (int64_t)idx * a.len;
            g.vlen = v < 0 ? 0 : (v < a.len ? v : a.len);
        }
        return g;
    }
    g.slot = a.ids ? (int64_t)a.ids[i] : i;
    const int64_t ss = a.sum_stride ? a.sum_stride : 32;
    if (a.chunk > 0) {
        // on-disk [sum][chunk]* shard file (bitrot-streaming.go:50-55)
        const int64_t f = g.slot / a.nchunks, c = g.slot - f * a.nchunks;
        const uint8_t* base = a.msgs + f * a.stride + c * (a.chunk + 32);
        g.exp = base;
        g.p = base + 32;
        g.len = c == a.nchunks - 1 ? a.last_len : a.chunk;
    } else {
        g.p = a.ptrs ? a.ptrs[i] : a.msgs + g.slot * a.stride;
        g.len = a.lens ? a.lens[i] : a.len;
        g.exp = a.expect ? a.expect + g.slot * ss : nullptr;
    }
    g.vlen = g.len;
    return g;
}

// NTP: non-temporal loads for 16-byte aligned message columns (bytes read once).
template <bool NTP = false>
__global__ void __launch_bounds__(256) k_hash_batch(HashArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[2][HB_CH * HB_TS];
    __shared__ int64_t s_len[HB_CH];
    const int tid = threadIdx.x;
    const int64_t m0 = (int64_t)blockIdx.x * HB_CH;
    const int chain = tid >> 2, lane = tid & 3;
    const uint32_t sel = zipper_sel(lane);
    HHLane st = hh_init(lane, a.key[0], a.key[1], a.key[2], a.key[3]);
    // geometry of this thread's hash chain and of the HB_PPT rows it loads
    const bool live = m0 + chain < a.n;
    const MsgGeom mine = live ? msg_geom(a, m0 + chain) : MsgGeom{nullptr, nullptr, 0, 0, 0};
    if (lane == 0) s_len[chain] = mine.len;
    const uint8_t* rp[HB_PPT];
    int64_t rl[HB_PPT];
#pragma unroll
    for (int q = 0; q < HB_PPT; ++q) {
        const int r = (tid + q * 256) / (HB_T / 16);
        const bool ok = m0 + r < a.n;
        const MsgGeom g = ok ? msg_geom(a, m0 + r) : MsgGeom{nullptr, nullptr, 0, 0, 0};
        rp[q] = g.p;
        rl[q] = g.vlen;  // loads stop at the valid bytes (zero past them); the chain hashes len
    }
    __syncthreads();
    int64_t maxlen = 0;
    for (int i = 0; i < HB_CH; ++i) maxlen = s_len[i] > maxlen ? s_len[i] : maxlen;
    const int64_t ntile = (maxlen + HB_T - 1) / HB_T;
    uint4 v[HB_PPT];
    auto load = [&](int64_t t0) {
#pragma unroll
        for (int q = 0; q < HB_PPT; ++q) {
            const int i = tid + q * 256;
            const int o = (i % (HB_T / 16)) * 16;
            const int64_t L = rl[q] - t0;
            v[q] = make_uint4(0, 0, 0, 0);
            if (o < L) {
                const uint8_t* src = rp[q] + t0 + o;
                if (o + 16 <= L) {
                    v[q] = (NTP && ((uintptr_t)src & 15) == 0) ? ld16_nt(src) : ld16(src);
                } else {
                    uint32_t w4[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int z = 0; z < 16; ++z)
                        if (z < L - o) w4[z >> 2] |= (uint32_t)src[z] << (8 * (z & 3));
                    v[q] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                }
            }
        }
    };
    auto stash = [&](uint8_t* tl) {
#pragma unroll
        for (int q = 0; q < HB_PPT; ++q) {
            const int i = tid + q * 256;
            const int r = i / (HB_T / 16), o = (i % (HB_T / 16)) * 16;
            *reinterpret_cast<uint4*>(tl + r * HB_TS + o) = v[q];
        }
    };
    if (ntile > 0) {
        load(0);
        stash(tile[0]);
        if (ntile > 1) load(HB_T);
    }
    lds_barrier();
    for (int64_t t = 0; t < ntile; ++t) {
        const int64_t t0 = t * HB_T;
        uint8_t* cur = tile[t & 1];
        // stash tile t+1 (registers) into the other buffer, then prefetch t+2
        if (t + 1 < ntile) {
            stash(tile[(t + 1) & 1]);
            if (t + 2 < ntile) load(t0 + 2 * HB_T);
        }
        const int64_t left = mine.len - t0;  // this chain's bytes from this tile on
        const uint8_t* row = cur + chain * HB_TS;
        if (left >= HB_T) {
            hh_packets_n<HB_T / 32>(st, row, lane, sel);
        } else if (left > 0) {
            const int L = (int)left;
            hh_packets(st, row, L >> 5, lane, sel);
            if (L & 31) hh_remainder(st, row + (L & ~31), (uint32_t)(L & 31), lane, sel);
        }
        lds_barrier();
    }
    const uint64_t h = hh_finalize256(st, lane, sel);
    if (live) {
        const int64_t ss = a.rps > 0 ? 32 : (a.sum_stride ? a.sum_stride : 32);
        const int64_t bs = a.rps > 0 ? 1 : (a.bad_stride ? a.bad_stride : 1);
        const int64_t out_i = a.chunk > 0 ? m0 + chain : mine.slot;
        if (a.sums) *reinterpret_cast<uint64_t*>(a.sums + out_i * ss + 8 * lane) = h;
        if (mine.exp && a.bad) {
            uint64_t want;
            __builtin_memcpy(&want, mine.exp + 8 * lane, 8);
            const unsigned long long mism = __ballot(want != h);
            const unsigned q = (unsigned)((mism >> (tid & 60)) & 0xFull);
            if (lane == 0) a.bad[out_i * bs] = q ? 1 : 0;
        }
    }
}

// ---------------------------------------------------------------------------
// GET / heal fused pass: per stripe, the k survivor rows the decode
// reads (ReconstructData's first k present shards, erasure-coding.go:108) are hashed
// and compared with their stored bitrot sums (streamingBitrotReader.ReadAt,
// bitrot-streaming.go:171-186: per-shard errFileCorrupt), and the e missing rows are
// rebuilt from the same registers (one HBM read of each survivor).  HOUT also hashes
// the rebuilt rows so a heal can write them with fresh sums (erasure-healing.go).
// Layout as k_encode_hash: G stripes per workgroup, T-byte tiles, each thread one
// CW-byte column, survivors (+ rebuilt rows) staged in LDS, one quad per hashed row.
// GX > 0 overrides the stripes per workgroup: with GX = 16 on a 4096-stripe batch the
// launch is one workgroup per CU (LDS padded so no two share a CU), all of a CU's
// waves in one barrier domain -- independent workgroups sharing a CU progress at very
// different rates under oldest-first issue and leave the CU under-occupied at the end
// (the fused encode kernel's finding, fused_v2.hip / scripts/stamps3.py).
template <int K, int EMAX, bool HOUT, int GX = 0>
struct VrShape {
    static constexpr int RH = K + (HOUT ? EMAX : 0);  // hashed rows per stripe
    static constexpr int G = GX > 0 ? GX : ((256 / (4 * RH)) > 0 ? 256 / (4 * RH) : 1);
    static constexpr int NT = round64(4 * G * RH);
    static constexpr int T = 256, CW = 8;
    static constexpr int TS = T + 32;
    static constexpr size_t TILE = (size_t)G * RH * TS;
};

template <int K, int EMAX, bool HOUT, int GX = 0>
__global__ void __launch_bounds__((VrShape<K, EMAX, HOUT, GX>::NT)) k_verify_reconstruct(VrArgs a) {
    using Sh = VrShape<K, EMAX, HOUT, GX>;
    constexpr int RH = Sh::RH, G = Sh::G, NT = Sh::NT, T = Sh::T, CW = Sh::CW;
    constexpr int NWd = CW / 4, TS = T + 32, CPB = T / CW, NCOL = G * CPB;
    constexpr int CPT = (NCOL + NT - 1) / NT;
    extern __shared__ __attribute__((aligned(16))) uint8_t vr_smem[];
    uint8_t* tile = vr_smem;  // [G * RH][TS], dynamic (may be padded to limit occupancy)
    __shared__ __attribute__((aligned(16))) uint32_t tabs[(EMAX > 0 ? EMAX : 1) * K * 8];
    __shared__ int32_t srows[K + EMAX];
    const int tid = threadIdx.x;
    const int E = a.e;
    for (int i = tid; i < E * K * 8; i += NT) tabs[i] = a.tables[i];
    for (int i = tid; i < K + E; i += NT) srows[i] = a.rows[i];
    const int64_t S = a.S;
    const int64_t blk0 = (int64_t)blockIdx.x * G;
    const int R = a.k + a.m;
    const int chain = tid >> 2, lane = tid & 3;
    const int cj = chain % RH;
    const bool chain_live = chain < G * RH && (blk0 + chain / RH) < a.n_blocks && (cj < K || cj - K < E);
    const int crow = chain < G * RH ? chain : 0;
    const uint32_t sel = zipper_sel(lane);
    HHLane st = hh_init(lane, a.key[0], a.key[1], a.key[2], a.key[3]);
    lds_barrier();
    int64_t roff[K];  // survivor row offsets (wave-uniform)
#pragma unroll
    for (int j = 0; j < K; ++j) roff[j] = (int64_t)__builtin_amdgcn_readfirstlane(srows[j]) * S;
    for (int64_t t0 = 0; t0 < S; t0 += T) {
        const int L = (int)((S - t0) < T ? (S - t0) : T);
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            const int col = tid + c * NT;
            if (col >= NCOL) continue;
            const int g = col / CPB;
            const int o = (col % CPB) * CW;
            if (o >= L) continue;
            const int64_t b = (blk0 + g) < a.n_blocks ? (blk0 + g) : (a.n_blocks - 1);
            uint8_t* blk = a.shards + (a.ids ? (int64_t)a.ids[b] : b) * a.block_stride + t0 + o;
            Col<NWd> x[K];
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = ldcol<NWd>(blk + roff[j]);
#pragma unroll
            for (int j = 0; j < K; ++j) stcol<NWd>(tile + (g * RH + j) * TS + o, x[j]);
            if constexpr (EMAX > 0) {
                const uint32_t* tb = tabs + opaque_zero();
#pragma unroll
                for (int r = 0; r < EMAX; ++r) {
                    if (r < E) {
                        GfAcc acc[NWd];
#pragma unroll
                        for (int w = 0; w < NWd; ++w) acc_init(acc[w]);
#pragma unroll
                        for (int j = 0; j < K; ++j) {
                            const CoefTab t = load_coef(tb, r * K + j);
#pragma unroll
                            for (int w = 0; w < NWd; ++w) acc_add(acc[w], gf_lookup(split_nibbles(x[j].w[w]), t));
                        }
                        Col<NWd> y;
#pragma unroll
                        for (int w = 0; w < NWd; ++w) y.w[w] = acc_done(acc[w]);
                        const int64_t orow = (int64_t)__builtin_amdgcn_readfirstlane(srows[K + r]);
                        stcol<NWd>(blk + orow * S, y);
                        if constexpr (HOUT) stcol<NWd>(tile + (g * RH + K + r) * TS + o, y);
                    }
                }
            }
        }
        lds_barrier();
        const uint8_t* row = tile + crow * TS;
        if (L == T)
            hh_packets_n<T / 32>(st, row, lane, sel);
        else
            hh_packets(st, row, L >> 5, lane, sel);
        if (t0 + L >= S && (L & 31)) hh_remainder(st, row + (L & ~31), (uint32_t)(L & 31), lane, sel);
        lds_barrier();
    }
    const uint64_t h = hh_finalize256(st, lane, sel);
    if (chain_live) {
        const int64_t b = a.ids ? (int64_t)a.ids[blk0 + chain / RH] : blk0 + chain / RH;
        const int64_t srow = srows[cj];
        if (cj < K) {
            uint64_t want;
            __builtin_memcpy(&want, a.expect + (b * R + srow) * 32 + 8 * lane, 8);
            const unsigned long long mism = __ballot(want != h);
            const unsigned q = (unsigned)((mism >> (tid & 60)) & 0xFull);
            if (lane == 0) a.bad[b * R + srow] = q ? 1 : 0;
        } else if (a.sums_out) {
            *reinterpret_cast<uint64_t*>(a.sums_out + (b * R + srow) * 32 + 8 * lane) = h;
        }
    }
}

// ---------------------------------------------------------------------------
// Synthetic input: counter-based splitmix64 (== oracle_fill in oracle/zs3_oracle.c).
__device__ __forceinline__ uint64_t sm_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_fill(uint8_t* out, int64_t stride, int64_t len, int64_t n,
                                              uint64_t seed, uint64_t obj0) {
    const int64_t nw = (len + 7) >> 3;
    for (int64_t b = blockIdx.y; b < n; b += gridDim.y) {
        const uint64_t s0 = seed + ((obj0 + (uint64_t)b) << 40);
        uint8_t* o = out + b * stride;
        const bool al = (((uintptr_t)o) & 7) == 0;
        for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (int64_t)gridDim.x * 256) {
            const uint64_t v = sm_mix(s0 + (uint64_t)(w + 1) * 0x9e3779b97f4a7c15ULL);
            if (al && w * 8 + 8 <= len) {
                *reinterpret_cast<uint64_t*>(o + w * 8) = v;
            } else {
                for (int i = 0; i < 8 && w * 8 + i < len; ++i) o[w * 8 + i] = (uint8_t)(v >> (8 * i));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Dispatch
template <int K, int M, int G, int T, int NBUF, int CW, int PF = 1, bool NTL = false, bool STAMP = false>
static void launch_fused(const EncArgs& a, hipStream_t s) {
    constexpr bool CAN_DY = (M == 2 || M == 4) && K % M == 0;
    constexpr int R = K + M;
    constexpr int NT = round64(4 * G * R);
    static_assert(T % CW == 0 && T % 32 == 0, "tile");
    const int64_t grid = (a.n_blocks + G - 1) / G;
    if constexpr (CAN_DY) {
        if (a.dyb == M) {
            hipLaunchKernelGGL((k_encode_hash<K, M, G, T, NBUF, NT, CW, PF, NTL, STAMP, M>), dim3((unsigned)grid),
                               dim3(NT), 0, s, a);
            return;
        }
    }
    hipLaunchKernelGGL((k_encode_hash<K, M, G, T, NBUF, NT, CW, PF, NTL, STAMP>), dim3((unsigned)grid), dim3(NT), 0, s, a);
}


template <int K, int M>
static hipError_t run_encode_fast(const EncArgs& a, hipStream_t s, int* path) {
    int p = PATH_NONE;
    if (a.sums) {
        constexpr int R = K + M;
        constexpr int G = pick_G<R>();
        constexpr int NBUF = 2;
        constexpr int T = pick_T<G * R, NBUF>();
        // Small batches are bound by one hash chain's latency, not by bytes: the split
        // path (encode-only pass + k_hash_lat) halves that (RS(8+4) 1 block: 0.23 vs
        // 0.53 ms; profiles/r02/sweep_sizes_small_v49.txt).  Not for RS(4+2), whose
        // quad-form k_ehx_ws chains run faster than k_hash_lat's at every size.
        if (a.variant == 0 && small_batch<K, M>(a.n_blocks, a.S)) {
            launch_encode_lat<K, M>(a, s);
            p = PATH_LATENCY;
        }
        // diagnostics 99: the product dispatch without the latency path (tests keep the
        // small-batch fused instances covered)
        const int fv = (ZS3_DIAG && a.variant == 99) ? 0 : a.variant;
#if ZS3_DIAG
        if (a.variant == 49) {  // force the small-batch split path
            launch_encode_lat<K, M>(a, s);
            p = PATH_LATENCY;
        }
        // the encode variants of fused_v2_diag.hip (PATH_NONE where one does not apply:
        // the first-generation launch below then serves the call)
        if (fv > 0 && p == PATH_NONE) p = launch_ehx(fv, a, s);
#endif
        // Dyadic shapes (RS(4+2), RS(8+4), RS(16+4), ...): the second-generation
        // kernels of fused_v2.hip pick their launch shape from (k, m, n_blocks).
        if (p == PATH_NONE && fv == 0) p = launch_ehx(0, a, s);
        if (p == PATH_NONE) {
            // First-generation kernel (profiles/r01 tuning): 8-byte columns so every
            // thread encodes, one 384-byte tile per step.  k <= 8: one LDS tile.
            // k > 8: two LDS tiles, so the next tile's encode does not wait for the
            // slower stripes' hashing.
            constexpr bool DY2 = K > 8 && (M == 2 || M == 4) && K % M == 0 &&
                                 2 * G * R * (384 + 32) + K * 32 <= 81920;
            if (DY2 && a.dyb == M) {
                if constexpr (DY2) launch_fused<K, M, G, 384, 2, 8>(a, s);
            } else if constexpr (G * R * (384 + 32) + M * K * 32 <= 40960) {
                launch_fused<K, M, G, 384, 1, 8>(a, s);
            } else {
                launch_fused<K, M, G, T, NBUF, 16>(a, s);
            }
            p = PATH_FIRSTGEN;
        }
    } else {
        const int64_t cols = (a.S + 15) >> 4;
        const unsigned gx = (unsigned)((cols + 255) / 256);
        const unsigned gy = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
        // non-temporal when every row is 16-byte aligned (diagnostics 98: plain)
        const bool al = (((uintptr_t)a.data | (uintptr_t)a.parity | (uint64_t)a.data_stride |
                          (uint64_t)a.parity_stride | (uint64_t)a.S) & 15) == 0;
        if (al && !(ZS3_DIAG && a.variant == 98))
            hipLaunchKernelGGL((k_encode_only<K, M, true>), dim3(gx, gy), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((k_encode_only<K, M>), dim3(gx, gy), dim3(256), 0, s, a);
        p = PATH_FIRSTGEN;
    }
    if (path) *path = p;
    return hipGetLastError();
}

#define ZS3_FAST_KM(X) \
    X(2, 1) X(2, 2) X(3, 2) X(3, 3) X(4, 2) X(4, 3) X(4, 4) X(5, 3) X(6, 2) X(6, 3) X(6, 4) \
    X(8, 2) X(8, 3) X(8, 4) X(10, 4) X(12, 4) X(16, 4)

// further geometries with an unaligned encode-only instance (the server defaults for
// 9-, 11-, 13- and 15-drive sets)
#define ZS3_UA_KM(X) X(5, 4) X(7, 4) X(9, 4) X(11, 4)

bool has_fast_encode(int k, int m) {
#define X(K, M) if (k == K && m == M) return true;
    ZS3_FAST_KM(X)
#undef X
    return false;
}

hipError_t launch_encode(const EncArgs& a, hipStream_t s, int* path) {
    if (path) *path = PATH_NONE;
    if (a.n_blocks <= 0 || a.S <= 0) return hipSuccess;
    // The server's non-dyadic default geometries (RS(6+4), RS(10+4), RS(3+3), ... and
    // RS(2+2) / RS(4+3)) on the warp-specialised kernel with a general matrix
    // (fused_v2_gen.hip) once the batch fills the chip (a workgroup takes 8-16 stripes);
    // smaller batches keep the latency-bound paths below.
    if (a.sums && a.variant == 0 && a.n_blocks >= 1024 && has_gen_encode(a.k, a.m)) {
        const int p = launch_ehx_gen(a, s);
        if (p != PATH_NONE) {
            if (path) *path = p;
            return hipGetLastError();
        }
    }
    // Vectorised kernels: 16-byte shard columns and no Split padding.
    const bool vec_ok = (a.S % 16) == 0 && a.n == (int64_t)a.k * a.S;
#define X(K, M)                                  \
    if (vec_ok && a.k == K && a.m == M) {        \
        return run_encode_fast<K, M>(a, s, path); \
    }
    ZS3_FAST_KM(X)
#undef X
    // fused encode + sums at shard sizes that are not a multiple of 16 (RS(12+4) on
    // 1 MiB blocks: S = 87 382)
    // (diagnostics: the RS(12+4) unaligned-row variants of fused_v2_diag.hip, same guard)
    if (a.sums && a.dyb && (a.variant == 0 || (ZS3_DIAG && a.variant >= 300))) {
        const int p = a.variant == 0 ? launch_ehx_ua(a, s) : launch_ehx(a.variant, a, s);
        if (p != PATH_NONE) {
            if (path) *path = p;
            return hipGetLastError();
        }
    }
    // Encode only at shard sizes that are not a multiple of 16 or with Split padding
    // (RS(12+4), RS(6+4), RS(10+4), ... on 1 MiB blocks): the specialised encode-only
    // kernel in UA mode (diagnostics 96: the any-geometry kernel below)
    // (a ragged column's 16-byte load ends at its row's valid end, so it starts at most 16
    // bytes before that end: inside the block when S >= 16 and n >= 16)
    if (!a.sums && a.S >= 16 && a.n >= 16 && !(ZS3_DIAG && (a.variant == 96 || a.variant == 97))) {
        const int64_t cols = (a.S + 15) >> 4;
        const unsigned gx = (unsigned)((cols + 255) / 256);
        const unsigned gy = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
#define X(K, M)                                                                               \
    if (a.k == K && a.m == M) {                                                               \
        hipLaunchKernelGGL((k_encode_only<K, M, false, true>), dim3(gx, gy), dim3(256), 0, s, a); \
        if (path) *path = PATH_FIRSTGEN;                                                      \
        return hipGetLastError();                                                             \
    }
        ZS3_FAST_KM(X)
        ZS3_UA_KM(X)
#undef X
    }
    if (path) *path = PATH_GENERIC;
    // any other geometry: encode (8-byte columns) + the batched hash in stripe mode;
    // diagnostics 97 keeps the byte kernel reachable
    if (encode_any_ok(a) && !(ZS3_DIAG && a.variant == 97)) return launch_encode_any(a, s);
    const int R = a.k + a.m;
    int nt = round64(4 * R);
    if (nt < 256) nt = 256;
    if (nt > 1024) nt = 1024;
    const size_t lds = (size_t)R * GEN_TS + 256 + 512 + (size_t)a.m * a.k;
    hipError_t e = ensure_dyn_lds((const void*)k_encode_hash_generic, lds);
    if (e != hipSuccess) return e;
    const unsigned grid = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
    hipLaunchKernelGGL(k_encode_hash_generic, dim3(grid), dim3(nt), lds, s, a);
    return hipGetLastError();
}

template <int K>
static hipError_t run_rec_fast(const RecArgs& a, hipStream_t s) {
    const int64_t cols = (a.S + 15) >> 4;
    const unsigned gx = (unsigned)((cols + 255) / 256);
    const unsigned gy = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
    // Default: non-temporal survivor loads and rebuilt-row stores (each byte is touched
    // once): RS(8+4) 4096 x 1 MiB {0,5} 1.016 -> 0.93 ms, {2,10} 0.905 -> 0.823 ms
    // (profiles/r02/ab_reconstruct_nt.jsonl).  Needs 16-byte aligned rows.
    if (((uintptr_t)a.shards & 15) == 0 && (a.block_stride & 15) == 0) {
        if (a.e <= 2)
            hipLaunchKernelGGL((k_reconstruct<K, 2, 1, true>), dim3(gx, gy), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((k_reconstruct<K, 4, 1, true>), dim3(gx, gy), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    if (a.e <= 2)
        hipLaunchKernelGGL((k_reconstruct<K, 2>), dim3(gx, gy), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_reconstruct<K, 4>), dim3(gx, gy), dim3(256), 0, s, a);
    return hipGetLastError();
}

template <int K>
static hipError_t run_rec_ua(const RecArgs& a, hipStream_t s) {
    const int64_t cols = (a.S + 15) >> 4;
    const unsigned gx = (unsigned)((cols + 255) / 256);
    const unsigned gy = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
    if (a.e <= 2)
        hipLaunchKernelGGL((k_reconstruct<K, 2, 1, false, true>), dim3(gx, gy), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_reconstruct<K, 4, 1, false, true>), dim3(gx, gy), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_reconstruct(const RecArgs& a, hipStream_t s, int* path) {
    if (path) *path = PATH_NONE;
    if (a.n_blocks <= 0 || a.S <= 0 || a.e <= 0) return hipSuccess;
    if (a.e <= 4 && (a.S % 16) == 0) {
        if (path) *path = PATH_FIRSTGEN;
        switch (a.k) {
            case 2: return run_rec_fast<2>(a, s);
            case 3: return run_rec_fast<3>(a, s);
            case 4: return run_rec_fast<4>(a, s);
            case 5: return run_rec_fast<5>(a, s);
            case 6: return run_rec_fast<6>(a, s);
            case 8: return run_rec_fast<8>(a, s);
            case 10: return run_rec_fast<10>(a, s);
            case 12: return run_rec_fast<12>(a, s);
            case 16: return run_rec_fast<16>(a, s);
            default: break;
        }
    }
    // unaligned shard sizes (1 MiB blocks of RS(12+4), RS(10+6), RS(5+4), ...): the same
    // specialised kernel with unaligned 16-byte accesses and a byte-wise last column
    // (diagnostics 97 keeps the any-geometry kernel reachable)
    if (a.e <= 4 && a.S >= 16 && !(ZS3_DIAG && a.variant == 97)) {
        if (path) *path = PATH_FIRSTGEN;
        switch (a.k) {
            case 2: return run_rec_ua<2>(a, s);
            case 3: return run_rec_ua<3>(a, s);
            case 4: return run_rec_ua<4>(a, s);
            case 5: return run_rec_ua<5>(a, s);
            case 6: return run_rec_ua<6>(a, s);
            case 8: return run_rec_ua<8>(a, s);
            case 10: return run_rec_ua<10>(a, s);
            case 12: return run_rec_ua<12>(a, s);
            case 16: return run_rec_ua<16>(a, s);
            default: break;
        }
    }
    if (path) *path = PATH_GENERIC;
    if (a.e <= AMAX && a.k <= 64 && !(ZS3_DIAG && a.variant == 97)) {
        const size_t lds = (size_t)a.e * a.k * 32 + 4 * (size_t)(a.k + a.e);
        hipError_t e = ensure_dyn_lds((const void*)k_reconstruct_any, lds);
        if (e != hipSuccess) return e;
        const int64_t gx = ((a.S + 7) / 8 + 255) / 256;
        const unsigned gy = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
        hipLaunchKernelGGL(k_reconstruct_any, dim3((unsigned)gx, gy), dim3(256), lds, s, a);
        return hipGetLastError();
    }
    const size_t lds = (size_t)((a.e * a.k + 3) & ~3) + 4 * (size_t)(a.k + a.e);
    hipError_t e = ensure_dyn_lds((const void*)k_reconstruct_generic, lds);
    if (e != hipSuccess) return e;
    const unsigned gx = (unsigned)((a.S + 255) / 256);
    const unsigned gy = (unsigned)(a.n_blocks < 65535 ? a.n_blocks : 65535);
    hipLaunchKernelGGL(k_reconstruct_generic, dim3(gx < 1024 ? gx : 1024, gy), dim3(256), lds, s, a);
    return hipGetLastError();
}

template <int K, int EMAX, bool HOUT>
static hipError_t run_vr(const VrArgs& a, hipStream_t s) {
    using Sh = VrShape<K, EMAX, HOUT>;
    static_assert(Sh::TILE <= 65536, "default GET tile fits the default LDS limit");
    const int64_t grid = (a.n_blocks + Sh::G - 1) / Sh::G;
    hipLaunchKernelGGL((k_verify_reconstruct<K, EMAX, HOUT>), dim3((unsigned)grid), dim3(Sh::NT), Sh::TILE, s, a);
    return hipGetLastError();
}

// The product GET / heal dispatch serves variant 0 and, in the diagnostics build, the
// variants that change a product shape's memory policy or layout (launch_vr_ws_t in
// fused_v2.hpp: 246 plain loads, 247 64-bit addresses, 420 the round-4 LDS stride,
// 423 high table dwords from LDS, 424 per-wave stamps, 429 the other rebuild-role
// priority, 431 / 433 timing ablations, 434 the other split placement, 440 the k_vr_ws
// instances for RS(16+4) rebuild / heal 4 instead of the survivor-quad kernel).
static bool product_get_variant(int v) {
    return v == 0 || (ZS3_DIAG && (v == 246 || v == 247 || v == 420 || v == 423 || v == 424 || v == 429 ||
                          v == 431 || v == 433 || v == 434 || v == 440 || v == 442 || v == 443 || v == 444 ||
                          v == 445 || v == 446 || v == 447));
}

// GET / heal small-batch path: k_reconstruct rebuilds the missing rows, then one chain
// per quad verifies the survivors (and, for heal, hashes the rebuilt rows).
static hipError_t launch_vr_lat(const VrArgs& a, hipStream_t s) {
    if (a.e > 0) {
        RecArgs r{};
        r.shards = a.shards;
        r.block_stride = a.block_stride;
        r.S = a.S;
        r.n_blocks = a.n_blocks;
        r.tables = a.tables;
        r.coef = a.coef;
        r.rows = a.rows;
        r.k = a.k;
        r.e = a.e;
        r.ids = a.ids;
        hipError_t e = launch_reconstruct(r, s, nullptr);
        if (e != hipSuccess) return e;
    }
    const int nr = a.k + (a.sums_out ? a.e : 0);
    const int64_t nch = a.n_blocks * nr;
    hipLaunchKernelGGL((k_vr_hash_lat<16, 3>), dim3((unsigned)((nch + 15) / 16)), dim3(64), 0, s, a, nr);
    return hipGetLastError();
}

// Crossover of the GET / heal latency path against the fused kernels (NOBJ sweeps of
// profiles/r02/get_lat_large_n.txt, get_small_batches.jsonl).  RS(4+2): the quad-form k_vr_ws
// chains are faster at every size.
static bool small_get(int k, int m, int e, bool heal, int64_t n, int64_t S) {
    if (k == 4 && m == 2) return false;
    if (k == 16 && m == 4) return n <= (e <= 1 ? 512 : 1024);
    if (k == 8 && m == 4) return n <= ((e <= 1 || (e == 2 && !heal)) ? 1024 : 2048);
    return n * k * S <= ((int64_t)1 << 30);
}

template <int K>
static hipError_t run_vr_k(const VrArgs& a, hipStream_t s, int* path) {
    if ((a.variant == 0 && small_get(a.k, a.m, a.e, a.sums_out != nullptr, a.n_blocks, a.S)) ||
        (ZS3_DIAG && a.variant == 230)) {  // 230: force it
        if (path) *path = PATH_LATENCY;
        return launch_vr_lat(a, s);
    }
    // Default for the RS(8+4)-, RS(4+2)- and RS(16+4)-shaped GETs: the warp-specialised
    // k_vr_ws (fused_v2.hip): RS(8+4) verify 0.85 -> 0.70 ms, verify + rebuild 2
    // 1.41 -> 1.13 ms on 4096 x 1 MiB (scripts/get_ab.py).  Diagnostics: 231 = the
    // product dispatch without the latency path; the variants of the product GET shapes
    // (product_get_variant) reach launch_vr_ws_t through the product dispatch; any other
    // variant runs the first-generation kernel.
    if (product_get_variant(a.variant) || (ZS3_DIAG && a.variant == 231))
        if (launch_vr_ws(0, a, s)) {
            if (path) *path = PATH_WS;
            return hipGetLastError();
        }
    if (path) *path = PATH_FIRSTGEN;
    const bool hout = a.sums_out != nullptr;
    if (a.e == 0) return run_vr<K, 0, false>(a, s);
    if (a.e <= 2) return hout ? run_vr<K, 2, true>(a, s) : run_vr<K, 2, false>(a, s);
    return hout ? run_vr<K, 4, true>(a, s) : run_vr<K, 4, false>(a, s);
}

hipError_t launch_verify_reconstruct(const VrArgs& a, hipStream_t s, int* path) {
    if (path) *path = PATH_NONE;
    if (a.n_blocks <= 0 || a.S <= 0) return hipSuccess;
    // Server-default geometries whose k is not 4, 8, 12 or 16 (RS(2+2), (3+2), (5+4),
    // (6+4), ...; fused_v2_get_gen.hip): rebuild / heal on the warp-specialised kernel
    // in one launch (4096 x 1 MiB: see that file); small batches keep the launches below
    if (product_get_variant(a.variant) && a.e >= 1 && a.e <= 4 && a.n_blocks >= 1024 && launch_vr_ws_gen(a, s)) {
        if (path) *path = PATH_WS;
        return hipGetLastError();
    }
    if (a.e <= 4 && (a.S % 16) == 0) {
        switch (a.k) {
            case 2: return run_vr_k<2>(a, s, path);
            case 4: return run_vr_k<4>(a, s, path);
            case 6: return run_vr_k<6>(a, s, path);
            case 8: return run_vr_k<8>(a, s, path);
            case 10: return run_vr_k<10>(a, s, path);
            case 12: return run_vr_k<12>(a, s, path);
            case 16: return run_vr_k<16>(a, s, path);
            default: break;
        }
    }
    // RS(12+4) on 1 MiB blocks (unaligned rows): the warp-specialised kernel in UA mode
    // (diagnostics 97: the any-geometry launches below)
    if (a.e <= 4 && a.k == 12 && !(ZS3_DIAG && a.variant == 97)) {
        if (launch_vr_ws(0, a, s)) {
            if (path) *path = PATH_WS;
            return hipGetLastError();
        }
    }
    // Any other shape: one verify launch per survivor row, then the reconstruct
    // kernel, then (heal) one hash launch per rebuilt row.
    if (path) *path = PATH_GENERIC;
    const int R = a.k + a.m;
    int32_t rows[256];
    if (a.h_rows) {
        for (int i = 0; i < a.k + a.e; ++i) rows[i] = a.h_rows[i];
    } else if (hipMemcpyAsync(rows, a.rows, (size_t)(a.k + a.e) * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
               hipStreamSynchronize(s) != hipSuccess) {
        return hipGetLastError();
    }
    if (a.k <= 64 && a.e <= 64 && !(ZS3_DIAG && a.variant == 97)) {
        // survivors verified in one launch (hash kernel, stripe mode), then the rebuild,
        // then (heal) the rebuilt rows hashed in one launch
        HashArgs h{};
        h.rps = a.k;
        h.kd = a.k + a.m;
        h.rtot = a.k + a.m;
        h.msgs = a.shards;
        h.stride = a.block_stride;
        h.len = a.S;
        h.n = a.n_blocks * a.k;
        h.expect = a.expect;
        h.bad = a.bad;
        h.ids = a.ids;
        for (int j = 0; j < a.k; ++j) h.rowmap[j] = (uint8_t)rows[j];
        for (int q = 0; q < 4; ++q) h.key[q] = a.key[q];
        hipError_t e = launch_hash(h, s);
        if (e != hipSuccess || a.e == 0) return e;
        RecArgs r{};
        r.shards = a.shards;
        r.block_stride = a.block_stride;
        r.S = a.S;
        r.n_blocks = a.n_blocks;
        r.tables = a.tables;
        r.coef = a.coef;
        r.rows = a.rows;
        r.k = a.k;
        r.e = a.e;
        r.ids = a.ids;
        e = launch_reconstruct(r, s, nullptr);
        if (e != hipSuccess || !a.sums_out) return e;
        HashArgs g{};
        g.rps = a.e;
        g.kd = a.k + a.m;
        g.rtot = a.k + a.m;
        g.msgs = a.shards;
        g.stride = a.block_stride;
        g.len = a.S;
        g.n = a.n_blocks * a.e;
        g.sums = a.sums_out;
        g.ids = a.ids;
        for (int j = 0; j < a.e; ++j) g.rowmap[j] = (uint8_t)rows[a.k + j];
        for (int q = 0; q < 4; ++q) g.key[q] = a.key[q];
        return launch_hash(g, s);
    }
    for (int j = 0; j < a.k; ++j) {
        HashArgs h{};
        h.msgs = a.shards + (int64_t)rows[j] * a.S;
        h.stride = a.block_stride;
        h.len = a.S;
        h.n = a.n_blocks;
        h.expect = a.expect + (int64_t)rows[j] * 32;
        h.bad = a.bad + rows[j];
        h.sum_stride = (int64_t)R * 32;
        h.bad_stride = R;
        h.ids = a.ids;
        for (int q = 0; q < 4; ++q) h.key[q] = a.key[q];
        hipError_t e = launch_hash(h, s);
        if (e != hipSuccess) return e;
    }
    if (a.e > 0) {
        RecArgs r{};
        r.shards = a.shards;
        r.block_stride = a.block_stride;
        r.S = a.S;
        r.n_blocks = a.n_blocks;
        r.tables = a.tables;
        r.coef = a.coef;
        r.rows = a.rows;
        r.k = a.k;
        r.e = a.e;
        r.ids = a.ids;
        hipError_t e = launch_reconstruct(r, s, nullptr);
        if (e != hipSuccess) return e;
        if (a.sums_out) {
            for (int i = 0; i < a.e; ++i) {
                HashArgs h{};
                h.msgs = a.shards + (int64_t)rows[a.k + i] * a.S;
                h.stride = a.block_stride;
                h.len = a.S;
                h.n = a.n_blocks;
                h.sums = a.sums_out + (int64_t)rows[a.k + i] * 32;
                h.sum_stride = (int64_t)R * 32;
                h.ids = a.ids;
                for (int q = 0; q < 4; ++q) h.key[q] = a.key[q];
                e = launch_hash(h, s);
                if (e != hipSuccess) return e;
            }
        }
    }
    return hipSuccess;
}

hipError_t launch_hash(const HashArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    const int64_t grid = (a.n + HB_CH - 1) / HB_CH;
    // (non-temporal loads here measured 1.11 -> 1.28 ms for 49 152 x 128 KiB and 0.70 ->
    // 1.28 ms for the deep scan: profiles/r02/ab_hash_nt.jsonl; not kept)
    hipLaunchKernelGGL(k_hash_batch<false>, dim3((unsigned)grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fill(uint8_t* out, int64_t stride, int64_t len, int64_t n, uint64_t seed,
                       uint64_t obj0, hipStream_t s) {
    if (n <= 0 || len <= 0) return hipSuccess;
    const int64_t nw = (len + 7) >> 3;
    const unsigned gx = (unsigned)((nw + 255) / 256 < 256 ? (nw + 255) / 256 : 256);
    const unsigned gy = (unsigned)(n < 65535 ? n : 65535);
    hipLaunchKernelGGL(k_fill, dim3(gx, gy), dim3(256), 0, s, out, stride, len, n, seed, obj0);
    return hipGetLastError();
}

// Rebuilt rows of a batch of stripes, device -> host (zs3_stream_decode on rows that are
// not 256-byte aligned, zs3gpu.hip stream_vr_range): for blocks b < nb and rows rs.row[],
// S bytes at b*E + row*S from src to the same offset of dst.  The two bases are congruent
// mod 16 (the caller checks), so each row is a ragged head, 16-byte words, a ragged tail.
// The HIP runtime's own D2H of the whole stripes moved 8x the bytes (profiles/r06/dma_sg).
__global__ void __launch_bounds__(256) k_rows_copy(const uint8_t* src, uint8_t* dst, int64_t E, int64_t S, int64_t nb,
                                                   RowSet rs) {
    for (int64_t p = blockIdx.y; p < nb * rs.n; p += gridDim.y) {
        const int64_t off = (p / rs.n) * E + (int64_t)rs.row[p % rs.n] * S;
        const uint8_t* sp = src + off;
        uint8_t* dp = dst + off;
        const int64_t h = std::min<int64_t>((16 - ((uintptr_t)dp & 15)) & 15, S);
        const int64_t nw = (S - h) >> 4;
        const int64_t t0 = h + nw * 16;
        if (blockIdx.x == 0 && threadIdx.x < h) dp[threadIdx.x] = sp[threadIdx.x];
        if (blockIdx.x == 0 && threadIdx.x < S - t0) dp[t0 + threadIdx.x] = sp[t0 + threadIdx.x];
        const uint4* s4 = reinterpret_cast<const uint4*>(sp + h);
        uint4* d4 = reinterpret_cast<uint4*>(dp + h);
        for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (int64_t)gridDim.x * 256) d4[w] = s4[w];
    }
    __threadfence_system();  // host-visible before the batch's completion event
}

hipError_t launch_rows_copy(const uint8_t* src, uint8_t* dst, int64_t E, int64_t S, int64_t nb, const RowSet& rs,
                            hipStream_t s) {
    if (nb <= 0 || rs.n <= 0 || S <= 0) return hipSuccess;
    if ((((uintptr_t)src - (uintptr_t)dst) & 15) != 0 || rs.n > 32) return hipErrorInvalidValue;
    const int64_t words = (S + 15) / 16;
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(64, (words + 255) / 256));
    const int64_t pairs = nb * rs.n;
    const unsigned gy = (unsigned)(pairs < 65535 ? pairs : 65535);
    hipLaunchKernelGGL(k_rows_copy, dim3(gx, gy), dim3(256), 0, s, src, dst, E, S, nb, rs);
    return hipGetLastError();
}

// One wavefront per row: OR of the row's flags (deep-scan: a file is corrupt when any
// of its chunks is).
__global__ void __launch_bounds__(256) k_any_rows(const int32_t* flags, int64_t rows, int64_t cols, int32_t* out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    int any = 0;
    for (int64_t c = threadIdx.x & 63; c < cols; c += 64) any |= flags[r * cols + c] != 0;
    const unsigned long long b = __ballot(any);
    if ((threadIdx.x & 63) == 0) out[r] = b ? 1 : 0;
}

hipError_t launch_any_rows(const int32_t* flags, int64_t rows, int64_t cols, int32_t* out, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_any_rows, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, flags, rows, cols, out);
    return hipGetLastError();
}

}  // namespace zs3k
