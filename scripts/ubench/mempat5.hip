// Memory-pattern probe, round 4 (third pass): the lockstep shape of the fused kernels with
// compiler-tracked loads only.  Loader waves read 8 data rows (16-byte columns, one tile
// of register prefetch) and XOR them into 4 parity columns that go to an LDS tile; storer
// waves of the same workgroup read the parity tile back and store it (one barrier per
// step).  No wave mixes loads and stores, so every s_waitcnt the compiler inserts is exact
// (no untracked loads, nothing for scripts/check_async_loads.py to guard).
// Probes whether the cap of this shape (65-68 % of 8 TB/s against 72 % for the streaming
// encode-only shape) comes from the power-of-two row stride of the Split layout:
//   rowpad  rows of a stripe S + pad apart (S = 2^17 in the reference layout)
//   skew    stripe stride (k+m)*S + skew
// Prints one JSON line per pattern: ms, algorithmic TB/s (data + parity bytes) and frac.
//   hipcc --offload-arch=gfx950 -O3 -o mempat5 mempat5.hip && ./mempat5
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int K = 8, M = 4, R = 12;
constexpr int64_t S0 = 131072, NOBJ = 16384;

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u4 ld_nt(const uint8_t* p) { return __builtin_nontemporal_load(reinterpret_cast<const u4*>(p)); }
__device__ __forceinline__ void st_nt(uint8_t* p, u4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u4*>(p)); }

// G stripes, NT loader threads + NT storer threads, T = NT*16/G bytes per row per step.
template <int G, int NT>
__global__ void __launch_bounds__(2 * NT) k_split(uint8_t* buf, int64_t stride, int64_t rs) {
    constexpr int CPB = NT / G;
    constexpr int T = CPB * 16;
    constexpr int64_t NST = S0 / T;  // full tiles only
    constexpr int PT = G * M * T;    // parity tile bytes
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x;
    const int lt = tid < NT ? tid : tid - NT;
    const int g = lt / CPB, o = (lt % CPB) * 16;
    uint8_t* base = buf + ((int64_t)blockIdx.x * G + g) * stride + o;
    u4* pt = reinterpret_cast<u4*>(lds);
    const int slot = (g * M * T + o) / 16;  // row r of the column at slot + r*T/16
    if (tid < NT) {
        u4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = ld_nt(base + j * rs);
        for (int64_t s = 0; s < NST; ++s) {
            u4 nx[K];
            if (s + 1 < NST) {
#pragma unroll
                for (int j = 0; j < K; ++j) nx[j] = ld_nt(base + j * rs + (s + 1) * T);
            }
            u4* tl = pt + (s & 1) * (PT / 16) + slot;
#pragma unroll
            for (int r = 0; r < M; ++r) tl[r * (T / 16)] = x[2 * r] ^ x[2 * r + 1];
            __syncthreads();
            if (s + 1 < NST) {
#pragma unroll
                for (int j = 0; j < K; ++j) x[j] = nx[j];
            }
        }
    } else {
        for (int64_t s = 0; s < NST; ++s) {
            __syncthreads();
            const u4* tl = pt + (s & 1) * (PT / 16) + slot;
#pragma unroll
            for (int r = 0; r < M; ++r) st_nt(base + (K + r) * rs + s * T, tl[r * (T / 16)]);
        }
    }
}

// k_split with PF tiles of loads in flight (a register ring, unrolled by PF so every
// register keeps its slot; the loader waves issue no stores, so the compiler's waits are
// exact) and NW workgroups' worth of stripes per launch row.
template <int G, int NT, int PF, int SM = 0>
__global__ void __launch_bounds__(2 * NT) k_split_pf(uint8_t* buf, int64_t stride, int64_t rs) {
    constexpr int CPB = NT / G;
    constexpr int T = CPB * 16;
    constexpr int64_t NST = S0 / T / 4 * 4;  // whole groups of 4 full tiles (PF and SM 2 / 4 divide it)
    constexpr int NB = SM >= 100 ? SM - 100 + 2 : SM >= 2 ? 2 * SM : 2;  // parity tiles in the LDS ring
    constexpr int PT = G * M * T;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x;
    const int lt = tid < NT ? tid : tid - NT;
    const int g = lt / CPB, o = (lt % CPB) * 16;
    uint8_t* base = buf + ((int64_t)blockIdx.x * G + g) * stride + o;
    u4* pt = reinterpret_cast<u4*>(lds);
    const int slot = (g * M * T + o) / 16;
    if (tid < NT) {
        u4 x[PF][K];
#pragma unroll
        for (int p = 0; p < PF; ++p)
#pragma unroll
            for (int j = 0; j < K; ++j) x[p][j] = ld_nt(base + j * rs + p * T);
        for (int64_t s0 = 0; s0 < NST; s0 += PF) {
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                const int64_t s = s0 + p;
                u4* tl = pt + (s % NB) * (PT / 16) + slot;
#pragma unroll
                for (int r = 0; r < M; ++r) tl[r * (T / 16)] = x[p][2 * r] ^ x[p][2 * r + 1];
                if (s + PF < NST) {
#pragma unroll
                    for (int j = 0; j < K; ++j) x[p][j] = ld_nt(base + j * rs + (s + PF) * T);
                }
                __syncthreads();
            }
        }
    } else {
        // storer lane mapping for batched stores: SM consecutive tiles of one parity row are
        // stored as one contiguous run (lane q of the stripe covers 16 B of the run)
        for (int64_t s = 0; s < NST; ++s) {
            __syncthreads();
            if constexpr (SM == 0) {
                const u4* tl = pt + (s % NB) * (PT / 16) + slot;
#pragma unroll
                for (int r = 0; r < M; ++r) st_nt(base + (K + r) * rs + s * T, tl[r * (T / 16)]);
            } else if constexpr (SM >= 100) {
                constexpr int D = SM - 100;
                for (int64_t tt = (s >= D ? s - D : NST); tt <= s - D || (s == NST - 1 && tt < NST); ++tt) {
                    const u4* tl = pt + (tt % NB) * (PT / 16) + slot;
#pragma unroll
                    for (int r = 0; r < M; ++r) st_nt(base + (K + r) * rs + tt * T, tl[r * (T / 16)]);
                }
            } else if constexpr (SM >= 2) {
                if ((s % SM) == SM - 1) {
                    const int64_t s0 = s - (SM - 1);
#pragma unroll
                    for (int u = 0; u < SM; ++u) {
                        // run byte offset u*T + o within the SM*T-byte run of row r
                        const int64_t tt = s0 + u;
                        const u4* tl = pt + (tt % NB) * (PT / 16) + slot;
#pragma unroll
                        for (int r = 0; r < M; ++r) st_nt(base + (K + r) * rs + tt * T, tl[r * (T / 16)]);
                    }
                }
            }
        }
    }
}

// encode_only-style: grid (S / (NT*16), NOBJ), one 16-B column per thread.
template <int NT>
__global__ void __launch_bounds__(NT) k_stream(uint8_t* buf, int64_t stride, int64_t rs) {
    uint8_t* base = buf + (int64_t)blockIdx.y * stride + ((int64_t)blockIdx.x * NT + threadIdx.x) * 16;
    u4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld_nt(base + j * rs);
    st_nt(base + (K + 0) * rs, x[0] ^ x[1]);
    st_nt(base + (K + 1) * rs, x[2] ^ x[3]);
    st_nt(base + (K + 2) * rs, x[4] ^ x[5]);
    st_nt(base + (K + 3) * rs, x[6] ^ x[7]);
}

// the same with the grid transposed: consecutive workgroups take consecutive stripes at
// the same 4 KiB chunk offset (thousands of stripes in flight, 4 KiB per row each)
template <int NT>
__global__ void __launch_bounds__(NT) k_stream_t(uint8_t* buf, int64_t stride, int64_t rs) {
    uint8_t* base = buf + (int64_t)blockIdx.x * stride + ((int64_t)blockIdx.y * NT + threadIdx.x) * 16;
    u4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld_nt(base + j * rs);
    st_nt(base + (K + 0) * rs, x[0] ^ x[1]);
    st_nt(base + (K + 1) * rs, x[2] ^ x[3]);
    st_nt(base + (K + 2) * rs, x[4] ^ x[5]);
    st_nt(base + (K + 3) * rs, x[6] ^ x[7]);
}

// stream with SPAN stripes interleaved: workgroup w takes chunk (w / SPAN) % CH of stripe
// (w % SPAN) + SPAN * (w / (SPAN * CH)): SPAN stripes are swept together, chunk by chunk
template <int NT, int SPAN>
__global__ void __launch_bounds__(NT) k_stream_span(uint8_t* buf, int64_t stride, int64_t rs) {
    constexpr int CH = (int)(S0 / (NT * 16));
    const int64_t w = blockIdx.x;
    const int64_t stripe = (w % SPAN) + (int64_t)SPAN * (w / ((int64_t)SPAN * CH));
    const int64_t chunk = (w / SPAN) % CH;
    uint8_t* base = buf + stripe * stride + (chunk * NT + threadIdx.x) * 16;
    u4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld_nt(base + j * rs);
    st_nt(base + (K + 0) * rs, x[0] ^ x[1]);
    st_nt(base + (K + 1) * rs, x[2] ^ x[3]);
    st_nt(base + (K + 2) * rs, x[4] ^ x[5]);
    st_nt(base + (K + 3) * rs, x[6] ^ x[7]);
}

template <typename F>
static void timeit(const char* name, F launch) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    launch();
    launch();
    (void)hipEventRecord(e0);
    const int reps = 6;
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        printf("%s: %s\n", name, hipGetErrorString(err));
        exit(2);  // sticky: stop at the first fault
    }
    ms /= reps;
    const double bytes = (double)NOBJ * (K + M) * S0;
    printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f, \"frac\": %.4f}\n", name, ms, bytes / ms / 1e9,
           bytes / ms / 1e9 / 8.0);
    fflush(stdout);
}

template <int G, int NT>
static void split(uint8_t* d, int64_t rowpad, int64_t skew, int lds) {
    constexpr int T = NT * 16 / G;
    const int need = 2 * G * M * T;
    const int dyn = need > lds ? need : lds;
    if (dyn > 163840) return;
    const int64_t rs = S0 + rowpad, stride = R * rs + skew;
    (void)hipFuncSetAttribute((const void*)k_split<G, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, dyn);
    char nm[160];
    snprintf(nm, sizeof nm, "split G%d T%d NT%d rowpad%lld skew%lld lds%dK", G, T, NT, (long long)rowpad, (long long)skew,
             dyn >> 10);
    timeit(nm, [&] { hipLaunchKernelGGL((k_split<G, NT>), dim3(NOBJ / G), dim3(2 * NT), dyn, 0, d, stride, rs); });
}

template <int NT>
static void stream(uint8_t* d, int64_t rowpad, int64_t skew) {
    const int64_t rs = S0 + rowpad, stride = R * rs + skew;
    char nm[160];
    snprintf(nm, sizeof nm, "stream NT%d rowpad%lld skew%lld", NT, (long long)rowpad, (long long)skew);
    timeit(nm, [&] { hipLaunchKernelGGL((k_stream<NT>), dim3(S0 / (NT * 16), NOBJ), dim3(NT), 0, 0, d, stride, rs); });
}

template <int G, int NT, int PF, int SM = 0>
static void splitpf(uint8_t* d, int lds) {
    constexpr int T = NT * 16 / G;
    constexpr int NB = SM >= 100 ? SM - 100 + 2 : SM >= 2 ? 2 * SM : 2;
    const int need = NB * G * M * T;
    const int dyn = need > lds ? need : lds;
    if (dyn > 163840 || 2 * NT > 1024) return;
    (void)hipFuncSetAttribute((const void*)k_split_pf<G, NT, PF, SM>, hipFuncAttributeMaxDynamicSharedMemorySize, dyn);
    char nm[160];
    snprintf(nm, sizeof nm, "splitpf G%d T%d NT%d PF%d stores%s lds%dK", G, T, NT, PF,
             SM == 0 ? "each" : SM == 1 ? "none" : SM == 2 ? "batch2" : SM == 4 ? "batch4" : SM == 104 ? "delay4" : "delay8",
             dyn >> 10);
    timeit(nm, [&] { hipLaunchKernelGGL((k_split_pf<G, NT, PF, SM>), dim3(NOBJ / G), dim3(2 * NT), dyn, 0, d, R * S0, S0); });
}

// stream without stores (the read half of the traffic alone)
template <int NT>
__global__ void __launch_bounds__(NT) k_stream_ro(uint8_t* buf, int64_t stride, int64_t rs) {
    uint8_t* base = buf + (int64_t)blockIdx.y * stride + ((int64_t)blockIdx.x * NT + threadIdx.x) * 16;
    u4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld_nt(base + j * rs);
    u4 a = x[0] ^ x[1] ^ x[2] ^ x[3] ^ x[4] ^ x[5] ^ x[6] ^ x[7];
    if (a.x == 0x9E3779B9u && a.y == 0x7F4A7C15u) buf[0] = 1;  // keep the loads
}

template <int NT, int SPAN>
static void span(uint8_t* d) {
    char nm[160];
    snprintf(nm, sizeof nm, "stream span%d NT%d", SPAN, NT);
    timeit(nm, [&] { hipLaunchKernelGGL((k_stream_span<NT, SPAN>), dim3(S0 / (NT * 16) * NOBJ), dim3(NT), 0, 0, d, R * S0, S0); });
}

int main() {
    uint8_t* d;
    const int64_t maxrow = S0 + 8192, maxskew = 1 << 20;
    const size_t bytes = (size_t)NOBJ * (R * maxrow + maxskew);
    if (hipMalloc(&d, bytes) != hipSuccess) return 1;
    (void)hipMemset(d, 1, bytes);
    const int ONE = 96 << 10;  // one workgroup per CU
    stream<256>(d, 0, 0);
    timeit("stream transposed NT256", [&] { hipLaunchKernelGGL((k_stream_t<256>), dim3(NOBJ, S0 / 4096), dim3(256), 0, 0, d, R * S0, S0); });
    timeit("stream no stores NT256 (read bytes only)", [&] { hipLaunchKernelGGL((k_stream_ro<256>), dim3(S0 / 4096, NOBJ), dim3(256), 0, 0, d, R * S0, S0); });
    splitpf<16, 384, 2, 0>(d, 96 << 10);
    splitpf<16, 384, 2, 104>(d, 96 << 10);
    splitpf<8, 384, 2, 104>(d, 96 << 10);
    splitpf<8, 384, 2, 108>(d, 96 << 10);
    splitpf<8, 384, 2, 0>(d, 96 << 10);
    // the product's memory shape: 16 stripes, 384-byte tiles, 6 loading waves (+6 storing)
    split<16, 384>(d, 0, 0, ONE);

    stream<256>(d, 0, 0);
    (void)hipFree(d);
    return 0;
}
