// Memory-pattern probe, round 4 (second pass).  mempat3 showed every lockstep shape
// (G stripes per workgroup stepping T-byte tiles, 4 to 32 stripes, 256 B to 4 KiB tiles,
// one tile or two in flight) at 64-67 % of 8 TB/s against 72 % for the encode-only
// streaming shape (each workgroup one 4 KiB column chunk of all rows of one stripe, then
// exit).  Here the lockstep loop issues its loads the way the fused kernel does (inline-asm
// non-temporal loads the compiler does not track, exact s_waitcnt vmcnt(N), stores of tile
// s after the loads of tile s+PF), and probes the address-mapping hypotheses:
//   rowpad   rows of a stripe S + pad apart instead of S = 2^17 (power-of-two row stride)
//   skew     stripe stride (k+m)*S + skew
//   stream1  the streaming shape at one workgroup of 1024 threads per CU
// Prints one JSON line per pattern: ms and algorithmic TB/s (data + parity bytes).
//   hipcc --offload-arch=gfx950 -O3 -o mempat4 mempat4.hip && ./mempat4
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int K = 8, M = 4, R = 12;
constexpr int64_t S0 = 131072, NOBJ = 16384;

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void ld_nt(u4& dst, const uint8_t* p) {
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(dst) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait(u4 (&xs)[K]) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
    for (int j = 0; j < K; ++j) asm volatile("" : "+v"(xs[j]));
}
__device__ __forceinline__ void st_nt(uint8_t* p, u4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u4*>(p)); }

// G stripes per workgroup, NT loading threads (16-byte columns), T = NT*16/G bytes per row
// per step, one tile of loads in flight (the fused kernel's steady step: wait for tile s,
// compute, issue the loads of tile s+1, store tile s).  Row j of stripe b at
// buf + b*stride + j*rs.
template <int G, int NT>
__global__ void __launch_bounds__(NT) k_lock(uint8_t* buf, int64_t stride, int64_t rs) {
    constexpr int CPB = NT / G;
    constexpr int T = CPB * 16;
    constexpr int64_t NST = S0 / T;  // full tiles only
    const int g = threadIdx.x / CPB, o = (threadIdx.x % CPB) * 16;
    uint8_t* base = buf + ((int64_t)blockIdx.x * G + g) * stride + o;
    u4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) ld_nt(x[j], base + j * rs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int64_t s = 0; s + 1 < NST; ++s) {
        vm_wait<M>(x);
        u4 par[M];
        par[0] = x[0] ^ x[1];
        par[1] = x[2] ^ x[3];
        par[2] = x[4] ^ x[5];
        par[3] = x[6] ^ x[7];
#pragma unroll
        for (int j = 0; j < K; ++j) ld_nt(x[j], base + j * rs + (s + 1) * T);
#pragma unroll
        for (int r = 0; r < M; ++r) st_nt(base + (K + r) * rs + s * T, par[r]);
    }
    vm_wait<0>(x);
#pragma unroll
    for (int r = 0; r < M; ++r) st_nt(base + (K + r) * rs + (NST - 1) * T, x[2 * r] ^ x[2 * r + 1]);
}

// encode_only-style: grid (S / (NT*16), NOBJ), one 16-B column per thread.
template <int NT>
__global__ void __launch_bounds__(NT) k_stream(uint8_t* buf, int64_t stride, int64_t rs) {
    uint8_t* base = buf + (int64_t)blockIdx.y * stride + ((int64_t)blockIdx.x * NT + threadIdx.x) * 16;
    u4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(base + j * rs));
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
static void lock(uint8_t* d, int64_t rowpad, int64_t skew, int lds) {
    const int64_t rs = S0 + rowpad, stride = R * rs + skew;
    (void)hipFuncSetAttribute((const void*)k_lock<G, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    char nm[160];
    snprintf(nm, sizeof nm, "lock G%d T%d NT%d rowpad%lld skew%lld lds%dK", G, NT * 16 / G, NT, (long long)rowpad,
             (long long)skew, lds >> 10);
    timeit(nm, [&] { hipLaunchKernelGGL((k_lock<G, NT>), dim3(NOBJ / G), dim3(NT), lds, 0, d, stride, rs); });
}

template <int NT>
static void stream(uint8_t* d, int64_t rowpad, int64_t skew, int lds) {
    const int64_t rs = S0 + rowpad, stride = R * rs + skew;
    (void)hipFuncSetAttribute((const void*)k_stream<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    char nm[160];
    snprintf(nm, sizeof nm, "stream NT%d rowpad%lld skew%lld lds%dK", NT, (long long)rowpad, (long long)skew, lds >> 10);
    timeit(nm, [&] { hipLaunchKernelGGL((k_stream<NT>), dim3(S0 / (NT * 16), NOBJ), dim3(NT), lds, 0, d, stride, rs); });
}

int main() {
    uint8_t* d;
    const int64_t maxrow = S0 + 8192, maxskew = 1 << 20;
    const size_t bytes = (size_t)NOBJ * (R * maxrow + maxskew);
    if (hipMalloc(&d, bytes) != hipSuccess) return 1;
    (void)hipMemset(d, 1, bytes);
    const int ONE = 96 << 10;  // one workgroup per CU
    stream<256>(d, 0, 0, 0);
    stream<1024>(d, 0, 0, ONE);
    stream<256>(d, 256, 0, 0);
    // the product's memory shape: 16 stripes, 384-byte tiles, 6 loading waves
    lock<16, 384>(d, 0, 0, ONE);
    lock<16, 384>(d, 256, 0, ONE);
    lock<16, 384>(d, 4096, 0, ONE);
    lock<16, 384>(d, 128, 0, ONE);
    lock<16, 384>(d, 0, 4096, ONE);
    lock<16, 384>(d, 0, 65536, ONE);
    lock<16, 384>(d, 0, 1 << 20, ONE);
    lock<16, 768>(d, 0, 0, ONE);
    lock<16, 768>(d, 256, 0, ONE);
    lock<8, 384>(d, 0, 0, ONE);
    lock<8, 384>(d, 256, 0, ONE);
    lock<4, 1024>(d, 0, 0, ONE);
    lock<4, 1024>(d, 256, 0, ONE);
    lock<16, 384>(d, 0, 0, 0);
    stream<256>(d, 0, 0, 0);
    (void)hipFree(d);
    return 0;
}
