// Memory-pattern probe for the fused encode+hash kernel (no GF, no hash): 4096
// stripes of 8 data rows read + 4 parity rows written, 128 KiB rows, in the access
// orders the fused kernel could use.  Prints ms and algorithmic TB/s per pattern.
//   hipcc --offload-arch=gfx950 -O3 -o mempat mempat.hip && ./mempat
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int K = 8, M = 4, R = 12;
constexpr int64_t S = 131072, NOBJ = 4096, STRIDE = R * S;

template <int CW> struct V;
template <> struct V<8> { typedef uint32_t t __attribute__((ext_vector_type(2))); };
template <> struct V<16> { typedef uint32_t t __attribute__((ext_vector_type(4))); };

// G stripes per workgroup, NT threads, CW bytes per lane -> T = NT*CW/G bytes per row per
// step.  BAR: __syncthreads() every step.  Loads of step i+1 are issued before the
// stores of step i (one tile of register prefetch).
// MAP 0: workgroup w owns stripes w*G..w*G+G-1; 1: stripes w + j*(NOBJ/G) (spread);
// 2: XCD-contiguous (w%8 picks a contiguous eighth of the batch).
template <int G, int NT, int CW, bool BAR, int MAP = 0>
__global__ void __launch_bounds__(NT) k_lockstep(uint8_t* buf) {
    typedef typename V<CW>::t VT;
    constexpr int CPB = NT / G;
    constexpr int T = CPB * CW;
    const int g = threadIdx.x / CPB, o = (threadIdx.x % CPB) * CW;
    const int64_t nwg = NOBJ / G, w = blockIdx.x;
    const int64_t stripe = MAP == 0 ? w * G + g
                         : MAP == 1 ? w + g * nwg
                                    : ((w % 8) * (nwg / 8) + w / 8) * G + g;
    uint8_t* base = buf + stripe * STRIDE + o;
    VT x[K];
    for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const VT*>(base + j * S);
    // full tiles only (T need not divide S): every access stays inside its row
    for (int64_t t0 = 0; t0 + T <= S; t0 += T) {
        VT p0 = x[0] ^ x[1], p1 = x[2] ^ x[3], p2 = x[4] ^ x[5], p3 = x[6] ^ x[7];
        if (t0 + 2 * T <= S)
            for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const VT*>(base + j * S + t0 + T);
        *reinterpret_cast<VT*>(base + (K + 0) * S + t0) = p0;
        *reinterpret_cast<VT*>(base + (K + 1) * S + t0) = p1;
        *reinterpret_cast<VT*>(base + (K + 2) * S + t0) = p2;
        *reinterpret_cast<VT*>(base + (K + 3) * S + t0) = p3;
        if (BAR) __syncthreads();
    }
}

// Lockstep with the parity writes deferred: every N steps, N tiles' parity (kept in
// registers) is written back-to-back, i.e. N*T contiguous bytes per parity row.
template <int N>
__global__ void __launch_bounds__(192) k_defer(uint8_t* buf) {
    typedef V<8>::t VT;
    constexpr int G = 4, NT = 192, CW = 8, CPB = NT / G, T = CPB * CW;
    const int g = threadIdx.x / CPB, o = (threadIdx.x % CPB) * CW;
    uint8_t* base = buf + ((int64_t)blockIdx.x * G + g) * STRIDE + o;
    VT x[K], p[N][M];
    for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const VT*>(base + j * S);
    constexpr int64_t NSTEP = S / T / N * N;
    for (int64_t s0 = 0; s0 < NSTEP; s0 += N) {
#pragma unroll
        for (int n = 0; n < N; ++n) {
            const int64_t t0 = (s0 + n) * T;
            p[n][0] = x[0] ^ x[1]; p[n][1] = x[2] ^ x[3]; p[n][2] = x[4] ^ x[5]; p[n][3] = x[6] ^ x[7];
            if ((s0 + n + 1) * T + T <= S)
                for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const VT*>(base + j * S + t0 + T);
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < M; ++r)
#pragma unroll
            for (int n = 0; n < N; ++n) *reinterpret_cast<VT*>(base + (K + r) * S + (s0 + n) * T) = p[n][r];
    }
}

// Lockstep G4/NT192/CW8 (T384) with PF tiles of loads in flight (register ring).
template <int PF>
__global__ void __launch_bounds__(192) k_lockpf(uint8_t* buf) {
    typedef V<8>::t VT;
    constexpr int G = 4, NT = 192, CW = 8, CPB = NT / G, T = CPB * CW;
    constexpr int64_t NST = S / T / PF * PF;  // whole PF-groups of full tiles
    const int g = threadIdx.x / CPB, o = (threadIdx.x % CPB) * CW;
    uint8_t* base = buf + ((int64_t)blockIdx.x * G + g) * STRIDE + o;
    VT x[PF][K];
#pragma unroll
    for (int p = 0; p < PF; ++p)
        for (int j = 0; j < K; ++j) x[p][j] = *reinterpret_cast<const VT*>(base + j * S + p * T);
    for (int64_t s0 = 0; s0 < NST; s0 += PF) {
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int64_t t0 = (s0 + p) * T;
            VT p0 = x[p][0] ^ x[p][1], p1 = x[p][2] ^ x[p][3], p2 = x[p][4] ^ x[p][5], p3 = x[p][6] ^ x[p][7];
            if (s0 + p + PF < NST)
                for (int j = 0; j < K; ++j) x[p][j] = *reinterpret_cast<const VT*>(base + j * S + t0 + PF * T);
            *reinterpret_cast<VT*>(base + (K + 0) * S + t0) = p0;
            *reinterpret_cast<VT*>(base + (K + 1) * S + t0) = p1;
            *reinterpret_cast<VT*>(base + (K + 2) * S + t0) = p2;
            *reinterpret_cast<VT*>(base + (K + 3) * S + t0) = p3;
            __syncthreads();
        }
    }
}

// Lockstep G4/NT192/CW8 (T384) with a runtime stripe stride (layout skew probe).
template <int POL>
__device__ __forceinline__ void st8(uint8_t* p, V<8>::t v) {
    if constexpr (POL == 0) {
        *reinterpret_cast<V<8>::t*>(p) = v;
    } else if constexpr (POL == 1) {
        __builtin_nontemporal_store(v, reinterpret_cast<V<8>::t*>(p));
    } else if constexpr (POL == 2) {
        asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    } else {
        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    }
}

template <int POL = 0>
__global__ void __launch_bounds__(192) k_lockskew(uint8_t* buf, int64_t stride) {
    typedef V<8>::t VT;
    constexpr int G = 4, NT = 192, CW = 8, CPB = NT / G, T = CPB * CW;
    const int g = threadIdx.x / CPB, o = (threadIdx.x % CPB) * CW;
    uint8_t* base = buf + ((int64_t)blockIdx.x * G + g) * stride + o;
    VT x[K];
    for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const VT*>(base + j * S);
    for (int64_t t0 = 0; t0 + T <= S; t0 += T) {
        VT p0 = x[0] ^ x[1], p1 = x[2] ^ x[3], p2 = x[4] ^ x[5], p3 = x[6] ^ x[7];
        if (t0 + 2 * T <= S)
            for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const VT*>(base + j * S + t0 + T);
        st8<POL>(base + (K + 0) * S + t0, p0);
        st8<POL>(base + (K + 1) * S + t0, p1);
        st8<POL>(base + (K + 2) * S + t0, p2);
        st8<POL>(base + (K + 3) * S + t0, p3);
        __syncthreads();
    }
}

// encode_only-style: grid (S / (256*16), NOBJ), one 16-B column per thread.
__global__ void __launch_bounds__(256) k_stream(uint8_t* buf) {
    typedef V<16>::t VT;
    uint8_t* base = buf + (int64_t)blockIdx.y * STRIDE + ((int64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    VT x[K];
    for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const VT*>(base + j * S);
    *reinterpret_cast<VT*>(base + (K + 0) * S) = x[0] ^ x[1];
    *reinterpret_cast<VT*>(base + (K + 1) * S) = x[2] ^ x[3];
    *reinterpret_cast<VT*>(base + (K + 2) * S) = x[4] ^ x[5];
    *reinterpret_cast<VT*>(base + (K + 3) * S) = x[6] ^ x[7];
}

template <typename F>
static void timeit(const char* name, F launch) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch();
    launch();
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        printf("%s: %s\n", name, hipGetErrorString(err));
        exit(2);  // sticky: stop at the first fault
    }
    ms /= reps;
    const double bytes = (double)NOBJ * (K + M) * S;
    printf("%-34s %.4f ms  %.2f TB/s\n", name, ms, bytes / ms / 1e9);
}

template <int G, int NT, int CW, bool BAR, int MAP = 0>
static void lock(const char* name, uint8_t* d, int lds = 0) {
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)k_lockstep<G, NT, CW, BAR, MAP>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    timeit(name, [&] { hipLaunchKernelGGL((k_lockstep<G, NT, CW, BAR, MAP>), dim3(NOBJ / G), dim3(NT), lds, 0, d); });
}

int main() {
    uint8_t* d;
    const int64_t maxskew = 2 << 20;
    if (hipMalloc(&d, NOBJ * (STRIDE + maxskew)) != hipSuccess) return 1;
    (void)hipMemset(d, 1, NOBJ * (STRIDE + maxskew));
    for (int64_t skew : {(int64_t)0, (int64_t)4096, (int64_t)65536, (int64_t)131072, (int64_t)262144,
                         (int64_t)524288, (int64_t)(1 << 20), (int64_t)(3 << 19), (int64_t)(2 << 20), (int64_t)0}) {
        char nm[64];
        snprintf(nm, sizeof nm, "lockskew +%lld", (long long)skew);
        timeit(nm, [&] { hipLaunchKernelGGL(k_lockskew<0>, dim3(NOBJ / 4), dim3(192), 0, 0, d, STRIDE + skew); });
    }
    timeit("lock stores nt", [&] { hipLaunchKernelGGL(k_lockskew<1>, dim3(NOBJ / 4), dim3(192), 0, 0, d, STRIDE); });
    timeit("lock stores sc1", [&] { hipLaunchKernelGGL(k_lockskew<2>, dim3(NOBJ / 4), dim3(192), 0, 0, d, STRIDE); });
    timeit("lock stores sc0 sc1", [&] { hipLaunchKernelGGL(k_lockskew<3>, dim3(NOBJ / 4), dim3(192), 0, 0, d, STRIDE); });
    timeit("stream (encode_only shape)", [&] { hipLaunchKernelGGL(k_stream, dim3(S / 4096, NOBJ), dim3(256), 0, 0, d); });
    lock<4, 192, 8, false>("lock G4 NT192 CW8 (T384)", d);
    timeit("defer N1", [&] { hipLaunchKernelGGL(k_defer<1>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    timeit("defer N2", [&] { hipLaunchKernelGGL(k_defer<2>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    timeit("defer N4", [&] { hipLaunchKernelGGL(k_defer<4>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    timeit("defer N8", [&] { hipLaunchKernelGGL(k_defer<8>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    timeit("defer N16", [&] { hipLaunchKernelGGL(k_defer<16>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    lock<4, 192, 8, true>("lock G4 NT192 CW8 (T384) bar", d);
    timeit("lockpf PF1 bar", [&] { hipLaunchKernelGGL(k_lockpf<1>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    timeit("lockpf PF2 bar", [&] { hipLaunchKernelGGL(k_lockpf<2>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    timeit("lockpf PF3 bar", [&] { hipLaunchKernelGGL(k_lockpf<3>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    timeit("lockpf PF4 bar", [&] { hipLaunchKernelGGL(k_lockpf<4>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    timeit("lockpf PF6 bar", [&] { hipLaunchKernelGGL(k_lockpf<6>, dim3(NOBJ / 4), dim3(192), 0, 0, d); });
    lock<1, 256, 16, false>("window G1 T4096 2/CU (512 live)", d, 80 * 1024);
    lock<1, 256, 16, false>("window G1 T4096 1/CU (256 live)", d, 150 * 1024);
    lock<1, 256, 16, false>("window G1 T4096 4/CU (1024 live)", d, 40 * 1024);
    lock<1, 256, 16, false>("window G1 T4096 8/CU (2048 live)", d, 20 * 1024);
    lock<4, 192, 8, true>("lock G4 T384 2/CU (2048 live)", d, 80 * 1024);
    lock<4, 192, 8, true>("lock G4 T384 1/CU (1024 live)", d, 150 * 1024);
    lock<4, 192, 8, true, 1>("lock ... bar map spread", d);
    lock<4, 192, 8, true, 2>("lock ... bar map xcd-contig", d);
    lock<1, 64, 16, true, 2>("lock G1 NT64 bar xcd-contig", d);
    lock<4, 192, 16, false>("lock G4 NT192 CW16 (T768)", d);
    lock<2, 256, 16, false>("lock G2 NT256 CW16 (T2048)", d);
    lock<1, 256, 16, false>("lock G1 NT256 CW16 (T4096)", d);
    lock<1, 256, 16, true>("lock G1 NT256 CW16 (T4096) bar", d);
    lock<8, 256, 8, false>("lock G8 NT256 CW8 (T256)", d);
    lock<16, 256, 8, false>("lock G16 NT256 CW8 (T128)", d);
    lock<4, 256, 16, false>("lock G4 NT256 CW16 (T1024)", d);
    lock<1, 64, 16, false>("lock G1 NT64 CW16 (T1024)", d);
    hipFree(d);
    return 0;
}
