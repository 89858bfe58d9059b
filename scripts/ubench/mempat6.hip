// Unaligned-row encode probe, round 4.  RS(12+4) on 1 MiB blocks has S = 87 382: every
// shard row starts 2-byte aligned, and the encode-only call on these rows runs at 42-45 %
// of HBM (any-geometry kernel, 8-byte columns) while the aligned streaming kernel runs at
// 70-75 %.  What do misaligned 16-byte loads and stores cost, separately, and does an
// aligned-access scheme (aligned loads + a neighbour lane's chunk over DPP + byte funnel
// shifts; the same for the stores) recover the aligned rate?
// Shape: the encode-only streaming kernel (grid = column chunks x stripes, one 16-byte
// column per lane), 12 data rows -> 4 parity rows (XOR: parity r = data r ^ r+4 ^ r+8),
// 4096 stripes of 16 x S bytes, rows contiguous.
//   load / store address modes: 0 = exact (misaligned), 1 = rounded down to 16 bytes,
//   2 = rounded down to 4 bytes (timing only: the data is not realigned)
//   realign16: loads/stores at 16-byte aligned addresses, the window of row offsets
//   [o, o+16) assembled from this lane's chunk and the next lane's (wave_shl:1 DPP), the
//   stored chunk from this lane's parity window and the previous lane's (wave_shr:1); 62
//   stored chunks per wave (lanes 0 and 63 are halo); exact, checked on the host.
//   realign4: the same at 4-byte granularity (dword-aligned vector accesses + alignbyte).
// Prints one JSON line per pattern: ms, algorithmic TB/s (data + parity bytes), check.
//   hipcc --offload-arch=gfx950 -O3 -o mempat6 mempat6.hip && ./mempat6
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

constexpr int K = 12, M = 4, R = 16;
constexpr int64_t NOBJ = 4096;

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u4 ldg(const uint8_t* p) { return __builtin_nontemporal_load(reinterpret_cast<const u4*>(p)); }
__device__ __forceinline__ void stg(uint8_t* p, u4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u4*>(p)); }

template <int MODE>
__device__ __forceinline__ const uint8_t* amode(const uint8_t* p) {
    if constexpr (MODE == 1) return reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)15);
    if constexpr (MODE == 2) return reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    return p;
}

// timing kernel: exact / rounded addresses, no realignment
template <int LM, int SM>
__global__ void __launch_bounds__(256) k_plain(uint8_t* buf, int64_t S) {
    const int64_t o = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (o + 16 > S) return;
    uint8_t* blk = buf + (int64_t)blockIdx.y * R * S;
    u4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ldg(amode<LM>(blk + j * S + o));
#pragma unroll
    for (int r = 0; r < M; ++r)
        stg(const_cast<uint8_t*>(amode<SM>(blk + (K + r) * S + o)), x[r] ^ x[r + 4] ^ x[r + 8]);
}

__device__ __forceinline__ uint32_t shl1(uint32_t v) {  // lane L <- lane L+1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t shr1(uint32_t v) {  // lane L <- lane L-1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ u4 shl1v(u4 v) { return u4{shl1(v.x), shl1(v.y), shl1(v.z), shl1(v.w)}; }
__device__ __forceinline__ u4 shr1v(u4 v) { return u4{shr1(v.x), shr1(v.y), shr1(v.z), shr1(v.w)}; }

// bytes [d, d + 16) of the 32 bytes lo ++ hi, d in [0, 16) wave-uniform
__device__ __forceinline__ u4 funnel16(u4 lo, u4 hi, uint32_t d) {
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const uint32_t q = d >> 2, r = d & 3;
    uint32_t s[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t a = q & 1 ? w[i + 1] : w[i];
        const uint32_t b = q & 1 ? w[i + 3 < 8 ? i + 3 : 7] : w[i + 2 < 8 ? i + 2 : 7];
        s[i] = q & 2 ? b : a;
    }
    return u4{__builtin_amdgcn_alignbyte(s[1], s[0], r), __builtin_amdgcn_alignbyte(s[2], s[1], r),
              __builtin_amdgcn_alignbyte(s[3], s[2], r), __builtin_amdgcn_alignbyte(s[4], s[3], r)};
}
// bytes [r, r + 16) of the 20 bytes v ++ e (one dword), r in [0, 4)
__device__ __forceinline__ u4 funnel4(u4 v, uint32_t e, uint32_t r) {
    return u4{__builtin_amdgcn_alignbyte(v.y, v.x, r), __builtin_amdgcn_alignbyte(v.z, v.y, r),
              __builtin_amdgcn_alignbyte(v.w, v.z, r), __builtin_amdgcn_alignbyte(e, v.w, r)};
}

// realign at granularity GR (16 or 4 bytes): wave w covers row offsets starting at
// base = w * 62 * 16 - 16, lane L at o = base + 16 L; lanes 1..62 store.
template <int GR>
__global__ void __launch_bounds__(256) k_realign(uint8_t* buf, int64_t S) {
    const int lane = threadIdx.x & 63;
    const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t o = wv * 62 * 16 - 16 + 16 * lane;
    if (wv * 62 * 16 >= S) return;
    uint8_t* blk = buf + (int64_t)blockIdx.y * R * S;
    const uintptr_t b0 = reinterpret_cast<uintptr_t>(blk);
    u4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        // lane 0 of the first wave would read before the row: its window only feeds bytes
        // before the row, which are never stored
        const int64_t oo = o < 0 ? 0 : o;
        const uintptr_t a = b0 + j * S + oo;
        const uint32_t d = (uint32_t)(a & (GR - 1));  // wave-uniform (o % 16 == 0)
        const u4 c = ldg(reinterpret_cast<const uint8_t*>(a - d));
        if constexpr (GR == 16)
            x[j] = funnel16(c, shl1v(c), d);
        else
            x[j] = funnel4(c, shl1(c.x), d);
    }
    const int64_t rem = S - o;  // bytes of the row from o on
#pragma unroll
    for (int r = 0; r < M; ++r) {
        const u4 p = x[r] ^ x[r + 4] ^ x[r + 8];
        const uintptr_t a = b0 + (K + r) * S + o;
        const uint32_t d = (uint32_t)(a & (GR - 1));
        u4 v;
        if constexpr (GR == 16)
            v = d ? funnel16(shr1v(p), p, 16 - d) : p;  // row offsets [o - d, o - d + 16)
        else
            v = d ? funnel4(u4{shr1(p.w), p.x, p.y, p.z}, p.w, 4 - d) : p;
        const bool inner = lane >= 1 && lane <= 62 && o - (int64_t)d >= 0 && rem - 16 + (int64_t)d >= 0;
        if (inner) {
            stg(reinterpret_cast<uint8_t*>(a - d), v);
        } else if (lane >= 1 && lane <= 62) {
            // edge chunk: only the bytes inside the row
            uint8_t* q = reinterpret_cast<uint8_t*>(a - d);
            const uint32_t wv4[4] = {v.x, v.y, v.z, v.w};
            for (int i = 0; i < 16; ++i) {
                const int64_t ro = o - (int64_t)d + i;
                if (ro >= 0 && ro < S) q[i] = (uint8_t)(wv4[i >> 2] >> (8 * (i & 3)));
            }
        }
    }
}

template <typename F>
static double timeit(F launch) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    launch();
    launch();
    (void)hipEventRecord(e0);
    const int reps = 8;
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        printf("{\"error\": \"%s\"}\n", hipGetErrorString(err));
        exit(2);
    }
    return ms / reps;
}

static void report(const char* name, int64_t S, double ms, long long bad) {
    const double bytes = (double)NOBJ * R * S;
    printf("{\"pattern\": \"%s\", \"S\": %lld, \"ms\": %.4f, \"TBps\": %.3f, \"frac\": %.4f, \"bad\": %lld}\n", name,
           (long long)S, ms, bytes / ms / 1e9, bytes / ms / 1e9 / 8.0, bad);
    fflush(stdout);
}

// host check of the parity rows of a few stripes
static long long check(const uint8_t* d, int64_t S) {
    const int64_t n = 3 * R * S;
    uint8_t* h = (uint8_t*)malloc(n);
    const int64_t objs[3] = {0, NOBJ / 2 + 1, NOBJ - 1};
    long long bad = 0;
    for (int t = 0; t < 3; ++t) {
        (void)hipMemcpy(h, d + objs[t] * R * S, R * S, hipMemcpyDeviceToHost);
        for (int r = 0; r < M; ++r)
            for (int64_t i = 0; i < S; ++i)
                bad += h[(K + r) * S + i] != (uint8_t)(h[r * S + i] ^ h[(r + 4) * S + i] ^ h[(r + 8) * S + i]);
    }
    free(h);
    return bad;
}

static void fill(uint8_t* d, size_t n) {
    uint8_t* h = (uint8_t*)malloc(n);
    for (size_t i = 0; i < n; ++i) h[i] = (uint8_t)((i * 2654435761u) >> 11);
    (void)hipMemcpy(d, h, n, hipMemcpyHostToDevice);
    free(h);
}

template <int LM, int SM>
static void plain(uint8_t* d, int64_t S) {
    const unsigned gx = (unsigned)((S / 16 + 255) / 256);
    const double ms = timeit([&] { hipLaunchKernelGGL((k_plain<LM, SM>), dim3(gx, NOBJ), dim3(256), 0, 0, d, S); });
    char nm[64];
    snprintf(nm, sizeof nm, "plain load%d store%d", LM, SM);
    report(nm, S, ms, (LM == 0 && SM == 0 && S % 16 == 0) ? check(d, S) : -1);
}

template <int GR>
static void realign(uint8_t* d, int64_t S) {
    const int64_t waves = (S + 62 * 16 - 1) / (62 * 16);
    const unsigned gx = (unsigned)((waves + 3) / 4);
    (void)hipMemset(d, 0, 16);
    const double ms = timeit([&] { hipLaunchKernelGGL((k_realign<GR>), dim3(gx, NOBJ), dim3(256), 0, 0, d, S); });
    char nm[64];
    snprintf(nm, sizeof nm, "realign%d", GR);
    report(nm, S, ms, check(d, S));
}

int main() {
    const int64_t Smax = 87392;
    const size_t bytes = (size_t)NOBJ * R * Smax + 4096;
    uint8_t* base;
    if (hipMalloc(&base, bytes) != hipSuccess) return 1;
    fill(base, bytes);
    uint8_t* d = base + 256;  // a 16-byte aligned buffer start
    for (int64_t S : {(int64_t)87392, (int64_t)87382, (int64_t)87381}) {
        plain<0, 0>(d, S);
        plain<1, 1>(d, S);
        plain<0, 1>(d, S);
        plain<1, 0>(d, S);
        plain<2, 2>(d, S);
        plain<2, 1>(d, S);
        fill(base, bytes);
        realign<16>(d, S);
        fill(base, bytes);
        realign<4>(d, S);
    }
    (void)hipFree(base);
    return 0;
}
