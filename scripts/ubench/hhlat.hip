// Dependent-chain time of one HighwayHash-256 packet update (hh256_dev.hpp) in the three
// thread mappings, at 1-4 waves per SIMD (the latency roof of the
// chain-bound paths, BASELINE config 2 = 6 144 chains of 8 192 packets).
//   quad : one HH lane per thread, 4 threads per chain (hh_update, DPP zipper partner)
//   pair : two HH lanes per thread, 2 threads per chain (hh2_update, no cross-lane move)
//   solo : four HH lanes per thread, 1 thread per chain (two hh2 pair updates, ILP 2)
// Packets come from registers (a per-packet counter mixed with the thread id), so the
// time is the update chain alone.  One workgroup of 4*W waves per CU (W waves per SIMD);
// ns per packet from s_memrealtime (100 MHz), cycles from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -I../../zs3server_amd/csrc -o hhlat hhlat.hip && ./hhlat
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "hh256_dev.hpp"

using namespace zs3dev;

#define NPK 4096

template <int FORM>
__global__ void k(uint64_t* out, uint64_t* clk) {
    const int tid = threadIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t res = 0;
    const uint64_t seed = 0x9e3779b97f4a7c15ULL * (blockIdx.x * 1024 + tid + 1);
    if constexpr (FORM == 0) {
        const int lane = tid & 3;
        HHLane s = hh_init(lane, 1, 2, 3, 4);
        const uint32_t sel = zipper_sel(lane);
        for (int i = 0; i < NPK; ++i) hh_update(s, seed + (uint64_t)i, sel);
        res = s.v0 ^ s.v1 ^ s.mul0 ^ s.mul1;
    } else if constexpr (FORM == 1) {
        HHPair s = hh2_init(tid & 1, 1, 2, 3, 4);
        for (int i = 0; i < NPK; ++i) hh2_update(s, seed + (uint64_t)i, seed ^ (uint64_t)i);
        res = s.v0[0] ^ s.v1[1] ^ s.mul0[0] ^ s.mul1[1];
    } else {
        HHPair a = hh2_init(0, 1, 2, 3, 4), b = hh2_init(1, 1, 2, 3, 4);
        for (int i = 0; i < NPK; ++i) {
            hh2_update(a, seed + (uint64_t)i, seed ^ (uint64_t)i);
            hh2_update(b, seed - (uint64_t)i, ~seed + (uint64_t)i);
        }
        res = a.v0[0] ^ b.v1[1] ^ a.mul0[1] ^ b.mul1[0];
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + tid] = res;
    if (tid == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int FORM>
void run(const char* name, int cus, int wps, uint64_t* d, uint64_t* clk) {
    const int threads = 256 * wps;
    hipLaunchKernelGGL(k<FORM>, dim3(cus), dim3(threads), 0, 0, d, clk);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k<FORM>, dim3(cus), dim3(threads), 0, 0, d, clk);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t h[2 * 1024];
    (void)hipMemcpy(h, clk, 2 * cus * sizeof(uint64_t), hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int i = 0; i < cus; ++i) {
        cyc += (double)h[2 * i];
        rt += (double)h[2 * i + 1];
    }
    cyc /= cus;
    rt /= cus;
    const double ns = rt * 10.0 / NPK;  // s_memrealtime: 100 MHz
    const int tpc = FORM == 0 ? 4 : FORM == 1 ? 2 : 1;
    const double chains_per_simd = 64.0 / tpc * wps;
    printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"chains_per_simd\": %.0f, \"ns_per_packet\": %.2f, "
           "\"cycles_per_packet\": %.1f, \"clock_GHz\": %.3f, \"ns_per_packet_per_chain_on_simd\": %.3f, "
           "\"kernel_ms\": %.3f}\n",
           name, wps, chains_per_simd, ns, cyc / NPK, cyc / rt / 10.0, ns / chains_per_simd, ms);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint64_t *d, *clk;
    (void)hipMalloc(&d, (size_t)cus * 1024 * 8);
    (void)hipMalloc(&clk, 2 * 1024 * 8);
    for (int w = 1; w <= 4; ++w) {
        run<0>("quad", cus, w, d, clk);
        run<1>("pair", cus, w, d, clk);
        run<2>("solo", cus, w, d, clk);
    }
    return 0;
}
