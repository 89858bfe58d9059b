// Issue cost of the VALU opcodes the fused RS-encode + HighwayHash kernel uses, at the
// kernel's occupancy (3 waves per SIMD) and at 8 waves per SIMD, plus the shader clock
// during the run (s_memtime ticks / s_memrealtime 100 MHz ticks).
//   hipcc --offload-arch=gfx950 -O3 -o opcost opcost.hip && ./opcost
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint32_t a[8], b[8];
    uint64_t q[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = seed * (threadIdx.x + i);
        b[i] = a[i] ^ 0x9e3779b9u;
        q[i] = ((uint64_t)a[i] << 32) | b[i];
    }
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) a[i] = __builtin_amdgcn_perm(a[i], b[i], a[(i + 1) & 7]);
            if constexpr (OP == 1) a[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], a[(i + 1) & 7], 0x96);
            if constexpr (OP == 2) { uint64_t r; asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(q[i]), "v"(q[(i+1)&7])); q[i] = r; }
            if constexpr (OP == 3) { uint64_t r, cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a[i]), "v"(b[i]), "v"(q[(i+1)&7])); q[i] = r; }
            if constexpr (OP == 4) { uint32_t r; asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(a[(i+1)&7])); a[i] = r; }
            if constexpr (OP == 5) { uint32_t r; asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(a[(i+1)&7])); a[i] = r; }
            if constexpr (OP == 6) { uint32_t r; asm volatile("v_and_b32 %0, 0x7070707, %1" : "=v"(r) : "v"(a[(i+1)&7])); a[i] ^= r; }
            if constexpr (OP == 7) { uint32_t r; asm volatile("v_lshrrev_b32 %0, 3, %1" : "=v"(r) : "v"(a[(i+1)&7])); a[i] = r; }
            if constexpr (OP == 8) { uint64_t r; asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "v"(q[(i+1)&7])); q[i] = r; }
            if constexpr (OP == 9) { uint32_t r; asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(a[(i+1)&7])); a[i] = r; }
            if constexpr (OP == 10) { uint32_t r; asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(a[(i+1)&7])); a[i] = r; }
            if constexpr (OP == 11) { uint32_t r; asm volatile("v_alignbit_b32 %0, %1, %2, 8" : "=v"(r) : "v"(a[i]), "v"(a[(i+1)&7])); a[i] = r; }
            if constexpr (OP == 12) { uint64_t r; asm volatile("v_lshrrev_b64 %0, 3, %1" : "=v"(r) : "v"(q[(i+1)&7])); q[i] = r ^ q[i]; }
            if constexpr (OP == 13) { uint64_t r; asm volatile("v_lshrrev_b64 %0, 3, %1" : "=v"(r) : "v"(q[(i+1)&7])); q[i] = r; }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + (uint32_t)q[i] + (uint32_t)(q[i] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int OP>
void run(const char* name, uint32_t* d, uint64_t* clk, int cus, int wps) {
    int blocks = cus * wps;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k<OP>), dim3(blocks), dim3(256), 0, 0, d, clk, 7u);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<OP>), dim3(blocks), dim3(256), 0, 0, d, clk, 7u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint64_t c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = c[1] ? (double)c[0] / c[1] * 0.1 : 0;
    const double per_simd = (double)wps * 5 * ITERS * 8;  // wave-instrs per SIMD
    const double ns = ms * 1e6 / per_simd;
    printf("%-16s waves/SIMD %d: %.3f ns/wave-instr  clk %.2f GHz  => %.2f cycles\n", name, wps, ns, ghz, ns * ghz);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    uint32_t* d;
    uint64_t* clk;
    int cus = p.multiProcessorCount;
    (void)hipMalloc(&d, cus * 8 * 256 * 4);
    (void)hipMalloc(&clk, 16);
    for (int w : {3, 8}) {
        run<0>("v_perm_b32", d, clk, cus, w);
        run<1>("v_bitop3_b32", d, clk, cus, w);
        run<2>("v_lshl_add_u64", d, clk, cus, w);
        run<3>("v_mad_u64_u32", d, clk, cus, w);
        run<4>("v_mov_b32_dpp", d, clk, cus, w);
        run<5>("v_xor_b32", d, clk, cus, w);
        run<6>("and+xor", d, clk, cus, w);
        run<7>("v_lshrrev_b32", d, clk, cus, w);
        run<8>("v_mov_b64", d, clk, cus, w);
        run<9>("v_add_u32", d, clk, cus, w);
        run<10>("v_mul_lo_u32", d, clk, cus, w);
        run<11>("v_alignbit_b32", d, clk, cus, w);
        run<12>("lshr_b64+xor64", d, clk, cus, w);
        run<13>("v_lshrrev_b64", d, clk, cus, w);
    }
    return 0;
}
