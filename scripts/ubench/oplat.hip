// Dependent-chain latency of the HighwayHash / GF opcodes with ONE wave per SIMD (the
// RS(4+2) config-2 regime: 384 chain waves for 1024 SIMDs), cycles per dependent op.
//   hipcc --offload-arch=gfx950 -O3 -o oplat oplat.hip && ./oplat
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint32_t a = seed * threadIdx.x, b = a ^ 0x9e3779b9u;
    uint64_t q = ((uint64_t)a << 32) | b, c = q * 3;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) a = __builtin_amdgcn_perm(a, b, a);
            if constexpr (OP == 1) a = __builtin_amdgcn_bitop3_b32(a, b, a, 0x96);
            if constexpr (OP == 2) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q) : "v"(c));
            if constexpr (OP == 3) { uint64_t r, cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"((uint32_t)q), "v"(b), "v"(c)); q = r; }
            if constexpr (OP == 4) a = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0xB1, 0xF, 0xF, false);
            if constexpr (OP == 5) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = a + (uint32_t)q;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

template <int OP>
void run(const char* name, uint32_t* d, uint64_t* clk, int cus) {
    hipLaunchKernelGGL((k<OP>), dim3(cus), dim3(256), 0, 0, d, clk, 7u);
    (void)hipDeviceSynchronize();
    uint64_t c;
    (void)hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
    printf("%-16s 1 wave/SIMD dependent chain: %.2f cycles per op\n", name, (double)c / (ITERS * 8.0));
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    uint32_t* d;
    uint64_t* clk;
    (void)hipMalloc(&d, p.multiProcessorCount * 256 * 4);
    (void)hipMalloc(&clk, 8);
    int cus = p.multiProcessorCount;
    run<0>("v_perm_b32", d, clk, cus);
    run<1>("v_bitop3_b32", d, clk, cus);
    run<2>("v_lshl_add_u64", d, clk, cus);
    run<3>("v_mad_u64_u32", d, clk, cus);
    run<4>("v_mov_b32_dpp", d, clk, cus);
    run<5>("v_xor_b32", d, clk, cus);
    return 0;
}
