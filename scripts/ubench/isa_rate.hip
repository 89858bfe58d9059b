// Throughput of the VALU ops the hot path is built from, on gfx950.
// 8 independent chains per thread, 8 waves per SIMD, cycles per wave-instruction
// per SIMD = elapsed_cycles * n_simds / (waves * iters * 8).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
    uint32_t a[8], b[8];
    uint64_t q[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = seed * (threadIdx.x + i);
        b[i] = a[i] ^ 0x9e3779b9u;
        q[i] = ((uint64_t)a[i] << 32) | b[i];
    }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) a[i] = a[i] ^ b[i];
            if constexpr (OP == 1) a[i] = __builtin_amdgcn_perm(a[i], b[i], a[i]);
            if constexpr (OP == 2) a[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], a[(i + 1) & 7], 0x96);
            if constexpr (OP == 3) { uint64_t r; asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(q[i]), "v"(q[(i+1)&7])); q[i] = r; }
            if constexpr (OP == 4) { q[i] = (uint64_t)(uint32_t)q[i] * (q[(i + 1) & 7] >> 32); }
            if constexpr (OP == 5) a[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a[(i + 3) & 7], 0xB1, 0xF, 0xF, false);
            if constexpr (OP == 6) { a[i] = a[i] + b[i]; }
            if constexpr (OP == 7) { q[i] = q[i] ^ q[(i + 1) & 7]; }
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + (uint32_t)q[i] + (uint32_t)(q[i] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
void run(const char* name, uint32_t* d, int cus) {
    int blocks = cus * 8;  // 8 x 256 threads per CU = 32 waves/CU = 8 per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 7u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double waves = blocks * 4.0 * 5;
    double instrs = waves * ITERS * 8;
    double simds = cus * 4.0;
    double ns_per = ms * 1e6 / (instrs / simds);
    printf("%-22s %.3f ns per wave-instr per SIMD (= %.2f cycles @2.0GHz)\n", name, ns_per, ns_per * 2.0);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    uint32_t* d;
    hipMalloc(&d, cus * 8 * 256 * 4);
    run<0>("v_xor_b32", d, cus);
    run<6>("v_add_u32", d, cus);
    run<1>("v_perm_b32", d, cus);
    run<2>("v_bitop3_b32", d, cus);
    run<3>("v_lshl_add_u64", d, cus);
    run<4>("v_mad_u64_u32", d, cus);
    run<5>("v_mov_b32_dpp", d, cus);
    run<7>("xor64 (2x v_xor)", d, cus);
    return 0;
}
