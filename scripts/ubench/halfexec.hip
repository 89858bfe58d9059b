// Does a wave64 VALU instruction with only lanes 0-31 active (EXEC hi = 0) issue faster
// than a full one on gfx950's 32-wide SIMDs?  8 waves per SIMD, 8 independent chains.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
template <int OP, int ACTIVE>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
    uint32_t a[8], b[8];
    uint64_t q[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = seed * (threadIdx.x + i);
        b[i] = a[i] ^ 0x9e3779b9u;
        q[i] = ((uint64_t)a[i] << 32) | b[i];
    }
    if ((threadIdx.x & 63) < ACTIVE) {
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (OP == 0) a[i] = __builtin_amdgcn_perm(a[i], b[i], a[(i + 1) & 7]);
                if constexpr (OP == 1) a[i] = __builtin_amdgcn_bitop3_b32(a[i], b[i], a[(i + 1) & 7], 0x96);
                if constexpr (OP == 2) { uint64_t r; asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(q[i]), "v"(q[(i+1)&7])); q[i] = r; }
            }
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + (uint32_t)q[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP, int ACTIVE>
void run(const char* name, uint32_t* d, int cus) {
    int blocks = cus * 8;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k<OP, ACTIVE>), dim3(blocks), dim3(256), 0, 0, d, 7u);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<OP, ACTIVE>), dim3(blocks), dim3(256), 0, 0, d, 7u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double instrs = blocks * 4.0 * 5 * ITERS * 8;
    printf("%-28s active %2d: %.3f ns per wave-instr per SIMD\n", name, ACTIVE, ms * 1e6 / (instrs / (cus * 4.0)));
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    uint32_t* d;
    (void)hipMalloc(&d, p.multiProcessorCount * 8 * 256 * 4);
    int cus = p.multiProcessorCount;
    run<0, 64>("v_perm_b32", d, cus);
    run<0, 32>("v_perm_b32", d, cus);
    run<0, 16>("v_perm_b32", d, cus);
    run<1, 64>("v_bitop3_b32", d, cus);
    run<1, 32>("v_bitop3_b32", d, cus);
    run<2, 64>("v_lshl_add_u64", d, cus);
    run<2, 32>("v_lshl_add_u64", d, cus);
    return 0;
}
