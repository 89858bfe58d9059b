// Are byte-misaligned global dwordx2 / dwordx4 loads and stores exact on this GPU, and
// what do they cost?  (RS(12+4) with 1 MiB blocks has S = 87 382: data and parity rows
// start at 2-byte-aligned offsets.)  Copies a 256 MiB buffer with 16-byte vector loads
// and stores offset by `mis` bytes, checks every byte on the host, reports GB/s.
//   hipcc --offload-arch=gfx950 -O3 -o unaligned unaligned.hip && ./unaligned
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

template <int W>
__global__ void __launch_bounds__(256) k_copy(const uint8_t* src, uint8_t* dst, size_t n_vec) {
    typedef uint32_t V __attribute__((ext_vector_type(W)));
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n_vec; i += (size_t)gridDim.x * 256) {
        V v;
        if constexpr (W == 4)
            asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(src + i * 16) : "memory");
        else
            asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(src + i * 8) : "memory");
        if constexpr (W == 4)
            asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(dst + i * 16), "v"(v) : "memory");
        else
            asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(dst + i * 8), "v"(v) : "memory");
    }
}

int main() {
    const size_t N = 256u << 20;
    uint8_t *h = (uint8_t*)malloc(N + 64), *g = (uint8_t*)malloc(N + 64);
    for (size_t i = 0; i < N + 64; ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
    uint8_t *ds, *dd;
    (void)hipMalloc(&ds, N + 64);
    (void)hipMalloc(&dd, N + 64);
    (void)hipMemcpy(ds, h, N + 64, hipMemcpyHostToDevice);
    const int mis_list[] = {0, 2, 6, 8, 14, 1};
    for (int w = 2; w <= 4; w += 2) {
        for (int mis : mis_list) {
            (void)hipMemset(dd, 0, N + 64);
            const size_t nv = N / (4 * w);
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            if (w == 4) hipLaunchKernelGGL(k_copy<4>, dim3(4096), dim3(256), 0, 0, ds + mis, dd + mis, nv);
            else hipLaunchKernelGGL(k_copy<2>, dim3(4096), dim3(256), 0, 0, ds + mis, dd + mis, nv);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(a, 0);
            for (int r = 0; r < 5; ++r) {
                if (w == 4) hipLaunchKernelGGL(k_copy<4>, dim3(4096), dim3(256), 0, 0, ds + mis, dd + mis, nv);
                else hipLaunchKernelGGL(k_copy<2>, dim3(4096), dim3(256), 0, 0, ds + mis, dd + mis, nv);
            }
            (void)hipEventRecord(b, 0);
            hipError_t e = hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            (void)hipMemcpy(g, dd, N + 64, hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (size_t i = 0; i < N; ++i) bad += g[mis + i] != h[mis + i];
            for (int i = 0; i < mis; ++i) bad += g[i] != 0;
            printf("{\"width_bytes\": %d, \"misalign\": %d, \"err\": \"%s\", \"bad_bytes\": %zu, \"GBps\": %.1f}\n", 4 * w,
                   mis, hipGetErrorString(e), bad, 2.0 * N * 5 / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
