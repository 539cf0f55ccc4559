// kend.hip -- TOOL (not shipped): per-launch overhead outside the waves' span for back-to-back persistent launches
// on MI355X, by how the kernel's last stores leave L2 (plain / nt / sc1 write-through), plus an empty kernel.
//   hipcc --offload-arch=gfx950 -O3 -o tools/kend tools/kend.hip && ./tools/kend
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ unsigned long long g_t0, g_t1;

template <int MODE>
__global__ void __launch_bounds__(1024) wr(float4* __restrict__ p, size_t n, int stamp) {
    extern __shared__ float4 lds[];
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (stamp && threadIdx.x == 0) atomicMin(&g_t0, t);
    if (threadIdx.x == 0) lds[0] = make_float4(0, 0, 0, 0);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = make_float4((float)i, 1.f, 2.f, 3.f);
        if constexpr (MODE == 0) {
            p[i] = v;
        } else if constexpr (MODE == 1) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w}, reinterpret_cast<f4*>(p + i));
        } else {
            typedef float f4 __attribute__((ext_vector_type(4)));
            const f4 w = {v.x, v.y, v.z, v.w};
            asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p + i), "v"(w) : "memory");
        }
    }
    if (stamp) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(&g_t1, __builtin_amdgcn_s_memrealtime());
    }
}

__global__ void __launch_bounds__(1024) empty_k(int) {}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <class F>
static float time_launches(F f, int K) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int i = 0; i < 20; i++) f();
    (void)hipEventRecord(a);
    for (int i = 0; i < K; i++) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / K;
}

int main() {
    const int grid = 256, block = 1024, lds = 160 * 1024;
    CK(hipFuncSetAttribute((const void*)wr<0>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CK(hipFuncSetAttribute((const void*)wr<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CK(hipFuncSetAttribute((const void*)wr<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    float4* p;
    for (size_t mb : {4, 16, 64, 100}) {
        const size_t n = mb * 1024 * 1024 / 16;
        CK(hipMalloc(&p, n * 16));
        for (int mode = 0; mode < 3; mode++) {
            auto f = [&]() {
                if (mode == 0) hipLaunchKernelGGL(wr<0>, dim3(grid), dim3(block), lds, 0, p, n, 0);
                else if (mode == 1) hipLaunchKernelGGL(wr<1>, dim3(grid), dim3(block), lds, 0, p, n, 0);
                else hipLaunchKernelGGL(wr<2>, dim3(grid), dim3(block), lds, 0, p, n, 0);
            };
            const float us = time_launches(f, 200);
            // span of one launch (first wave entry -> last block exit), s_memrealtime at 100 MHz
            double span = 0;
            for (int r = 0; r < 5; r++) {
                unsigned long long hi = ~0ull, lo = 0;
                CK(hipMemcpyToSymbol(HIP_SYMBOL(g_t0), &hi, 8));
                CK(hipMemcpyToSymbol(HIP_SYMBOL(g_t1), &lo, 8));
                if (mode == 0) hipLaunchKernelGGL(wr<0>, dim3(grid), dim3(block), lds, 0, p, n, 1);
                else if (mode == 1) hipLaunchKernelGGL(wr<1>, dim3(grid), dim3(block), lds, 0, p, n, 1);
                else hipLaunchKernelGGL(wr<2>, dim3(grid), dim3(block), lds, 0, p, n, 1);
                CK(hipDeviceSynchronize());
                unsigned long long t0, t1;
                CK(hipMemcpyFromSymbol(&t0, HIP_SYMBOL(g_t0), 8));
                CK(hipMemcpyFromSymbol(&t1, HIP_SYMBOL(g_t1), 8));
                span += (double)(t1 - t0) * 0.01 / 5;
            }
            printf("{\"MB\": %zu, \"mode\": \"%s\", \"us_per_launch\": %.2f, \"span_us\": %.2f, \"outside_us\": %.2f}\n", mb,
                   mode == 0 ? "plain" : mode == 1 ? "nt" : "sc1", us, span, us - span);
        }
        CK(hipFree(p));
    }
    auto fe = [&]() { hipLaunchKernelGGL(empty_k, dim3(grid), dim3(block), 0, 0, 0); };
    printf("{\"empty_kernel_us_per_launch\": %.2f}\n", time_launches(fe, 500));
    return 0;
}
