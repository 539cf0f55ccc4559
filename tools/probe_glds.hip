// TOOL: probe of global_load_lds_dwordx4 placement on gfx950 (where lane l's 16 bytes land in LDS).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ void glds16(const float* src, float* lds_wave_base) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)lds_wave_base, 16, 0, 0);
#endif
}
__global__ void k(const float* src, float* out) {
    __shared__ float S[1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) S[i] = -1.0f;
    __syncthreads();
    // wave w loads 256 floats: lane l reads src[w*256 + 4*perm(l)] where perm reverses lanes
    glds16(src + w * 256 + 4 * (63 - lane), S + w * 256);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) out[i] = S[i];
}
int main() {
    float h[1024], o[1024];
    for (int i = 0; i < 1024; i++) h[i] = (float)i;
    float *d, *e;
    hipMalloc(&d, 4096); hipMalloc(&e, 4096);
    hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, e);
    hipMemcpy(o, e, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int w = 0; w < 4; w++)
        for (int l = 0; l < 64; l++)
            for (int c = 0; c < 4; c++) {
                const float want = (float)(w * 256 + 4 * (63 - l) + c);
                if (o[w * 256 + 4 * l + c] != want) bad++;
            }
    printf("lane-linear placement mismatches: %d; first values:", bad);
    for (int i = 0; i < 12; i++) printf(" %g", o[i]);
    printf("\n");
    return 0;
}
