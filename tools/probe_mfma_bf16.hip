// TOOL: probe of v_mfma_f32_32x32x16_bf16 operand / result lane maps on gfx950 with exact integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// A[32][16], B[16][32] (row-major), C = A B: lane l holds A[l&31][8(l>>5)+j], B[8(l>>5)+j][l&31]
__global__ void k(const float* A, const float* B, float* C) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    bf16x8 a, b;
    for (int j = 0; j < 8; j++) {
        a[j] = (__bf16)A[r * 16 + 8 * h + j];
        b[j] = (__bf16)B[(8 * h + j) * 32 + r];
    }
    floatx16 c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    for (int q = 0; q < 16; q++) C[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = c[q];
}
int main() {
    float A[512], B[512], C[1024], R[1024];
    for (int i = 0; i < 512; i++) { A[i] = (float)((i * 7) % 13 - 6); B[i] = (float)((i * 5) % 11 - 5); }
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) {
            float s = 0;
            for (int kk = 0; kk < 16; kk++) s += A[i * 16 + kk] * B[kk * 32 + j];
            R[i * 32 + j] = s;
        }
    float *dA, *dB, *dC;
    (void)hipMalloc(&dA, 2048); (void)hipMalloc(&dB, 2048); (void)hipMalloc(&dC, 4096);
    (void)hipMemcpy(dA, A, 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B, 2048, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    (void)hipMemcpy(C, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; i++) bad += C[i] != R[i];
    printf("mfma_f32_32x32x16_bf16 documented-map mismatches: %d / 1024 (C[0]=%g want %g, C[33]=%g want %g)\n", bad, C[0],
           R[0], C[33], R[33]);
    return 0;
}
