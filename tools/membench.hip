// membench.hip -- TOOL (not shipped): memory-only twins of g2048_step to calibrate the achievable bandwidth of
// its access pattern on MI355X.  Same per-lane loads and stores as the PCG64 + log2-obs step (173 B/board), no
// game logic; plus a float4 stream copy for the chip's streaming rate.
#include <hip/hip_runtime.h>
#include <stdint.h>

struct Bufs {
    uint64_t* board; uint8_t* status; const uint8_t* action; uint32_t* sc; uint8_t* mt; uint32_t* score;
    ulonglong2* rs; const ulonglong2* inc; uint64_t* buf; float* reward; uint8_t* flags; uint32_t* mask; float4* obs;
    uint32_t n;
};

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

template <bool COOP, int WORK>
__global__ void __launch_bounds__(1024) twin(Bufs a) {
    const int lane = threadIdx.x & 63;
    const uint32_t wf = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u;
    const uint32_t ws = gridDim.x * blockDim.x;
    for (uint32_t w0 = wf; w0 < a.n; w0 += ws) {
        const uint32_t i = w0 + lane;
        uint64_t b = 0;
        if (i < a.n) {
            b = a.board[i];
            const uint32_t st = a.status[i], act = a.action[i], sc = a.sc[i], mt = a.mt[i], score = a.score[i];
            ulonglong2 r = a.rs[i];
            const ulonglong2 c = a.inc[i];
            const uint64_t bf = a.buf[i];
            r.x += c.x; r.y ^= c.y;
            // synthetic ALU work: WORK iterations of 4 independent 32-bit chains (~8 VALU each)
            uint32_t x0 = (uint32_t)b, x1 = (uint32_t)(b >> 32), x2 = sc ^ score, x3 = (uint32_t)r.x;
            for (int w = 0; w < WORK; w++) {
                x0 = x0 * 0x9E3779B1u + x1; x1 = (x1 ^ (x0 >> 7)) * 0x85EBCA77u;
                x2 = x2 * 0xC2B2AE3Du + x3; x3 = (x3 ^ (x2 >> 9)) * 0x27D4EB2Fu;
            }
            b ^= (uint64_t)(x0 ^ x1 ^ x2 ^ x3) << 1;
            b ^= (uint64_t)act << 60 | st;
            a.board[i] = b;
            a.sc[i] = sc + 1;
            a.score[i] = score + act;
            a.mt[i] = (uint8_t)(mt + 1);
            a.rs[i] = r;
            a.buf[i] = bf + 1;
            a.reward[i] = (float)act;
            a.flags[i] = (uint8_t)st;
            a.mask[i] = (uint32_t)b;
            if (!COOP) {
#pragma unroll
                for (int k = 0; k < 4; k++) a.obs[(size_t)i * 4 + k] = make_float4((float)(b >> k & 15), 0.f, 1.f, 2.f);
            }
        }
        if (COOP) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int q = k * 64 + lane;
                const uint64_t bb = shfl64(b, q >> 2);
                if (w0 + (q >> 2) < a.n) a.obs[(size_t)w0 * 4 + q] = make_float4((float)(bb & 15), 0.f, 1.f, 2.f);
            }
        }
    }
}

__global__ void __launch_bounds__(256) stream_copy(const float4* __restrict__ src, float4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// read one float4, write two (the step kernel's 1:2 read:write byte mix): dst[2i], dst[2i+1] from src[i]
__global__ void __launch_bounds__(256) stream_rw12(const float4* __restrict__ src, float4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = src[i];
        dst[i] = v;
        dst[n + i] = make_float4(v.w, v.z, v.y, v.x);
    }
}

// write-only stream (the one-hot obs bound): float4 stores, plain or non-temporal
template <bool NT>
__global__ void __launch_bounds__(256) stream_fill(float4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 v = {0.f, 1.f, 0.f, (float)(i & 7)};
        f4* p = reinterpret_cast<f4*>(dst) + i;
        if constexpr (NT) __builtin_nontemporal_store(v, p);
        else *p = v;
    }
}

template <int W>
void launch_twin(Bufs* a, int coop, int grid, int block, int lds, void* stream) {
    if (coop) hipLaunchKernelGGL((twin<true, W>), dim3(grid), dim3(block), lds, (hipStream_t)stream, *a);
    else hipLaunchKernelGGL((twin<false, W>), dim3(grid), dim3(block), lds, (hipStream_t)stream, *a);
}

// work: 0, 16, 32, 64 iterations; lds: dynamic LDS bytes per block (to force 1 block/CU like the real kernel)
extern "C" int mb_twin(Bufs* a, int coop, int grid, int block, int work, int lds, void* stream) {
    switch (work) {
        case 16: launch_twin<16>(a, coop, grid, block, lds, stream); break;
        case 32: launch_twin<32>(a, coop, grid, block, lds, stream); break;
        case 64: launch_twin<64>(a, coop, grid, block, lds, stream); break;
        default: launch_twin<0>(a, coop, grid, block, lds, stream); break;
    }
    return (int)hipGetLastError();
}

extern "C" int mb_copy(const void* src, void* dst, size_t n16, int grid, void* stream) {
    hipLaunchKernelGGL(stream_copy, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float4*)src, (float4*)dst, n16);
    return (int)hipGetLastError();
}

extern "C" int mb_rw12(const void* src, void* dst, size_t n16, int grid, void* stream) {
    hipLaunchKernelGGL(stream_rw12, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float4*)src, (float4*)dst, n16);
    return (int)hipGetLastError();
}
extern "C" int mb_fill(void* dst, size_t n16, int grid, int nt, void* stream) {
    if (nt) hipLaunchKernelGGL(stream_fill<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (float4*)dst, n16);
    else hipLaunchKernelGGL(stream_fill<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (float4*)dst, n16);
    return (int)hipGetLastError();
}
