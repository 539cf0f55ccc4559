// g2048_dw2.hip -- the layer-2 weight / bias gradient of the fused update (part of libg2048.so).
//
// update_batch accumulates, per valid step, the outer product a1 d2^T into dW2 and d2 into db2
// (src/reinforce_agent.py:536-555 -> _backpropagation :639-678).  The fused gradient kernels (g2048_policy.hip)
// write every sample's a1 and d2 as columns of a1^T and d2^T, stored in 16-column blocks (element (row, col) at
// ((col >> 4) R + row) 16 + (col & 15), R = max(H1p, H2p)); this kernel sums dW2 = a1^T d2 over a column range and
// db2 = the row sums of d2^T, split over workgroups (one fp32 partial [H1p + 1][H2p] slab per workgroup, rows
// 0..H1p-1 = dW2, row H1p = db2; the caller sums the slabs in fp64).
//
// gfx950 design: the product is HBM-bound at 2 KiB of columns per sample only if the arithmetic runs faster than
// the fp32 MFMA (64 FLOP/clk/SIMD would make it compute-bound at 2x the HBM time).  Every fp32 operand is split
// exactly into three bf16 planes (x = x0 + x1 + x2, 8 significant bits each) and the six plane products of order
// <= 2 run on v_mfma_f32_32x32x16_bf16 (16x the fp32 MFMA rate) into fp32 accumulators: fp32-accurate products
// (the dropped terms are < 2^-24 |x y|), at 6 x 32 cycles per 32x32x16 step against 8 x 64 for fp32 MFMA.
// Columns are staged global -> LDS by LDS-DMA (global_load_lds_dwordx4), 16 samples per stage -- one block of each
// buffer, so every stage reads two contiguous runs (the row-major [row][ld] layout read 64 B from each of 512 rows
// 4 MB apart per stage and ran at 2 TB/s) -- in a 4-slot ring with two stages in flight (counted vmcnt + raw
// barrier); the 16-B chunks of a staged row are XOR-swizzled by row so that the fragment reads (ds_read_b128) are
// bank-conflict free.  One 256-thread workgroup per CU: the 4 waves own 2 x 2 blocks of the output tiles (4 x 4
// tiles of 32 x 32, 256 accumulator registers each for a 256 x 256 layer).  Software-pipelined: each loop step reads
// and splits stage it + 1 into a second register set while the 96 MFMAs of stage it run, with the interleave pinned
// by sched_group_barrier (8 LDS reads up front, then per MFMA one LDS read and 4 VALU) -- hipcc otherwise issues the
// whole split (~360 VALU) ahead of the first MFMA.  Measured at 2^20 columns of a 256 x 256 layer: 905 us with the
// split in front, 690-750 us pipelined; PMC: MFMA busy 3072 of 4090 cycles per wave-stage, the chip holding ~1.5 GHz
// under this load (profiles/round3/).
#include <hip/hip_runtime.h>

#include "g2048.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kBK = 16;                     // samples (columns) per stage = one 32x32x16 MFMA k-step
constexpr int kAhead = 2;                   // stages in flight beyond the one being split
constexpr int kStages = kAhead + 2;         // LDS ring (a slot is refilled two barriers after its last read)
constexpr int kThreads = 256;  // 4 waves

__host__ __device__ inline int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// one LDS-DMA of 16 B per lane: lane l's 16 bytes land at lds_wave_base + 16 l (lds_wave_base wave-uniform).
// Issued through inline asm so that hipcc does not track it: the compiler otherwise treats every pending LDS-DMA as
// an LDS write and drains the whole ring (s_waitcnt vmcnt(0)) before each ds_read, serialising the pipeline; the
// kernel counts these loads itself (vmcnt(N) + barrier before a stage is read).  M0 is written and restored in the
// same statement (the compiler reserves it).  Device-only body: the host pass of a template kernel that names the
// address-space-3 cast drops the kernel's host stub without a diagnostic.
__device__ __forceinline__ void glds16(const float* src, float* lds_wave_base) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds_wave_base);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
#else
    (void)src;
    (void)lds_wave_base;
#endif
}

// 256-wide second layers: one 8-wave workgroup per column range (2 waves per SIMD, 8 accumulator tiles each, one
// register set of planes).  (Round 4: the 4-wave kernel with all 256 output columns spilled ~145 VGPRs; with the
// columns split over two workgroups each re-read the a1 rows -- both slower, profiles/round4/r4c10/.)
__host__ __device__ constexpr int dw2_threads(int nt2) { return nt2 >= 8 ? 512 : 256; }

// MODE: 0 = d2 columns; 1 = the ReLU critic's factored records (mask words + scalar g); 2 = the ReLU actor's
// records (mask words + the 4 values of g per sample; d2 rebuilt here)
template <int NT1, int NT2, int MODE>
struct Dw2 {
    static constexpr bool FAC = MODE != 0;             // a record per block instead of d2 rows
    static constexpr int H1 = 32 * NT1, H2 = 32 * NT2;
    static constexpr int RB = H1 > H2 ? H1 : H2;        // rows per 16-column block of both column buffers
    static constexpr bool WIDE = NT2 >= 8;
    static constexpr int CS = 1;                        // output column ranges per column range (blockIdx.y)
    static constexpr int kW = WIDE ? 8 : 4;             // waves: a WR x WC grid over the output tiles
    static constexpr int WR = 2, WC = kW / 2;
    static constexpr int kThr = 64 * kW;
    static_assert(kThr == dw2_threads(NT2), "launch bounds");
    static constexpr int NT2h = NT2 / CS, H2h = H2 / CS;
    static constexpr int kRows = FAC ? H1 : H1 + H2h;   // staged rows: a1 rows, then this half's d2 rows
    static constexpr int kRecFloats = FAC ? 256 : 0;    // FAC: the block's 1 KiB record (mask words, g)
    static constexpr int kStageFloats = kRows * kBK + kRecFloats;   // 64 B per staged row
    static constexpr int kRowGlds = kRows / 16;         // 1 KiB LDS-DMA instructions per stage (16 rows each)
    static constexpr int kGlds = kRowGlds + (FAC ? 1 : 0);          // + the record
    static constexpr int kGldsPerWave = (kGlds + kW - 1) / kW;
    static constexpr int TR = NT1 >= WR ? NT1 / WR : 1;   // row tiles per wave
    static constexpr int TC = NT2h >= WC ? NT2h / WC : 1;  // column tiles per wave
};

struct Dw2Args {
    const float* a1t;   // a1^T, 16-column blocks of RB rows
    const float* d2t;   // d2^T, the same layout (factored form: the 1 KiB block records)
    const float* w3;    // MODE 1: W3[:, 0] padded to H2p; MODE 2: W3 [H2p][4] padded
    float* part;        // [nparts][H1p + 1][H2p]
    uint32_t ld, col0, ncols, kb;   // column range [col0, col0 + ncols); workgroup p takes kb columns from col0 + p kb
};


// exact split of 8 fp32 values into three bf16 planes (x = p0 + p1 + p2 exactly)
__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
#pragma unroll
    for (int j = 0; j < 8; j++) {   // round to nearest even at each step
        const __bf16 h = (__bf16)v[j];
        const float r = v[j] - (float)h;
        const __bf16 m = (__bf16)r;
        const float r2 = r - (float)m;
        p0[j] = h;
        p1[j] = m;
        p2[j] = (__bf16)r2;
    }
}

// 8 consecutive columns k = 8h .. 8h+7 of staged row `row` (two 16-B chunks, swizzled slot = chunk ^ ((row >> 2) & 3))
__device__ __forceinline__ void read_frag(const float* stage, int row, int h, float (&v)[8]) {
    const int f = (row >> 2) & 3;
    const float4 x = *reinterpret_cast<const float4*>(stage + row * kBK + (((2 * h) ^ f) << 2));
    const float4 y = *reinterpret_cast<const float4*>(stage + row * kBK + (((2 * h + 1) ^ f) << 2));
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}

// FAC: the ReLU critic's factored form (g2048_critic_grad d2_form 1): d2 = m * (W3 g) with a 0/1 mask m and a scalar
// g per sample, so dW2 = W3[j] * sum (a1 g) m^T and db2 = W3[j] * sum g m: the A operand is a1 * g (one fp32 product,
// split exactly into three planes), the B operand the mask (exact in bf16), three MFMAs per step instead of six.
template <int NT1, int NT2, int MODE>
__global__ void __launch_bounds__(dw2_threads(NT2), 1) dw2_kernel(Dw2Args a) {
    using G = Dw2<NT1, NT2, MODE>;
    constexpr bool FAC = G::FAC;
    __shared__ float S[kStages * G::kStageFloats];   // the only LDS object (see the glds / second-object rule)
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, r = lane & 31;
    const int wr = w / G::WC, wc = w % G::WC;
    const uint32_t k_begin = a.col0 + blockIdx.x * a.kb;
    const uint32_t k_end = min(k_begin + a.kb, a.col0 + a.ncols);
    const int iters = k_end > k_begin ? (int)((k_end - k_begin) / kBK) : 0;
    const int c0 = (int)blockIdx.y * G::H2h;            // this workgroup's first output column (unit of layer 2)

    // this lane's LDS-DMA sources: instruction g (wave w issues g = w, w + 4, ...; past the end: the last one
    // again, an identical rewrite) covers staged rows 16 g .. 16 g + 15; lane -> row 16 g + (lane >> 2), slot
    // lane & 3, which holds the row's chunk (slot ^ ((row >> 2) & 3))
    // (FAC: instruction kRowGlds copies the block's record, 16 B per lane, unswizzled, after the staged rows; which
    // instruction that is depends only on the wave, so the per-stage source stride is a scalar)
    const int ws = __builtin_amdgcn_readfirstlane(w);
    const auto glds_index = [&](int i) {
        const int g = ws + G::kW * i;
        return g < G::kGlds ? g : G::kGlds - 1;
    };
    const float* src[G::kGldsPerWave];
#pragma unroll
    for (int i = 0; i < G::kGldsPerWave; i++) {
        const int g = glds_index(i);
        if (FAC && g == G::kRowGlds) {
            src[i] = a.d2t + (size_t)(k_begin / kBK) * 256 + 4 * lane;
        } else {
            const int row = 16 * g + (lane >> 2);
            const int chunk = (lane & 3) ^ ((lane >> 4) & 3);
            const float* base = row < G::H1 ? a.a1t + row * kBK : a.d2t + (row - G::H1 + c0) * kBK;
            src[i] = base + (size_t)(k_begin / kBK) * G::RB * kBK + 4 * chunk;   // block k_begin / 16
        }
    }
    const auto issue_to = [&](int slot, int stage_idx) {
        float* dst = S + slot * G::kStageFloats;
#pragma unroll
        for (int i = 0; i < G::kGldsPerWave; i++) {
            const int g = glds_index(i);
            const uint32_t stride = (FAC && g == G::kRowGlds) ? 256u : (uint32_t)(G::RB * kBK);
            glds16(src[i] + (size_t)stage_idx * stride, dst + 16 * g * kBK);
        }
    };

    floatx16 acc[G::TR][G::TC];
#pragma unroll
    for (int i = 0; i < G::TR; i++)
#pragma unroll
        for (int j = 0; j < G::TC; j++) acc[i][j] = floatx16{};
    const bool rows_mine = NT1 >= G::WR || wr == 0, cols_mine = G::NT2h >= G::WC || wc == 0;
    // db2: thread t sums d2 row c0 + t (threads past H2h sum the half's last row and never store: no branch in the
    // loop body)
    const int drow = G::H1 + (t < G::H2h ? t : G::H2h - 1);
    const int dunit = c0 + (t < G::H2h ? t : G::H2h - 1);
    float dsum = 0.0f;
    // MODE 2: the W3 rows this thread rebuilds d2 with -- its db2 unit and its B-fragment units
    float4 w3d = make_float4(0.f, 0.f, 0.f, 0.f), w3c[G::TC];
    if constexpr (MODE == 2) {
        const float4* w3v = reinterpret_cast<const float4*>(a.w3);
        w3d = w3v[dunit];
#pragma unroll
        for (int j = 0; j < G::TC; j++) w3c[j] = w3v[c0 + 32 * ((G::NT2h >= G::WC ? wc : 0) * G::TC + j) + r];
    }
    // d2 = act'(a2) (W3 g) exactly as grad_kernel forms it: fl(g0 w0), three fmaf, times 1.0 or 0.0
    const auto d2_of = [](const float4 g, const float4 w, bool m) {
        float dh = g.x * w.x;
        dh = fmaf(g.y, w.y, dh);
        dh = fmaf(g.z, w.z, dh);
        dh = fmaf(g.w, w.w, dh);
        return dh * (m ? 1.0f : 0.0f);
    };

    // the bf16 planes of one stage's operand fragments (this wave's A rows and B rows), double-buffered: the loop
    // reads and splits stage it + 1 while the MFMAs of stage it run from registers
    struct Planes {
        bf16x8 a0[G::TR], a1[G::TR], a2[G::TR], b0[G::TC], b1[G::TC], b2[G::TC];
    };
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const auto load = [&](const float* st, Planes& p) {
        if constexpr (MODE == 2) {
            const float* rec = st + G::kRows * kBK;
            const uint16_t* mw = reinterpret_cast<const uint16_t*>(rec);
            const float4* gv = reinterpret_cast<const float4*>(rec + 128);   // byte 512: g of sample s at gv[s]
            {   // db2: the d2 of unit `dunit` over the block's 16 samples, in sample order (as the column sum)
                const uint32_t m = mw[dunit];
#pragma unroll
                for (int e = 0; e < 16; e++) dsum += d2_of(gv[e], w3d, (m >> e) & 1u);
            }
            if (rows_mine && cols_mine) {
#pragma unroll
                for (int i = 0; i < G::TR; i++) {
                    float v[8];
                    read_frag(st, 32 * (wr * G::TR + i) + r, h, v);
                    split3(v, p.a0[i], p.a1[i], p.a2[i]);
                }
                float4 gk[8];
#pragma unroll
                for (int e = 0; e < 8; e++) gk[e] = gv[8 * h + e];
#pragma unroll
                for (int j = 0; j < G::TC; j++) {
                    const uint32_t m = (uint32_t)mw[c0 + 32 * (wc * G::TC + j) + r] >> (8 * h);
                    float v[8];
#pragma unroll
                    for (int e = 0; e < 8; e++) v[e] = d2_of(gk[e], w3c[j], (m >> e) & 1u);
                    split3(v, p.b0[j], p.b1[j], p.b2[j]);
                }
            }
            return;
        }
        if constexpr (MODE == 1) {
            const float* rec = st + G::kRows * kBK;
            const uint16_t* mw = reinterpret_cast<const uint16_t*>(rec);
            const float* gv = rec + 128;   // byte 512: g of the block's 16 samples
            {   // db2 (before the W3 scaling): sum over the samples of g where unit `dunit`'s mask bit is set
                const uint32_t m = mw[dunit];
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const float4 x = *reinterpret_cast<const float4*>(gv + 4 * c);
                    dsum += ((m >> (4 * c + 0)) & 1u) ? x.x : 0.0f;
                    dsum += ((m >> (4 * c + 1)) & 1u) ? x.y : 0.0f;
                    dsum += ((m >> (4 * c + 2)) & 1u) ? x.z : 0.0f;
                    dsum += ((m >> (4 * c + 3)) & 1u) ? x.w : 0.0f;
                }
            }
            if (rows_mine && cols_mine) {
                const float4 g0 = *reinterpret_cast<const float4*>(gv + 8 * h);
                const float4 g1 = *reinterpret_cast<const float4*>(gv + 8 * h + 4);
                const float gk[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
                for (int i = 0; i < G::TR; i++) {
                    float v[8];
                    read_frag(st, 32 * (wr * G::TR + i) + r, h, v);
#pragma unroll
                    for (int e = 0; e < 8; e++) v[e] *= gk[e];   // a1 g: the one rounding of the factored form
                    split3(v, p.a0[i], p.a1[i], p.a2[i]);
                }
#pragma unroll
                for (int j = 0; j < G::TC; j++) {   // mask bits 8h .. 8h+7 of unit n as bf16 1.0 (0x3F80) / 0
                    const uint32_t m = (uint32_t)mw[c0 + 32 * (wc * G::TC + j) + r] >> (8 * h);
                    u32x4 q;
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        q[e] = (((m >> (2 * e)) & 1u) * 0x3F80u) | (((m >> (2 * e + 1)) & 1u) * 0x3F800000u);
                    p.b0[j] = __builtin_bit_cast(bf16x8, q);
                }
            }
            return;
        }
        const float* rowp = st + drow * kBK;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const float4 x = *reinterpret_cast<const float4*>(rowp + 4 * c);
            dsum += x.x;
            dsum += x.y;
            dsum += x.z;
            dsum += x.w;
        }
        if (rows_mine && cols_mine) {
#pragma unroll
            for (int i = 0; i < G::TR; i++) {
                float v[8];
                read_frag(st, 32 * (wr * G::TR + i) + r, h, v);
                split3(v, p.a0[i], p.a1[i], p.a2[i]);
            }
#pragma unroll
            for (int j = 0; j < G::TC; j++) {
                float v[8];
                read_frag(st, G::H1 + 32 * (wc * G::TC + j) + r, h, v);
                split3(v, p.b0[j], p.b1[j], p.b2[j]);
            }
        }
    };
    const auto mfma = [&](const Planes& p) {
        if (rows_mine && cols_mine) {
#pragma unroll
            for (int i = 0; i < G::TR; i++)
#pragma unroll
                for (int j = 0; j < G::TC; j++) {
                    floatx16 c = acc[i][j];   // smallest terms first
                    if constexpr (MODE == 1) {   // (a1 g) m: the mask is exact in one plane
                        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a2[i], p.b0[j], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a1[i], p.b0[j], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a0[i], p.b0[j], c, 0, 0, 0);
                        acc[i][j] = c;
                        continue;
                    }
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a2[i], p.b0[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a1[i], p.b1[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a0[i], p.b2[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a1[i], p.b0[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a0[i], p.b1[j], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(p.a0[i], p.b0[j], c, 0, 0, 0);
                    acc[i][j] = c;
                }
        }
    };
    // one loop step: refill the slot of stage it + 1 + kAhead (past the end: stage iters - 1 again into a slot
    // nobody reads, so the wait count stays uniform), wait for stage it + 1, then split it into `nxt` while the
    // MFMAs of stage it (`cur`) run; the interleave is pinned (1 MFMA, then up to 4 VALU) since hipcc otherwise
    // puts the whole split ahead of the first MFMA
    const auto step = [&](int it, const Planes& cur, Planes& nxt) {
        const int q = it + 1 + kAhead;
        issue_to(q % kStages, q < iters ? q : iters - 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kAhead * G::kGldsPerWave) : "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        load(S + ((it + 1) % kStages) * G::kStageFloats, nxt);
        mfma(cur);
        constexpr int kMfma = (MODE == 1 ? 3 : 6) * G::TR * G::TC;
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);   // DS read: the first fragments' reads up front
#pragma unroll
        for (int m = 0; m < kMfma; m++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // VALU
        }
    };

    if constexpr (G::WIDE) {
        // two waves per SIMD, one register set of planes (a second set does not fit 256 registers): each step waits
        // for stage it, splits it and runs its MFMAs; the SIMD's other wave fills the gaps
        Planes pa;
        if (iters > 0) {
#pragma unroll
            for (int q = 0; q < kAhead; q++) issue_to(q, q < iters ? q : iters - 1);
            for (int it = 0; it < iters; it++) {
                const int q = it + kAhead;
                issue_to(q % kStages, q < iters ? q : iters - 1);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kAhead * G::kGldsPerWave) : "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                load(S + (it % kStages) * G::kStageFloats, pa);
                mfma(pa);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    } else {
    Planes pa, pb;
    if (iters > 0) {
#pragma unroll
        for (int q = 0; q <= kAhead; q++) issue_to(q, q < iters ? q : iters - 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kAhead * G::kGldsPerWave) : "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        load(S, pa);
        int it = 0;
        for (; it + 2 < iters; it += 2) {
            step(it, pa, pb);
            step(it + 1, pb, pa);
        }
        if (it + 1 < iters) {
            step(it, pa, pb);
            mfma(pb);
        } else {
            mfma(pa);
        }
        // the LDS-DMA refills issued past the last stage (kept so the wait count stays uniform) are not tracked
        // by the compiler: drain them before the workgroup ends, so its LDS is never handed on with writes in flight
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    }
    // this workgroup's slab: dW2 rows from the accumulators (C/D layout: column = lane & 31, row = acc_row), db2
    // (FAC: each column scaled by W3[j] -- the one multiply of the factored form)
    float* out = a.part + (size_t)blockIdx.x * (G::H1 + 1) * G::H2;
    if (rows_mine && cols_mine) {
#pragma unroll
        for (int j = 0; j < G::TC; j++) {
            const float ws = MODE == 1 ? a.w3[c0 + 32 * (wc * G::TC + j) + r] : 1.0f;
#pragma unroll
            for (int i = 0; i < G::TR; i++)
#pragma unroll
                for (int q = 0; q < 16; q++)
                    out[(size_t)(32 * (wr * G::TR + i) + acc_row(q, h)) * G::H2 + c0 + 32 * (wc * G::TC + j) + r] =
                        MODE == 1 ? acc[i][j][q] * ws : acc[i][j][q];
        }
    }
    if (t < G::H2h) out[(size_t)G::H1 * G::H2 + dunit] = MODE == 1 ? dsum * a.w3[dunit] : dsum;
}

template <int NT1, int MODE>
void launch_nt2(const Dw2Args& a, int nt2, int grid, hipStream_t s) {
    switch (nt2) {   // grid.y = the output column halves (Dw2::CS)
        case 1: hipLaunchKernelGGL((dw2_kernel<NT1, 1, MODE>), dim3(grid, Dw2<NT1, 1, MODE>::CS), dim3(Dw2<NT1, 1, MODE>::kThr), 0, s, a); break;
        case 2: hipLaunchKernelGGL((dw2_kernel<NT1, 2, MODE>), dim3(grid, Dw2<NT1, 2, MODE>::CS), dim3(Dw2<NT1, 2, MODE>::kThr), 0, s, a); break;
        case 4: hipLaunchKernelGGL((dw2_kernel<NT1, 4, MODE>), dim3(grid, Dw2<NT1, 4, MODE>::CS), dim3(Dw2<NT1, 4, MODE>::kThr), 0, s, a); break;
        default: hipLaunchKernelGGL((dw2_kernel<NT1, 8, MODE>), dim3(grid, Dw2<NT1, 8, MODE>::CS), dim3(Dw2<NT1, 8, MODE>::kThr), 0, s, a); break;
    }
}

template <int NT1>
void launch_mode(const Dw2Args& a, int mode, int nt2, int grid, hipStream_t s) {
    if (mode == 1) launch_nt2<NT1, 1>(a, nt2, grid, s);
    else if (mode == 2) launch_nt2<NT1, 2>(a, nt2, grid, s);
    else launch_nt2<NT1, 0>(a, nt2, grid, s);
}

int tiles_of(int hsize) {   // as g2048_policy.hip: 32-unit tiles rounded up to 1, 2, 4 or 8
    const int t = (hsize + 31) / 32;
    return t <= 1 ? 1 : t <= 2 ? 2 : t <= 4 ? 4 : 8;
}

// acc[i] += sum_p part[p slab + i] in fp64.  A workgroup of 64 G threads takes 64 consecutive elements: wave g
// sums the slabs p = g, g + G, g + 2G, ... (8 loads in flight; each load instruction reads 256 contiguous bytes),
// then the G wave sums are added in order of g through LDS -- a fixed order, so the result is deterministic.
// G (1..16) grows as the slab shrinks, so that small slabs with many parts still put enough waves on the chip.
__global__ void __launch_bounds__(1024) fold_kernel(const float* __restrict__ part, uint32_t nparts, uint32_t slab,
                                                    double* __restrict__ acc) {
    __shared__ double ws[16][64];
    const uint32_t G = blockDim.x >> 6, g = threadIdx.x >> 6, e = threadIdx.x & 63u;
    const uint32_t i = blockIdx.x * 64u + e;
    const uint32_t ic = i < slab ? i : slab - 1u;
    double s = 0.0;
    uint32_t p = g;
    for (; p + 7u * G < nparts; p += 8u * G) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = part[(size_t)(p + q * G) * slab + ic];
#pragma unroll
        for (int q = 0; q < 8; q++) s += (double)v[q];
    }
    for (; p < nparts; p += G) s += (double)part[(size_t)p * slab + ic];
    ws[g][e] = s;
    __syncthreads();
    if (g == 0 && i < slab) {
        double t = ws[0][e];
        for (uint32_t k = 1; k < G; k++) t += ws[k][e];
        acc[i] += t;
    }
}

}  // namespace

namespace g2048_internal {
int set_error(int code, const char* msg);
}

static int dw2_launch(const float* a1t, const float* d2t, const float* w3, int mode, int h1, int h2, int64_t ld,
                      int64_t col0, int64_t ncols, int64_t cols_per_part, float* partials, int64_t nparts, void* stream) {
    using g2048_internal::set_error;
    if (h1 < 1 || h1 > 256 || h2 < 1 || h2 > 256) return set_error(G2048_EINVAL, "dw2: hidden sizes must be in 1..256");
    if (!a1t || !d2t || !partials || (mode && !w3)) return set_error(G2048_EINVAL, "dw2: NULL buffer");
    if (ld <= 0 || (ld & 15) || ld > ((int64_t)1 << 28)) return set_error(G2048_EINVAL, "dw2: ld must be a positive multiple of 16");
    if (col0 < 0 || (col0 & 15) || ncols < 0 || (ncols & 15) || col0 + ncols > ld)
        return set_error(G2048_EINVAL, "dw2: column range must be multiples of 16 inside ld");
    if (cols_per_part <= 0 || (cols_per_part & 15)) return set_error(G2048_EINVAL, "dw2: cols_per_part must be a positive multiple of 16");
    if (nparts != (ncols + cols_per_part - 1) / cols_per_part || nparts > 65535)
        return set_error(G2048_EINVAL, "dw2: nparts must be ceil(ncols / cols_per_part) (<= 65535)");
    if (nparts == 0) return G2048_OK;
    Dw2Args a{a1t, d2t, w3, partials, (uint32_t)ld, (uint32_t)col0, (uint32_t)ncols, (uint32_t)cols_per_part};
    const int nt1 = tiles_of(h1), nt2 = tiles_of(h2);
    hipStream_t s = (hipStream_t)stream;
    const int grid = (int)nparts;
    switch (nt1) {
        case 1: launch_mode<1>(a, mode, nt2, grid, s); break;
        case 2: launch_mode<2>(a, mode, nt2, grid, s); break;
        case 4: launch_mode<4>(a, mode, nt2, grid, s); break;
        default: launch_mode<8>(a, mode, nt2, grid, s); break;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(G2048_EHIP, hipGetErrorString(e));
    return G2048_OK;
}

extern "C" int g2048_dw2(const float* a1t, const float* d2t, int h1, int h2, int64_t ld, int64_t col0, int64_t ncols,
                         int64_t cols_per_part, float* partials, int64_t nparts, void* stream) {
    return dw2_launch(a1t, d2t, nullptr, 0, h1, h2, ld, col0, ncols, cols_per_part, partials, nparts, stream);
}

extern "C" int g2048_dw2_factored(const float* a1t, const float* records, const float* w3, int h1, int h2, int64_t ld,
                                  int64_t col0, int64_t ncols, int64_t cols_per_part, float* partials, int64_t nparts,
                                  void* stream) {
    return dw2_launch(a1t, records, w3, 1, h1, h2, ld, col0, ncols, cols_per_part, partials, nparts, stream);
}

extern "C" int g2048_dw2_actor(const float* a1t, const float* records, const float* w3, int h1, int h2, int64_t ld,
                               int64_t col0, int64_t ncols, int64_t cols_per_part, float* partials, int64_t nparts,
                               void* stream) {
    return dw2_launch(a1t, records, w3, 2, h1, h2, ld, col0, ncols, cols_per_part, partials, nparts, stream);
}

extern "C" int g2048_fold_partials(const float* partials, int64_t nparts, int64_t slab, double* acc, void* stream) {
    using g2048_internal::set_error;
    if (!partials || !acc) return set_error(G2048_EINVAL, "fold_partials: NULL buffer");
    if (nparts < 0 || slab < 0 || nparts > ((int64_t)1 << 24) || slab > ((int64_t)1 << 28))
        return set_error(G2048_EINVAL, "fold_partials: nparts / slab out of range");
    if (nparts == 0 || slab == 0) return G2048_OK;
    // waves per workgroup: enough that ~4 waves per SIMD (4096 on 256 CUs) each sum at least 8 slabs
    const int64_t blocks = (slab + 63) / 64;
    int G = 1;
    while (G < 16 && blocks * G < 4096 && nparts >= 16 * G) G *= 2;
    hipLaunchKernelGGL(fold_kernel, dim3((unsigned)blocks), dim3(64 * G), 0, (hipStream_t)stream, partials,
                       (uint32_t)nparts, (uint32_t)slab, acc);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(G2048_EHIP, hipGetErrorString(e));
    return G2048_OK;
}
