// g2048_deep.hip -- the policy / value MLP of ANY depth for the rollout and the update (part of libg2048.so).
//
// The reference's forward (forward_logits, src/MLP.py:159-196) is generic in depth: hidden_sizes is a list, and
// runner.py documents [256, 128, 64] on one-hot obs (runner.py:10-47).  g2048_policy.hip's kernels are register-
// specialised for two hidden layers of log2 / raw obs; this file covers the rest:
//   * g2048_deep_policy: forward of 1..4 hidden layers of 1..256 units (ReLU / Sigmoid) + masked softmax +
//     select_action's choice (src/reinforce_agent.py:178-190), straight from the bitboards -- no obs buffer.  One
//     256-thread workgroup (4 waves) per group of 32 boards, two workgroups per CU: every layer's activations live
//     in LDS ([unit][board], row stride 33 floats), its 32-unit output tiles are split over the 4 waves and run on
//     v_mfma_f32_32x32x2_f32 (exact fp32, a k-ordered fmaf chain) with the weight fragments streamed from L2 in
//     A-fragment order (one 16-B load per lane = four k-steps) and the activations as the B operand read from LDS;
//     bias + activation in registers on the way back to LDS; the output layer (4 logits, or the value) on VALU.
//   * the one-hot first layer (obs_mode "onehot": 16 cells x 17 one-hot features, src/env.py:131-150) is NOT a
//     272-wide fp32 GEMM: x has exactly one 1 per cell, so each cell's slice of x is an exact bf16 operand, and W1 is
//     packed as three exact bf16 planes (w = p0 + p1 + p2): per cell and 32-unit tile 3 v_mfma_f32_32x32x16_bf16
//     (onehot_l0_tile / deep_forward), every product exact, act((hi + lo) + b1) -- the same bits in the rollout, the
//     policy and (since round 6, no separate layer-0 kernel) inside the gradient kernel.
//   * g2048_onehot_layer1 / g2048_onehot_dw1: the update's layer-1 activations for the hipBLASLt path (a gather of the
//     16 W1 rows a board selects), and dW1 = X^T D1 of a one-hot X on the bf16 MFMA (A = the exact one-hot of two
//     cells, B = the deltas split into three exact bf16 planes), one fp32 partial slab per workgroup, the slabs summed
//     in fp64 by g2048_fold_partials.
// Roofline: the dense layers are fp32-MFMA bound (157.3 TFLOP/s dense fp32 on MI355X); the one-hot layer 0 and dW1
// run on the bf16 MFMA at 3 planes per product; the gather of g2048_onehot_layer1 is L2-bound (16 rows x 4 H1 B per
// sample).
#include <hip/hip_runtime.h>

#include <atomic>
#include <type_traits>

#include "g2048.h"
#include "g2048_core.h"

using namespace g2048;

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// two floats rounded to nearest even into one dword of bf16 (a in the low half): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}

// exact split of 8 floats into three bf16 planes (x = p0 + p1 + p2; each residual is exact in fp32), packed two
// values per dword: 11 VALU per pair
__device__ __forceinline__ void split3_bf16(const float (&v)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 h, m, l;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const float x0 = v[2 * j], x1 = v[2 * j + 1];
        const uint32_t hh = pk_bf16(x0, x1);
        const float r0 = x0 - __uint_as_float(hh << 16), r1 = x1 - __uint_as_float(hh & 0xFFFF0000u);
        const uint32_t mm = pk_bf16(r0, r1);
        const float t0 = r0 - __uint_as_float(mm << 16), t1 = r1 - __uint_as_float(mm & 0xFFFF0000u);
        h[j] = hh;
        m[j] = mm;
        l[j] = pk_bf16(t0, t1);
    }
    p0 = __builtin_bit_cast(bf16x8, h);
    p1 = __builtin_bit_cast(bf16x8, m);
    p2 = __builtin_bit_cast(bf16x8, l);
}


constexpr int kMaxHidden = G2048_DEEP_MAX_HIDDEN;   // hidden layers
constexpr int kDeepBlock = 256;                      // 4 waves; two workgroups per CU
constexpr int kActStride = 33;                       // LDS activation row stride in floats: [unit][32 boards + 1]
constexpr int kOneHotRows = 272;                     // 16 cells x 17 one-hot features (src/env.py:143-150)
constexpr int kOneHotPlaneFloats = 16 * 3 * 64 * 4;   // one unit tile's W1 plane fragments

// the hidden unit held by accumulator register r of lane half h of a v_mfma_f32_32x32x2_f32 result tile
__host__ __device__ inline int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Packed net layout (floats; nt[l] = 32-unit tiles of hidden layer l, zero padded -- exact, a padded unit's
// outgoing weights are zero):
//   layer 0 weights   one-hot: table [272][32 nt0] row-major (row 17 c + e = W1[17 c + e, :]);
//                     else:    A fragments [nt0][8][64] (k-step s, lane l: W1[2 s + (l >> 5)][32 t + (l & 31)])
//   layer l >= 1      A fragments [nt_l][nt_{l-1}][4][64][4]: output tile o, k-tile t, lane l, k-step s = 4 q + u at
//                     [o][t][q][l][u] = W_l[32 t + tile_row(s, l >> 5)][32 o + (l & 31)] -- k-step s takes the input
//                     units an MFMA result tile holds in its register s (round 5), so a wave's accumulator tile of
//                     layer l - 1 can be the B operand of layer l register for register (the two-layer
//                     g2048_policy's layout); the LDS-fed chains read the same rows (frag_chain)
//   bias l            [32 nt_l]
//   output layer      [32 nt_{L-1}][4] row-major (a value head is output 0), bias [4]
//   one-hot W1 planes [nt0][16 cells][3 planes][64 lanes] dwords x 4 (round 5): the A fragment of
//                     v_mfma_f32_32x32x16_bf16 for unit tile t, cell c, plane p -- lane l holds bf16 plane p of
//                     W1[17 c + 8 (l >> 5) + j][32 t + (l & 31)], j = 0..7 (split3_bf16: w = p0 + p1 + p2 exactly)
struct DeepNet {
    int L;                            // hidden layers
    int onehot;                       // first layer is the one-hot bf16-plane table
    int nt[kMaxHidden];
    int64_t w[kMaxHidden + 1], b[kMaxHidden + 1];
    int64_t wpl;                      // one-hot: W1's bf16-plane A fragments (see the layout note above)
    int64_t total;
};

int tiles_of(int h) { return (h + 31) / 32; }

bool deep_layout(int L, const int* hidden, int onehot, DeepNet& n) {
    if (L < 1 || L > kMaxHidden || !hidden) return false;
    n = DeepNet{};
    n.L = L;
    n.onehot = onehot;
    int64_t off = 0;
    for (int l = 0; l < L; l++) {
        if (hidden[l] < 1 || hidden[l] > 256) return false;
        n.nt[l] = tiles_of(hidden[l]);
        n.w[l] = off;
        if (l == 0) off += onehot ? (int64_t)kOneHotRows * 32 * n.nt[0] : (int64_t)n.nt[0] * 8 * 64;
        else off += (int64_t)n.nt[l] * n.nt[l - 1] * 1024;
        n.b[l] = off;
        off += 32 * n.nt[l];
    }
    n.w[L] = off;
    off += (int64_t)32 * n.nt[L - 1] * 4;
    n.b[L] = off;
    off += 4;
    n.wpl = onehot ? off : -1;
    if (onehot) off += (int64_t)n.nt[0] * kOneHotPlaneFloats;
    n.total = off;
    return true;
}

struct DeepPackArgs {
    DeepNet net;
    const float* W[kMaxHidden + 1];
    const float* B[kMaxHidden + 1];
    int h[kMaxHidden];
    int out;
    float* dst;
};

// one thread per packed float
__global__ void __launch_bounds__(256) deep_pack_kernel(DeepPackArgs a) {
    const DeepNet& n = a.net;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n.total; q += (int64_t)gridDim.x * blockDim.x) {
        if (n.onehot && q >= n.wpl) {   // W1 plane fragment dword (split3_bf16: w = p0 + p1 + p2 exactly)
            const int64_t x = q - n.wpl;
            const int d = (int)(x & 3), lane = (int)((x >> 2) & 63);
            const int64_t r = x >> 8;
            const int p = (int)(r % 3), c = (int)((r / 3) % 16), t = (int)(r / 48);
            const int hh = lane >> 5, j = 32 * t + (lane & 31);
            float v8[8];
#pragma unroll
            for (int jj = 0; jj < 8; jj++) v8[jj] = j < a.h[0] ? a.W[0][(int64_t)(17 * c + 8 * hh + jj) * a.h[0] + j] : 0.0f;
            bf16x8 p0, p1, p2;
            split3_bf16(v8, p0, p1, p2);
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 pv = __builtin_bit_cast(u32x4, p == 0 ? p0 : (p == 1 ? p1 : p2));
            a.dst[q] = __uint_as_float(pv[d]);
            continue;
        }
        float v = 0.0f;
        int l = n.L;
        while (l > 0 && q < n.w[l]) l--;          // the segment: [w[l], b[l]) weights, [b[l], w[l+1]) bias
        if (l == n.L) {
            if (q < n.b[l]) {
                const int64_t x = q - n.w[l];
                const int j = (int)(x >> 2), o = (int)(x & 3);
                v = (j < a.h[n.L - 1] && o < a.out) ? a.W[n.L][(int64_t)j * a.out + o] : 0.0f;
            } else {
                const int o = (int)(q - n.b[l]);
                v = o < a.out ? a.B[n.L][o] : 0.0f;
            }
        } else if (q >= n.b[l]) {
            const int j = (int)(q - n.b[l]);
            v = j < a.h[l] ? a.B[l][j] : 0.0f;
        } else if (l == 0) {
            const int64_t x = q - n.w[0];
            if (n.onehot) {
                const int H = 32 * n.nt[0];
                const int row = (int)(x / H), j = (int)(x % H);
                v = j < a.h[0] ? a.W[0][(int64_t)row * a.h[0] + j] : 0.0f;
            } else {
                const int lane = (int)(x & 63), s = (int)((x >> 6) & 7), t = (int)(x >> 9);
                const int k = 2 * s + (lane >> 5), j = 32 * t + (lane & 31);
                v = j < a.h[0] ? a.W[0][k * a.h[0] + j] : 0.0f;
            }
        } else {
            const int64_t x = q - n.w[l];
            const int u = (int)(x & 3), lane = (int)((x >> 2) & 63), qq = (int)((x >> 8) & 3);
            const int64_t tt = x >> 10;
            const int t = (int)(tt % n.nt[l - 1]), o = (int)(tt / n.nt[l - 1]);
            const int k = 32 * t + tile_row(4 * qq + u, lane >> 5), j = 32 * o + (lane & 31);
            v = (k < a.h[l - 1] && j < a.h[l]) ? a.W[l][(int64_t)k * a.h[l] + j] : 0.0f;
        }
        a.dst[q] = v;
    }
}

template <int ACT>
__device__ __forceinline__ float activate(float z) {
    if constexpr (ACT == 0) return fmaxf(z, 0.0f);
    else return 1.0f / (1.0f + expf(-z));
}

template <int OBS>
__device__ __forceinline__ float obs_value(uint64_t b, int cell, float scale) {
    const uint32_t e = (uint32_t)(b >> (4 * cell)) & 15u;
    if constexpr (OBS == G2048_OBS_LOG2) return (float)e * scale;
    else return e ? (float)(1u << e) : 0.0f;
}

// (Always the static struct: passing the forward its LDS as pointers -- for a rollout layout sized to the net --
// made hipcc emit FLAT instead of LDS instructions for the forward's accesses, in every form tried, and the
// rollout ran 0.318-0.348 s against 0.275 s; `profiles/round5/r5u/`, `r5v/`.)
struct DeepSmem {
    float act[2][256 * kActStride];   // ping-pong activations [unit][board]
    float part[8][32][4];             // output-layer partial sums [unit slice][board][output]
    uint64_t board[32];               // the group's boards
};

// The k-ordered MFMA chain of one output tile over k-tiles [t0, t1): A = the tile's weight fragments `fo` (4 float4
// per lane per k-tile, streamed from L2), B = the activation rows `in` (LDS).  Two fragment register sets, fa for
// the even and fb for the odd k-tiles, refilled as a sliding window: as soon as fragment q of k-tile t has fed its 4
// MFMAs, its register is reloaded with fragment q of k-tile t + 2 (a scheduling barrier keeps the load there), so
// every fragment load is issued two k-tiles (~2,000 cycles) before its use -- L2 latency under the gradient kernel's
// load exceeded the one k-tile of round 4's double buffer.  Past the end the window reloads the last k-tile
// (harmless, an L1 hit).  (Without a barrier hipcc sank every fragment load next to its MFMA and waited for it there:
// four L2 round trips per k-tile.)  The B operands run one segment (4 k-steps) ahead: the next segment's two
// ds_read2 are issued before this segment's MFMAs, so no segment waits for LDS reads issued next to its own first
// MFMA (round 6: runner-config update 1.215 -> 1.179 s, rollout 0.252 -> 0.240 s, `profiles/round6/r7h/`).  Same
// MFMAs in the same order as a plain loop.  (Also round 6, in the 64-sample gradient kernel: k-tile 0's fragments of
// each wave's first item loaded before the barrier that opens the phase -- 92 spilled SGPRs, update 1.259-1.264 s
// against 1.119-1.123 s; the hidden biases staged in LDS for the epilogues -- 1.119-1.120 s, even; neither kept,
// `profiles/round6/s3/`.)
template <int STRIDE = kActStride>
__device__ __forceinline__ floatx16 frag_chain(const float4* __restrict__ fo, const float* in, int t0, int t1, int h,
                                               int col) {
    floatx16 c = {};
    if (t0 >= t1) return c;
    float4 fa[4], fb[4];
    const int last = t1 - 1;
    // the B operands (4 LDS values per segment) one segment ahead: the next segment's reads are issued before this
    // segment's MFMAs, so a segment waits for reads issued ~4 MFMAs earlier instead of its own
    const float* base = in + 4 * h * STRIDE + col;
    const auto ld4 = [&](float (&v)[4], int t, int q) {
        const float* ib = base + (32 * t + 8 * q) * STRIDE;   // k-step 4 q + u: row 8 q + u + 4 h
        v[0] = ib[0 * STRIDE];
        v[1] = ib[1 * STRIDE];
        v[2] = ib[2 * STRIDE];
        v[3] = ib[3 * STRIDE];
    };
    float bc[4], bn[4];
    ld4(bc, t0, 0);
    const auto seg = [&](float4& f, int t, int q, int tn) {
        ld4(bn, q < 3 ? t : (t + 1 < t1 ? t + 1 : last), (q + 1) & 3);   // past the end: a harmless re-read
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(f.x, bc[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(f.y, bc[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(f.z, bc[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(f.w, bc[3], c, 0, 0, 0);
        f = fo[tn * 256 + q * 64];
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // the next segment's 2 ds_read2 first,
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // then this segment's 4 MFMAs,
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // then the fragment reload
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; i++) bc[i] = bn[i];
    };
#pragma unroll
    for (int q = 0; q < 4; q++) fa[q] = fo[t0 * 256 + q * 64];
#pragma unroll
    for (int q = 0; q < 4; q++) fb[q] = fo[(t0 + 1 < t1 ? t0 + 1 : last) * 256 + q * 64];
    __builtin_amdgcn_sched_barrier(0);
    int t = t0;
    for (; t + 1 < t1; t += 2) {
        const int ta = t + 2 < t1 ? t + 2 : last, tb = t + 3 < t1 ? t + 3 : last;
#pragma unroll
        for (int q = 0; q < 4; q++) seg(fa[q], t, q, ta);
#pragma unroll
        for (int q = 0; q < 4; q++) seg(fb[q], t + 1, q, tb);
    }
    if (t < t1) {
#pragma unroll
        for (int q = 0; q < 4; q++) seg(fa[q], t, q, last);
    }
    return c;
}

// frag_chain over k-tiles [0, nt) with k-tile 0's fragments carried across a wave's items: fa holds k-tile 0 of `fo`
// on entry, and its window reload past the end fetches k-tile 0 of `fo_next` (the wave's next item; NULL: the last
// k-tile again) -- so the next item's first MFMAs do not wait an L2 round trip behind this item's epilogue.  The
// same MFMAs in the same order as frag_chain(fo, in, 0, nt, h, col).
template <int STRIDE = kActStride>
__device__ __forceinline__ floatx16 frag_chain_carry(const float4* __restrict__ fo, const float* in, int nt, int h,
                                                     int col, float4 (&fa)[4], const float4* __restrict__ fo_next) {
    floatx16 c = {};
    float4 fb[4];
    const int last = nt - 1;
    const float* base = in + 4 * h * STRIDE + col;
    const auto ld4 = [&](float (&v)[4], int t, int q) {
        const float* ib = base + (32 * t + 8 * q) * STRIDE;
        v[0] = ib[0 * STRIDE];
        v[1] = ib[1 * STRIDE];
        v[2] = ib[2 * STRIDE];
        v[3] = ib[3 * STRIDE];
    };
    float bc[4], bn[4];
    ld4(bc, 0, 0);
    const auto seg = [&](float4& f, int t, int q, const float4* nf) {
        ld4(bn, q < 3 ? t : (t + 1 < nt ? t + 1 : last), (q + 1) & 3);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(f.x, bc[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(f.y, bc[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(f.z, bc[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(f.w, bc[3], c, 0, 0, 0);
        f = nf[q * 64];
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; i++) bc[i] = bn[i];
    };
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; q++) fb[q] = fo[(nt > 1 ? 256 : 0) + q * 64];   // k-tile 1 (needed 16 MFMAs later)
    int t = 0;
    for (; t + 1 < nt; t += 2) {
        const float4* na = t + 2 < nt ? fo + (t + 2) * 256 : (fo_next ? fo_next : fo + last * 256);
        const float4* nb = t + 3 < nt ? fo + (t + 3) * 256 : fo + last * 256;
#pragma unroll
        for (int q = 0; q < 4; q++) seg(fa[q], t, q, na);
#pragma unroll
        for (int q = 0; q < 4; q++) seg(fb[q], t + 1, q, nb);
    }
    if (t < nt) {   // odd nt: the last k-tile from fa, which then takes the next item's k-tile 0
#pragma unroll
        for (int q = 0; q < 4; q++) seg(fa[q], t, q, fo_next ? fo_next : fo + last * 256);
    }
    return c;
}

// One dense hidden layer (in -> out, [unit][board] stride kActStride) whose k range is split in two halves when it
// has fewer output tiles than 8 (the gradient kernel's waves) and at least 2 k-tiles: output tile o is
// act(fl(c0 + c1) + b) with c0 / c1 the k-ordered MFMA chains over k-tiles [0, ntin/2) and [ntin/2, ntin) -- the
// same values for any wave count NW, so deep_grad_kernel (8 waves) and its pattern probe deep_hidden_kernel (4 waves)
// agree bit for bit; the halves' items keep the idle waves of a 2- or 4-tile layer busy.  The second half's chain
// is parked in the output tile's own LDS cells until the first half adds it (one barrier inside).  The rollout /
// policy kernels keep the single chain (their layers are already spread over their 4 waves).
// MODE 1 (the 8-wave gradient kernels): split when ntout < 8 (and ntin >= 2); MODE 2 (the 4-wave one): split only
// when the two halves of every output tile give each of the 4 waves at most one item (2 ntout <= 4) -- the 64-unit
// layer of [256, 128, 64] -- so a wave keeps one chain in registers.
template <int ACT, int NW, int MODE = 1>
__device__ __forceinline__ void dense_fwd_split(const float* in, float* out, const float4* __restrict__ frag,
                                                const float* bias, int ntin, int ntout, int w) {
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const auto chain = [&](int o, int t0, int t1) {
        return frag_chain(frag + (int64_t)o * ntin * 256, in, t0, t1, h, col);
    };
    const auto cell = [&](int o, int r) { return out + (32 * o + tile_row(r, h)) * kActStride + col; };
    const auto finish = [&](int o, const floatx16& c) {
        const float* bb = bias + 32 * o;
        float bv[16];   // all 16 bias loads issued before the first use (one L2 round trip, not four)
#pragma unroll
        for (int r = 0; r < 16; r++) bv[r] = bb[tile_row(r, h)];
#pragma unroll
        for (int r = 0; r < 16; r++) *cell(o, r) = activate<ACT>(c[r] + bv[r]);
    };
    const bool split = ntin >= 2 && (MODE == 1 ? ntout < 8 : 2 * ntout <= 4);
    if (!split) {
        for (int o = w; o < ntout; o += NW) finish(o, chain(o, 0, ntin));
        return;
    }
    const int kh = ntin >> 1;
    constexpr int kKeep = MODE == 1 ? (7 + NW - 1) / NW : 1;      // first-half items per wave
    constexpr int kSecond = MODE == 1 ? (14 + NW - 1) / NW : 1;   // item slots per wave that may hold a second half
    floatx16 c0[kKeep];
#pragma unroll
    for (int r = 0; r < kKeep; r++) {
        const int o = w + NW * r;
        if (o < ntout) c0[r] = chain(o, 0, kh);
    }
#pragma unroll
    for (int r = 0; r < kSecond; r++) {
        const int i = w + NW * r;
        if (i >= ntout && i < 2 * ntout) {
            const floatx16 c1 = chain(i - ntout, kh, ntin);
#pragma unroll
            for (int q = 0; q < 16; q++) *cell(i - ntout, q) = c1[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kKeep; r++) {
        const int o = w + NW * r;
        if (o < ntout) {
            floatx16 c = c0[r];
#pragma unroll
            for (int q = 0; q < 16; q++) c[q] = c[q] + *cell(o, q);
            finish(o, c);
        }
    }
}

// The forward of the group's 32 boards (S.board) through every hidden layer, leaving the output layer's 8 partial
// sums per board in S.part (the caller adds them in order p = 0..7 plus the output bias).  Every thread of the
// workgroup calls it; it ends with a barrier.

// Entry 2 e + hh of the one-hot B-operand table: exponent e as 8 bf16 (1.0 at k = e, else 0) for the lane half hh
// (k = 8 hh .. 8 hh + 7).  Looked up per cell from LDS by the 64-slot rollout's layer 0: built by compares and
// selects it was ~21 VALU per cell and operand (round 5, the then layer-0 kernel of the update was VALU-bound).
__device__ __forceinline__ uint4 onehot_entry(uint32_t idx) {
    const uint32_t e = idx >> 1, hh = idx & 1;
    uint32_t d[4];
#pragma unroll
    for (int jj = 0; jj < 4; jj++)
        d[jj] = (e == 8 * hh + 2 * jj ? 0x3F80u : 0u) | (e == 8 * hh + 2 * jj + 1 ? 0x3F800000u : 0u);
    return make_uint4(d[0], d[1], d[2], d[3]);
}


// Tools-only phase clock (-DG2048_DEEP_DIAG=1 builds; see deep_grad_kernel's DEEP_STAMP): deep_forward stamps its
// layer phases into it when the caller passes one (the rollout kernel), an empty type in the product.
constexpr int kDiagSlots = 15;
#if G2048_DEEP_DIAG
struct DiagClock {
    uint64_t ph[kDiagSlots];
    uint64_t last;
    __device__ void stamp(int i) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        ph[i] += t - last;
        last = t;
    }
};
#define FWD_STAMP(dc, i)          \
    do {                          \
        if (dc) (dc)->stamp(i);   \
    } while (0)
#else
struct DiagClock {};
#define FWD_STAMP(dc, i) \
    do {                 \
    } while (0)
#endif

// KSPLIT: the dense layers by dense_fwd_split (the gradient kernel's forward, for the pattern probe).
template <int OBS, int ACT, int KSPLIT = 0>
__device__ void deep_forward(const DeepNet& net, const float* __restrict__ P, DeepSmem& S, float obs_scale,
                             DiagClock* dc = nullptr) {
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31, w = threadIdx.x >> 6;
    // ---- first hidden layer -> S.act[0]
    {
        float* out = S.act[0];
        const int nt0 = net.nt[0];
        if constexpr (OBS == G2048_OBS_ONEHOT) {
            // the one-hot layer-0 arithmetic of every kernel (onehot_l0_tile), W1's plane fragments streamed from the
            // packed net: wave w, unit tiles w, w + 4; per cell one exact one-hot B operand and 3 MFMAs (hi plane
            // into `hi`, the mid and lo planes into `lo`), cell by cell; act((hi + lo) + b1) -- the same bits in
            // rollout, policy, probe and update, and 32 x 16 x 3 fragments of 1 KiB per tile instead of 16 KiB of
            // W1 rows per board gathered from L2.  Fragments stream two cells ahead.
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const uint64_t b = S.board[col];
            const u32x4* fr = reinterpret_cast<const u32x4*>(P + net.wpl) + lane;
            for (int t = w; t < nt0; t += 4) {   // wave-uniform
                const u32x4* ft = fr + (int64_t)t * (kOneHotPlaneFloats / 4);
                float bv[16];
#pragma unroll
                for (int i = 0; i < 16; i++) bv[i] = P[net.b[0] + 32 * t + tile_row(i, h)];
                u32x4 f[3][3];
#pragma unroll
                for (int q = 0; q < 2; q++)
#pragma unroll
                    for (int pl = 0; pl < 3; pl++) f[q][pl] = ft[(q * 3 + pl) * 64];
                floatx16 hi = {}, lo = {};
#pragma unroll
                for (int c = 0; c < 16; c++) {
                    if (c + 2 < 16) {
#pragma unroll
                        for (int pl = 0; pl < 3; pl++) f[(c + 2) % 3][pl] = ft[((c + 2) * 3 + pl) * 64];
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    const uint32_t nib = (uint32_t)(b >> (4 * c)) & 15u;
                    u32x4 dv;
#pragma unroll
                    for (int jj = 0; jj < 4; jj++)
                        dv[jj] = (nib == (uint32_t)(8 * h + 2 * jj) ? 0x3F80u : 0u) |
                                 (nib == (uint32_t)(8 * h + 2 * jj + 1) ? 0x3F800000u : 0u);
                    const bf16x8 bvv = __builtin_bit_cast(bf16x8, dv);
                    hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c % 3][0]), bvv, hi, 0, 0, 0);
                    lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c % 3][1]), bvv, lo, 0, 0, 0);
                    lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c % 3][2]), bvv, lo, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 16; i++)
                    out[(32 * t + tile_row(i, h)) * kActStride + col] = activate<ACT>((hi[i] + lo[i]) + bv[i]);
            }
        } else {
            const uint64_t b = S.board[col];
            float x[8];
#pragma unroll
            for (int s = 0; s < 8; s++) x[s] = obs_value<OBS>(b, 2 * s + h, obs_scale);
            const float* w1f = P + net.w[0];
            for (int t = w; t < nt0; t += 4) {
                floatx16 acc = {};
#pragma unroll
                for (int s = 0; s < 8; s++)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1f[(t * 8 + s) * 64 + lane], x[s], acc, 0, 0, 0);
                const float* bb = P + net.b[0] + 32 * t;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int u = tile_row(r, h);
                    out[(32 * t + u) * kActStride + col] = activate<ACT>(acc[r] + bb[u]);
                }
            }
        }
    }
    __syncthreads();
    FWD_STAMP(dc, 1);
    // ---- dense hidden layers 1 .. L-1 (ping-pong)
    for (int l = 1; l < net.L; l++) {
        const float* in = S.act[(l - 1) & 1];
        float* out = S.act[l & 1];
        const int ntin = net.nt[l - 1], ntout = net.nt[l];
        const float4* __restrict__ frag = reinterpret_cast<const float4*>(P + net.w[l]) + lane;
        const float* bias = P + net.b[l];
        if constexpr (KSPLIT != 0) {
            dense_fwd_split<ACT, kDeepBlock / 64, KSPLIT>(in, out, frag, bias, ntin, ntout, w);
            __syncthreads();
            continue;
        }
        for (int o = w; o < ntout; o += 4) {
            const floatx16 acc = frag_chain(frag + (int64_t)o * ntin * 256, in, 0, ntin, h, col);
            const float* bb = bias + 32 * o;
            float bv[16];   // the 16 bias loads issued before the first use
#pragma unroll
            for (int r = 0; r < 16; r++) bv[r] = bb[tile_row(r, h)];
#pragma unroll
            for (int r = 0; r < 16; r++) out[(32 * o + tile_row(r, h)) * kActStride + col] = activate<ACT>(acc[r] + bv[r]);
        }
        __syncthreads();
    }
    FWD_STAMP(dc, 2);
    // ---- output layer partials: thread (p = tid >> 5, board = tid & 31) sums units [p Hp / 8, (p + 1) Hp / 8)
    {
        const float* in = S.act[(net.L - 1) & 1];
        const int Hp = 32 * net.nt[net.L - 1];
        const int p = threadIdx.x >> 5, bb = threadIdx.x & 31, per = Hp >> 3;
        const float4* wo = reinterpret_cast<const float4*>(P + net.w[net.L]);
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        for (int j = p * per; j < (p + 1) * per; j++) {
            const float x = in[j * kActStride + bb];
            const float4 wv = wo[j];
            s0 = fmaf(x, wv.x, s0);
            s1 = fmaf(x, wv.y, s1);
            s2 = fmaf(x, wv.z, s2);
            s3 = fmaf(x, wv.w, s3);
        }
        S.part[p][bb][0] = s0;
        S.part[p][bb][1] = s1;
        S.part[p][bb][2] = s2;
        S.part[p][bb][3] = s3;
    }
    __syncthreads();
    FWD_STAMP(dc, 3);
}

// ---- 64 boards per workgroup (the one-hot rollout, round 5): one 8-wave workgroup per CU over 64 episode slots
// instead of two 4-wave workgroups of 32 -- every weight fragment (W1 planes, dense layers) is read from L2 once per
// 64 boards instead of once per 32, and the slot owners' step (logits, choice, env step, trajectory row) runs on
// all 64 lanes of wave 0.  The same arithmetic per board as deep_forward (one-hot layer 0 by the plane MFMAs, each
// dense output tile a k-ordered chain, the output partials over the same 8 unit slices), so the rollout stays bit
// for bit the per-step policy path.
constexpr int kAct64 = 65;   // LDS row stride in floats: [unit][64 boards + 1]
struct DeepSmem64 {
    float act[2][256 * kAct64];
    float part[8][64][4];
    uint64_t board[64];
    uint4 oh[32];   // the one-hot B-operand table (onehot_entry), filled at kernel start
};

template <int ACT>
__device__ void deep_forward64(const DeepNet& net, const float* __restrict__ P, DeepSmem64& S, DiagClock* dc) {
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31, w = threadIdx.x >> 6;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    // ---- layer 0: wave w owns unit tile w for both 32-board column tiles (one fragment stream, two B operands;
    //      fragments one cell ahead; the bias is loaded after the chain, beside which the four
    //      accumulator tiles are live)
    {
        float* out = S.act[0];
        const int nt0 = net.nt[0];
        if (w < nt0) {   // wave-uniform
            const int t = w;
            const uint64_t b0 = S.board[col], b1 = S.board[32 + col];
            const u32x4* ft = reinterpret_cast<const u32x4*>(P + net.wpl) + lane + (int64_t)t * (kOneHotPlaneFloats / 4);
            constexpr int kAhead = 1;   // cells of fragments in flight ahead of the MFMAs
            u32x4 f[kAhead + 1][3];
#pragma unroll
            for (int q = 0; q < kAhead; q++)
#pragma unroll
                for (int pl = 0; pl < 3; pl++) f[q][pl] = ft[(q * 3 + pl) * 64];
            floatx16 hi0 = {}, lo0 = {}, hi1 = {}, lo1 = {};
            const auto onehot_b = [&](uint64_t b, int c) {   // from the LDS table (same operand as the compares)
                const uint32_t nib = (uint32_t)(b >> (4 * c)) & 15u;
                return __builtin_bit_cast(bf16x8, S.oh[(nib << 1) | (uint32_t)h]);
            };
#pragma unroll
            for (int c = 0; c < 16; c++) {
                if (c + kAhead < 16) {
#pragma unroll
                    for (int pl = 0; pl < 3; pl++) f[(c + kAhead) % (kAhead + 1)][pl] = ft[((c + kAhead) * 3 + pl) * 64];
                }
                __builtin_amdgcn_sched_barrier(0);
                const bf16x8 x0 = onehot_b(b0, c), x1 = onehot_b(b1, c);
                const int fs = c % (kAhead + 1);
                const bf16x8 wh = __builtin_bit_cast(bf16x8, f[fs][0]), wm = __builtin_bit_cast(bf16x8, f[fs][1]),
                             wl = __builtin_bit_cast(bf16x8, f[fs][2]);
                hi0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, x0, hi0, 0, 0, 0);
                hi1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, x1, hi1, 0, 0, 0);
                lo0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, x0, lo0, 0, 0, 0);
                lo1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, x1, lo1, 0, 0, 0);
                lo0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, x0, lo0, 0, 0, 0);
                lo1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, x1, lo1, 0, 0, 0);
            }
            float bv[16];
#pragma unroll
            for (int i = 0; i < 16; i++) bv[i] = P[net.b[0] + 32 * t + tile_row(i, h)];
#pragma unroll
            for (int i = 0; i < 16; i++) {
                float* o = out + (32 * t + tile_row(i, h)) * kAct64 + col;
                o[0] = activate<ACT>((hi0[i] + lo0[i]) + bv[i]);
                o[32] = activate<ACT>((hi1[i] + lo1[i]) + bv[i]);
            }
        }
    }
    __syncthreads();
    FWD_STAMP(dc, 1);
    // ---- dense layers: item i = (output tile i >> 1, column tile i & 1), items w, w + 8, ..: the two column tiles
    //      of one output tile on neighbouring waves (other SIMDs), so the second read of each fragment hits L1
    for (int l = 1; l < net.L; l++) {
        const float* in = S.act[(l - 1) & 1];
        float* out = S.act[l & 1];
        const int ntin = net.nt[l - 1], ntout = net.nt[l];
        const float4* __restrict__ frag = reinterpret_cast<const float4*>(P + net.w[l]) + lane;
        for (int i = w; i < 2 * ntout; i += 8) {
            const int o = i >> 1, cc = i & 1;
            const floatx16 acc = frag_chain<kAct64>(frag + (int64_t)o * ntin * 256, in + 32 * cc, 0, ntin, h, col);
            const float* bb = P + net.b[l] + 32 * o;
            float bv[16];
#pragma unroll
            for (int r = 0; r < 16; r++) bv[r] = bb[tile_row(r, h)];
#pragma unroll
            for (int r = 0; r < 16; r++) out[(32 * o + tile_row(r, h)) * kAct64 + 32 * cc + col] = activate<ACT>(acc[r] + bv[r]);
        }
        __syncthreads();
    }
    FWD_STAMP(dc, 2);
    // ---- output layer partials: thread (p = tid >> 6, board = tid & 63), units [p Hp / 8, (p + 1) Hp / 8)
    {
        const float* in = S.act[(net.L - 1) & 1];
        const int Hp = 32 * net.nt[net.L - 1];
        const int p = threadIdx.x >> 6, bb = threadIdx.x & 63, per = Hp >> 3;
        const float4* wo = reinterpret_cast<const float4*>(P + net.w[net.L]);
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        for (int j = p * per; j < (p + 1) * per; j++) {
            const float x = in[j * kAct64 + bb];
            const float4 wv = wo[j];
            s0 = fmaf(x, wv.x, s0);
            s1 = fmaf(x, wv.y, s1);
            s2 = fmaf(x, wv.z, s2);
            s3 = fmaf(x, wv.w, s3);
        }
        S.part[p][bb][0] = s0;
        S.part[p][bb][1] = s1;
        S.part[p][bb][2] = s2;
        S.part[p][bb][3] = s3;
    }
    __syncthreads();
    FWD_STAMP(dc, 3);
}

// the 4 outputs of board `bb` from the partials (threads 0..31 after deep_forward)
template <class Smem>
__device__ __forceinline__ void deep_logits(const DeepNet& net, const float* __restrict__ P, const Smem& S, int bb,
                                            float lg[4]) {
    const float* bo = P + net.b[net.L];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        float v = S.part[0][bb][k];
#pragma unroll
        for (int p = 1; p < 8; p++) v += S.part[p][bb][k];
        lg[k] = v + bo[k];
    }
}

struct DeepPolArgs {
    DeepNet net;
    const float* packed;
    const uint64_t* boards;
    const uint32_t* lane_state;   // env lane state words (G2048_LS_ACTIVE, step count) or NULL
    const int32_t* lane_index;    // entry j -> lane lane_index[j] (NULL: lane j)
    uint64_t *rs, *inc, *buf;
    uint64_t key;
    const uint64_t* lane_seed;
    float* probs_out;
    float* logits_out;
    uint8_t* actions;             // NULL: forward only (logits_out / the value of a critic net)
    float obs_scale;
    uint32_t n;
    int use_mask, greedy;
};

__device__ __forceinline__ uint32_t mask_word_of(uint64_t b) {
    const uint32_t m = action_mask(b);   // int8[4] as one word: byte a = bit a
    return (m & 1u) | ((m & 2u) << 7) | ((m & 4u) << 14) | ((m & 8u) << 21);
}

template <int OBS, int ACT, int RNG>
__global__ void __launch_bounds__(kDeepBlock, 2) deep_policy_kernel(DeepPolArgs a) {
    __shared__ DeepSmem S;
    const uint32_t groups = (a.n + 31u) >> 5;
    const int tid = threadIdx.x;
    for (uint32_t gi = blockIdx.x; gi < groups; gi += gridDim.x) {
        const uint32_t j = gi * 32u + (uint32_t)(tid & 31);
        const uint32_t jc = j < a.n ? j : a.n - 1u;
        const uint32_t i = a.lane_index ? (uint32_t)a.lane_index[jc] : jc;
        if (tid < 32) S.board[tid] = a.boards[i];
        __syncthreads();
        deep_forward<OBS, ACT>(a.net, a.packed, S, a.obs_scale);
        if (tid < 32 && j < a.n) {
            const uint32_t ls = a.lane_state ? a.lane_state[i] : G2048_LS_ACTIVE;
            if (ls & G2048_LS_ACTIVE) {
                float lg[4];
                deep_logits(a.net, a.packed, S, tid, lg);
                if (a.logits_out) reinterpret_cast<float4*>(a.logits_out)[i] = make_float4(lg[0], lg[1], lg[2], lg[3]);
                if (a.actions) {
                    const uint32_t mw = a.use_mask ? mask_word_of(S.board[tid]) : 0x01010101u;
                    double u = 0.0;
                    if (!a.greedy) {
                        if constexpr (RNG == G2048_RNG_PCG64) {
                            Pcg64 g;
                            const ulonglong2 sv = reinterpret_cast<const ulonglong2*>(a.rs)[i];
                            const ulonglong2 iv = reinterpret_cast<const ulonglong2*>(a.inc)[i];
                            const uint64_t bf = a.buf[i];
                            g.s_lo = sv.x; g.s_hi = sv.y; g.i_lo = iv.x; g.i_hi = iv.y;
                            g.has_uint32 = (uint32_t)(bf >> 32); g.uinteger = (uint32_t)bf;
                            u = pcg_random(g);
                            reinterpret_cast<ulonglong2*>(a.rs)[i] = make_ulonglong2(g.s_lo, g.s_hi);
                        } else {
                            const uint64_t sd = a.lane_seed ? a.lane_seed[i] : (uint64_t)i;
                            U4 c{(uint32_t)sd, (uint32_t)(sd >> 32), ls & G2048_LS_STEP_MASK, 3u};
                            const U4 r = philox4x32(c, (uint32_t)a.key, (uint32_t)(a.key >> 32));
                            const uint64_t xx = ((uint64_t)r.x << 32) | r.y;
                            u = (double)(xx >> 11) * (1.0 / 9007199254740992.0);
                        }
                    }
                    float p[4];
                    const uint32_t act = softmax_select(lg, mw, a.use_mask != 0, a.greedy != 0, u, p);
                    if (a.probs_out) reinterpret_cast<float4*>(a.probs_out)[i] = make_float4(p[0], p[1], p[2], p[3]);
                    a.actions[i] = (uint8_t)act;
                }
            }
        }
        // S.board is rewritten by threads 0..31 only, after they finished with it; every other LDS buffer is
        // rewritten only after the next group's first barrier
    }
}

// The activations of hidden layer `layer` (the net truncated after it runs deep_forward; its output-layer partials
// are unused): out[j * ld + u] for u < 32 nt[layer] -- bit for bit what deep_grad_kernel computes (dense layers by
// dense_fwd_split when the net's gradient instantiation splits k, else deep_forward's chain), for tests that impose
// the gradient kernel's own activation pattern on an fp64 evaluation.
template <int OBS, int ACT, int KSPLIT>
__global__ void __launch_bounds__(kDeepBlock, 2) deep_hidden_kernel(DeepNet net, const float* packed,
                                                                     const uint64_t* boards, uint32_t n, float obs_scale,
                                                                     float* out, uint32_t ld) {
    __shared__ DeepSmem S;
    const uint32_t groups = (n + 31u) >> 5;
    const int tid = threadIdx.x, layer = net.L - 1, H = 32 * net.nt[layer];
    for (uint32_t gi = blockIdx.x; gi < groups; gi += gridDim.x) {
        if (tid < 32) {
            const uint32_t j = gi * 32u + (uint32_t)tid;
            S.board[tid] = boards[j < n ? j : n - 1u];
        }
        __syncthreads();
        deep_forward<OBS, ACT, KSPLIT>(net, packed, S, obs_scale);
        const float* act = S.act[layer & 1];
        for (int e = tid; e < 32 * H; e += kDeepBlock) {
            const int b = e / H, u = e % H;
            const uint32_t j = gi * 32u + (uint32_t)b;
            if (j < n) out[(size_t)j * ld + u] = act[u * kActStride + b];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------ rollout
// The whole batched rollout (ReinforceAgent.run_episode, src/reinforce_agent.py:195-252, for n (env_seed,
// policy_seed) pairs) for a net of any depth / one-hot obs, in one persistent launch: a workgroup runs 32 episode
// slots, every step is deep_forward over the 32 slots' boards, then the slot owners (lanes 0..31 of wave 0) choose
// (softmax_select on the slot's policy stream), step the env in registers (env_step_pcg, row tables through L1/L2)
// and write the trajectory row; a finished slot takes the next episode from the queue.  Unbounded episodes
// (max_steps None, src/env.py:289-296): an episode that reaches row `cap` without ending is SUSPENDED -- its board,
// counters, running total and both streams are written back per episode and the episode is listed -- and the host
// grows the trajectory buffer and resumes the listed episodes (resume = 1) from row cap on.
struct GLine {
    const uint16_t* p;
    __device__ uint32_t operator()(uint32_t o) const { return p[o]; }
};
struct GCode {
    const uint8_t* p;
    __device__ uint32_t operator()(uint32_t o) const { return (p[o >> 1] >> ((o & 1u) << 2)) & 15u; }
};

struct DeepRollArgs {
    DeepNet net;
    const float* packed;
    const uint8_t* tab;
    RewardCfg rc;
    int64_t max_steps;
    float obs_scale;
    int use_mask, greedy;
    uint64_t* env_rs;
    const uint64_t* env_inc;
    uint64_t* env_buf;
    uint64_t* pol_rs;
    const uint64_t* pol_inc;
    uint64_t* pol_buf;
    uint32_t* next;
    const int32_t* order;
    uint32_t n_order;
    int resume;
    g2048_suspend sus;
    g2048_traj tr;
    uint32_t n, cap;
    uint64_t* diag;   // -DG2048_DEEP_DIAG=1 builds only: per-wave phase cycles (tools/diag_deep.py --rollout)
};

__device__ __forceinline__ Pcg64 load_stream(const uint64_t* rs, const uint64_t* inc, const uint64_t* buf, uint32_t e) {
    Pcg64 g;
    const ulonglong2 s = reinterpret_cast<const ulonglong2*>(rs)[e];
    const ulonglong2 c = reinterpret_cast<const ulonglong2*>(inc)[e];
    const uint64_t bf = buf[e];
    g.s_lo = s.x;
    g.s_hi = s.y;
    g.i_lo = c.x;
    g.i_hi = c.y;
    g.has_uint32 = (uint32_t)(bf >> 32);
    g.uinteger = (uint32_t)bf;
    return g;
}

__device__ __forceinline__ void store_stream(uint64_t* rs, uint64_t* buf, uint32_t e, const Pcg64& g) {
    reinterpret_cast<ulonglong2*>(rs)[e] = make_ulonglong2(g.s_lo, g.s_hi);
    buf[e] = ((uint64_t)g.has_uint32 << 32) | g.uinteger;
}

constexpr uint32_t kNoEpisode = 0xFFFFFFFFu;

// NB = 32: 4-wave workgroups, two per CU, deep_forward; NB = 64 (one-hot nets): one 8-wave workgroup per CU,
// deep_forward64 (above).  Slot owners: lanes 0 .. NB - 1 of wave 0.  Their phase is ~6.9 k of a step's ~47 k
// cycles at 64 slots (the other waves wait for it at the step's first barrier; round 6 stamps, profiles/round6/s5/:
// logits + choice 2.2 k, env step 2.5 k, trajectory row 0.5 k, claim 1.3 k).  Tried in round 6 and not kept
// (runner config, 1M episodes, interleaved on one box, profiles/round6/s6/, s7/): all four actions' row-table reads
// issued before the choice (32 scattered loads per lane: logits + choice 2.2 k -> 6.5 k cycles, rollout 0.241 ->
// 0.263 s); the move by line_move_alu instead of the tables (env step 2.5 k -> 3.0 k, 0.241 -> 0.243 s); the output
// bias from LDS and the fp64 division of k = 3 skipped (0.241 -> 0.242 s).
template <int OBS, int ACT, int NB>
__global__ void __launch_bounds__(NB * 8, NB == 64 ? 1 : 2) deep_rollout_kernel(DeepRollArgs a) {
    static_assert(NB == 32 || (NB == 64 && OBS == G2048_OBS_ONEHOT), "64 slots: one-hot nets");
    typedef typename std::conditional<NB == 64, DeepSmem64, DeepSmem>::type Smem;
    __shared__ Smem S;
    __shared__ int go;
    __shared__ uint32_t park[NB == 64 ? 28 : 1][64];
    const int tid = threadIdx.x;
    if constexpr (NB == 64) {
        if (tid < 32) S.oh[tid] = onehot_entry((uint32_t)tid);   // read after the first forward's barriers
    }
    const bool owner = tid < NB;
    const GLine lut{reinterpret_cast<const uint16_t*>(a.tab)};
    const GCode code{a.tab + 2 * 65536};
    uint32_t ep = kNoEpisode, t = 0, sc = 0, mt = 2;
    uint64_t b = 0;
    double total = 0.0;
    Pcg64 ge{}, gp{};
    bool drained = false;                              // wave-0-uniform: the queue is empty (claims only grow)
    const auto start = [&](uint32_t e) {
        ep = e;
        ge = load_stream(a.env_rs, a.env_inc, a.env_buf, e);
        gp = load_stream(a.pol_rs, a.pol_inc, a.pol_buf, e);
        if (a.resume) {
            b = a.sus.board[e];
            t = a.sus.meta[3 * (size_t)e];
            sc = a.sus.meta[3 * (size_t)e + 1];
            mt = a.sus.meta[3 * (size_t)e + 2];
            total = a.sus.total[e];
        } else {
            b = spawn_pcg(spawn_pcg(0ull, ge), ge);    // Game2048.reset (src/game2048.py:26-34)
            t = 0;
            sc = 0;
            mt = 2;                                   // max_tile_seen = 4 (src/env.py:188)
            total = 0.0;
        }
    };
    const auto claim = [&]() {                         // wave 0 only
        if (drained) return;
        const bool need = owner && ep == kNoEpisode;
        const uint64_t bal = __ballot(need);
        if (!bal) return;
        const int leader = __builtin_ctzll(bal);
        uint32_t base = 0;
        if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(a.next, (uint32_t)__popcll(bal));
        base = (uint32_t)__shfl((int)base, leader, 64);
        const uint32_t idx =
            base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (need && idx < a.n_order) start(a.order ? (uint32_t)a.order[idx] : idx);
        drained = __ballot(need && idx >= a.n_order) != 0ull;
    };
#if G2048_DEEP_DIAG
    DiagClock dclk{};
    dclk.last = __builtin_amdgcn_s_memtime();
    DiagClock* dc = a.diag ? &dclk : nullptr;
#else
    DiagClock* dc = nullptr;
#endif
    if (tid < 64) claim();
    while (true) {
        if (tid < 64) {
            const uint64_t live = __ballot(owner && ep != kNoEpisode);
            if (tid == 0) go = live != 0ull;
            if (owner) S.board[tid] = ep != kNoEpisode ? b : 0ull;
        }
        __syncthreads();
        FWD_STAMP(dc, 0);
        if (!go) break;                                // block-uniform
        if constexpr (NB == 64) {
            // the slots' episode state (28 words) parked in LDS across the forward and read back by every thread
            // (the non-owners' copies are never used), so its registers are free for the forward's fragment
            // windows -- the 8-wave kernel is at 256 VGPRs
            const int sl = tid & 63;
            const auto put = [&](int k, uint32_t v) { park[k][sl] = v; };
            const auto put64 = [&](int k, uint64_t v) { put(k, (uint32_t)v); put(k + 1, (uint32_t)(v >> 32)); };
            if (owner) {
                put(0, ep); put(1, t); put(2, sc); put(3, mt);
                put64(4, b); put64(6, (uint64_t)__double_as_longlong(total));
                put64(8, ge.s_lo); put64(10, ge.s_hi); put64(12, ge.i_lo); put64(14, ge.i_hi);
                put(16, ge.has_uint32); put(17, ge.uinteger);
                put64(18, gp.s_lo); put64(20, gp.s_hi); put64(22, gp.i_lo); put64(24, gp.i_hi);
                put(26, gp.has_uint32); put(27, gp.uinteger);
            }
            deep_forward64<ACT>(a.net, a.packed, S, dc);   // (its barriers order the parking)
            const auto get = [&](int k) { return park[k][sl]; };
            const auto get64 = [&](int k) { return (uint64_t)get(k) | ((uint64_t)get(k + 1) << 32); };
            ep = get(0); t = get(1); sc = get(2); mt = get(3);
            b = get64(4); total = __longlong_as_double((long long)get64(6));
            ge.s_lo = get64(8); ge.s_hi = get64(10); ge.i_lo = get64(12); ge.i_hi = get64(14);
            ge.has_uint32 = get(16); ge.uinteger = get(17);
            gp.s_lo = get64(18); gp.s_hi = get64(20); gp.i_lo = get64(22); gp.i_hi = get64(24);
            gp.has_uint32 = get(26); gp.uinteger = get(27);
        } else {
            deep_forward<OBS, ACT>(a.net, a.packed, S, a.obs_scale, dc);
        }
        if (owner && ep != kNoEpisode) {
            float lg[4];
            deep_logits(a.net, a.packed, S, tid, lg);
            const uint32_t mw = a.use_mask ? mask_word_of(b) : 0x01010101u;
            const double u = a.greedy ? 0.0 : pcg_random(gp);
            float p[4];
            const uint32_t act = softmax_select(lg, mw, a.use_mask != 0, a.greedy != 0, u, p);
            FWD_STAMP(dc, 6);
            const StepValues ov = env_step_pcg(b, act, sc, mt, ge, a.rc, a.max_steps, lut, code);
#if G2048_DEEP_DIAG
            asm volatile("" ::"v"(ov.board), "v"(ov.reward), "v"(ov.flags));
#endif
            FWD_STAMP(dc, 7);
            const size_t row = (size_t)t * a.n + ep;
            a.tr.boards[row] = b;
            a.tr.actions[row] = (uint8_t)act;
            a.tr.rewards[row] = ov.reward;
            a.tr.flags[row] = (uint8_t)ov.flags;
            if (a.tr.probs) reinterpret_cast<float4*>(a.tr.probs)[row] = make_float4(p[0], p[1], p[2], p[3]);
            total += ov.reward;                        // total_reward += float(reward) (src/reinforce_agent.py:233)
            b = ov.board;
            t += 1;
            if ((ov.flags & (kFTerminated | kFTruncated)) != 0u) {
                a.tr.lengths[ep] = (int32_t)t;
                a.tr.totals[ep] = total;
                a.tr.max_tile[ep] = (uint8_t)mt;
                a.tr.final_board[ep] = b;
                ep = kNoEpisode;
            } else if (t >= a.cap) {                   // out of trajectory rows: suspend for the host to resume
                store_stream(a.env_rs, a.env_buf, ep, ge);
                store_stream(a.pol_rs, a.pol_buf, ep, gp);
                a.sus.board[ep] = b;
                a.sus.meta[3 * (size_t)ep] = t;
                a.sus.meta[3 * (size_t)ep + 1] = sc;
                a.sus.meta[3 * (size_t)ep + 2] = mt;
                a.sus.total[ep] = total;
                a.sus.list[atomicAdd(a.sus.count, 1u)] = (int32_t)ep;
                ep = kNoEpisode;
            }
            FWD_STAMP(dc, 8);
        }
        FWD_STAMP(dc, 4);
        if (tid < 64) claim();
        FWD_STAMP(dc, 5);
#if G2048_DEEP_DIAG
        dclk.ph[kDiagSlots - 1] += 1;
#endif
    }
#if G2048_DEEP_DIAG
    if (a.diag && (tid & 63) == 0) {
        uint64_t* slot = a.diag + ((size_t)blockIdx.x * (NB / 8) + (tid >> 6)) * kDiagSlots;
#pragma unroll
        for (int i = 0; i < kDiagSlots; i++) slot[i] += dclk.ph[i];
    }
#endif
}

// ------------------------------------------------------------------------------------ update (fused, any depth)
// The actor / critic branch of update_batch (src/reinforce_agent.py:403-555; _backpropagation :639-678) for a net
// of any depth whose dense weight-gradient tiles fit the workgroup's accumulator registers (see kGradTilesPerWave):
// one 512-thread workgroup (8 waves, 2 per SIMD) per CU takes 32 samples at a time --
//   * forward as deep_forward, every hidden layer's activations kept in LDS ([unit][sample], stride 33);
//   * g = (onehot(a) - p) coef (actor: masked softmax of the logits) or dL/dV coef (critic: MSE / Huber on V - target);
//   * output layer on VALU: dW_out += a^T g per thread (unit = thread), delta = (W_out g) act'(a) in place;
//   * each dense layer l (top down): dW_l += a_{l-1}^T delta_l on v_mfma_f32_32x32x2_f32 with the 32 samples as the
//     contraction (A = a_{l-1}, B = delta_l, both from LDS), accumulated in registers across the workgroup's groups
//     (tile f of the flattened tile list belongs to wave f % 8); then delta_{l-1} = (W_l delta_l) act'(a_{l-1}) as
//     the forward's MFMA chain on the backward fragments (W_l in A-fragment order, streamed from L2), written over
//     a_{l-1} in LDS;
//   * first layer: log2 / raw obs: dW_0 += x^T delta_0 on MFMA (x rebuilt from the boards); one-hot obs: delta_0 is
//     written out ([n][H0p], row-major) for g2048_onehot_dw1's bf16 MFMA;
//   * biases: per-thread sums (unit = thread).
// Every workgroup writes one fp32 partial slab (g2048_fold_partials sums them in fp64).
// Three instantiations by the net's dense dW tile count (deep_grad_variant), every one at two waves per SIMD so that
// one wave's MFMA chains run while the other's gathers, epilogues and barriers do:
//   * NB = 64, NW = 8, TPW = 5 (one-hot nets of <= 40 tiles whose LDS fits 160 KiB at 64 samples: the runner config's
//     [256, 128, 64] has exactly 40 tiles; round 6): one 8-wave workgroup per CU on 64-sample groups (two 32-sample
//     column tiles, LDS rows of 65 floats) -- every weight fragment (W1 planes, forward and backward dense
//     fragments) is read from L2 once per 64 samples instead of 32, the two column tiles of one output tile on
//     neighbouring waves (the second read hits L1), and a group's barriers are paid once per 64 samples; each dW tile
//     contracts over 64 samples (32 k-steps) in its 5-tile register budget.  Every output tile of a dense layer is the
//     plain k-ordered chain (deep_forward's), so its activations are bit for bit the rollout / policy kernels'.
//     Runner config, 1M episodes, interleaved on one box: update 1.1524-1.1553 s against 1.1784-1.1808 s for round
//     5's two 4-wave workgroups per CU on 32-sample groups (NW = 4, TPW = 10; profiles/round6/r7n/), which it
//     replaces (no net reaches that form's LDS bound without exceeding this one's).
//   * NW = 8, TPW = 6 (<= 48 tiles): 32-sample groups on one 8-wave workgroup per CU (round 4); dense layers with
//     fewer than 8 output tiles split k in two halves (dense_fwd_split) to keep the idle waves busy.
//   * NW = 8, TPW = 8 (<= 64 tiles: one-hot / log2 [256, 256] and [256, 256, x] nets, round 5): as above with 128
//     accumulator registers per wave.
// (A 4-wave workgroup alone per CU with 12 tiles per wave took the whole register file, one wave per SIMD.)
constexpr int kDeepGradMaxBlock = 512;
// Tried, not kept (measured on the runner config; the A/B switches are gone from the source): the 4-wave
// instantiation's 64-unit layer as a 4-way k split (no change, round 5); log2 / raw nets of 49..64 dense tiles on the 8 x 8
// instantiation (spills ~300 VGPRs; the two-layer cooperative kernel runs them); the delta_0 rows by 16-byte stores
// (a quarter of the store instructions): 1.2535-1.2542 s against 1.2499-1.2517 s (profiles/round6/r7b/d0b128_*).
// The one-hot layer 0 is computed here (onehot_l0_tile) since round 6: with the per-phase lane ids below the kernel
// no longer spills, and the fused form measured equal to reading back a separate layer-0 kernel's 1 KiB / sample
// blocks (1.2167-1.2200 s against 1.2167-1.2181 s, profiles/round6/r7f/; it had been 2 % slower while it spilled 30
// VGPRs, r7a/l0fused_*), so that kernel and its 2 KiB / sample-pass of HBM traffic are gone.

// One unit tile t of a one-hot layer 0 for 32 boards (lane col: board b) by the exact bf16-plane MFMAs: per cell one
// exact one-hot B operand, hi plane into `hi`, mid and lo planes into `lo` (deep_forward's arithmetic, the same
// bits), W1's plane fragments streamed from the packed net one cell ahead, the bias loaded after the chain; writes
// act((hi + lo) + b1) to out[unit * stride + col].  The gradient kernel's layer 0.  (Two cells ahead -- with one
// accumulator to fit the registers -- measured the same: 1.175-1.180 s against 1.179-1.180 s, profiles/round6/r7k/.)
template <int ACT>
__device__ __forceinline__ void onehot_l0_tile(const float* __restrict__ P, const DeepNet& net, int t, uint64_t b,
                                               float* out, int stride) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    int tq = (int)threadIdx.x;
    asm volatile("" : "+v"(tq));   // lane ids derived here, not hoisted out of the caller's group loop
    const int lane = tq & 63, h = lane >> 5, col = lane & 31;
    const u32x4* ft = reinterpret_cast<const u32x4*>(P + net.wpl) + lane + (int64_t)t * (kOneHotPlaneFloats / 4);
    u32x4 f[2][3];
#pragma unroll
    for (int pl = 0; pl < 3; pl++) f[0][pl] = ft[pl * 64];
    floatx16 hi = {}, lo = {};
#pragma unroll
    for (int c = 0; c < 16; c++) {
        if (c + 1 < 16) {
#pragma unroll
            for (int pl = 0; pl < 3; pl++) f[(c + 1) & 1][pl] = ft[((c + 1) * 3 + pl) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t nib = (uint32_t)(b >> (4 * c)) & 15u;
        u32x4 dv;
#pragma unroll
        for (int jj = 0; jj < 4; jj++)
            dv[jj] = (nib == (uint32_t)(8 * h + 2 * jj) ? 0x3F80u : 0u) | (nib == (uint32_t)(8 * h + 2 * jj + 1) ? 0x3F800000u : 0u);
        const bf16x8 bvv = __builtin_bit_cast(bf16x8, dv);
        hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c & 1][0]), bvv, hi, 0, 0, 0);
        lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c & 1][1]), bvv, lo, 0, 0, 0);
        lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c & 1][2]), bvv, lo, 0, 0, 0);
    }
    float bv[16];
#pragma unroll
    for (int i = 0; i < 16; i++) bv[i] = P[net.b[0] + 32 * t + tile_row(i, h)];
#pragma unroll
    for (int i = 0; i < 16; i++) out[(32 * t + tile_row(i, h)) * stride + col] = activate<ACT>((hi[i] + lo[i]) + bv[i]);
}

// The same for CT column tiles of 32 boards (the 64-sample gradient groups): one fragment stream, CT B operands
// (as deep_forward64).  (A separate function: the CT = 1 case written this way compiled to other registers and made
// round 5's 4 x 10 gradient kernel spill 22 VGPRs.)  Two cells ahead spills 5 VGPRs and measured slower: 1.169-1.172 s
// against 1.150-1.153 s (profiles/round6/r7p/).  With `oh` (the gradient kernel's 64-sample form) the B operands come
// from the LDS table of onehot_entry instead of the compares and selects (~20 VALU per cell and column tile): update
// 1.133-1.138 -> 1.121-1.124 s on one box (profiles/round6/s2/).
template <int ACT, int CT>
__device__ __forceinline__ void onehot_l0_tile_cols(const float* __restrict__ P, const DeepNet& net, int t,
                                               const uint64_t (&b)[CT], float* out, int stride,
                                               const uint4* oh = nullptr) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    int tq = (int)threadIdx.x;
    asm volatile("" : "+v"(tq));   // lane ids derived here, not hoisted out of the caller's group loop
    const int lane = tq & 63, h = lane >> 5, col = lane & 31;
    const u32x4* ft = reinterpret_cast<const u32x4*>(P + net.wpl) + lane + (int64_t)t * (kOneHotPlaneFloats / 4);
    u32x4 f[2][3];
#pragma unroll
    for (int pl = 0; pl < 3; pl++) f[0][pl] = ft[pl * 64];
    floatx16 hi[CT], lo[CT];
#pragma unroll
    for (int cc = 0; cc < CT; cc++) hi[cc] = lo[cc] = floatx16{};
#pragma unroll
    for (int c = 0; c < 16; c++) {
        if (c + 1 < 16) {
#pragma unroll
            for (int pl = 0; pl < 3; pl++) f[(c + 1) & 1][pl] = ft[((c + 1) * 3 + pl) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 bvv[CT];
#pragma unroll
        for (int cc = 0; cc < CT; cc++) {
            const uint32_t nib = (uint32_t)(b[cc] >> (4 * c)) & 15u;
            if (oh) {   // the table (same operand as the compares)
                bvv[cc] = __builtin_bit_cast(bf16x8, oh[(nib << 1) | (uint32_t)h]);
                continue;
            }
            u32x4 dv;
#pragma unroll
            for (int jj = 0; jj < 4; jj++)
                dv[jj] = (nib == (uint32_t)(8 * h + 2 * jj) ? 0x3F80u : 0u) | (nib == (uint32_t)(8 * h + 2 * jj + 1) ? 0x3F800000u : 0u);
            bvv[cc] = __builtin_bit_cast(bf16x8, dv);
        }
#pragma unroll
        for (int cc = 0; cc < CT; cc++)
            hi[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c & 1][0]), bvv[cc], hi[cc], 0, 0, 0);
#pragma unroll
        for (int cc = 0; cc < CT; cc++)
            lo[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c & 1][1]), bvv[cc], lo[cc], 0, 0, 0);
#pragma unroll
        for (int cc = 0; cc < CT; cc++)
            lo[cc] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f[c & 1][2]), bvv[cc], lo[cc], 0, 0, 0);
    }
    float bv[16];
#pragma unroll
    for (int i = 0; i < 16; i++) bv[i] = P[net.b[0] + 32 * t + tile_row(i, h)];
#pragma unroll
    for (int cc = 0; cc < CT; cc++)
#pragma unroll
        for (int i = 0; i < 16; i++)
            out[(32 * t + tile_row(i, h)) * stride + 32 * cc + col] = activate<ACT>((hi[cc][i] + lo[cc][i]) + bv[i]);
}

struct DeepGradVariant {
    int nw, tpw, ksplit, per_cu, passes;   // passes > 1: the dense dW tiles in ranges of nw x tpw, one launch each
    int nb = 32;                           // samples per group
};

struct DeepGradArgs {
    DeepNet net;
    const float* packed;          // forward layout (g2048_deep_pack)
    const float* bpacked;         // backward fragments (g2048_deep_grad_pack)
    int64_t boff[kMaxHidden];     // per dense layer l >= 1: offset of its backward fragments
    int64_t pw[kMaxHidden + 1], pb[kMaxHidden + 1];   // partial-slab offsets: dW_l, db_l (l = L: the output layer)
    int64_t pslab;                // floats per partial slab
    const uint64_t* boards;
    const uint8_t* actions;
    const float* coef;            // actor: advantage x step weight; critic: step weight
    int critic, huber;
    float huber_delta;
    const float* target;          // critic: r + gamma V(s') m
    float* delta_out;             // critic: target - V (NULL ok)
    float* v_out;                 // critic: V (NULL ok)
    float* d0_out;                // one-hot: delta_0 [n][H0p] for g2048_onehot_dw1
    g2048_td_rows td;             // has_td: the critic's target and V(s) through lane-indexed values
    int has_td;
    float* part;                  // [gridDim.x][pslab]
    float obs_scale;
    uint32_t n;
    int use_mask;
    int ntiles;                   // dense dW tiles in all
    int tile_begin[kMaxHidden];   // flattened tile index of layer l's first tile (l >= 1)
    int aoff[kMaxHidden];         // LDS float offset of layer l's activations / deltas
    int lds_tail;                 // LDS float offset of the output partials, g, boards and bias sums
    uint64_t* diag;               // -DG2048_DEEP_DIAG=1 builds only (tools/diag_deep.py): per-wave phase cycles
    int tile0;                    // this launch's dense dW tiles: [tile0, tile0 + NW TPW) (nets past one pass)
    int first_pass, last_pass;    // first: writes the bias / output-layer / first-layer partials; last: delta_0 rows
};

// Phase-time attribution (tools-only build, -DG2048_DEEP_DIAG=1): each wave adds the s_memtime cycles of every
// phase (ending at the barrier that closes it, so a phase includes waiting for the slowest wave) to its own slot
// diag[(block * NW + wave) * kDiagSlots + phase]; slot kDiagSlots - 1 counts the groups.  No stamp in the product.
#if G2048_DEEP_DIAG
#define DEEP_STAMP(i)                                             \
    do {                                                          \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();         \
        dph[i] += t_ - dlast;                                     \
        dlast = t_;                                               \
    } while (0)
#else
#define DEEP_STAMP(i) \
    do {              \
    } while (0)
#endif

// The gradient kernel's in-loop barriers order LDS accesses only: a raw s_barrier behind lgkmcnt(0).
// __syncthreads() adds a workgroup release fence, i.e. vmcnt(0): every barrier would wait for the wave's global
// stores (the V(s) / delta_0 rows) and for the weight-fragment loads a chain's window left in flight, none of which
// another wave reads (loaded values are waited for at their use, as always).  The group's first barrier keeps
// __syncthreads() (the loads of the group's inputs).  (__syncthreads() everywhere measured the same, round 5; the
// group's first barrier and the 64-slot rollout's barriers as LDS-only ones measured the same too, round 6 r7l/.)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int ACT>
__device__ __forceinline__ float act_deriv(float a) {   // from the activation (src/reinforce_agent.py:624-636)
    if constexpr (ACT == 0) return a > 0.0f ? 1.0f : 0.0f;
    else return a * (1.0f - a);
}

// threadIdx.x through an empty asm: every call is a new value to the compiler, so the per-lane LDS / global
// addresses a phase derives from it are computed in that phase -- derived once from threadIdx.x, hipcc hoisted them
// out of the group loop and kept them live across all of it, and the 4 x 10 instantiation spilled them to scratch
// (whose reloads, vector-memory ops, then waited behind the in-order vmcnt of the phase's stores / LDS-DMA)
__device__ __forceinline__ int fresh_tid() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
#define DEEP_LANE_IDS                                                                    \
    const int tid = fresh_tid(), lane = tid & 63, h = lane >> 5, col = lane & 31; \
    (void)lane;                                                                          \
    (void)h;                                                                             \
    (void)col

template <int OBS, int ACT, int NW, int TPW, int KSPLIT, int NB = 32>
__global__ void __launch_bounds__(64 * NW, 8 / NW) deep_grad_kernel(DeepGradArgs a) {
    static_assert(NB == 32 || (NB == 64 && NW == 8 && KSPLIT == 0 && OBS == G2048_OBS_ONEHOT), "64-sample groups");
    constexpr int kBlock = 64 * NW;
    constexpr int SS = NB + 1;    // LDS row stride in floats: [unit][NB samples + 1]
    constexpr int CT = NB / 32;   // 32-sample column tiles per group
    extern __shared__ float dyn[];
    const DeepNet& net = a.net;
    const int L = net.L;
    // w through readfirstlane: the wave index and everything derived from it (tile ranges, LDS bases) live in
    // SGPRs -- as a per-lane value hipcc kept them in VGPRs and the 4 x 10 instantiation spilled 41 of them
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31,
              w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // LDS: the hidden layers' activations (deltas overwrite them top down; layer l at aoff[l]), the output
    // partials, g, the boards and each thread's bias-gradient sums
    const auto actl = [&](int l) { return dyn + a.aoff[l]; };
    float* lds_end = dyn + a.lds_tail;
    float (*part)[NB][4] = reinterpret_cast<float (*)[NB][4]>(lds_end);          // [8][NB][4]
    float (*gs)[4] = reinterpret_cast<float (*)[4]>(lds_end + 8 * NB * 4);       // [NB][4]
    uint64_t* bds = reinterpret_cast<uint64_t*>(lds_end + 8 * NB * 4 + NB * 4);  // [NB]
    float* dbs = lds_end + 8 * NB * 4 + NB * 4 + 2 * NB;                         // [kMaxHidden][256]: db_l of unit tid
    float* wol = dbs + kMaxHidden * 256;                                         // [HL][4] output weights, then [4] bias
    // the group's per-sample inputs (coef, action, target / TD row: [7][32]) and the db_out sums ([32][4]) in LDS
    // instead of registers across the forward and delta chains (round 5: 29 -> 16 spilled VGPRs)
    float* smp_in = wol + 256 * 4 + 4;
    float* dbo_l = smp_in + 7 * NB;
    // (64-sample form) the one-hot B-operand table (onehot_entry), as the 64-slot rollout's layer 0
    const uint4* ohl = reinterpret_cast<const uint4*>(dbo_l + 4 * NB);
    if (tid < 256)
        for (int l = 0; l < kMaxHidden; l++) dbs[l * 256 + tid] = 0.0f;
    if (tid < 4 * NB) dbo_l[tid] = 0.0f;
    const float* P = a.packed;
    {   // the output layer's weights and bias in LDS for the whole launch (its phases read them every group)
        const int HLw = 32 * net.nt[L - 1] * 4;
        for (int i = tid; i < HLw + 4; i += kBlock) wol[i] = i < HLw ? P[net.w[L] + i] : P[net.b[L] + (i - HLw)];
    }
    floatx16 acc[TPW];
#pragma unroll
    for (int k = 0; k < TPW; k++) acc[k] = floatx16{};
    constexpr int kA0 = 8 / NW;   // log2 / raw first layer: dW_0^T tiles t = w + NW i
    floatx16 acc0[kA0];
#pragma unroll
    for (int i = 0; i < kA0; i++) acc0[i] = floatx16{};
    // dW_out / db_{L-1} partials of this thread's (unit, sample range); db_out: threads 0..31 sum their sample slot's
    // g over the groups (the slots are added in order at the end)
    float dwo[4] = {0.f, 0.f, 0.f, 0.f}, dbl = 0.f;
    const int HL = 32 * net.nt[L - 1];
    const int oq = kBlock / HL, oper = (NB + oq - 1) / oq;   // sample ranges of the output layer
    const float4* wout = reinterpret_cast<const float4*>(wol);
    const float* bo = wol + 4 * HL;
    const uint32_t groups = (a.n + (uint32_t)(NB - 1)) / (uint32_t)NB;
    // A group's per-sample inputs (threads 0..NB-1): board, coefficient, action, critic target or TD row.  The
    // 64-sample form loads group g + gridDim.x's at the end of group g, ahead of g's delta_0 stores, and puts them in
    // LDS behind those stores: the loads are older than the stores in the in-order vmcnt, so neither the next
    // group's top nor this group's end drains the stores or waits a full load latency (the 32-sample forms load at
    // the group's top behind a fence).  Round 6: the group top's 2.7 k cycles (of 104 k) -> 0.3 k; runner-config 1M
    // update 1.168-1.172 -> 1.133-1.138 s on one box (profiles/round6/s2/).
    struct GroupIn {
        uint64_t board;
        float cf, tg, td_r, td_h;
        uint32_t act;
        int64_t td_l;
        bool valid;
    };
    const auto load_in = [&](uint32_t g) {
        GroupIn v{0ull, 0.0f, 0.0f, 0.0f, 0.0f, 0u, 0, false};
        const int t = fresh_tid();
        if (t < NB && a.n > 0) {
            const uint32_t j = g * (uint32_t)NB + (uint32_t)t;
            const bool valid = j < a.n;
            const uint32_t jc = valid ? j : a.n - 1u;
            // every field loaded from valid memory whatever the launch's mode, then selected: no branch per mode,
            // so the loads issue together (merged per-mode paths made the wait-count pass drain the board and
            // coefficient loads before the action load was issued)
            const uint8_t* pact = a.critic ? reinterpret_cast<const uint8_t*>(a.boards) : a.actions;
            const float* ptg = a.critic && !a.has_td ? a.target : a.coef;
            const int64_t* ptl = a.has_td ? a.td.lane : reinterpret_cast<const int64_t*>(a.boards);
            const float* ptr = a.has_td ? a.td.reward : a.coef;
            const float* pth = a.has_td ? a.td.has_next : a.coef;
            // raw values here, the selects at put_in: a select next to its load would wait for the load there
            v.board = a.boards[jc];
            v.cf = a.coef[jc];
            v.tg = ptg[jc];
            v.td_r = ptr[jc];
            v.td_h = pth[jc];
            v.act = pact[jc];
            v.td_l = ptl[jc];
            v.valid = valid;
        }
        return v;
    };
    const auto put_in = [&](const GroupIn& v) {
        const int t = fresh_tid();
        if (t < NB) {
            const bool use_tg = a.critic && !a.has_td;
            const int64_t tl = a.has_td ? v.td_l : 0;
            bds[t] = v.valid ? v.board : 0ull;
            smp_in[t] = v.valid ? v.cf : 0.0f;
            smp_in[NB + t] = __uint_as_float(a.critic ? 0u : v.act);
            smp_in[2 * NB + t] = use_tg ? v.tg : 0.0f;
            smp_in[3 * NB + t] = a.has_td ? v.td_r : 0.0f;
            smp_in[4 * NB + t] = a.has_td ? v.td_h : 0.0f;
            smp_in[5 * NB + t] = __uint_as_float((uint32_t)tl);
            smp_in[6 * NB + t] = __uint_as_float((uint32_t)((uint64_t)tl >> 32));
        }
    };
    if constexpr (NB == 64) {
        if (tid < 32) const_cast<uint4*>(ohl)[tid] = onehot_entry((uint32_t)tid);
        put_in(load_in(blockIdx.x));
        __syncthreads();   // (also orders the LDS initialisation above)
    }
#if G2048_DEEP_DIAG
    uint64_t dph[kDiagSlots] = {};
    uint64_t dlast = __builtin_amdgcn_s_memtime();
#endif
    for (uint32_t gi = blockIdx.x; gi < groups; gi += gridDim.x) {
        float td_v = 0.0f;   // V(s') of the critic's TD row (loaded after layer 0, used at the logits)
        if constexpr (NB != 64) {
            DEEP_LANE_IDS;
            const uint32_t j = gi * (uint32_t)NB + (uint32_t)(tid & (NB - 1));
            const bool valid = j < a.n;
            const uint32_t jc = valid ? j : a.n - 1u;
            if (tid < NB) bds[tid] = valid ? a.boards[j] : 0ull;
            // the sample's coefficient / action / target, loaded now so that the forward covers their latency
            const float cf = (tid < NB && valid) ? a.coef[jc] : 0.0f;
            const uint32_t act_j = (tid < NB && !a.critic) ? a.actions[jc] : 0u;
            // the critic's target, or (TD rows) its reward / has-next / lane now and V(s') once layer 0 is done (the
            // lane index has arrived by then: no dependent load in front of the first barrier)
            float tg = 0.0f, td_r = 0.0f, td_h = 0.0f;
            int64_t td_l = 0;
            if (tid < NB && a.critic) {
                if (a.has_td) {
                    td_l = a.td.lane[jc];
                    td_r = a.td.reward[jc];
                    td_h = a.td.has_next[jc];
                } else {
                    tg = a.target[jc];
                }
            }
            __syncthreads();   // (a fence: vmcnt(0) -- the loads above have arrived)
            if (tid < NB) {   // read back at the logits: their registers are free until then
                smp_in[tid] = cf;
                smp_in[NB + tid] = __uint_as_float(act_j);
                smp_in[2 * NB + tid] = tg;
                smp_in[3 * NB + tid] = td_r;
                smp_in[4 * NB + tid] = td_h;
                smp_in[5 * NB + tid] = __uint_as_float((uint32_t)td_l);
                smp_in[6 * NB + tid] = __uint_as_float((uint32_t)((uint64_t)td_l >> 32));
            }
        }
        DEEP_STAMP(0);
        // ---- forward: layer 0
        {
            DEEP_LANE_IDS;
            float* out = actl(0);
            const int nt0 = net.nt[0];
            if constexpr (OBS == G2048_OBS_ONEHOT) {
                if constexpr (CT == 1) {
                    for (int t = w; t < nt0; t += NW) onehot_l0_tile<ACT>(P, net, t, bds[col], out, SS);
                } else {
                    uint64_t bc[CT];
#pragma unroll
                    for (int cc = 0; cc < CT; cc++) bc[cc] = bds[32 * cc + col];
                    for (int t = w; t < nt0; t += NW) onehot_l0_tile_cols<ACT, CT>(P, net, t, bc, out, SS, ohl);
                }
            } else {
                const uint64_t b = bds[col];
                float x[8];
#pragma unroll
                for (int s2 = 0; s2 < 8; s2++) x[s2] = obs_value<OBS>(b, 2 * s2 + h, a.obs_scale);
                const float* w1f = P + net.w[0];
                for (int t = w; t < nt0; t += NW) {
                    floatx16 c = {};
#pragma unroll
                    for (int s2 = 0; s2 < 8; s2++)
                        c = __builtin_amdgcn_mfma_f32_32x32x2f32(w1f[(t * 8 + s2) * 64 + lane], x[s2], c, 0, 0, 0);
                    const float* bb = P + net.b[0] + 32 * t;
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        const int u = tile_row(r, h);
                        out[(32 * t + u) * SS + col] = activate<ACT>(c[r] + bb[u]);
                    }
                }
            }
        }
        lds_barrier();
        DEEP_STAMP(1);
        {
            DEEP_LANE_IDS;
            if (tid < NB && a.critic && a.has_td) {
                const int64_t tl = (int64_t)((uint64_t)__float_as_uint(smp_in[5 * NB + tid]) |
                                             ((uint64_t)__float_as_uint(smp_in[6 * NB + tid]) << 32));
                td_v = a.td.v_next[tl];
            }
        }
        // ---- forward: dense layers (each into its own region)
        for (int l = 1; l < L; l++) {
            DEEP_LANE_IDS;
            const float* in = actl(l - 1);
            float* out = actl(l);
            const int ntin = net.nt[l - 1], ntout = net.nt[l];
            const float4* __restrict__ frag = reinterpret_cast<const float4*>(P + net.w[l]) + lane;
            if constexpr (KSPLIT != 0) {
                dense_fwd_split<ACT, NW, KSPLIT>(in, out, frag, P + net.b[l], ntin, ntout, w);
            } else {   // deep_forward's chain: the rollout / policy kernels' bits
                // item i = (output tile i / CT, column tile i % CT): the column tiles of one output tile on
                // neighbouring waves, so the second read of each fragment hits L1 (as deep_forward64)
                for (int i = w; i < CT * ntout; i += NW) {
                    const int o = i >> (CT - 1), cc = i & (CT - 1);
                    const floatx16 c = frag_chain<SS>(frag + (int64_t)o * ntin * 256, in + 32 * cc, 0, ntin, h, col);
                    const float* bb = P + net.b[l] + 32 * o;
                    float bv[16];
#pragma unroll
                    for (int r = 0; r < 16; r++) bv[r] = bb[tile_row(r, h)];
#pragma unroll
                    for (int r = 0; r < 16; r++) out[(32 * o + tile_row(r, h)) * SS + 32 * cc + col] = activate<ACT>(c[r] + bv[r]);
                }
            }
            lds_barrier();
            DEEP_STAMP(l == 1 ? 2 : 9);
        }
        // ---- output layer partials (as deep_forward; threads 0..255).  (Round 6: the same sums from the last dense
        //      layer's epilogue registers, the chain handed across the lane halves -- same bits, no pass and barrier
        //      here -- measured 0.4 % slower: the epilogue lengthens the 2-tile layer's waves while the pass here
        //      uses all four; profiles/round6/r7c/, r7d/)
        {
            DEEP_LANE_IDS;
            if (tid < 8 * NB) {
                const float* in = actl(L - 1);
                const int pp = tid >> (CT + 4), bb = tid & (NB - 1), per = HL >> 3;
                float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
                if (per == 8) {   // a 64-unit last layer: the slice's 8 reads in flight, then the same chain
                    float x[8];
                    float4 wv[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        x[i] = in[(8 * pp + i) * SS + bb];
                        wv[i] = wout[8 * pp + i];
                    }
                    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        s0 = fmaf(x[i], wv[i].x, s0);
                        s1 = fmaf(x[i], wv[i].y, s1);
                        s2 = fmaf(x[i], wv[i].z, s2);
                        s3 = fmaf(x[i], wv[i].w, s3);
                    }
                } else
                for (int u = pp * per; u < (pp + 1) * per; u++) {
                    const float x = in[u * SS + bb];
                    const float4 wv = wout[u];
                    s0 = fmaf(x, wv.x, s0);
                    s1 = fmaf(x, wv.y, s1);
                    s2 = fmaf(x, wv.z, s2);
                    s3 = fmaf(x, wv.w, s3);
                }
                part[pp][bb][0] = s0;
                part[pp][bb][1] = s1;
                part[pp][bb][2] = s2;
                part[pp][bb][3] = s3;
            }
            lds_barrier();
        }
        DEEP_STAMP(3);
        // ---- logits -> g (threads 0..31, one sample each)
        {
            DEEP_LANE_IDS;
            const uint32_t j = gi * (uint32_t)NB + (uint32_t)(tid & (NB - 1));
            const bool valid = j < a.n;
            if (tid < NB) {
                const float cf_ = smp_in[tid];
                const uint32_t act_j_ = __float_as_uint(smp_in[NB + tid]);
                float tg_ = smp_in[2 * NB + tid];
                const float td_r_ = smp_in[3 * NB + tid], td_h_ = smp_in[4 * NB + tid];
                float lg[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    float v = part[0][tid][k];
#pragma unroll
                    for (int q = 1; q < 8; q++) v += part[q][tid][k];
                    lg[k] = v + bo[k];
                }
                float g[4];
                if (!a.critic) {
                    // logits_to_probs (src/MLP.py:139-156) and the policy-gradient logits delta (:328-354)
                    const uint32_t mw = a.use_mask ? mask_word_of(bds[tid]) : 0x01010101u;
                    const uint32_t act = valid ? act_j_ : 0u;
                    float l4[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) l4[k] = ((mw >> (8 * k)) & 0xFFu) ? lg[k] : -1e9f;
                    const float mx = fmaxf(fmaxf(l4[0], l4[1]), fmaxf(l4[2], l4[3]));
                    float e[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) e[k] = expf(l4[k] - mx);
                    const float es = ((e[0] + e[1]) + e[2]) + e[3];
#pragma unroll
                    for (int k = 0; k < 4; k++) g[k] = (((uint32_t)k == act ? 1.0f : 0.0f) - e[k] / es) * cf_;
                } else {
                    // the critic's value-loss gradient (update_batch :403-498, _get_grad_logits_critic :884-910)
                    if (a.has_td) tg_ = ((td_v * a.td.gamma) * td_h_) + td_r_;   // the host's fp32 operation order
                    const float diff = lg[0] - tg_;
                    const float gd = (a.huber && fabsf(diff) > a.huber_delta) ? copysignf(a.huber_delta, diff) : diff;
                    g[0] = gd * cf_;
                    g[1] = g[2] = g[3] = 0.0f;
                    if (valid && a.delta_out) a.delta_out[j] = tg_ - lg[0];
                    if (valid) {
                        if (a.has_td) a.td.v_out[a.td.lane[j]] = lg[0];
                        else if (a.v_out) a.v_out[j] = lg[0];
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    gs[tid][k] = g[k];
                    dbo_l[tid * 4 + k] += g[k];
                }
            }
            lds_barrier();
        }
        DEEP_STAMP(4);
        {
            DEEP_LANE_IDS;
            // ---- output layer backward: dW_out, db_{L-1}, delta_{L-1} in place; thread (unit u, sample range q) of
            //      oq ranges, so every thread works (one thread per unit ran 32 serial steps on one or two waves)
            if (tid < oq * HL) {
                const int u = tid % HL, q = tid / HL, n0 = q * oper, n1 = n0 + oper < NB ? n0 + oper : NB;
                float* arow = actl(L - 1) + u * SS;
                const float4 wv = wout[u];
                float d0 = dwo[0], d1 = dwo[1], d2 = dwo[2], d3 = dwo[3], db = dbl;
                const auto step = [&](int n2, float x, float4 g4) {
                    d0 = fmaf(x, g4.x, d0);
                    d1 = fmaf(x, g4.y, d1);
                    d2 = fmaf(x, g4.z, d2);
                    d3 = fmaf(x, g4.w, d3);
                    float dh = g4.x * wv.x;
                    dh = fmaf(g4.y, wv.y, dh);
                    dh = fmaf(g4.z, wv.z, dh);
                    dh = fmaf(g4.w, wv.w, dh);
                    const float dl = dh * act_deriv<ACT>(x);
                    db += dl;
                    arow[n2] = dl;
                };
                if (n1 - n0 == 8) {   // the runner net's 64-unit layer on 4 waves: 4 samples' reads in flight per wait
#pragma unroll
                    for (int b0 = 0; b0 < 8; b0 += 4) {
                        float x[4];
                        float4 g4[4];
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            x[i] = arow[n0 + b0 + i];
                            g4[i] = *reinterpret_cast<const float4*>(gs[n0 + b0 + i]);
                        }
                        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
                        for (int i = 0; i < 4; i++) step(n0 + b0 + i, x[i], g4[i]);
                    }
                } else
                for (int n2 = n0; n2 < n1; n2++) {
                    const float x = arow[n2];
                    const float4 g4 = *reinterpret_cast<const float4*>(gs[n2]);
                    d0 = fmaf(x, g4.x, d0);
                    d1 = fmaf(x, g4.y, d1);
                    d2 = fmaf(x, g4.z, d2);
                    d3 = fmaf(x, g4.w, d3);
                    float dh = g4.x * wv.x;
                    dh = fmaf(g4.y, wv.y, dh);
                    dh = fmaf(g4.z, wv.z, dh);
                    dh = fmaf(g4.w, wv.w, dh);
                    const float dl = dh * act_deriv<ACT>(x);
                    db += dl;
                    arow[n2] = dl;
                }
                dwo[0] = d0; dwo[1] = d1; dwo[2] = d2; dwo[3] = d3;
                dbl = db;
            }
            lds_barrier();
        }
        DEEP_STAMP(5);
        // ---- dense layers top down: dW_l (MFMA over the 32 samples), then delta_{l-1} (MFMA chain) in place
        for (int l = L - 1; l >= 1; l--) {
            DEEP_LANE_IDS;
            const float* A = actl(l - 1);
            const float* D = actl(l);
            const int ntin = net.nt[l - 1], ntout = net.nt[l];
            const int f0 = a.tile_begin[l], f1 = f0 + ntin * ntout;
#pragma unroll
            for (int k = 0; k < TPW; k++) {
                const int f = a.tile0 + w + NW * k;
                if (f >= f0 && f < f1) {                     // wave-uniform
                    const int ti = (f - f0) / ntout, tj = (f - f0) % ntout;
                    const float* ap = A + (32 * ti + col) * SS + h;
                    const float* dp = D + (32 * tj + col) * SS + h;
                    floatx16 c = acc[k];
                    // in chunks of 8 k-steps, the next chunk's operands read while this chunk's MFMAs run (the same
                    // MFMAs, same order)
                    constexpr int NCH = NB / 16;
                    float av[2][8], dv[2][8];
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        av[0][i] = ap[2 * i];
                        dv[0][i] = dp[2 * i];
                    }
#pragma unroll
                    for (int hh = 0; hh < NCH; hh++) {
                        if (hh + 1 < NCH) {
#pragma unroll
                            for (int i = 0; i < 8; i++) {
                                av[(hh + 1) & 1][i] = ap[2 * (8 * (hh + 1) + i)];
                                dv[(hh + 1) & 1][i] = dp[2 * (8 * (hh + 1) + i)];
                            }
                        }
#pragma unroll
                        for (int i = 0; i < 8; i++)
                            c = __builtin_amdgcn_mfma_f32_32x32x2f32(av[hh & 1][i], dv[hh & 1][i], c, 0, 0, 0);
                        if (hh + 1 < NCH) {
                            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);   // the next chunk's reads first
                            __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);   // then this chunk's MFMAs
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
                    acc[k] = c;
                }
            }
            // delta_{l-1} = (W_l delta_l) act'(a_{l-1}): output tiles = layer l-1's units, k = layer l's units
            const float4* __restrict__ frag = reinterpret_cast<const float4*>(a.bpacked + a.boff[l]) + lane;
            float* Aw = actl(l - 1);
            // (64-sample form, ReLU) k-tile 0's fragments of the wave's first item, loaded before the barrier below
            // (in flight across it: update 1.121-1.123 -> 1.116-1.118 s on one box, profiles/round6/s12/; the same
            // for the dense forward's first chains -- after layer 0 / before each layer's barrier -- measured much
            // slower, 1.177 against 1.115-1.117 s, s13/, as in s3/)
            float4 fa[4];
            const auto load_fa = [&]() {
                if (w < CT * ntin) {
                    const float4* f0 = frag + (int64_t)(w >> (CT - 1)) * ntout * 256;
#pragma unroll
                    for (int q = 0; q < 4; q++) fa[q] = f0[q * 64];
                }
            };
            if constexpr (ACT == 0 && NB == 64) load_fa();
            lds_barrier();                               // every read of a_{l-1} by the dW tiles is done
            DEEP_STAMP(l == L - 1 ? 6 : 10);
            if constexpr (ACT == 0 && NB == 64) {
                // ReLU, 64-sample form (round 6): per item act'(a) read as a 16-bit mask BEFORE the chain (its LDS
                // reads under the chain's first fragment loads, not after its last MFMA), then only the stores after
                // it -- the same products c * 1 or c * 0 (update 1.120-1.124 -> 1.115-1.118 s on one box,
                // profiles/round6/s8/); and k-tile 0's fragments carried from one item of the wave to the next
                // (frag_chain_carry: 1.112-1.113 -> 1.105-1.107 s, s11/).  (The 64-unit layer's forward as two
                // half-k chains on all 8 waves measured slower, 1.126-1.132 s, s8/.)
                for (int i = w; i < CT * ntin; i += NW) {
                    const int o = i >> (CT - 1), cc = i & (CT - 1);
                    uint32_t pos = 0;
#pragma unroll
                    for (int r = 0; r < 16; r++)
                        pos |= (Aw[(32 * o + tile_row(r, h)) * SS + 32 * cc + col] > 0.0f ? 1u : 0u) << r;
                    const int inext = i + NW;
                    const float4* fnext = inext < CT * ntin ? frag + (int64_t)(inext >> (CT - 1)) * ntout * 256 : nullptr;
                    const floatx16 c = frag_chain_carry<SS>(frag + (int64_t)o * ntout * 256, D + 32 * cc, ntout, h, col,
                                                            fa, fnext);
#pragma unroll
                    for (int r = 0; r < 16; r++)
                        Aw[(32 * o + tile_row(r, h)) * SS + 32 * cc + col] = c[r] * (((pos >> r) & 1u) ? 1.0f : 0.0f);
                }
            } else
            for (int i = w; i < CT * ntin; i += NW) {
                const int o = i >> (CT - 1), cc = i & (CT - 1);
                const floatx16 c = frag_chain<SS>(frag + (int64_t)o * ntout * 256, D + 32 * cc, 0, ntout, h, col);
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    float* pa = Aw + (32 * o + tile_row(r, h)) * SS + 32 * cc + col;
                    *pa = c[r] * act_deriv<ACT>(*pa);
                }
            }
            lds_barrier();
            DEEP_STAMP(l == L - 1 ? 11 : 12);
            // db_{l-1} of unit tid
            if (tid < 32 * ntin) {
                const float* drow = Aw + tid * SS;
                float db = dbs[(l - 1) * 256 + tid];
                // 8 rows' reads in flight per wait (the same adds in the same order)
#pragma unroll
                for (int n0 = 0; n0 < NB; n0 += 8) {
                    float v[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) v[i] = drow[n0 + i];
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
                    for (int i = 0; i < 8; i++) db += v[i];
                }
                dbs[(l - 1) * 256 + tid] = db;
            }
            DEEP_STAMP(l == L - 1 ? 7 : 13);
        }
        // ---- first layer's weight gradient
        {
            DEEP_LANE_IDS;
            if constexpr (NB == 64) {
                // (one launch: last_pass) the next group's inputs first (see load_in), then delta_0 out for the
                // one-hot dW1 over all 8 waves: thread (unit u, half hf) stores rows 32 hf .. 32 hf + 31 of unit u.
                // Through a buffer resource over the group's rows: rows past a ragged group's end, and threads past
                // 2 H0, fall outside num_records (the row offset runs in the VGPR offset, one add per store).
                const GroupIn nx = load_in(gi + gridDim.x);
                const int H0 = 32 * net.nt[0];
                const int hf = tid >= H0 ? 1 : 0, u = tid - hf * H0;
                const bool live = tid < 2 * H0;
                const float* drow = actl(0) + (live ? u : 0) * SS + 32 * hf;
                const uint32_t left = a.n - gi * (uint32_t)NB < (uint32_t)NB ? a.n - gi * (uint32_t)NB : (uint32_t)NB;
                const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
                    a.d0_out + (size_t)gi * (uint32_t)NB * (uint32_t)H0, 0, (int)(left * (uint32_t)H0 * 4u), 0x00020000);
                const int rowb = __builtin_amdgcn_readfirstlane(H0 * 4);
                int vo = live ? (u + 32 * hf * H0) * 4 : 0x40000000;
#pragma unroll
                for (int n0 = 0; n0 < 32; n0 += 8) {
                    float v[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) v[i] = drow[n0 + i];
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);   // the 4 ds_read2 first
                    __builtin_amdgcn_sched_group_barrier(0x040, 8, 0);   // then the 8 stores
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i]), rd, vo, 0, 0);
                        vo += rowb;
                        asm volatile("" : "+v"(vo));   // one running offset, not 32 hoisted constants
                    }
                }
                put_in(nx);
            } else if constexpr (OBS == G2048_OBS_ONEHOT) {
                // delta_0 out for the one-hot dW1 (g2048_onehot_dw1): row j, unit tid (coalesced rows) -- by the last
                // launch of a multi-launch net only (each launch recomputes the same rows)
                const int H0 = 32 * net.nt[0];
                if (tid < H0 && a.last_pass) {
                    // through a buffer resource over the group's rows (base and row offsets in SGPRs, no 64-bit
                    // per-lane address to keep live; the rows past a ragged group's end fall outside num_records)
                    const float* drow = actl(0) + tid * SS;
                    const uint32_t left = a.n - gi * (uint32_t)NB < (uint32_t)NB ? a.n - gi * (uint32_t)NB : (uint32_t)NB;
                    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
                        a.d0_out + (size_t)gi * (uint32_t)NB * (uint32_t)H0, 0, (int)(left * (uint32_t)H0 * 4u), 0x00020000);
                    // in batches of 8: the batch's LDS reads issued together, one wait, then its stores (hipcc otherwise
                    // alternated one ds_read2 / one wait / two stores, 16 LDS round trips in series); the row offset
                    // advances by one scalar add per store (as 32 distinct offsets hipcc hoisted them out of the group
                    // loop and spilled them to VGPR lanes)
                    const int rowb = __builtin_amdgcn_readfirstlane(H0 * 4);
                    int so = 0;
#pragma unroll
                    for (int n0 = 0; n0 < NB; n0 += 8) {
                        float v[8];
#pragma unroll
                        for (int i = 0; i < 8; i++) v[i] = drow[n0 + i];
                        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);   // the 4 ds_read2 first
                        __builtin_amdgcn_sched_group_barrier(0x040, 8, 0);   // then the 8 stores
#pragma unroll
                        for (int i = 0; i < 8; i++) {
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i]), rd, tid * 4, so, 0);
                            so += rowb;
                            asm volatile("" : "+s"(so));   // one running offset, not 32 hoisted constants
                        }
                    }
                }
            } else {
                // dW_0^T tile t (32 units x 32 features, features >= 16 zero): A = delta_0 [unit][sample], B = x [sample][feature]
                const float* D0 = actl(0);
#pragma unroll
                for (int i = 0; i < kA0; i++) {
                    const int t = w + NW * i;
                    if (t < net.nt[0]) {
                        floatx16 c = acc0[i];
                        const float* dp = D0 + (32 * t + col) * SS + h;
#pragma unroll
                        for (int s2 = 0; s2 < 16; s2++) {
                            const float xv = col < 16 ? obs_value<OBS>(bds[2 * s2 + h], col, a.obs_scale) : 0.0f;
                            c = __builtin_amdgcn_mfma_f32_32x32x2f32(dp[2 * s2], xv, c, 0, 0, 0);
                        }
                        acc0[i] = c;
                    }
                }
            }
            lds_barrier();   // the next group rewrites the boards and layer 0: every LDS access done
        }
        DEEP_STAMP(8);
#if G2048_DEEP_DIAG
        dph[kDiagSlots - 1] += 1;
#endif
    }
#if G2048_DEEP_DIAG
    if (a.diag && lane == 0) {
        uint64_t* slot = a.diag + ((size_t)blockIdx.x * NW + w) * kDiagSlots;
#pragma unroll
        for (int i = 0; i < kDiagSlots; i++) slot[i] += dph[i];
    }
#endif
    // ---- the output layer's (unit, range) partials summed per unit in range order (LDS: the activation area,
    //      at least kOutRed floats), db_out's 32 sample slots in slot order, then this workgroup's partial slab
    float dbo = 0.0f;
    {
        float* red = dyn;                                   // [oq][HL][5]
        if (tid < NB) {
#pragma unroll
            for (int k = 0; k < 4; k++) gs[tid][k] = dbo_l[tid * 4 + k];
        }
        if (tid < oq * HL) {
#pragma unroll
            for (int k = 0; k < 4; k++) red[tid * 5 + k] = dwo[k];
            red[tid * 5 + 4] = dbl;
        }
        __syncthreads();
        if (tid < HL) {
            float sum[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
            for (int q = 0; q < oq; q++)
#pragma unroll
                for (int k = 0; k < 5; k++) sum[k] += red[(q * HL + tid) * 5 + k];
#pragma unroll
            for (int k = 0; k < 4; k++) dwo[k] = sum[k];
            dbs[(L - 1) * 256 + tid] = sum[4];
        }
        if (tid < 4)
            for (int q = 0; q < NB; q++) dbo += gs[q][tid];
        __syncthreads();
    }
    float* out = a.part + (size_t)blockIdx.x * a.pslab;
#pragma unroll
    for (int k = 0; k < TPW; k++) {
        const int f = a.tile0 + w + NW * k;
        if (f < a.ntiles) {
            int l = 1;
            while (l + 1 < L && f >= a.tile_begin[l + 1]) l++;
            const int ntout = net.nt[l], f0 = a.tile_begin[l];
            const int ti = (f - f0) / ntout, tj = (f - f0) % ntout;
            const int Ho = 32 * ntout;
#pragma unroll
            for (int r = 0; r < 16; r++)
                out[a.pw[l] + (int64_t)(32 * ti + tile_row(r, h)) * Ho + 32 * tj + col] = acc[k][r];
        }
    }
    if (!a.first_pass) return;   // the launches after the first write their dense tiles only
    if constexpr (OBS != G2048_OBS_ONEHOT) {
        const int H0 = 32 * net.nt[0];
#pragma unroll
        for (int i = 0; i < kA0; i++) {
            const int t = w + NW * i;
            if (t < net.nt[0] && col < 16) {               // C[unit][feature]: dW_0[feature][unit]
#pragma unroll
                for (int r = 0; r < 16; r++) out[a.pw[0] + (int64_t)col * H0 + 32 * t + tile_row(r, h)] = acc0[i][r];
            }
        }
    }
    for (int l = 0; l < L; l++)
        if (tid < 32 * net.nt[l]) out[a.pb[l] + tid] = dbs[l * 256 + tid];
    if (tid < HL) {
#pragma unroll
        for (int k = 0; k < 4; k++) out[a.pw[L] + (int64_t)tid * 4 + k] = dwo[k];
    }
    if (tid < 4) out[a.pb[L] + tid] = dbo;
}

// backward fragments of the dense layers: layer l (1..L-1) at boff[l], [nt_{l-1}][nt_l][4][64][4]: output tile o
// (a unit tile of layer l-1), k-tile t (of layer l), lane, k-step s = 4 q + u -> W_l[32 o + (lane & 31)][32 t + tile_row(s, lane >> 5)]
// (the k order of frag_chain, as the forward fragments)
struct DeepGradPackArgs {
    const float* W[kMaxHidden];
    int h[kMaxHidden];
    int nt[kMaxHidden];
    int64_t boff[kMaxHidden + 1];
    int L;
    float* dst;
};

__global__ void __launch_bounds__(256) deep_grad_pack_kernel(DeepGradPackArgs a) {
    const int64_t total = a.boff[a.L];
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
        int l = a.L - 1;
        while (l > 1 && q < a.boff[l]) l--;
        const int64_t x = q - a.boff[l];
        const int u = (int)(x & 3), lane = (int)((x >> 2) & 63), qq = (int)((x >> 8) & 3);
        const int64_t tt = x >> 10;
        const int t = (int)(tt % a.nt[l]), o = (int)(tt / a.nt[l]);
        const int i = 32 * o + (lane & 31), k = 32 * t + tile_row(4 * qq + u, lane >> 5);
        a.dst[q] = (i < a.h[l - 1] && k < a.h[l]) ? a.W[l][(int64_t)i * a.h[l] + k] : 0.0f;
    }
}

// partial-slab layout of deep_grad_kernel: dense dW_l [H_{l-1}p][H_lp] + db_l for l >= 1, dW_0 ([16][H0p], log2 /
// raw only) + db_0, dW_out [H_{L-1}p][4] + db_out [4]
struct DeepGradLayout {
    int64_t pw[kMaxHidden + 1], pb[kMaxHidden + 1], pslab;
    int64_t boff[kMaxHidden + 1];
    int ntiles;
    int tile_begin[kMaxHidden];
};

DeepGradLayout deep_grad_layout(const DeepNet& n) {
    DeepGradLayout g{};
    int64_t off = 0;
    for (int l = 0; l < n.L; l++) {
        g.pw[l] = off;
        if (l == 0) off += n.onehot ? 0 : (int64_t)16 * 32 * n.nt[0];
        else off += (int64_t)32 * n.nt[l - 1] * 32 * n.nt[l];
        g.pb[l] = off;
        off += 32 * n.nt[l];
    }
    g.pw[n.L] = off;
    off += (int64_t)32 * n.nt[n.L - 1] * 4;
    g.pb[n.L] = off;
    off += 4;
    g.pslab = off;
    int64_t bo = 0;
    int tiles = 0;
    for (int l = 1; l < n.L; l++) {
        g.boff[l] = bo;
        bo += (int64_t)n.nt[l - 1] * n.nt[l] * 1024;
        g.tile_begin[l] = tiles;
        tiles += n.nt[l - 1] * n.nt[l];
    }
    g.boff[n.L] = bo;
    if (n.L == 1) g.boff[1] = 0;
    g.ntiles = tiles;
    return g;
}

// floats of the hidden layers' activations, at least the output layer's final reduction (deep_grad_kernel:
// [oq][HL][5], oq HL <= the block size)
int64_t deep_grad_act_floats(const DeepNet& n, int nw, int nb = 32) {
    int64_t units = 0;
    for (int l = 0; l < n.L; l++) units += 32 * n.nt[l];
    int64_t f = units * (nb + 1);
    const int64_t red = 5 * 64 * nw;
    if (red > f) f = red;
    return f;
}
// + part, g, boards, bias sums, output weights / bias, the per-sample inputs, the db_out sums
int64_t deep_grad_lds_bytes(const DeepNet& n, int nw, int nb = 32) {
    return (deep_grad_act_floats(n, nw, nb) + 8 * nb * 4 + nb * 4 + 2 * nb + kMaxHidden * 256 + 256 * 4 + 4 +
            7 * nb + nb * 4 + (nb == 64 ? 32 * 4 : 0)) * 4;
}

// the instantiation that covers the net (nw = 0: none; see deep_grad_kernel).  The 4-wave and the 64-tile ones are
// one-hot only: with the log2 / raw first layer's MFMA tiles (dW_0 accumulators, the obs rebuilt per k-step) on top
// of 10 or 8 dense tiles per wave, hipcc spills whole accumulator tiles (~300-650 VGPRs).
DeepGradVariant deep_grad_variant(const DeepNet& n) {
    const int tiles = deep_grad_layout(n).ntiles;
    if (n.onehot && tiles <= 40 && deep_grad_lds_bytes(n, 8, 64) <= 160 * 1024)
        return {8, 5, 0, 1, 1, 64};
    if (tiles <= 48 && deep_grad_lds_bytes(n, 8) <= 160 * 1024) return {8, 6, 1, 1, 1};
    if (n.onehot && tiles <= 64 && deep_grad_lds_bytes(n, 8) <= 160 * 1024) return {8, 8, 1, 1, 1};
    // past one launch's accumulator budget (round 5; e.g. one-hot [256, 256, 256], log2 [256, 256]): the dense dW
    // tiles in ranges, one launch per range, each redoing the forward and the delta chains (the dW MFMAs, a third
    // of the work, are split); 64 tiles per launch on one-hot nets, 48 on log2 / raw (whose 8 x 8 instantiation
    // spills)
    if (deep_grad_lds_bytes(n, 8) <= 160 * 1024) {
        const int cap = n.onehot ? 64 : 48;
        return {8, n.onehot ? 8 : 6, 1, 1, (tiles + cap - 1) / cap};
    }
    return {0, 0, 0, 0, 0};
}

// ------------------------------------------------------------------------------------ one-hot layer 1 (update)
// a1[s][j] = act(b1[j] + sum_c W1[17 c + e_c(s)][j]) for samples s < m, units j < h1: one wave per sample (lanes =
// units, 64 at a time), rows read coalesced from the unpadded [272][h1] weight (the torch parameter itself).
template <int ACT>
__global__ void __launch_bounds__(256) onehot_l1_kernel(const float* __restrict__ W1, const float* __restrict__ b1,
                                                         const uint64_t* __restrict__ boards, int h1, int64_t m,
                                                         int64_t ld, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t s = wave; s < m; s += waves) {
        const uint64_t b = boards[s];
        for (int j0 = 0; j0 < h1; j0 += 64) {
            const int j = j0 + lane;
            if (j < h1) {
                float acc = 0.0f;
#pragma unroll
                for (int c = 0; c < 16; c++) acc += W1[(int64_t)(17 * c + (int)((b >> (4 * c)) & 15u)) * h1 + j];
                out[s * ld + j] = activate<ACT>(acc + b1[j]);
            }
        }
    }
}

// dW1 / db1 of a one-hot first layer on the bf16 MFMA (round 5; replaces onehot_dw1_kernel's register scatter on
// the update path).  dW1 = X^T D1 with X the [samples][272] one-hot of the boards is a GEMM whose A operand is exact
// in bf16 (0 / 1): v_mfma_f32_32x32x16_bf16 with A = X^T of two cells (row 16 q + e: cell 2 p + q, exponent e; k = 16
// samples) and B = the samples' deltas split exactly into three bf16 planes (d = d0 + d1 + d2, 8 significant bits
// each), so every product is exact and only the fp32 accumulation rounds, as the sequential sum does.  Wave w owns
// the 32 units 32 w .. 32 w + 31 (one column tile) x all 16 cells (8 cell pairs): 8 accumulator tiles = 128
// registers, two waves per SIMD (16 tiles = 256 AGPRs per wave made hipcc spill ~250 VGPRs), one 8-wave workgroup
// per CU and sample range (always 8 waves: the units past h1 compute zeros and store nothing).  Per 16 samples: 24 MFMAs per wave (8 pairs x 3 planes), 1,536 cycles per SIMD for 256 units,
// against 16 KiB of deltas read per workgroup.  The one-hot A fragments (the same for every wave) are built once per
// workgroup: wave w builds pair w (from byte w of each board) into a double-buffered LDS image that every wave
// reads back (one ds_read_b128 per pair, one pair ahead of its MFMAs).  db1 is each lane's sum of its B values (samples 8 h .. 8 h + 7 of each step, in order), the
// two lane halves added at the end.  Deltas and boards are loaded three steps ahead (a four-slot register ring)
// through buffer resources.
// Rows 17 c + 16 (exponent 16, never on a bitboard) are written as zeros.
constexpr int kDw1Rows = kOneHotRows + 1;   // a dW1 partial slab: 272 rows of dW1, then db1
constexpr int kDw1Step = 16;        // samples per MFMA k-step
constexpr int kDw1MaxWaves = 8;     // 32 units per wave

struct Dw1Slot {
    float v[8];       // deltas of this lane's unit, samples 8 h .. 8 h + 7 of the step (0 past the range)
    uint32_t bw[8];   // byte w of the same samples' boards: cells 2 w, 2 w + 1 (this wave's cell pair)
};

// Loads through two buffer resources over this workgroup's sample range [s0, s1): a lane's voffset plus a scalar
// per-sample offset, so a step's 16 loads need no address arithmetic (64-bit per-load addresses cost ~80 VALU per
// step), and a load past s1 returns 0 (num_records), which is the tail's zero delta.
__global__ void __launch_bounds__(64 * kDw1MaxWaves, 1) onehot_dw1_mfma_kernel(
    const uint64_t* __restrict__ boards, const float* __restrict__ d1, int h1, int64_t m, int64_t ld, int64_t per,
    float* __restrict__ part) {
    __shared__ uint4 abuf[2][8][64];   // [buffer][cell pair][lane]: the A fragment (8 bf16) of `lane`
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int64_t s0 = (int64_t)blockIdx.x * per, s1 = s0 + per < m ? s0 + per : m;
    const int u = 32 * w + r;
    const bool live = u < h1;
    const uint32_t q = (uint32_t)r >> 4, e = (uint32_t)r & 15u;
    const int nsteps = s1 > s0 ? (int)((s1 - s0 + kDw1Step - 1) / kDw1Step) : 0;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(d1 + s0 * ld), 0, (int)((s1 - s0) * ld * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint64_t*>(boards + s0), 0, (int)((s1 - s0) * 8), 0x00020000);
    const uint32_t ld4 = (uint32_t)ld * 4u;
    // this lane's first delta; a unit past h1 reads past num_records (0) instead of being masked per load
    const uint32_t dvo = live ? (uint32_t)(8 * h) * ld4 + (uint32_t)u * 4u : 0x80000000u;
    const uint32_t bvo = (uint32_t)(8 * h) * 8u + (uint32_t)w;                      // its first board byte
    floatx16 acc[8];
#pragma unroll
    for (int p = 0; p < 8; p++) acc[p] = floatx16{};
    float db = 0.0f;
    const auto load = [&](int st, Dw1Slot& sl) {
        const uint32_t so = (uint32_t)(st * kDw1Step);   // the step's first sample, relative to s0
#pragma unroll
        for (int k = 0; k < 8; k++) {
            sl.v[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rd, (int)dvo, (int)((so + k) * ld4), 0));
            sl.bw[k] = __builtin_amdgcn_raw_buffer_load_b8(rb, (int)bvo, (int)((so + k) * 8u), 0);
        }
    };
    const auto build_a = [&](const Dw1Slot& sl, int buf) {   // this wave's cell pair of the step's one-hot
        uint32_t d[4];
#pragma unroll
        for (int k2 = 0; k2 < 4; k2++) {
            const uint32_t x0 = (sl.bw[2 * k2] >> (4u * q)) & 15u, x1 = (sl.bw[2 * k2 + 1] >> (4u * q)) & 15u;
            d[k2] = (x0 == e ? 0x3F80u : 0u) | (x1 == e ? 0x3F800000u : 0u);   // bf16 1.0 / 0 per sample
        }
        abuf[buf][w][lane] = make_uint4(d[0], d[1], d[2], d[3]);
    };
    // step st: the MFMAs of `cur` (its A image in `buf`) while the loads of three steps ahead are in flight and the
    // next step's A image is built
    const auto step = [&](Dw1Slot& cur, Dw1Slot& nxt, Dw1Slot& ahead, int st, int buf) {
        if (st + 3 < nsteps) load(st + 3, ahead);
#pragma unroll
        for (int k = 0; k < 8; k++) db += cur.v[k];
        bf16x8 pl[3];
        split3_bf16(cur.v, pl[0], pl[1], pl[2]);
        if (st + 1 < nsteps) build_a(nxt, buf ^ 1);
        uint4 a = abuf[buf][0][lane];
#pragma unroll
        for (int p = 0; p < 8; p++) {
            const bf16x8 av = __builtin_bit_cast(bf16x8, a);
            if (p < 7) a = abuf[buf][p + 1][lane];
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, pl[0], acc[p], 0, 0, 0);
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, pl[1], acc[p], 0, 0, 0);
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, pl[2], acc[p], 0, 0, 0);
        }
        __syncthreads();   // the next step's A image is complete; this one is free to be rewritten
    };
    Dw1Slot sl0, sl1, sl2, sl3;
    if (nsteps > 0) load(0, sl0);
    if (nsteps > 1) load(1, sl1);
    if (nsteps > 2) load(2, sl2);
    if (nsteps > 0) build_a(sl0, 0);
    __syncthreads();
    for (int st = 0; st < nsteps; st += 4) {   // block-uniform trip count; the four slots rotate
        step(sl0, sl1, sl3, st, 0);
        if (st + 1 >= nsteps) break;
        step(sl1, sl2, sl0, st + 1, 1);
        if (st + 2 >= nsteps) break;
        step(sl2, sl3, sl1, st + 2, 0);
        if (st + 3 >= nsteps) break;
        step(sl3, sl0, sl2, st + 3, 1);
    }
    db += __shfl_xor(db, 32);   // lane half 0 + half 1 (addition commutes: both halves hold the same bits)
    if (!live) return;
    float* slab = part + (int64_t)blockIdx.x * kDw1Rows * h1;
#pragma unroll
    for (int p = 0; p < 8; p++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int row = tile_row(i, h);                       // 16 q' + e' of the pair
            slab[(int64_t)(17 * (2 * p + (row >> 4)) + (row & 15)) * h1 + u] = acc[p][i];
        }
    }
    if (h == 0) {
#pragma unroll
        for (int c = 0; c < 16; c++) slab[(int64_t)(17 * c + 16) * h1 + u] = 0.0f;   // exponent 16: never on a bitboard
        slab[(int64_t)kOneHotRows * h1 + u] = db;
    }
}

// onehot_dw1_mfma_kernel with its deltas and boards staged through an LDS ring by LDS-DMA (round 5; the shipped
// dW1 path when d1 rows are 16-byte aligned; any other stride takes the register form).  The register form kept three
// steps of loads in flight on paper, but the register allocator reused in-flight load destinations as temporaries,
// so the wait-count pass drained every load each step (vmcnt(0) in the loop): 2.9 TB/s, MFMA busy 0.40.  Here a
// step's 16 rows (16 KiB at h1 = 256) and 16 boards go straight to LDS (global_load_lds_dwordx4: no registers) in
// an 8-slot ring, five steps in flight across each step's raw barrier (s_waitcnt vmcnt(15): 5 steps x 3 DMA
// instructions per wave).  Row r's 16-byte chunks are stored XOR-swizzled by 8 chunks when r >= 8 so the two lane
// halves (rows 8 h + k) read disjoint banks.  Rows past the range are clamped loads (valid memory) masked to 0 at
// the read, and their boards to 0: the same operands, MFMAs and order as onehot_dw1_mfma_kernel, the same bits.
constexpr int kDw1Slots = 8;
#define G2048_DW1_STEP_WAIT "s_waitcnt vmcnt(15)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier"
static_assert((kDw1Slots - 3) * 3 == 15, "G2048_DW1_STEP_WAIT: (slots - 3) steps x 3 DMA instructions in flight");

__global__ void __launch_bounds__(64 * kDw1MaxWaves, 1) onehot_dw1_ring_kernel(
    const uint64_t* __restrict__ boards, const float* __restrict__ d1, int h1, int64_t m, int64_t ld, int64_t per,
    float* __restrict__ part) {
    __shared__ float ring[kDw1Slots][kDw1Step * 256];            // [slot][row][16-byte chunk (swizzled)][4]
    __shared__ uint32_t bring[kDw1Slots][kDw1MaxWaves][64];      // [slot][wave: its own copy][16 boards, twice]
    __shared__ uint4 abuf[2][8][64];                             // as onehot_dw1_mfma_kernel's
    typedef __attribute__((address_space(3))) void lvoid;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int64_t s0 = (int64_t)blockIdx.x * per, s1 = s0 + per < m ? s0 + per : m;
    const int u = 32 * w + r;
    const bool live = u < h1;
    const uint32_t q = (uint32_t)r >> 4, e = (uint32_t)r & 15u;
    const int nsteps = s1 > s0 ? (int)((s1 - s0 + kDw1Step - 1) / kDw1Step) : 0;
    const int nch = (h1 + 3) >> 2;                                   // 16-byte chunks per row
    const int word = (((u >> 2) ^ (h << 3)) << 2) | (u & 3);        // unit u of rows 8 h .. 8 h + 7 in the slot
    floatx16 acc[8];
#pragma unroll
    for (int p = 0; p < 8; p++) acc[p] = floatx16{};
    float db = 0.0f;
    if (nsteps > 0) {   // block-uniform
        const int64_t slast = s1 - 1;
        // The DMA is issued from inline asm: with the builtin, the wait-count pass cannot tell the ring slots (or
        // abuf) apart from the slot being filled and put vmcnt(0) before every LDS read.  The asm barrier below
        // (vmcnt(15), "memory") is the only ordering these reads need.  M0 is not in the clobber lists (hipcc
        // reserves it and ignores such a clobber): nothing the compiler emits in this kernel reads M0 (the ISA's
        // only M0 writes are these asm statements' own).
        const uint32_t ring_lds = (uint32_t)(uintptr_t)(lvoid*)&ring[0][0], bring_lds = (uint32_t)(uintptr_t)(lvoid*)&bring[0][0][0];
        const int wu = __builtin_amdgcn_readfirstlane(w);
        const auto issue = [&](int st) {   // step st into slot st % kDw1Slots: wave w rows 2 w, 2 w + 1, its boards
            const int sl = st % kDw1Slots;
            const int64_t base = s0 + (int64_t)st * kDw1Step;
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int row = 2 * w + i;
                const int64_t smp = base + row < slast ? base + row : slast;
                const int g = lane ^ (((row >> 3) & 1) << 3);
                const float* src = d1 + smp * ld + 4 * (g < nch ? g : 0);
                const uint32_t dst = ring_lds + (uint32_t)((sl * kDw1Step + 2 * wu + i) * 256 * 4);
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(dst)
                             : "memory");
            }
            const int j = (lane & 31) >> 1;   // lanes 32 .. 63 load the same 16 boards again (one DMA shape per wave)
            const int64_t smp = base + j < slast ? base + j : slast;
            const uint32_t* src = reinterpret_cast<const uint32_t*>(boards + smp) + (lane & 1);
            const uint32_t dst = bring_lds + (uint32_t)((sl * kDw1MaxWaves + wu) * 64 * 4);
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(dst)
                         : "memory");
        };
        const auto build_a = [&](int st, int buf) {   // this wave's cell pair of step st's one-hot (0 past the range)
            const int sl = st % kDw1Slots;
            const int64_t lim = s1 - s0 - (int64_t)st * kDw1Step;
            const uint8_t* bb = reinterpret_cast<const uint8_t*>(&bring[sl][w][0]);
            uint32_t d[4];
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) {
                const int j0 = 8 * h + 2 * k2, j1 = j0 + 1;
                const uint32_t b0 = bb[8 * j0 + w] & (j0 < lim ? 0xFFu : 0u), b1 = bb[8 * j1 + w] & (j1 < lim ? 0xFFu : 0u);
                const uint32_t x0 = (b0 >> (4u * q)) & 15u, x1 = (b1 >> (4u * q)) & 15u;
                d[k2] = (x0 == e ? 0x3F80u : 0u) | (x1 == e ? 0x3F800000u : 0u);
            }
            abuf[buf][w][lane] = make_uint4(d[0], d[1], d[2], d[3]);
        };
        for (int j = 0; j < kDw1Slots - 1; j++) issue(j);
        asm volatile(G2048_DW1_STEP_WAIT ::: "memory");   // steps 0, 1 landed
        build_a(0, 0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (int st = 0; st < nsteps; st++) {
            const int buf = st & 1;
            issue(st + kDw1Slots - 1);   // into the slot step st - 1 read (its end barrier passed); clamped past the end
            const int sl = st % kDw1Slots;
            const int64_t lim = s1 - s0 - (int64_t)st * kDw1Step;
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t x = __float_as_uint(ring[sl][(8 * h + k) * 256 + word]);   // masked, not branched
                v[k] = __uint_as_float(x & (live && 8 * h + k < lim ? 0xFFFFFFFFu : 0u));
            }
#pragma unroll
            for (int k = 0; k < 8; k++) db += v[k];
            bf16x8 pl[3];
            split3_bf16(v, pl[0], pl[1], pl[2]);
            build_a(st + 1, buf ^ 1);   // past the last step: an image nobody reads
            uint4 a = abuf[buf][0][lane];
#pragma unroll
            for (int p = 0; p < 8; p++) {
                const bf16x8 av = __builtin_bit_cast(bf16x8, a);
                if (p < 7) a = abuf[buf][p + 1][lane];
                acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, pl[0], acc[p], 0, 0, 0);
                acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, pl[1], acc[p], 0, 0, 0);
                acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, pl[2], acc[p], 0, 0, 0);
            }
            asm volatile(G2048_DW1_STEP_WAIT ::: "memory");   // steps <= st + 2 landed; this step's slots free
        }
    }
    db += __shfl_xor(db, 32);
    if (!live) return;
    float* slab = part + (int64_t)blockIdx.x * kDw1Rows * h1;
#pragma unroll
    for (int p = 0; p < 8; p++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int row = tile_row(i, h);
            slab[(int64_t)(17 * (2 * p + (row >> 4)) + (row & 15)) * h1 + u] = acc[p][i];
        }
    }
    if (h == 0) {
#pragma unroll
        for (int c = 0; c < 16; c++) slab[(int64_t)(17 * c + 16) * h1 + u] = 0.0f;
        slab[(int64_t)kOneHotRows * h1 + u] = db;
    }
}

int device_cus() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0) cus = c;
    }
    return cus;
}

template <int OBS, int ACT>
void launch_deep_rng(const DeepPolArgs& a, int rng, int grid, hipStream_t s) {
    if (rng == G2048_RNG_PCG64)
        hipLaunchKernelGGL((deep_policy_kernel<OBS, ACT, G2048_RNG_PCG64>), dim3(grid), dim3(kDeepBlock), 0, s, a);
    else
        hipLaunchKernelGGL((deep_policy_kernel<OBS, ACT, G2048_RNG_PHILOX>), dim3(grid), dim3(kDeepBlock), 0, s, a);
}

template <int OBS>
void launch_deep_act(const DeepPolArgs& a, int act, int rng, int grid, hipStream_t s) {
    if (act == G2048_ACT_RELU) launch_deep_rng<OBS, 0>(a, rng, grid, s);
    else launch_deep_rng<OBS, 1>(a, rng, grid, s);
}

}  // namespace

namespace g2048_internal {   // g2048.hip
int set_error(int code, const char* msg);
int device_tables(const uint8_t*& tab, int& cus);
int check_env_cfg(const g2048_env_cfg* c);
g2048::RewardCfg reward_cfg_of(const g2048_env_cfg& c);
}  // namespace g2048_internal

namespace {
int dfail(int code, const char* msg) { return g2048_internal::set_error(code, msg); }
int check_hip() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : dfail(G2048_EHIP, hipGetErrorString(e));
}
template <int OBS, int ACT, int NB>
int launch_deep_roll(const DeepRollArgs& a, int grid, hipStream_t s) {
    hipLaunchKernelGGL((deep_rollout_kernel<OBS, ACT, NB>), dim3(grid), dim3(NB * 8), 0, s, a);
    return check_hip();
}

}  // namespace

#if G2048_DEEP_DIAG
namespace {
uint64_t* g_deep_diag = nullptr;
}
extern "C" void g2048_diag_deep_stamps(uint64_t* p) { g_deep_diag = p; }   // tools-only build (no header entry)
#endif

extern "C" {

int64_t g2048_deep_packed_size(int obs_mode, int n_hidden, const int32_t* hidden) {
    DeepNet n;
    if (obs_mode != G2048_OBS_LOG2 && obs_mode != G2048_OBS_RAW && obs_mode != G2048_OBS_ONEHOT) return -1;
    if (!deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, n)) return -1;
    return n.total;
}

int g2048_deep_pack(const float* const* W, const float* const* b, int obs_mode, int n_hidden, const int32_t* hidden,
                    int out_dim, float* packed, int64_t packed_len, void* stream) {
    DeepNet n;
    if (obs_mode != G2048_OBS_LOG2 && obs_mode != G2048_OBS_RAW && obs_mode != G2048_OBS_ONEHOT)
        return dfail(G2048_EINVAL, "deep policy: obs_mode must be log2, raw or onehot");
    if (!deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, n))
        return dfail(G2048_EINVAL, "deep policy: 1..4 hidden layers of 1..256 units");
    if (out_dim != 1 && out_dim != 4) return dfail(G2048_EINVAL, "deep policy: output width must be 4 or 1");
    if (!W || !b || !packed) return dfail(G2048_EINVAL, "deep policy: NULL buffer");
    if (packed_len < n.total) return dfail(G2048_EINVAL, "deep policy: packed buffer too small");
    DeepPackArgs a{};
    a.net = n;
    for (int l = 0; l <= n_hidden; l++) {
        if (!W[l] || !b[l]) return dfail(G2048_EINVAL, "deep policy: NULL weight");
        a.W[l] = W[l];
        a.B[l] = b[l];
    }
    for (int l = 0; l < n_hidden; l++) a.h[l] = hidden[l];
    a.out = out_dim;
    a.dst = packed;
    const int grid = (int)((n.total + 255) / 256 < 4096 ? (n.total + 255) / 256 : 4096);
    hipLaunchKernelGGL(deep_pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    return check_hip();
}

int g2048_deep_policy(const float* packed, int n_hidden, const int32_t* hidden, int activation, const uint64_t* boards,
                      const uint32_t* lane_state, const int32_t* lane_index, int obs_mode, float obs_scale, int use_mask,
                      int greedy, int rng_mode, uint64_t* rng_state, const uint64_t* rng_inc, const uint64_t* rng_buf,
                      uint64_t philox_key, const uint64_t* lane_seed, float* probs_out, float* logits_out,
                      uint8_t* actions, int64_t n, void* stream) {
    if (n < 0 || n > (int64_t)0xFFFFFFE0) return dfail(G2048_EINVAL, "n out of range");
    if (obs_mode != G2048_OBS_LOG2 && obs_mode != G2048_OBS_RAW && obs_mode != G2048_OBS_ONEHOT)
        return dfail(G2048_EINVAL, "deep policy: obs_mode must be log2, raw or onehot");
    DeepNet net;
    if (!deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, net))
        return dfail(G2048_EINVAL, "deep policy: 1..4 hidden layers of 1..256 units");
    if (activation != G2048_ACT_RELU && activation != G2048_ACT_SIGMOID)
        return dfail(G2048_EINVAL, "Unsupported activation");
    if (rng_mode != G2048_RNG_PCG64 && rng_mode != G2048_RNG_PHILOX) return dfail(G2048_EINVAL, "Unsupported rng_mode");
    if (!packed || !boards || (!actions && !logits_out))
        return dfail(G2048_EINVAL, "deep policy: packed / boards and actions or logits_out are required");
    if (actions && !greedy && rng_mode == G2048_RNG_PCG64 && (!rng_state || !rng_inc || !rng_buf))
        return dfail(G2048_EINVAL, "PCG64 sampling needs rng_state / rng_inc / rng_buf");
    if (n == 0) return G2048_OK;
    DeepPolArgs a;
    a.net = net;
    a.packed = packed;
    a.boards = boards;
    a.lane_state = lane_state;
    a.lane_index = lane_index;
    a.rs = rng_state;
    a.inc = const_cast<uint64_t*>(rng_inc);
    a.buf = const_cast<uint64_t*>(rng_buf);
    a.key = philox_key;
    a.lane_seed = lane_seed;
    a.probs_out = probs_out;
    a.logits_out = logits_out;
    a.actions = actions;
    a.obs_scale = obs_scale;
    a.n = (uint32_t)n;
    a.use_mask = use_mask;
    a.greedy = greedy;
    const int64_t groups = (n + 31) / 32;
    const int64_t cap = 2 * (int64_t)device_cus();   // persistent: two workgroups per CU
    const int grid = (int)(groups < cap ? groups : cap);
    hipStream_t s = (hipStream_t)stream;
    if (obs_mode == G2048_OBS_ONEHOT) launch_deep_act<G2048_OBS_ONEHOT>(a, activation, rng_mode, grid, s);
    else if (obs_mode == G2048_OBS_LOG2) launch_deep_act<G2048_OBS_LOG2>(a, activation, rng_mode, grid, s);
    else launch_deep_act<G2048_OBS_RAW>(a, activation, rng_mode, grid, s);
    return check_hip();
}

int g2048_deep_rollout(const float* packed, int n_hidden, const int32_t* hidden, int activation, const g2048_env_cfg* cfg,
                       int greedy, uint64_t* env_state, const uint64_t* env_inc, uint64_t* env_buf, uint64_t* pol_state,
                       const uint64_t* pol_inc, uint64_t* pol_buf, uint32_t* queue, const int32_t* order,
                       int64_t n_order, int resume, const g2048_suspend* sus, int64_t n, int64_t cap,
                       const g2048_traj* traj, void* stream) {
    int rc = g2048_internal::check_env_cfg(cfg);
    if (rc) return rc;
    if (n < 0 || n > (int64_t)0x7FFFFFFF) return dfail(G2048_EINVAL, "n out of range");
    if (n_order < 0 || n_order > n || (!order && n_order != n) || (resume && !order))
        return dfail(G2048_EINVAL, "deep rollout: order must list n_order <= n episodes (all n when NULL; resume needs a list)");
    if (cap < 1 || cap > (int64_t)0x7FFFFFFF || n * cap > ((int64_t)1 << 40)) return dfail(G2048_EINVAL, "deep rollout: bad cap");
    DeepNet net;
    if (!deep_layout(n_hidden, hidden, cfg->obs_mode == G2048_OBS_ONEHOT, net))
        return dfail(G2048_EINVAL, "deep policy: 1..4 hidden layers of 1..256 units");
    if (activation != G2048_ACT_RELU && activation != G2048_ACT_SIGMOID)
        return dfail(G2048_EINVAL, "Unsupported activation");
    if (!packed || !env_state || !env_inc || !env_buf || !pol_state || !pol_inc || !pol_buf || !queue || !sus || !traj ||
        !sus->board || !sus->meta || !sus->total || !sus->list || !sus->count || !traj->boards || !traj->actions ||
        !traj->rewards || !traj->flags || !traj->lengths || !traj->totals || !traj->max_tile || !traj->final_board)
        return dfail(G2048_EINVAL, "deep rollout: a required buffer is NULL");
    if (n_order == 0) return G2048_OK;
    const uint8_t* tab = nullptr;
    int cus = 256;
    if ((rc = g2048_internal::device_tables(tab, cus))) return rc;
    DeepRollArgs a;
#if G2048_DEEP_DIAG
    a.diag = g_deep_diag;
#else
    a.diag = nullptr;
#endif
    a.net = net;
    a.packed = packed;
    a.tab = tab;
    a.rc = g2048_internal::reward_cfg_of(*cfg);
    a.max_steps = cfg->max_steps;
    a.obs_scale = cfg->obs_log2_scale;
    a.use_mask = cfg->use_action_mask;
    a.greedy = greedy;
    a.env_rs = env_state;
    a.env_inc = env_inc;
    a.env_buf = env_buf;
    a.pol_rs = pol_state;
    a.pol_inc = pol_inc;
    a.pol_buf = pol_buf;
    a.next = queue;
    a.order = order;
    a.n_order = (uint32_t)n_order;
    a.resume = resume;
    a.sus = *sus;
    a.tr = *traj;
    a.n = (uint32_t)n;
    a.cap = (uint32_t)cap;
    hipStream_t s = (hipStream_t)stream;
    const int obs = cfg->obs_mode;
    if (obs == G2048_OBS_ONEHOT) {   // persistent: one workgroup per CU, 64 slots each
        int64_t grid = (n_order + 63) / 64;
        if (grid > (int64_t)cus) grid = cus;
        return activation == G2048_ACT_RELU ? launch_deep_roll<G2048_OBS_ONEHOT, 0, 64>(a, (int)grid, s)
                                            : launch_deep_roll<G2048_OBS_ONEHOT, 1, 64>(a, (int)grid, s);
    }
    int64_t grid = (n_order + 31) / 32;
    if (grid > 2 * (int64_t)cus) grid = 2 * (int64_t)cus;   // persistent; the slots refill from the queue
    if (obs == G2048_OBS_LOG2)
        return activation == G2048_ACT_RELU ? launch_deep_roll<G2048_OBS_LOG2, 0, 32>(a, (int)grid, s)
                                            : launch_deep_roll<G2048_OBS_LOG2, 1, 32>(a, (int)grid, s);
    return activation == G2048_ACT_RELU ? launch_deep_roll<G2048_OBS_RAW, 0, 32>(a, (int)grid, s)
                                        : launch_deep_roll<G2048_OBS_RAW, 1, 32>(a, (int)grid, s);
}

int g2048_deep_hidden(const float* packed, int n_hidden, const int32_t* hidden, int activation, int obs_mode,
                      float obs_scale, const uint64_t* boards, int64_t n, int layer, float* out, int64_t ld,
                      void* stream) {
    DeepNet net;
    if (obs_mode != G2048_OBS_LOG2 && obs_mode != G2048_OBS_RAW && obs_mode != G2048_OBS_ONEHOT)
        return dfail(G2048_EINVAL, "deep policy: obs_mode must be log2, raw or onehot");
    if (!deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, net))
        return dfail(G2048_EINVAL, "deep policy: 1..4 hidden layers of 1..256 units");
    if (layer < 0 || layer >= n_hidden || ld < 32 * net.nt[layer] || n < 0 || n > (int64_t)0xFFFFFFE0)
        return dfail(G2048_EINVAL, "deep hidden: bad layer / ld / n");
    if (activation != G2048_ACT_RELU && activation != G2048_ACT_SIGMOID)
        return dfail(G2048_EINVAL, "Unsupported activation");
    if (!packed || (n > 0 && (!boards || !out))) return dfail(G2048_EINVAL, "deep hidden: NULL buffer");
    if (n == 0) return G2048_OK;
    const int ksplit = deep_grad_variant(net).ksplit;   // the full net's gradient instantiation's k-split rule
    hipStream_t s = (hipStream_t)stream;
    net.L = layer + 1;   // truncated: deep_forward stops after `layer` (offsets of the kept layers unchanged)
    const int64_t groups = (n + 31) / 32, cap = 2 * (int64_t)device_cus();
    const int grid = (int)(groups < cap ? groups : cap);
#define G2048_HIDDEN(O, A)                                                                                      \
    do {                                                                                                            \
        if (ksplit == 1)                                                                                            \
            hipLaunchKernelGGL((deep_hidden_kernel<O, A, 1>), dim3(grid), dim3(kDeepBlock), 0, s, net,          \
                               packed, boards, (uint32_t)n, obs_scale, out, (uint32_t)ld);                      \
        else if (ksplit == 2)                                                                                       \
            hipLaunchKernelGGL((deep_hidden_kernel<O, A, 2>), dim3(grid), dim3(kDeepBlock), 0, s, net,          \
                               packed, boards, (uint32_t)n, obs_scale, out, (uint32_t)ld);                      \
        else                                                                                                        \
            hipLaunchKernelGGL((deep_hidden_kernel<O, A, 0>), dim3(grid), dim3(kDeepBlock), 0, s, net,          \
                               packed, boards, (uint32_t)n, obs_scale, out, (uint32_t)ld);                      \
    } while (0)
    if (obs_mode == G2048_OBS_ONEHOT) {
        if (activation == G2048_ACT_RELU) G2048_HIDDEN(G2048_OBS_ONEHOT, 0); else G2048_HIDDEN(G2048_OBS_ONEHOT, 1);
    } else if (obs_mode == G2048_OBS_LOG2) {
        if (activation == G2048_ACT_RELU) G2048_HIDDEN(G2048_OBS_LOG2, 0); else G2048_HIDDEN(G2048_OBS_LOG2, 1);
    } else {
        if (activation == G2048_ACT_RELU) G2048_HIDDEN(G2048_OBS_RAW, 0); else G2048_HIDDEN(G2048_OBS_RAW, 1);
    }
#undef G2048_HIDDEN
    return check_hip();
}

int64_t g2048_deep_grad_pack_size(int obs_mode, int n_hidden, const int32_t* hidden) {
    DeepNet n;
    if (!deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, n)) return -1;
    const int64_t s = deep_grad_layout(n).boff[n.L];
    return s > 0 ? s : 1;
}

int64_t g2048_deep_grad_slab(int obs_mode, int n_hidden, const int32_t* hidden) {
    DeepNet n;
    if (obs_mode != G2048_OBS_LOG2 && obs_mode != G2048_OBS_RAW && obs_mode != G2048_OBS_ONEHOT) return -1;
    if (!deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, n)) return -1;
    if (deep_grad_variant(n).nw == 0) return -1;   // not covered
    return deep_grad_layout(n).pslab;
}

int g2048_deep_grad_parts(int obs_mode, int n_hidden, const int32_t* hidden) {
    DeepNet n;
    if (g2048_deep_grad_slab(obs_mode, n_hidden, hidden) < 0) return -1;
    deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, n);
    return deep_grad_variant(n).per_cu * device_cus();
}

int g2048_deep_grad_passes(int obs_mode, int n_hidden, const int32_t* hidden) {
    DeepNet n;
    if (g2048_deep_grad_slab(obs_mode, n_hidden, hidden) < 0) return -1;
    deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, n);
    return deep_grad_variant(n).passes;
}

int g2048_deep_grad_pack(const float* const* W, int obs_mode, int n_hidden, const int32_t* hidden, float* packed,
                         int64_t packed_len, void* stream) {
    DeepNet n;
    if (!deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, n))
        return dfail(G2048_EINVAL, "deep gradient: 1..4 hidden layers of 1..256 units");
    const DeepGradLayout g = deep_grad_layout(n);
    if (!W || !packed) return dfail(G2048_EINVAL, "deep gradient: NULL buffer");
    if (packed_len < g.boff[n.L]) return dfail(G2048_EINVAL, "deep gradient: packed buffer too small");
    if (g.boff[n.L] == 0) return G2048_OK;   // one hidden layer: no dense backward fragments
    DeepGradPackArgs a{};
    for (int l = 0; l < n_hidden; l++) {
        if (l >= 1 && !W[l]) return dfail(G2048_EINVAL, "deep gradient: NULL weight");
        a.W[l] = W[l];
        a.h[l] = hidden[l];
        a.nt[l] = n.nt[l];
    }
    for (int l = 0; l <= n_hidden; l++) a.boff[l] = g.boff[l];
    a.L = n_hidden;
    a.dst = packed;
    const int64_t total = g.boff[n.L];
    const int grid = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(deep_grad_pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    return check_hip();
}

}  // extern "C"

namespace {
template <int OBS, int ACT, int NW, int TPW, int KSPLIT, int NB = 32>
int launch_deep_grad_v(const DeepGradArgs& a, int grid, int64_t lds, hipStream_t s) {
    // the dynamic-LDS attribute is per kernel and device: one bit per device id, set on the first launch there
    // (two threads racing both set it, which is harmless)
    static std::atomic<uint64_t> attr_set{0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return dfail(G2048_EHIP, "deep gradient: hipGetDevice failed");
    const uint64_t bit = 1ull << (dev & 63);
    if (!(attr_set.load(std::memory_order_acquire) & bit)) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&deep_grad_kernel<OBS, ACT, NW, TPW, KSPLIT, NB>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return (void)hipGetLastError(), dfail(G2048_EHIP, "deep gradient: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
        attr_set.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL((deep_grad_kernel<OBS, ACT, NW, TPW, KSPLIT, NB>), dim3(grid), dim3(64 * NW), (unsigned)lds, s, a);
    return check_hip();
}

template <int OBS, int ACT>
int launch_deep_grad_pass(const DeepGradArgs& a, const DeepGradVariant& v, int grid, int64_t lds, hipStream_t s) {
    if constexpr (OBS == G2048_OBS_ONEHOT) {
        if (v.nb == 64) return launch_deep_grad_v<OBS, ACT, 8, 5, 0, 64>(a, grid, lds, s);
        if (v.tpw == 8) return launch_deep_grad_v<OBS, ACT, 8, 8, 1>(a, grid, lds, s);
    }
    return launch_deep_grad_v<OBS, ACT, 8, 6, 1>(a, grid, lds, s);
}
// one launch per range of dense dW tiles (v.passes; one for every net within the accumulator budget): each writes
// its tiles' partials, the first also the bias / output / first-layer ones, so the slab is complete after the last
template <int OBS, int ACT>
int launch_deep_grad(const DeepGradArgs& a0, const DeepGradVariant& v, int grid, int64_t lds, hipStream_t s) {
    DeepGradArgs a = a0;
    for (int p = 0; p < v.passes; p++) {
        a.tile0 = p * v.nw * v.tpw;
        a.first_pass = p == 0;
        a.last_pass = p == v.passes - 1;
        const int rc = launch_deep_grad_pass<OBS, ACT>(a, v, grid, lds, s);
        if (rc) return rc;
    }
    return G2048_OK;
}
}  // namespace


extern "C" {

int g2048_deep_grad(const float* packed, const float* grad_packed, int n_hidden, const int32_t* hidden,
                    int activation, int obs_mode, float obs_scale, int use_mask, const uint64_t* boards,
                    const uint8_t* actions, const float* coef, int critic, int loss, float huber_delta,
                    const float* target, float* delta_out, float* value_out, float* d0_out, int64_t n,
                    float* partials, int64_t nparts, const g2048_td_rows* td, void* stream) {
    if (n < 0 || n > (int64_t)0x7FFFFFE0) return dfail(G2048_EINVAL, "n out of range");
    if (activation != G2048_ACT_RELU && activation != G2048_ACT_SIGMOID)
        return dfail(G2048_EINVAL, "Unsupported activation");
    if (g2048_deep_grad_slab(obs_mode, n_hidden, hidden) < 0)
        return dfail(G2048_EINVAL, "deep gradient: net not covered (obs mode one-hot / log2 / raw, 1..4 hidden "
                                   "layers of 1..256 units)");
    if (critic && loss != 0 && loss != 1) return dfail(G2048_EINVAL, "Unknown critic loss type");
    if (!packed || !partials || (n > 0 && (!boards || !coef)) || (n > 0 && !critic && !actions) ||
        (n > 0 && critic && !target && !td) || (n > 0 && obs_mode == G2048_OBS_ONEHOT && !d0_out))
        return dfail(G2048_EINVAL, "deep gradient: NULL buffer");
    if (td && (!critic || (n > 0 && (!td->lane || !td->reward || !td->has_next || !td->v_next || !td->v_out))))
        return dfail(G2048_EINVAL, "deep gradient: TD rows are for the critic, with every buffer set");
    if (nparts < 1 || nparts > 65535) return dfail(G2048_EINVAL, "deep gradient: nparts out of range");
    DeepNet net;
    deep_layout(n_hidden, hidden, obs_mode == G2048_OBS_ONEHOT, net);
    const DeepGradLayout g = deep_grad_layout(net);
    if (g.boff[net.L] > 0 && !grad_packed) return dfail(G2048_EINVAL, "deep gradient: NULL backward fragments");
    DeepGradArgs a{};
    a.net = net;
    a.packed = packed;
    a.bpacked = grad_packed;
    const DeepGradVariant v = deep_grad_variant(net);
    int off = 0;
    for (int l = 0; l < net.L; l++) {
        a.boff[l] = g.boff[l];
        a.tile_begin[l] = g.tile_begin[l];
        a.aoff[l] = off;
        off += 32 * net.nt[l] * (v.nb + 1);
    }
    a.lds_tail = (int)deep_grad_act_floats(net, v.nw, v.nb);   // >= off: room for the output layer's reduction
    for (int l = 0; l <= net.L; l++) {
        a.pw[l] = g.pw[l];
        a.pb[l] = g.pb[l];
    }
    a.pslab = g.pslab;
    a.ntiles = g.ntiles;
    a.boards = boards;
    a.actions = actions;
    a.coef = coef;
    a.critic = critic;
    a.huber = loss == 1;
    a.huber_delta = huber_delta;
    a.target = target;
    a.delta_out = delta_out;
    a.v_out = value_out;
    a.d0_out = d0_out;
    a.has_td = td != nullptr;
    if (td) a.td = *td;
    a.part = partials;
    a.obs_scale = obs_scale;
    a.n = (uint32_t)n;
    a.use_mask = use_mask;
#if G2048_DEEP_DIAG
    a.diag = g_deep_diag;
#endif
    const int64_t lds = deep_grad_lds_bytes(net, v.nw, v.nb);
    hipStream_t s = (hipStream_t)stream;
    const int grid = (int)nparts;   // every workgroup writes its slab (zeros when it gets no group)
    if (obs_mode == G2048_OBS_ONEHOT)
        return activation == G2048_ACT_RELU ? launch_deep_grad<G2048_OBS_ONEHOT, 0>(a, v, grid, lds, s)
                                            : launch_deep_grad<G2048_OBS_ONEHOT, 1>(a, v, grid, lds, s);
    if (obs_mode == G2048_OBS_LOG2)
        return activation == G2048_ACT_RELU ? launch_deep_grad<G2048_OBS_LOG2, 0>(a, v, grid, lds, s)
                                            : launch_deep_grad<G2048_OBS_LOG2, 1>(a, v, grid, lds, s);
    return activation == G2048_ACT_RELU ? launch_deep_grad<G2048_OBS_RAW, 0>(a, v, grid, lds, s)
                                        : launch_deep_grad<G2048_OBS_RAW, 1>(a, v, grid, lds, s);
}

int g2048_onehot_layer1(const float* W1, const float* b1, int h1, int activation, const uint64_t* boards, int64_t m,
                        int64_t ld, float* out, void* stream) {
    if (m < 0 || h1 < 1 || ld < h1) return dfail(G2048_EINVAL, "one-hot layer 1: bad m / h1 / ld");
    if (activation != G2048_ACT_RELU && activation != G2048_ACT_SIGMOID)
        return dfail(G2048_EINVAL, "Unsupported activation");
    if (!W1 || !b1 || (m > 0 && (!boards || !out))) return dfail(G2048_EINVAL, "one-hot layer 1: NULL buffer");
    if (m == 0) return G2048_OK;
    const int64_t blocks = (m + 3) / 4;
    const int grid = (int)(blocks < 8 * device_cus() ? blocks : 8 * device_cus());
    hipStream_t s = (hipStream_t)stream;
    if (activation == G2048_ACT_RELU)
        hipLaunchKernelGGL(onehot_l1_kernel<0>, dim3(grid), dim3(256), 0, s, W1, b1, boards, h1, m, ld, out);
    else
        hipLaunchKernelGGL(onehot_l1_kernel<1>, dim3(grid), dim3(256), 0, s, W1, b1, boards, h1, m, ld, out);
    return check_hip();
}

int64_t g2048_onehot_dw1_slab(int h1) { return h1 < 1 || h1 > 256 ? -1 : (int64_t)kDw1Rows * h1; }

int g2048_onehot_dw1(const uint64_t* boards, const float* d1, int h1, int64_t m, int64_t ld, int64_t per,
                     float* partials, int64_t nparts, void* stream) {
    if (h1 < 1 || h1 > 256 || m < 0 || ld < h1 || per < 1) return dfail(G2048_EINVAL, "one-hot dW1: bad sizes");
    if (nparts != (m + per - 1) / per || nparts > 65535) return dfail(G2048_EINVAL, "one-hot dW1: nparts != ceil(m / per)");
    if (per * ld * 4 >= ((int64_t)1 << 31)) return dfail(G2048_EINVAL, "one-hot dW1: per x ld too large (2 GiB per slab range)");
    if (m > 0 && (!boards || !d1 || !partials)) return dfail(G2048_EINVAL, "one-hot dW1: NULL buffer");
    if (m == 0) return G2048_OK;
    // 16-byte rows for the LDS-DMA ring, whose whole 16-byte chunks end exactly at unit h1 (h1 % 4 == 0: a row's
    // last chunk never reads past s * ld + h1 - 1, which the header promises is valid memory)
    if (ld % 4 == 0 && h1 % 4 == 0 && ((uintptr_t)d1 & 15u) == 0)
        hipLaunchKernelGGL(onehot_dw1_ring_kernel, dim3((unsigned)nparts), dim3(64 * kDw1MaxWaves), 0,
                           (hipStream_t)stream, boards, d1, h1, m, ld, per, partials);
    else
        hipLaunchKernelGGL(onehot_dw1_mfma_kernel, dim3((unsigned)nparts), dim3(64 * kDw1MaxWaves), 0,
                           (hipStream_t)stream, boards, d1, h1, m, ld, per, partials);
    return check_hip();
}

}  // extern "C"
