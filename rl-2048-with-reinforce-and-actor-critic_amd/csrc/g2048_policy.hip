// g2048_policy.hip -- fused policy forward + action selection for the rollout (part of libg2048.so).
//
// Replaces, for the batched rollout, the chain forward_logits (src/MLP.py:159-196) -> logits_to_probs
// (:139-156) -> select_action's choice (src/reinforce_agent.py:178-190) for the reference's 2-hidden-layer MLP
// (obs width 16: "log2" / "raw"; hidden sizes <= 256; ReLU or Sigmoid; 4 actions).  One wave takes 32 boards:
//   * the obs are built in registers from the bitboards (no obs buffer round trip through HBM);
//   * layer 1 (H1^T = W1^T X^T) and layer 2 (H2^T = W2^T H1^T) run on v_mfma_f32_32x32x2_f32 -- exact fp32,
//     a k-ordered fmaf chain (cdna_hip_programming.md "FP32-input MFMA") -- with hidden units on the MFMA rows
//     and boards on its columns, so each layer-1 accumulator tile is, register for register, the B operand of a
//     layer-2 k-step (k order permuted consistently on both operands; no LDS round trip);
//   * bias + activation are applied to the accumulators in registers; layer 3 (4 outputs) is VALU fmaf over each
//     layer-2 tile as it completes, the two lane halves' partial sums are added by a cross-lane swap;
//   * the action is chosen by the same device code as g2048_sample (softmax_select in g2048_core.h).
// Weights are pre-packed (g2048_policy_pack) in MFMA fragment order, so every A fragment is one coalesced load
// (the packed net, <= 290 KB, stays L2-resident).  Hidden sizes are zero-padded to whole 32-unit tiles, which is
// exact: a padded unit's outgoing weights are zero.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>

#include "g2048.h"
#include "g2048_core.h"

using namespace g2048;

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// grad_kernel column stores are issued inside the MFMA loops that follow the values' computation, so they drain
// under the MFMAs (with one wave per SIMD a phase that stores its own 128 columns per lane stalls on the VMEM
// queue: vmcnt caps outstanding ops at 63): the d2^T values through the d1 loop (2 per k-tile; they are its B
// operand, already in registers), the a1^T values as the first output tile of the layer-2 loop reads them from LDS
// (DESIGN.md section 3 has the measured alternatives).
#ifndef G2048_DIAG
#define G2048_DIAG 0
#endif
#if G2048_DIAG
// diag build only: per-workgroup sums of rollout phase durations (s_memrealtime ticks): layer 1 + barrier,
// layer 2 + barrier, logits + choice + env step, claims; [4] = steps
constexpr int kRollDiagBlocks = 4096;
__device__ unsigned long long g_roll_ph[kRollDiagBlocks * 5];
// per-workgroup (wave 0) sums of grad_kernel phase durations: layer 1 (+ a1 columns), layer 2 + logits,
// softmax / loss + dW3, d2 (+ d2 columns), d1 + db1 + dW1; [5] = groups
__device__ unsigned long long g_grad_ph[kRollDiagBlocks * 6];
#endif

constexpr int kPolBlock = 256;   // 4 waves; two workgroups per CU (2 waves per SIMD)

// packed layout (floats), nt1 / nt2 = hidden tiles of 32:
//   w1f [nt1][8][64]         lane l of k-step s: W1[2s + (l>>5)][32t + (l&31)]
//   b1p [nt1][2][16]         half h, register r: b1[32t + row(r, h)]
//   w2f [nt2][nt1][4][64][4] lane l, k-step (t, r = 4q + u) at [o][t][q][l][u]: W2[32t + row(r, l>>5)][32o + (l&31)]
//                            (one 16-B load per lane fetches four consecutive k-steps)
//   b2p [nt2][2][16]
//   w3p [nt2][2][16][4]      W3[32o + row(r, h)][a]
//   b3  [4]
// row(r, h) = (r & 3) + 8 (r >> 2) + 4 h: the hidden unit held by accumulator register r in lane half h.
__host__ __device__ inline int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

struct PolLayout {
    int64_t w1f, b1p, w2f, b2p, w3p, b3, total;
};

__host__ __device__ constexpr PolLayout pol_layout(int nt1, int nt2) {
    PolLayout L{};
    L.w1f = 0;
    L.b1p = L.w1f + (int64_t)nt1 * 8 * 64;
    L.w2f = L.b1p + (int64_t)nt1 * 32;
    L.b2p = L.w2f + (int64_t)nt2 * nt1 * 16 * 64;
    L.w3p = L.b2p + (int64_t)nt2 * 32;
    L.b3 = L.w3p + (int64_t)nt2 * 32 * 4;
    L.total = L.b3 + 4;
    return L;
}

struct PackArgs {
    const float *W1, *b1, *W2, *b2, *W3, *b3;
    int h1, h2, nt1, nt2;
    float* out;
    int64_t total;
};

// one thread per packed float
__global__ void __launch_bounds__(256) pack_kernel(PackArgs a) {
    const PolLayout L = pol_layout(a.nt1, a.nt2);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.total; q += (int64_t)gridDim.x * blockDim.x) {
        float v = 0.0f;
        if (q < L.b1p) {
            const int64_t x = q - L.w1f;
            const int lane = (int)(x & 63), s = (int)((x >> 6) & 7), t = (int)(x >> 9);
            const int k = 2 * s + (lane >> 5), j = 32 * t + (lane & 31);
            v = j < a.h1 ? a.W1[k * a.h1 + j] : 0.0f;
        } else if (q < L.w2f) {
            const int64_t x = q - L.b1p;
            const int r = (int)(x & 15), h = (int)((x >> 4) & 1), t = (int)(x >> 5);
            const int j = 32 * t + acc_row(r, h);
            v = j < a.h1 ? a.b1[j] : 0.0f;
        } else if (q < L.b2p) {
            const int64_t x = q - L.w2f;
            const int u = (int)(x & 3), lane = (int)((x >> 2) & 63), r = 4 * (int)((x >> 8) & 3) + u;
            const int64_t tt = x >> 10;
            const int t = (int)(tt % a.nt1), o = (int)(tt / a.nt1);
            const int k = 32 * t + acc_row(r, lane >> 5), j = 32 * o + (lane & 31);
            v = (k < a.h1 && j < a.h2) ? a.W2[(int64_t)k * a.h2 + j] : 0.0f;
        } else if (q < L.w3p) {
            const int64_t x = q - L.b2p;
            const int r = (int)(x & 15), h = (int)((x >> 4) & 1), o = (int)(x >> 5);
            const int j = 32 * o + acc_row(r, h);
            v = j < a.h2 ? a.b2[j] : 0.0f;
        } else if (q < L.b3) {
            const int64_t x = q - L.w3p;
            const int act = (int)(x & 3), r = (int)((x >> 2) & 15), h = (int)((x >> 6) & 1), o = (int)(x >> 7);
            const int j = 32 * o + acc_row(r, h);
            v = j < a.h2 ? a.W3[j * 4 + act] : 0.0f;
        } else {
            v = a.b3[q - L.b3];
        }
        a.out[q] = v;
    }
}

struct PolArgs {
    const float* net;
    const uint64_t* boards;
    const uint32_t* lane_state;   // env lane state words (G2048_LS_ACTIVE, step count) or NULL
    const int32_t* lane_index;   // entry j -> lane lane_index[j] (NULL: lane j)
    uint64_t *rs, *inc, *buf;
    uint64_t key;
    const uint64_t* lane_seed;
    float* probs_out;
    float* logits_out;
    uint8_t* actions;
    float obs_scale;
    uint32_t n;
    int use_mask, greedy;
};

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

// Waves per SIMD: 2 while the layer-1 activations (16 x NT1 registers) leave room; the 256-unit first layer
// (128 registers of activations + the layer-2 A fragments in flight) takes the whole 512-register file.
template <int NT1>
constexpr int pol_waves_per_simd() { return NT1 >= 8 ? 1 : 2; }

// Small tensors of the packed net staged in LDS (layer-1 fragments, biases, layer 3: <= 22.5 KB); the
// layer-2 fragments (the bulk, up to 256 KB) stay in L2 and are streamed by mlp_logits.
template <int NT1, int NT2>
struct NetSmem {
    static constexpr PolLayout L = pol_layout(NT1, NT2);
    static constexpr int kFloats = (int)(L.w2f - L.w1f) + (int)(L.total - L.b2p);
    float v[kFloats];
    __device__ void load(const float* net) {   // whole workgroup; caller syncs
        for (int k = threadIdx.x; k < kFloats; k += blockDim.x) v[k] = k < (int)L.w2f ? net[k] : net[L.b2p + (k - (int)L.w2f)];
    }
    __device__ const float* w1f() const { return v; }
    __device__ const float* b1p() const { return v + L.b1p; }
    __device__ const float* b2p() const { return v + L.w2f; }
    __device__ const float* w3p() const { return v + L.w2f + (L.w3p - L.b2p); }
    __device__ const float* b3() const { return v + L.w2f + (L.b3 - L.b2p); }
};

// The 4 logits of board b (this lane's column; both lane halves return the same values) for one wave of 32
// boards: layer 1 and 2 on fp32 MFMA, layer 3 on VALU (see the file comment).  w2q: the layer-2 fragments
// (float4) offset by this lane.
template <int NT1, int NT2, int ACT, int OBS>
__device__ __forceinline__ void mlp_logits(const NetSmem<NT1, NT2>& sm, const float4* __restrict__ w2q, uint64_t b,
                                           float obs_scale, int lane, float lg[4]) {
    const int h = lane >> 5;
    // first layer-2 fragments in flight while layer 1 runs
    float4 fa[4];
#pragma unroll
    for (int q = 0; q < 4; q++) fa[q] = w2q[q * 64];
    // X^T k-step s: row k = 2s + h (obs feature), column = board
    float x[8];
#pragma unroll
    for (int s = 0; s < 8; s++) x[s] = obs_value<OBS>(b, 2 * s + h, obs_scale);
    // layer 1: H1^T tile t (32 hidden x 32 boards), bias + activation in registers
    float h1[NT1][16];
    const float* w1f = sm.w1f();
#pragma unroll
    for (int t = 0; t < NT1; t++) {
        floatx16 acc = {};
#pragma unroll
        for (int s = 0; s < 8; s++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1f[(t * 8 + s) * 64 + lane], x[s], acc, 0, 0, 0);
        const float4* bb = reinterpret_cast<const float4*>(sm.b1p() + (t * 2 + h) * 16);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float4 bv = bb[q];
            h1[t][4 * q + 0] = activate<ACT>(acc[4 * q + 0] + bv.x);
            h1[t][4 * q + 1] = activate<ACT>(acc[4 * q + 1] + bv.y);
            h1[t][4 * q + 2] = activate<ACT>(acc[4 * q + 2] + bv.z);
            h1[t][4 * q + 3] = activate<ACT>(acc[4 * q + 3] + bv.w);
        }
    }
    // layer 2 tile by tile (A fragments of k-tile t+1 loaded while tile t's 16 MFMAs run, across tiles),
    // each output tile folded into the 4 logits as soon as it is done
    lg[0] = lg[1] = lg[2] = lg[3] = 0.0f;
#pragma unroll 1
    for (int o = 0; o < NT2; o++) {
        floatx16 acc = {};
        const float4* wo = w2q + o * NT1 * 4 * 64;
#pragma unroll
        for (int t = 0; t < NT1; t++) {
            float4 fb[4];
            const float4* nx = (t + 1 < NT1) ? wo + (t + 1) * 4 * 64 : (o + 1 < NT2 ? wo + NT1 * 4 * 64 : w2q);
#pragma unroll
            for (int q = 0; q < 4; q++) fb[q] = nx[q * 64];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, h1[t][4 * q + 0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, h1[t][4 * q + 1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, h1[t][4 * q + 2], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, h1[t][4 * q + 3], acc, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) fa[q] = fb[q];
        }
        const float4* bb = reinterpret_cast<const float4*>(sm.b2p() + (o * 2 + h) * 16);
        const float4* w3 = reinterpret_cast<const float4*>(sm.w3p() + (o * 2 + h) * 64);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float4 bv = bb[q];
            const float hv[4] = {activate<ACT>(acc[4 * q + 0] + bv.x), activate<ACT>(acc[4 * q + 1] + bv.y),
                                 activate<ACT>(acc[4 * q + 2] + bv.z), activate<ACT>(acc[4 * q + 3] + bv.w)};
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const float4 wv = w3[4 * q + u];
                lg[0] = fmaf(hv[u], wv.x, lg[0]);
                lg[1] = fmaf(hv[u], wv.y, lg[1]);
                lg[2] = fmaf(hv[u], wv.z, lg[2]);
                lg[3] = fmaf(hv[u], wv.w, lg[3]);
            }
        }
    }
    // the two lane halves hold different hidden units of the same board
    const float* b3 = sm.b3();
#pragma unroll
    for (int k = 0; k < 4; k++) lg[k] = (lg[k] + __shfl_xor(lg[k], 32, 64)) + b3[k];
}

__device__ __forceinline__ uint64_t shfl64_(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t mask_word_of(uint64_t b) {
    const uint32_t m = action_mask(b);   // int8[4] as one word: byte a = bit a
    return (m & 1u) | ((m & 2u) << 7) | ((m & 4u) << 14) | ((m & 8u) << 21);
}

template <int NT1, int NT2, int ACT, int OBS, int RNG>
__global__ void __launch_bounds__(kPolBlock, pol_waves_per_simd<NT1>()) policy_kernel(PolArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    __shared__ NetSmem<NT1, NT2> sm;
    sm.load(a.net);
    __syncthreads();
    const float4* __restrict__ w2q = reinterpret_cast<const float4*>(a.net + NetSmem<NT1, NT2>::L.w2f) + lane;
    const uint32_t waves = gridDim.x * (kPolBlock / 64);
    const uint32_t groups = (a.n + 31u) >> 5;
    for (uint32_t gi = blockIdx.x * (kPolBlock / 64) + (threadIdx.x >> 6); gi < groups; gi += waves) {
        const uint32_t j = gi * 32u + (uint32_t)col;            // this lane's entry (both halves)
        const uint32_t jc = j < a.n ? j : a.n - 1u;
        const uint32_t i = a.lane_index ? (uint32_t)a.lane_index[jc] : jc;   // its board / lane
        const uint64_t b = a.boards[i];
        float lg[4];
        mlp_logits<NT1, NT2, ACT, OBS>(sm, w2q, b, a.obs_scale, lane, lg);
        const uint32_t ls = a.lane_state ? a.lane_state[i] : G2048_LS_ACTIVE;
        if (h == 0 && j < a.n && (ls & G2048_LS_ACTIVE)) {
            if (a.logits_out) reinterpret_cast<float4*>(a.logits_out)[i] = make_float4(lg[0], lg[1], lg[2], lg[3]);
            const uint32_t mw = a.use_mask ? mask_word_of(b) : 0x01010101u;
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


// ---------------------------------------------------------------------------------------------------- rollout
// The whole batched rollout (ReinforceAgent.run_episode, src/reinforce_agent.py:195-252, for n (env_seed,
// policy_seed) pairs) in one persistent launch: each wave runs 32 episode slots; per step the MLP above picks
// every slot's action (Generator.choice on the slot's policy stream, or greedy), Game2048Env.step runs in
// registers (env_step_pcg, row tables read through L1/L2), and the step's trajectory row is written.  A slot
// whose episode ends writes the episode's results and takes the next episode from a.next (one atomic per
// episode), so no work is spent on finished episodes and there is no per-step host round trip.  Both lane halves
// carry every slot (the MFMA layout); the lower half writes.
struct RolloutArgs {
    const float* net;
    const uint8_t* tab;
    RewardCfg rc;
    int64_t max_steps;
    float obs_scale;
    int use_mask, greedy;
    const uint64_t *env_rs, *env_inc, *env_buf;   // default_rng(env_seed) per episode (g2048_seed_pcg64)
    const uint64_t *pol_rs, *pol_inc, *pol_buf;   // default_rng(policy_seed) per episode
    uint32_t* next;                               // episode queue (zero before the launch)
    uint64_t* boards;                             // [cap, n] time-major trajectory rows
    uint8_t* actions;
    double* rewards;                              // fp64: the Python float run_episode records
    uint8_t* flags;
    float* probs;                                 // [cap, n, 4] or NULL
    int32_t* lengths;                             // per episode
    double* totals;
    uint8_t* max_tile;
    uint64_t* final_board;
    uint32_t n, cap;
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

struct GLine {
    const uint16_t* p;
    __device__ uint32_t operator()(uint32_t o) const { return p[o]; }
};
struct GCode {
    const uint8_t* p;
    __device__ uint32_t operator()(uint32_t o) const { return (p[o >> 1] >> ((o & 1u) << 2)) & 15u; }
};

// LDS of one rollout workgroup: the small net tensors, the layer-1 activations of the current step in
// layer-2 B-fragment order, the per-wave partial logits and the episode-claim broadcast.
template <int NT1, int NT2>
struct RollSmem {
    NetSmem<NT1, NT2> net;
    float4 h1f[NT1][4][64];      // [k-tile t][r / 4][lane]: registers 4q..4q+3 of layer-1 tile t
    float part[4][32][4];        // [wave][slot][action]
    uint32_t claim[32];
};

// One workgroup = 32 episode slots, TWO workgroups per CU; its 4 waves split every step's MLP: wave w computes the
// layer-1 tiles and the layer-2 output tiles congruent to w mod 4 (a quarter of the MFMAs), exchanging the layer-1
// activations and the partial logits through LDS (two barriers per step), so a step takes about a quarter of the
// one-wave latency.  Each wave streams its quarter of the layer-2 weight fragments from L2 every step (the next k-tile
// in flight; the first issued before layer 1), which leaves the registers for a second workgroup per CU: the
// two workgroups' steps interleave on every SIMD, so one's MFMAs run while the other's env step, layer 1 and
// barriers do (one workgroup per CU with the weights resident in registers left the MFMAs idle for those phases).
// Every wave holds the same logits and runs the same choice and env step on the same slot state (so no per-slot
// state is broadcast); wave 0 writes the trajectory and claims episodes for the workgroup.
constexpr int kRollBlocksPerCU = 2;

template <int NT1, int NT2, int ACT, int OBS>
__global__ void __launch_bounds__(kPolBlock, kRollBlocksPerCU) rollout_kernel(RolloutArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31, w = threadIdx.x >> 6;
    __shared__ RollSmem<NT1, NT2> S;
    S.net.load(a.net);
    const GLine lut{reinterpret_cast<const uint16_t*>(a.tab)};
    const GCode code{a.tab + 2 * 65536};
    // this wave's layer-2 fragment stream: output tiles o = w + 4 k2 (those < NT2), k-tiles tt; stream index
    // i = k2 * NT1 + tt; the index past the end re-reads the first k-tile (unused)
    constexpr int kOwn = (NT2 + 3) / 4;
    // Loads through a buffer resource: this lane's voffset (lane * 16) plus a scalar k-tile offset -- 64-bit
    // per-fragment addresses were hoisted out of the step loop (128 registers) and spilled.
    const int ws = __builtin_amdgcn_readfirstlane(w);
    const int nown = (NT2 - ws + 3) / 4;                  // own output tiles (0 when w >= NT2)
    const int nkt = nown * NT1;
    const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.net + NetSmem<NT1, NT2>::L.w2f), 0, NT2 * NT1 * 1024 * 4, 0x00020000);
    const uint32_t fvo = (uint32_t)lane * 16u;
    const auto frag = [&](int i, float4 f[4]) {
        const int ii = i < nkt ? i : 0;
        const int o = ws + 4 * (ii / NT1), tt = ii % NT1;
        const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(((o < NT2 ? o : 0) * NT1 + tt) * 4096));
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rw2, (int)fvo, (int)(base + 1024u * q), 0);
            f[q] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
        }
    };
    // episode claims for the slots that need one (identical `need` in all waves): wave 0 takes them with one
    // atomic and publishes them; every wave must call this together (it contains barriers)
    const auto claim = [&](bool need, uint32_t cur) -> uint32_t {
        if (w == 0) {
            const uint64_t bal = __ballot(need && h == 0);
            uint32_t base = 0;
            if (bal) {
                const int leader = __builtin_ctzll(bal);
                if (lane == leader) base = atomicAdd(a.next, (uint32_t)__popcll(bal));
                base = (uint32_t)__shfl((int)base, leader, 64);
            }
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            if (h == 0) S.claim[col] = need ? base + rank : cur;
        }
        __syncthreads();
        const uint32_t v = S.claim[col];
        __syncthreads();
        return v;
    };
    uint32_t ep = claim(true, 0u);
    bool drained = __ballot(ep >= a.n) != 0ull;           // block-uniform: the queue is empty (claims only grow)
    uint32_t t = 0, sc = 0, mt = 2;
    uint64_t b = 0;
    double total = 0.0;
    Pcg64 ge{}, gp{};
    const auto start = [&]() {
        if (ep < a.n) {
            ge = load_stream(a.env_rs, a.env_inc, a.env_buf, ep);
            gp = load_stream(a.pol_rs, a.pol_inc, a.pol_buf, ep);
            b = spawn_pcg(spawn_pcg(0ull, ge), ge);       // Game2048.reset (src/game2048.py:26-34)
            t = 0;
            sc = 0;
            mt = 2;                                       // max_tile_seen = 4 (src/env.py:188)
            total = 0.0;
        }
    };
    start();
#if G2048_DIAG
    unsigned long long ph[5] = {0, 0, 0, 0, 0};
    unsigned long long tp = __builtin_amdgcn_s_memrealtime();
#define ROLL_PH(k)                                                        \
    do {                                                                  \
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();  \
        ph[k] += tn - tp;                                                 \
        tp = tn;                                                          \
    } while (0)
#else
#define ROLL_PH(k) \
    do {           \
    } while (0)
#endif
    while (__ballot(ep < a.n)) {                         // block-uniform (all waves hold the same slot state)
        float4 fa[4];                                     // layer-2 k-tile 0, in flight through layer 1
        frag(0, fa);
        // ---- layer 1: this wave's tiles -> LDS
        float x[8];
#pragma unroll
        for (int s2 = 0; s2 < 8; s2++) x[s2] = obs_value<OBS>(b, 2 * s2 + h, a.obs_scale);
        const float* w1f = S.net.w1f();
#pragma unroll
        for (int tt = 0; tt < NT1; tt++) {
            if ((tt & 3) != w) continue;
            floatx16 acc = {};
#pragma unroll
            for (int s2 = 0; s2 < 8; s2++)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1f[(tt * 8 + s2) * 64 + lane], x[s2], acc, 0, 0, 0);
            const float4* bb = reinterpret_cast<const float4*>(S.net.b1p() + (tt * 2 + h) * 16);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4 bv = bb[q];
                S.h1f[tt][q][lane] = make_float4(activate<ACT>(acc[4 * q + 0] + bv.x), activate<ACT>(acc[4 * q + 1] + bv.y),
                                                 activate<ACT>(acc[4 * q + 2] + bv.z), activate<ACT>(acc[4 * q + 3] + bv.w));
            }
        }
        __syncthreads();
        ROLL_PH(0);
        // ---- layer 2: this wave's output tiles (B from LDS, A streamed), folded into partial logits
        float lgp[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k2 = 0; k2 < kOwn; k2++) {
            const int o = ws + 4 * k2;
            if (o >= NT2) continue;                         // wave-uniform
            // a compiler memory barrier: otherwise the layer-1 activations' LDS reads (the same for every own
            // tile) are kept from the first tile for the next, 128 registers, which spill at 2 waves per SIMD
            asm volatile("" ::: "memory");
            floatx16 acc = {};
#pragma unroll
            for (int tt = 0; tt < NT1; tt++) {
                asm volatile("" ::: "memory");              // (the same per k-tile: its 4 LDS reads stay here)
                float4 fb[4];                               // k-tile i + 1 of the stream
                frag(k2 * NT1 + tt + 1, fb);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4 hb = S.h1f[tt][q][lane];
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, hb.x, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, hb.y, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, hb.z, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, hb.w, acc, 0, 0, 0);
                }
#pragma unroll
                for (int q = 0; q < 4; q++) fa[q] = fb[q];
            }
            const float4* bb = reinterpret_cast<const float4*>(S.net.b2p() + (o * 2 + h) * 16);
            const float4* w3 = reinterpret_cast<const float4*>(S.net.w3p() + (o * 2 + h) * 64);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4 bv = bb[q];
                const float hv[4] = {activate<ACT>(acc[4 * q + 0] + bv.x), activate<ACT>(acc[4 * q + 1] + bv.y),
                                     activate<ACT>(acc[4 * q + 2] + bv.z), activate<ACT>(acc[4 * q + 3] + bv.w)};
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const float4 wv = w3[4 * q + u];
                    lgp[0] = fmaf(hv[u], wv.x, lgp[0]);
                    lgp[1] = fmaf(hv[u], wv.y, lgp[1]);
                    lgp[2] = fmaf(hv[u], wv.z, lgp[2]);
                    lgp[3] = fmaf(hv[u], wv.w, lgp[3]);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) lgp[k] += __shfl_xor(lgp[k], 32, 64);
        if (h == 0) {
#pragma unroll
            for (int k = 0; k < 4; k++) S.part[w][col][k] = lgp[k];
        }
        __syncthreads();
        ROLL_PH(1);
        // ---- every wave: the same logits, choice and env step
        const float* b3 = S.net.b3();
        float lg[4];
#pragma unroll
        for (int k = 0; k < 4; k++) lg[k] = (((S.part[0][col][k] + S.part[1][col][k]) + S.part[2][col][k]) + S.part[3][col][k]) + b3[k];
        if (ep < a.n) {
            const uint32_t mw = a.use_mask ? mask_word_of(b) : 0x01010101u;
            const double u = a.greedy ? 0.0 : pcg_random(gp);
            float p[4];
            const uint32_t act = softmax_select(lg, mw, a.use_mask != 0, a.greedy != 0, u, p);
            const StepValues ov = env_step_pcg(b, act, sc, mt, ge, a.rc, a.max_steps, lut, code);
            const double r = ov.reward;
            total += r;                            // total_reward += float(reward) (src/reinforce_agent.py:233)
            if (w == 0 && h == 0) {
                const size_t row = (size_t)t * a.n + ep;
                a.boards[row] = b;
                a.actions[row] = (uint8_t)act;
                a.rewards[row] = r;
                a.flags[row] = (uint8_t)ov.flags;
                if (a.probs) reinterpret_cast<float4*>(a.probs)[row] = make_float4(p[0], p[1], p[2], p[3]);
            }
            b = ov.board;
            t += 1;
            if ((ov.flags & (kFTerminated | kFTruncated)) != 0u || t >= a.cap) {
                if (w == 0 && h == 0) {
                    a.lengths[ep] = (int32_t)t;
                    a.totals[ep] = total;
                    a.max_tile[ep] = (uint8_t)mt;
                    a.final_board[ep] = b;
                }
                ep = a.n;
            }
        }
        ROLL_PH(2);
        const bool need = ep >= a.n;
        if (!drained && __ballot(need)) {                // block-uniform
            const uint32_t fresh = claim(need, ep);
            if (need && fresh < a.n) {
                ep = fresh;
                start();
            }
            drained = __ballot(need && fresh >= a.n) != 0ull;
        }
        ROLL_PH(3);
#if G2048_DIAG
        ph[4] += 1;
#endif
    }
#if G2048_DIAG
    if (threadIdx.x == 0 && blockIdx.x < kRollDiagBlocks)
        for (int k = 0; k < 5; k++) g_roll_ph[blockIdx.x * 5 + k] = ph[k];
#endif
}

template <int NT1, int NT2, int ACT, int OBS>
void launch_pol_rng(const PolArgs& a, int rng, int grid, hipStream_t s) {
    if (rng == G2048_RNG_PCG64)
        hipLaunchKernelGGL((policy_kernel<NT1, NT2, ACT, OBS, G2048_RNG_PCG64>), dim3(grid), dim3(kPolBlock), 0, s, a);
    else
        hipLaunchKernelGGL((policy_kernel<NT1, NT2, ACT, OBS, G2048_RNG_PHILOX>), dim3(grid), dim3(kPolBlock), 0, s, a);
}

template <int NT1, int NT2, int ACT>
void launch_pol_obs(const PolArgs& a, int obs, int rng, int grid, hipStream_t s) {
    if (obs == G2048_OBS_LOG2) launch_pol_rng<NT1, NT2, ACT, G2048_OBS_LOG2>(a, rng, grid, s);
    else launch_pol_rng<NT1, NT2, ACT, G2048_OBS_RAW>(a, rng, grid, s);
}

template <int NT1, int NT2>
void launch_pol_act(const PolArgs& a, int act, int obs, int rng, int grid, hipStream_t s) {
    if (act == G2048_ACT_RELU) launch_pol_obs<NT1, NT2, 0>(a, obs, rng, grid, s);
    else launch_pol_obs<NT1, NT2, 1>(a, obs, rng, grid, s);
}

template <int NT1>
void launch_pol_nt2(const PolArgs& a, int nt2, int act, int obs, int rng, int grid, hipStream_t s) {
    switch (nt2) {
        case 1: launch_pol_act<NT1, 1>(a, act, obs, rng, grid, s); break;
        case 2: launch_pol_act<NT1, 2>(a, act, obs, rng, grid, s); break;
        case 4: launch_pol_act<NT1, 4>(a, act, obs, rng, grid, s); break;
        default: launch_pol_act<NT1, 8>(a, act, obs, rng, grid, s); break;
    }
}

// ---------------------------------------------------------------------------------------------------- gradient
// The actor branch of update_batch (src/reinforce_agent.py:502-555: _policy_gradient_step :328-354,
// _backpropagation :639-678, _activation_derivative :624-636) for a batch of samples (valid steps), one wave per
// 32 samples, fused: forward (as mlp_logits, keeping both hidden layers in registers), masked softmax,
// g = (onehot(a) - p) * coef (coef = advantage * rank_w / (T_i * n), from the host), the output-layer delta
// d2 = act'(a2) * (W3 g) on VALU, the input delta d1 = act'(a1) * (W2 d2) on MFMA (W2 packed by g2048_grad_pack
// in A-fragment order; d2 tiles are its B operands register for register, like layer 2 of the forward), and the
// small weight gradients dW1 (x^T d1), db1, dW3 (a2^T g), db3 on v_mfma_f32_16x16x4f32 through a per-wave LDS
// transpose, accumulated per wave in LDS across the wave's sample groups.  The one large weight gradient,
// dW2 = a1^T d2 and db2 = sum d2, is left to g2048_dw2 (g2048_dw2.hip) over the a1^T / d2^T columns this kernel
// writes (the accumulator layout puts 32 consecutive samples of one unit in a lane half: two 64-B runs, one in
// each of two 16-column blocks).
// Packed input-delta weights: w2b [nt1][nt2][4][64][4]: lane l, k-step (t2, r = 4q + u) of output tile o1 at
// [o1][t2][q][l][u]: W2[32 o1 + (l & 31)][32 t2 + row(r, l >> 5)].
struct GradPackArgs {
    const float* W2;
    int h1, h2, nt1, nt2;
    float* out;
    int64_t total;
};

__global__ void __launch_bounds__(256) grad_pack_kernel(GradPackArgs a) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.total; q += (int64_t)gridDim.x * blockDim.x) {
        const int u = (int)(q & 3), lane = (int)((q >> 2) & 63), r = 4 * (int)((q >> 8) & 3) + u;
        const int64_t tt = q >> 10;
        const int t2 = (int)(tt % a.nt2), o1 = (int)(tt / a.nt2);
        const int i = 32 * o1 + (lane & 31), k = 32 * t2 + acc_row(r, lane >> 5);
        a.out[q] = (i < a.h1 && k < a.h2) ? a.W2[(int64_t)i * a.h2 + k] : 0.0f;
    }
}

// floats of one wave's partial gradients: dW1 [16][H1p], db1 [H1p], dW3 [H2p][4], db3 [4]
__host__ __device__ constexpr int64_t grad_part_floats(int nt1, int nt2) { return 17 * 32 * nt1 + 4 * 32 * nt2 + 4; }

struct GradArgs {
    const float* net;        // g2048_policy_pack layout
    const float* w2b;        // g2048_grad_pack layout
    const uint64_t* boards;  // [n] sample boards (the obs of each step)
    const uint8_t* actions;  // [n]
    const float* coef;       // [n] advantage * step weight
    float* a1t;              // a1^T: [R][ld] in 16-column blocks (col_store), R = 32 max(NT1, NT2)
    float* d2t;              // d2^T: the same layout
    float* part;             // [waves][grad_part_floats]
    uint32_t n, ld;          // samples; columns (a multiple of 32, >= n): samples n..ld-1 have coef 0
    float obs_scale;
    int use_mask;
    // critic mode (value head = output 0 of the packed net, outputs 1..3 zero): g0 = dL/dV * coef with
    // L = MSE or Huber on V - target; delta_out = target - V (the TD error)
    int critic, huber;
    float huber_delta;
    const float* target;     // [n]
    float* delta_out;        // [n] or NULL
    float* v_out;            // [n] or NULL: V(s) of each sample (critic mode)
    g2048_td_rows td;        // has_td: target and V(s) through the lane-indexed value buffers (g2048_td_rows)
    int has_td;
    // column window: sample j's a1^T / d2^T column is col_off + j; groups of 32 processed: ngroups (columns
    // col_off .. col_off + 32 ngroups - 1; those past n are written as zero-coefficient padding)
    uint32_t col_off, ngroups;
    int part_accum;          // add this launch's per-wave partials to `part` instead of overwriting it
    int d2_form;             // 1 (critic, ReLU) / 2 (actor, ReLU): d2t receives one 1 KiB record per 16-column block
                             // instead of d2 columns (include/g2048.h; the FAC kernel variants)
};

// the critic's TD target of sample j: given, or r + (gamma V(s')) m from the lane-indexed values (g2048_td_rows; the
// host's fp32 operation order -- the TU is built with -ffp-contract=off, so nothing fuses)
__device__ __forceinline__ float td_target(const GradArgs& a, uint32_t j) {
    if (!a.has_td) return a.target[j];
    return ((a.td.v_next[a.td.lane[j]] * a.td.gamma) * a.td.has_next[j]) + a.td.reward[j];
}

template <int NT1, int NT2>
struct GradSmem {
    static constexpr int kStage = NT1 * 4 * 64 * 4 > 32 * 33 ? NT1 * 4 * 64 * 4 : 32 * 33;   // floats per wave
    NetSmem<NT1, NT2> net;
    float stage[4][kStage];            // per wave: the layer-1 activations in layer-2 B-fragment order, then (after
                                       // the forward) the backward's transpose tile [unit][sample], stride 33
    float g[4][32][4];                 // per-wave g of the group [sample][action]
    float db1[4][32 * NT1];            // per-wave db1 partial
};

__device__ __forceinline__ void lds_fence() {   // order this wave's LDS writes / reads (a wave's LDS ops retire in order)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int ACT>
__device__ __forceinline__ float activation_derivative(float a) {   // from the activation (src/reinforce_agent.py:624-636)
    if constexpr (ACT == 0) return a > 0.0f ? 1.0f : 0.0f;
    else return a * (1.0f - a);
}

// The a1^T / d2^T column buffers are addressed as buffer resources: element (row, column) at voffset = this lane's
// column byte offset (one VGPR for every access) + soffset = row * ld * 4 (scalar), so no per-row 64-bit vector
// address is ever formed (those kept 2 VGPRs live per row across the whole group and spilled the large nets).
// Column buffers fp32 in 16-column blocks (include/g2048.h): element (row, col) at ((col >> 4) * R + row) * 16 +
// (col & 15), R = 32 max(NT1, NT2) rows per block for both buffers, so one stage of 16 samples of every row is
// one contiguous 64 R bytes (g2048_dw2 streams them; a wave's column stores stay inside two blocks).  Row `row` of
// this lane's column at scalar offset row * ld4 (ld4 = 64 bytes, the row stride inside a block).
// The caller re-opaques ld4 per tile (opaque_sgpr): otherwise the compiler hoists every row's offset out of the
// group loop into its own SGPR (hundreds of them), spills them to VGPR lanes, and pays a v_readlane + hazard nops
// before every column store.
__device__ __forceinline__ void col_store(__amdgpu_buffer_rsrc_t r, uint32_t row, uint32_t ld4, uint32_t voff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)voff, (int)(row * ld4), 0);
}
__device__ __forceinline__ float col_load(__amdgpu_buffer_rsrc_t r, uint32_t row, uint32_t ld4, uint32_t voff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)(row * ld4), 0));
}
__device__ __forceinline__ void opaque_sgpr(uint32_t& v) { asm volatile("" : "+s"(v)); }
// packed weight fragment `idx` (64 lanes x float4) at this lane's voffset (lane * 16): the same one-VGPR addressing
// for the fragment streams (per-fragment 64-bit pointers were hoisted out of the group loop, 2 registers each)
__device__ __forceinline__ float4 frag_load(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t idx) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)(idx * 1024u), 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// FAC (critic, ReLU): d2 = m * (W3 g) with m = [a2 > 0] and a scalar g per sample, so instead of the d2 columns the
// kernel writes, per 16-column block, a 1 KiB record: the ReLU mask as one 16-bit word per second-layer unit (bit k =
// sample 16 c + k) at bytes [0, 2 H2p), and g of the 16 samples at bytes [512, 576); g2048_dw2_factored rebuilds
// dW2 = W3 * sum (a1 g) m^T from it (64 B per sample written and read instead of 1 KiB).
// FAC 2 (actor, ReLU): the same mask words plus the 4 values of g per sample (float4 at byte 512 + 16 (c & 15));
// g2048_dw2_actor rebuilds d2 = fl(fl(g0 W3[j,0]) + g1 W3[j,1] ...) * m exactly as below (64 B per sample).
template <int NT1, int NT2, int ACT, int OBS, int FAC = 0>
__global__ void __launch_bounds__(kPolBlock, 1) grad_kernel(GradArgs a) {
    typedef float floatx4 __attribute__((ext_vector_type(4)));
    constexpr int H1p = 32 * NT1, H2p = 32 * NT2;
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31, w = threadIdx.x >> 6;
    const int l16 = lane & 15, q16 = lane >> 4;
    __shared__ GradSmem<NT1, NT2> S;
    S.net.load(a.net);
    for (int k = lane; k < H1p; k += 64) S.db1[w][k] = 0.0f;
    __syncthreads();
    const NetSmem<NT1, NT2>& sm = S.net;
    const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.net + NetSmem<NT1, NT2>::L.w2f), 0, NT2 * NT1 * 1024 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.w2b), 0, NT1 * NT2 * 1024 * 4,
                                                                         0x00020000);
    const uint32_t fvo = (uint32_t)lane * 16u;
    float4* h1f = reinterpret_cast<float4*>(S.stage[w]);             // [t][q][lane] during the forward
    float (*T)[33] = reinterpret_cast<float (*)[33]>(S.stage[w]);     // [unit][sample] during the backward
    float gsum[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // db3 partial (lanes of half 0)
    constexpr uint32_t RB = 32u * (NT1 > NT2 ? NT1 : NT2);   // rows per 16-column block of both column buffers
    const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc(a.a1t, 0, (int)(RB * a.ld * 4u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd2 = __builtin_amdgcn_make_buffer_rsrc(
        a.d2t, 0, FAC ? (int)((a.ld >> 4) * 1024u) : (int)(RB * a.ld * 4u), 0x00020000);
    floatx4 dw1acc[2 * NT1], dw3acc[2 * NT2];  // dW1^T / dW3^T 16x16 accumulator blocks, across the wave's groups
#pragma unroll
    for (int k = 0; k < 2 * NT1; k++) dw1acc[k] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 2 * NT2; k++) dw3acc[k] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    const uint32_t waves = gridDim.x * (kPolBlock / 64);
    const uint32_t groups = a.ngroups;
#if G2048_DIAG
    unsigned long long gph[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long gtp = __builtin_amdgcn_s_memrealtime();
#define GRAD_PH(k)                                                        \
    do {                                                                  \
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();  \
        gph[k] += tn - gtp;                                               \
        gtp = tn;                                                         \
    } while (0)
#else
#define GRAD_PH(k) \
    do {           \
    } while (0)
#endif
    for (uint32_t gi = blockIdx.x * (kPolBlock / 64) + w; gi < groups; gi += waves) {
        const uint32_t j = gi * 32u + (uint32_t)col;   // this lane's sample (both halves)
        // a compiler memory barrier per group: without it the net tensors' LDS reads (loop-invariant) are hoisted
        // out of the group loop into hundreds of registers
        asm volatile("" ::: "memory");
        const uint32_t cj = a.col_off + j;                        // this sample's column
        // byte offset of column cj's row 4h (acc_row's lane-half rows) in its 16-column block
        const uint32_t off = (((cj >> 4) * RB + 4u * (uint32_t)h) * 16u + (cj & 15u)) * 4u;
        uint32_t ld4 = 64u;                                          // row stride inside a block (see col_store)
        const bool valid = j < a.n;
        const uint64_t b = valid ? a.boards[j] : 0ull;
        const uint32_t act = (valid && !a.critic) ? a.actions[j] : 0u;   // no actions in critic mode
        const float cf = valid ? a.coef[j] : 0.0f;
        // ---- forward (mlp_logits, keeping a2 = h2); each a1 tile goes to its a1^T columns when done (a1 is
        //      re-read from there for the input delta, so it is not held across the backward)
        // weight fragments: two k-tiles in flight (fa = this one, fn = the next; the one after is loaded while this
        // tile's MFMAs run).  Stream order: the forward's (o, t) tiles, then the input-delta's (o1, t2) tiles.
        constexpr int KF = NT2 * NT1, KB = NT1 * NT2;
        const auto stream_frag = [&](int kt, int q) -> float4 {   // k-tiles past the stream's end re-read tile 0
            return kt < KF ? frag_load(rw2, fvo, kt * 4 + q) : frag_load(rwb, fvo, (kt - KF < KB ? kt - KF : 0) * 4 + q);
        };
        float4 fa[4], fn[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            fa[q] = stream_frag(0, q);
            fn[q] = stream_frag(1, q);
        }
        lds_fence();   // the previous group's reads of the stage are done
        {
            float x[8];
#pragma unroll
            for (int s = 0; s < 8; s++) x[s] = obs_value<OBS>(b, 2 * s + h, a.obs_scale);
#pragma unroll
            for (int t = 0; t < NT1; t++) {
                opaque_sgpr(ld4);
                floatx16 acc = {};
#pragma unroll
                for (int s = 0; s < 8; s++)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sm.w1f()[(t * 8 + s) * 64 + lane], x[s], acc, 0, 0, 0);
                const float4* bb = reinterpret_cast<const float4*>(sm.b1p() + (t * 2 + h) * 16);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4 bv = bb[q];
                    const float4 hv = make_float4(activate<ACT>(acc[4 * q + 0] + bv.x), activate<ACT>(acc[4 * q + 1] + bv.y),
                                                  activate<ACT>(acc[4 * q + 2] + bv.z), activate<ACT>(acc[4 * q + 3] + bv.w));
                    h1f[(t * 4 + q) * 64 + lane] = hv;
                }
            }
        }
        lds_fence();
        GRAD_PH(0);
        float h2[NT2][16];
        float lg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int o = 0; o < NT2; o++) {
            floatx16 acc = {};
#pragma unroll
            for (int t = 0; t < NT1; t++) {
                float4 fb[4];   // k-tile kt + 2 of the stream (the last ones run into the input-delta stream)
#pragma unroll
                for (int q = 0; q < 4; q++) fb[q] = stream_frag(o * NT1 + t + 2, q);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4 hb = h1f[(t * 4 + q) * 64 + lane];
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, hb.x, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, hb.y, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, hb.z, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, hb.w, acc, 0, 0, 0);
                    if (o == 0) {   // the a1 values of tile t go out with the first output tile
                        const float hv[4] = {hb.x, hb.y, hb.z, hb.w};
#pragma unroll
                        for (int c = 0; c < 4; c++) {
                            opaque_sgpr(ld4);
                            col_store(ra1, 32 * t + acc_row(4 * q + c, 0), ld4, off, hv[c]);
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    fa[q] = fn[q];
                    fn[q] = fb[q];
                }
            }
            const float4* bb = reinterpret_cast<const float4*>(sm.b2p() + (o * 2 + h) * 16);
            const float4* w3 = reinterpret_cast<const float4*>(sm.w3p() + (o * 2 + h) * 64);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4 bv = bb[q];
                h2[o][4 * q + 0] = activate<ACT>(acc[4 * q + 0] + bv.x);
                h2[o][4 * q + 1] = activate<ACT>(acc[4 * q + 1] + bv.y);
                h2[o][4 * q + 2] = activate<ACT>(acc[4 * q + 2] + bv.z);
                h2[o][4 * q + 3] = activate<ACT>(acc[4 * q + 3] + bv.w);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const float4 wv = w3[4 * q + u];
                    lg[0] = fmaf(h2[o][4 * q + u], wv.x, lg[0]);
                    lg[1] = fmaf(h2[o][4 * q + u], wv.y, lg[1]);
                    lg[2] = fmaf(h2[o][4 * q + u], wv.z, lg[2]);
                    lg[3] = fmaf(h2[o][4 * q + u], wv.w, lg[3]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);   // keep the scheduler from hoisting later tiles' LDS reads
        }
#pragma unroll
        for (int k = 0; k < 4; k++) lg[k] = (lg[k] + __shfl_xor(lg[k], 32, 64)) + sm.b3()[k];
        GRAD_PH(1);
        float g[4];
        if (!a.critic) {
            // ---- logits_to_probs (src/MLP.py:139-156) and the policy-gradient logits delta (:328-354)
            const uint32_t mw = a.use_mask ? mask_word_of(b) : 0x01010101u;
            float l[4];
#pragma unroll
            for (int k = 0; k < 4; k++) l[k] = ((mw >> (8 * k)) & 0xFFu) ? lg[k] : -1e9f;
            const float mx = fmaxf(fmaxf(l[0], l[1]), fmaxf(l[2], l[3]));
            float e[4];
#pragma unroll
            for (int k = 0; k < 4; k++) e[k] = expf(l[k] - mx);
            const float es = ((e[0] + e[1]) + e[2]) + e[3];
#pragma unroll
            for (int k = 0; k < 4; k++) g[k] = (((uint32_t)k == act ? 1.0f : 0.0f) - e[k] / es) * cf;
        } else {
            // ---- the critic's value-loss gradient (update_batch :403-498, _get_grad_logits_critic :884-910)
            const float tg = valid ? td_target(a, j) : 0.0f;
            const float diff = lg[0] - tg;
            const float gd = (a.huber && fabsf(diff) > a.huber_delta) ? copysignf(a.huber_delta, diff) : diff;
            g[0] = gd * cf;
            g[1] = g[2] = g[3] = 0.0f;
            if (valid && h == 0 && a.delta_out) a.delta_out[j] = tg - lg[0];
            if (valid && h == 0) {
                if (a.has_td) a.td.v_out[a.td.lane[j]] = lg[0];
                else if (a.v_out) a.v_out[j] = lg[0];
            }
        }
        lds_fence();   // the previous group's reads of S.g are done
        if (h == 0) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                gsum[k] += g[k];
                S.g[w][col][k] = g[k];
            }
        }
        // a1 of the first h1 tile for the input delta, re-read from its columns well ahead of its use (each tile's
        // reload is issued one tile ahead: loaded at the point of use it cost a full memory latency per register)
        float a1n[16];
        opaque_sgpr(ld4);
#pragma unroll
        for (int r = 0; r < 16; r++) a1n[r] = col_load(ra1, acc_row(r, 0), ld4, off);
        // ---- dW3 += a2^T g: per h2 tile, a2 transposed through LDS, 16x16x4 MFMAs over the 32 samples
        //      (A = g^T [action][sample], B = a2^T [sample][unit]; only the 4 action rows are kept)
#pragma unroll
        for (int o = 0; o < NT2; o++) {
            lds_fence();
#pragma unroll
            for (int r = 0; r < 16; r++) T[acc_row(r, h)][col] = h2[o][r];
            lds_fence();
#pragma unroll
            for (int kk = 0; kk < 8; kk++) {
                const int s = 4 * kk + q16;
                const float av = l16 < 4 ? S.g[w][s][l16 & 3] : 0.0f;
#pragma unroll
                for (int c = 0; c < 2; c++)
                    dw3acc[2 * o + c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, T[16 * c + l16][s], dw3acc[2 * o + c], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        GRAD_PH(2);
        // ---- d2 = act'(a2) * (W3 g), in place; d2^T columns (FAC: the block records' mask words and g instead)
        if constexpr (FAC == 1) {
            if (h == 0) {   // g of this lane's sample at byte 512 + 4 (cj & 15) of its block's record
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g[0]), rd2, (int)((cj >> 4) * 1024u + 512u + (cj & 15u) * 4u),
                                                      0, 0);
            }
        } else if constexpr (FAC == 2) {
            if (h == 0) {   // the 4 values of g of this lane's sample at byte 512 + 16 (cj & 15)
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 gv = {__float_as_uint(g[0]), __float_as_uint(g[1]), __float_as_uint(g[2]), __float_as_uint(g[3])};
                __builtin_amdgcn_raw_buffer_store_b128(gv, rd2, (int)((cj >> 4) * 1024u + 512u + (cj & 15u) * 16u), 0, 0);
            }
        }
#pragma unroll
        for (int o = 0; o < NT2; o++) {
            opaque_sgpr(ld4);
            if constexpr (FAC) {
                // ballot of a2 > 0 per register r: bits 0..31 = samples of unit acc_row(r, 0), 32..63 = of unit
                // acc_row(r, 1); lane L = 4 r + 2 h' + b stores the 16-bit word of unit 32 o + acc_row(r, h') for
                // the group's block b (one 16-bit store per lane covers the tile's 32 units x 32 samples)
                uint32_t mv = 0u;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const uint64_t bal = __ballot(h2[o][r] > 0.0f);
                    const uint32_t hw = (uint32_t)(bal >> (32 * ((lane >> 1) & 1)));
                    const uint32_t part = (hw >> (16 * (lane & 1))) & 0xFFFFu;
                    mv = (lane >> 2) == r ? part : mv;
                }
                const uint32_t unit = 32u * (uint32_t)o + (uint32_t)acc_row(lane >> 2, (lane >> 1) & 1);
                const uint32_t blk = ((a.col_off + gi * 32u) >> 4) + (uint32_t)(lane & 1);
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)mv, rd2, (int)(blk * 1024u + unit * 2u), 0, 0);
            }
            const float4* w3 = reinterpret_cast<const float4*>(sm.w3p() + (o * 2 + h) * 64);
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const float4 wv = w3[r];
                float dh = g[0] * wv.x;
                dh = fmaf(g[1], wv.y, dh);
                dh = fmaf(g[2], wv.z, dh);
                dh = fmaf(g[3], wv.w, dh);
                h2[o][r] = dh * activation_derivative<ACT>(h2[o][r]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        GRAD_PH(3);
        // ---- d1 = act'(a1) * (W2 d2) per h1 tile, then db1 and dW1 += x^T d1 (16x16x4 MFMAs: A = x^T
        //      [feature][sample] built from the group's boards, B = d1^T [sample][unit] through LDS)
        float xa[8];
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const uint64_t bs = shfl64_(b, 4 * kk + q16);
            xa[kk] = obs_value<OBS>(bs, l16, a.obs_scale);
        }
        float4 fw[4];
#pragma unroll
        for (int q = 0; q < 4; q++) fw[q] = fa[q];   // input-delta k-tiles 0 and 1, prefetched by the forward
#pragma unroll
        for (int o1 = 0; o1 < NT1; o1++) {
            opaque_sgpr(ld4);
            float a1v[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                a1v[r] = a1n[r];
                if (o1 + 1 < NT1) a1n[r] = col_load(ra1, 32 * (o1 + 1) + acc_row(r, 0), ld4, off);
            }
            floatx16 acc = {};
#pragma unroll
            for (int t2 = 0; t2 < NT2; t2++) {
                float4 fb[4];
#pragma unroll
                for (int q = 0; q < 4; q++)   // k-tile + 2 (past the end: tile 0 again, unused)
                    fb[q] = stream_frag(KF + o1 * NT2 + t2 + 2, q);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fw[q].x, h2[t2][4 * q + 0], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fw[q].y, h2[t2][4 * q + 1], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fw[q].z, h2[t2][4 * q + 2], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fw[q].w, h2[t2][4 * q + 3], acc, 0, 0, 0);
                }
                // d2 value r of tile t2 goes out at input tile (r * NT1) / 16
                if constexpr (!FAC) {
#pragma unroll
                    for (int r = 0; r < 16; r++)
                        if ((r * NT1) / 16 == o1) {
                            opaque_sgpr(ld4);
                            col_store(rd2, 32 * t2 + acc_row(r, 0), ld4, off, h2[t2][r]);
                        }
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    fw[q] = fn[q];
                    fn[q] = fb[q];
                }
            }
            lds_fence();
#pragma unroll
            for (int r = 0; r < 16; r++) T[acc_row(r, h)][col] = acc[r] * activation_derivative<ACT>(a1v[r]);
            lds_fence();
            float bs = 0.0f;   // db1: unit col of this tile, samples 16h .. 16h+15, then both halves
#pragma unroll
            for (int s = 0; s < 16; s++) bs += T[col][16 * h + s];
            bs += __shfl_xor(bs, 32, 64);
            if (h == 0) S.db1[w][32 * o1 + col] += bs;
#pragma unroll
            for (int kk = 0; kk < 8; kk++)
#pragma unroll
                for (int c = 0; c < 2; c++)
                    dw1acc[2 * o1 + c] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[kk], T[16 * c + l16][4 * kk + q16],
                                                                            dw1acc[2 * o1 + c], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        GRAD_PH(4);
#if G2048_DIAG
        gph[5] += 1;
#endif
    }
#if G2048_DIAG
    if (threadIdx.x == 0 && blockIdx.x < kRollDiagBlocks)
        for (int k = 0; k < 6; k++) g_grad_ph[blockIdx.x * 6 + k] = gph[k];
#endif
#undef GRAD_PH
    // ---- this wave's partial gradients
    const uint32_t wg = blockIdx.x * (kPolBlock / 64) + w;
    float* out = a.part + (size_t)wg * grad_part_floats(NT1, NT2);
    const bool acc = a.part_accum != 0;   // this wave owns its row: a plain read-modify-write
    lds_fence();
#pragma unroll
    for (int k = 0; k < 2 * NT1; k++)   // block k: h1 units 16k..16k+15; row 4 q16 + r = feature
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float* p = out + (4 * q16 + r) * H1p + 16 * k + l16;
            *p = (acc ? *p : 0.0f) + dw1acc[k][r];
        }
    for (int k = lane; k < H1p; k += 64) out[16 * H1p + k] = (acc ? out[16 * H1p + k] : 0.0f) + S.db1[w][k];
    if (q16 == 0) {                     // rows 0..3 = actions
#pragma unroll
        for (int k = 0; k < 2 * NT2; k++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float* p = out + 17 * H1p + (16 * k + l16) * 4 + r;
                *p = (acc ? *p : 0.0f) + dw3acc[k][r];
            }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        float v = h == 0 ? gsum[k] : 0.0f;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if (lane == 0) out[17 * H1p + 4 * H2p + k] = (acc ? out[17 * H1p + 4 * H2p + k] : 0.0f) + v;
    }
}

// ---------------------------------------------------------------------------------------------------- gradient, cooperative
// grad_coop_kernel: grad_kernel's computation and outputs (a1^T columns, d2^T columns or records, the per-row
// partials) with the 4 waves of a workgroup splitting each 32-sample group's MFMAs instead of each wave taking a group
// of its own.  Wave w owns the layer-1 / input-delta tiles and the layer-2 output tiles congruent to w mod 4; the
// layer-1 activations and d2 are exchanged through LDS in B-fragment order and the partial logits through LDS (four
// workgroup barriers per group).  A wave then holds a quarter of grad_kernel's per-group registers, so TWO
// workgroups run per CU (2 waves per SIMD): one workgroup's MFMAs run while the other's epilogues, softmax, column
// stores and barriers do, where grad_kernel's single wave per SIMD leaves the MFMAs idle for those phases (the
// rollout kernel's arrangement).  Dynamic LDS (CoopLds: 74 KiB at 256 x 256).  Partials: workgroup b writes rows 2b
// and 2b + 1 -- wave w adds its own tiles' entries to row 2b + (w >> 1) and (unless accumulating) zeros the same
// entries of the other row -- so the row count is g2048_actor_grad_waves() as for grad_kernel.  The logits are the
// sum of the four waves' partials in wave order (grad_kernel sums the output tiles in order), so the two kernels'
// forwards round differently; each is checked against fp64 under its own ReLU pattern (tests/exact_grad.py).
template <int NT1, int NT2>
struct CoopLds {
    static constexpr PolLayout P = pol_layout(NT1, NT2);
    static constexpr int kA = NT1 * 1024 > 4 * 32 * 33 ? NT1 * 1024 : 4 * 32 * 33;   // h1f, later the transpose tiles
    static constexpr int oD2 = kA;                                                   // d2f [NT2][4][64] float4
    static constexpr int oPart = oD2 + NT2 * 1024;                                   // [4][32][4] partial logits
    static constexpr int oG = oPart + 4 * 32 * 4;                                    // [4][32][4] per-wave g
    static constexpr int oB1 = oG + 4 * 32 * 4;                                      // b1p
    static constexpr int oB2 = oB1 + (int)(P.w2f - P.b1p);                           // b2p, w3p, b3
    static constexpr int kFloats = oB2 + (int)(P.total - P.b2p);
    static constexpr int kBytes = kFloats * 4;
};

template <int NT1, int NT2, int ACT, int OBS, int FAC>
__global__ void __launch_bounds__(kPolBlock, 2) grad_coop_kernel(GradArgs a) {
    static_assert(NT1 % 4 == 0 && NT2 % 4 == 0, "every wave owns NT / 4 tiles of each layer");
    typedef float floatx4 __attribute__((ext_vector_type(4)));
    using C = CoopLds<NT1, NT2>;
    constexpr int H1p = 32 * NT1, H2p = 32 * NT2, KO1 = NT1 / 4, KO2 = NT2 / 4;
    constexpr int KF = KO2 * NT1, KB = KO1 * NT2;     // this wave's forward / input-delta k-tiles
    extern __shared__ float coop_lds[];
    float4* h1f = reinterpret_cast<float4*>(coop_lds);              // [t][q][lane]: registers 4q..4q+3 of a1 tile t
    float4* d2f = reinterpret_cast<float4*>(coop_lds + C::oD2);     // [t2][q][lane]: the same for d2
    float (*part)[32][4] = reinterpret_cast<float (*)[32][4]>(coop_lds + C::oPart);
    float (*gs)[32][4] = reinterpret_cast<float (*)[32][4]>(coop_lds + C::oG);
    const float* b1p = coop_lds + C::oB1;
    const float* b2p = coop_lds + C::oB2;
    const float* w3p = b2p + (C::P.w3p - C::P.b2p);
    const float* b3 = b2p + (C::P.b3 - C::P.b2p);
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int l16 = lane & 15, q16 = lane >> 4;
    float (*T)[33] = reinterpret_cast<float (*)[33]>(coop_lds + w * 32 * 33);   // inside h1f: used after layer 2
    for (int k = threadIdx.x; k < C::kFloats - C::oB1; k += kPolBlock)
        coop_lds[C::oB1 + k] = k < C::oB2 - C::oB1 ? a.net[C::P.b1p + k] : a.net[C::P.b2p + (k - (C::oB2 - C::oB1))];
    // this wave's layer-1 A fragments (tiles w + 4k), resident for the whole launch
    float w1own[KO1][8];
#pragma unroll
    for (int k = 0; k < KO1; k++)
#pragma unroll
        for (int s = 0; s < 8; s++) w1own[k][s] = a.net[C::P.w1f + ((w + 4 * k) * 8 + s) * 64 + lane];
    // The wave-dependent parts of every address go into per-wave bases (fragment resources starting at the wave's
    // first own tile, the column offset advanced by its first own row block), so the per-fragment / per-row offsets
    // are compile-time constants: with `w` in them the compiler hoists ~150 distinct scalar offsets out of the
    // group loop and spills them.
    const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.net + C::P.w2f + (size_t)w * NT1 * 1024), 0, (NT2 - w) * NT1 * 1024 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w2b + (size_t)w * NT2 * 1024), 0, (NT1 - w) * NT2 * 1024 * 4, 0x00020000);
    const uint32_t fvo = (uint32_t)lane * 16u;
    constexpr uint32_t RB = 32u * (NT1 > NT2 ? NT1 : NT2);
    const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc(a.a1t, 0, (int)(RB * a.ld * 4u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd2 = __builtin_amdgcn_make_buffer_rsrc(
        a.d2t, 0, FAC ? (int)((a.ld >> 4) * 1024u) : (int)(RB * a.ld * 4u), 0x00020000);
    floatx4 dw1acc[2 * KO1], dw3acc[2 * KO2];
#pragma unroll
    for (int k = 0; k < 2 * KO1; k++) dw1acc[k] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 2 * KO2; k++) dw3acc[k] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    float db1r[KO1];
#pragma unroll
    for (int k = 0; k < KO1; k++) db1r[k] = 0.0f;
    float gsum[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // db3 (wave 0, lanes of half 0)
    // this wave's fragment stream: the forward's (own output tile w + 4 k2, k-tile) pairs, then the input delta's
    // (own input tile w + 4 k1, k-tile), relative to the per-wave bases; past the end: fragment 0 again (unused)
    const auto stream_frag = [&](int i, int q) -> float4 {
        if (i < KF) return frag_load(rw2, fvo, (uint32_t)((4 * (i / NT1) * NT1 + i % NT1) * 4 + q));
        if (i < KF + KB) {
            const int ii = i - KF;
            return frag_load(rwb, fvo, (uint32_t)((4 * (ii / NT2) * NT2 + ii % NT2) * 4 + q));
        }
        return frag_load(rw2, fvo, (uint32_t)q);
    };
    for (uint32_t gi = blockIdx.x; gi < a.ngroups; gi += gridDim.x) {   // workgroup-uniform
        const uint32_t j = gi * 32u + (uint32_t)col;
        asm volatile("" ::: "memory");
        const uint32_t cj = a.col_off + j;
        // this lane's column, rows 4h + 32 w (the wave's first own row block) on: own rows are 32 (4 k) + acc_row
        const uint32_t off = (((cj >> 4) * RB + 4u * (uint32_t)h + 32u * (uint32_t)w) * 16u + (cj & 15u)) * 4u;
        uint32_t ld4 = 64u;
        const bool valid = j < a.n;
        const uint64_t b = valid ? a.boards[j] : 0ull;
        const uint32_t act = (valid && !a.critic) ? a.actions[j] : 0u;
        const float cf = valid ? a.coef[j] : 0.0f;
        float4 fa[4], fn[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            fa[q] = stream_frag(0, q);
            fn[q] = stream_frag(1, q);
        }
        __syncthreads();   // every wave is done with the previous group's transpose tiles (in h1f) and d2f
        // ---- layer 1: own tiles, kept in registers and published to h1f
        float a1own[KO1][16];
        {
            float x[8];
#pragma unroll
            for (int s = 0; s < 8; s++) x[s] = obs_value<OBS>(b, 2 * s + h, a.obs_scale);
#pragma unroll
            for (int k = 0; k < KO1; k++) {
                const int t = w + 4 * k;
                floatx16 acc = {};
#pragma unroll
                for (int s = 0; s < 8; s++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1own[k][s], x[s], acc, 0, 0, 0);
                const float4* bb = reinterpret_cast<const float4*>(b1p + (t * 2 + h) * 16);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4 bv = bb[q];
                    a1own[k][4 * q + 0] = activate<ACT>(acc[4 * q + 0] + bv.x);
                    a1own[k][4 * q + 1] = activate<ACT>(acc[4 * q + 1] + bv.y);
                    a1own[k][4 * q + 2] = activate<ACT>(acc[4 * q + 2] + bv.z);
                    a1own[k][4 * q + 3] = activate<ACT>(acc[4 * q + 3] + bv.w);
                    h1f[(t * 4 + q) * 64 + lane] = make_float4(a1own[k][4 * q + 0], a1own[k][4 * q + 1],
                                                               a1own[k][4 * q + 2], a1own[k][4 * q + 3]);
                }
            }
        }
        __syncthreads();   // h1f complete
        // ---- layer 2: own output tiles (B = a1 from LDS, A streamed), folded into partial logits; the own a1
        //      columns are stored through it (kS1 per k-tile)
        constexpr int kS1 = (KO1 * 16 + KF - 1) / KF;
        float h2[KO2][16];
        float lgp[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k2 = 0; k2 < KO2; k2++) {
            const int o = w + 4 * k2;
            floatx16 acc = {};
#pragma unroll
            for (int tt = 0; tt < NT1; tt++) {
                const int i = k2 * NT1 + tt;
                float4 fb[4];
#pragma unroll
                for (int q = 0; q < 4; q++) fb[q] = stream_frag(i + 2, q);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4 hb = h1f[(tt * 4 + q) * 64 + lane];
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, hb.x, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, hb.y, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, hb.z, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, hb.w, acc, 0, 0, 0);
                }
#pragma unroll
                for (int v = i * kS1; v < (i + 1) * kS1; v++)
                    if (v < KO1 * 16) {
                        opaque_sgpr(ld4);
                        col_store(ra1, 128 * (v / 16) + acc_row(v % 16, 0), ld4, off, a1own[v / 16][v % 16]);
                    }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    fa[q] = fn[q];
                    fn[q] = fb[q];
                }
            }
            const float4* bb = reinterpret_cast<const float4*>(b2p + (o * 2 + h) * 16);
            const float4* w3 = reinterpret_cast<const float4*>(w3p + (o * 2 + h) * 64);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4 bv = bb[q];
                h2[k2][4 * q + 0] = activate<ACT>(acc[4 * q + 0] + bv.x);
                h2[k2][4 * q + 1] = activate<ACT>(acc[4 * q + 1] + bv.y);
                h2[k2][4 * q + 2] = activate<ACT>(acc[4 * q + 2] + bv.z);
                h2[k2][4 * q + 3] = activate<ACT>(acc[4 * q + 3] + bv.w);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const float4 wv = w3[4 * q + u];
                    lgp[0] = fmaf(h2[k2][4 * q + u], wv.x, lgp[0]);
                    lgp[1] = fmaf(h2[k2][4 * q + u], wv.y, lgp[1]);
                    lgp[2] = fmaf(h2[k2][4 * q + u], wv.z, lgp[2]);
                    lgp[3] = fmaf(h2[k2][4 * q + u], wv.w, lgp[3]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int k = 0; k < 4; k++) lgp[k] += __shfl_xor(lgp[k], 32, 64);
        if (h == 0) {
#pragma unroll
            for (int k = 0; k < 4; k++) part[w][col][k] = lgp[k];
        }
        __syncthreads();   // partial logits complete; h1f is free from here (the transpose tiles live in it)
        float lg[4];
#pragma unroll
        for (int k = 0; k < 4; k++) lg[k] = (((part[0][col][k] + part[1][col][k]) + part[2][col][k]) + part[3][col][k]) + b3[k];
        float g[4];
        if (!a.critic) {
            const uint32_t mw = a.use_mask ? mask_word_of(b) : 0x01010101u;
            float l[4];
#pragma unroll
            for (int k = 0; k < 4; k++) l[k] = ((mw >> (8 * k)) & 0xFFu) ? lg[k] : -1e9f;
            const float mx = fmaxf(fmaxf(l[0], l[1]), fmaxf(l[2], l[3]));
            float e[4];
#pragma unroll
            for (int k = 0; k < 4; k++) e[k] = expf(l[k] - mx);
            const float es = ((e[0] + e[1]) + e[2]) + e[3];
#pragma unroll
            for (int k = 0; k < 4; k++) g[k] = (((uint32_t)k == act ? 1.0f : 0.0f) - e[k] / es) * cf;
        } else {
            const float tg = valid ? td_target(a, j) : 0.0f;
            const float diff = lg[0] - tg;
            const float gd = (a.huber && fabsf(diff) > a.huber_delta) ? copysignf(a.huber_delta, diff) : diff;
            g[0] = gd * cf;
            g[1] = g[2] = g[3] = 0.0f;
            if (valid && w == 0 && h == 0 && a.delta_out) a.delta_out[j] = tg - lg[0];
            if (valid && w == 0 && h == 0) {
                if (a.has_td) a.td.v_out[a.td.lane[j]] = lg[0];
                else if (a.v_out) a.v_out[j] = lg[0];
            }
        }
        if (h == 0) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (w == 0) gsum[k] += g[k];
                gs[w][col][k] = g[k];
            }
        }
        // ---- dW3 += a2^T g over the own h2 tiles (a2 transposed through this wave's tile, 16x16x4 MFMAs)
#pragma unroll
        for (int k2 = 0; k2 < KO2; k2++) {
            lds_fence();
#pragma unroll
            for (int r = 0; r < 16; r++) T[acc_row(r, h)][col] = h2[k2][r];
            lds_fence();
#pragma unroll
            for (int kk = 0; kk < 8; kk++) {
                const int s = 4 * kk + q16;
                const float av = l16 < 4 ? gs[w][s][l16 & 3] : 0.0f;
#pragma unroll
                for (int c = 0; c < 2; c++)
                    dw3acc[2 * k2 + c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, T[16 * c + l16][s], dw3acc[2 * k2 + c], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // ---- d2 = act'(a2) * (W3 g) over the own tiles -> d2f (and the records' mask words / g)
        if constexpr (FAC == 1) {
            if (w == 0 && h == 0)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g[0]), rd2, (int)((cj >> 4) * 1024u + 512u + (cj & 15u) * 4u),
                                                      0, 0);
        } else if constexpr (FAC == 2) {
            if (w == 0 && h == 0) {
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 gv = {__float_as_uint(g[0]), __float_as_uint(g[1]), __float_as_uint(g[2]), __float_as_uint(g[3])};
                __builtin_amdgcn_raw_buffer_store_b128(gv, rd2, (int)((cj >> 4) * 1024u + 512u + (cj & 15u) * 16u), 0, 0);
            }
        }
#pragma unroll
        for (int k2 = 0; k2 < KO2; k2++) {
            const int o = w + 4 * k2;
            if constexpr (FAC) {
                uint32_t mv = 0u;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const uint64_t bal = __ballot(h2[k2][r] > 0.0f);
                    const uint32_t hw = (uint32_t)(bal >> (32 * ((lane >> 1) & 1)));
                    const uint32_t pt = (hw >> (16 * (lane & 1))) & 0xFFFFu;
                    mv = (lane >> 2) == r ? pt : mv;
                }
                const uint32_t unit = 32u * (uint32_t)o + (uint32_t)acc_row(lane >> 2, (lane >> 1) & 1);
                const uint32_t blk = ((a.col_off + gi * 32u) >> 4) + (uint32_t)(lane & 1);
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)mv, rd2, (int)(blk * 1024u + unit * 2u), 0, 0);
            }
            const float4* w3 = reinterpret_cast<const float4*>(w3p + (o * 2 + h) * 64);
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const float4 wv = w3[r];
                float dh = g[0] * wv.x;
                dh = fmaf(g[1], wv.y, dh);
                dh = fmaf(g[2], wv.z, dh);
                dh = fmaf(g[3], wv.w, dh);
                h2[k2][r] = dh * activation_derivative<ACT>(h2[k2][r]);
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                d2f[(o * 4 + q) * 64 + lane] = make_float4(h2[k2][4 * q + 0], h2[k2][4 * q + 1], h2[k2][4 * q + 2], h2[k2][4 * q + 3]);
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();   // d2f complete
        // ---- d1 = act'(a1) * (W2 d2) over the own input tiles (B = d2 from LDS), then db1 and dW1 += x^T d1;
        //      the own d2 columns (FAC 0) are stored through it (kS2 per k-tile)
        float xa[8];
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const uint64_t bs = shfl64_(b, 4 * kk + q16);
            xa[kk] = obs_value<OBS>(bs, l16, a.obs_scale);
        }
        constexpr int kS2 = (KO2 * 16 + KB - 1) / KB;
#pragma unroll
        for (int k1 = 0; k1 < KO1; k1++) {
            floatx16 acc = {};
#pragma unroll
            for (int t2 = 0; t2 < NT2; t2++) {
                const int i = k1 * NT2 + t2;
                float4 fb[4];
#pragma unroll
                for (int q = 0; q < 4; q++) fb[q] = stream_frag(KF + i + 2, q);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4 db = d2f[(t2 * 4 + q) * 64 + lane];
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, db.x, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, db.y, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, db.z, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, db.w, acc, 0, 0, 0);
                }
                if constexpr (!FAC) {
#pragma unroll
                    for (int v = i * kS2; v < (i + 1) * kS2; v++)
                        if (v < KO2 * 16) {
                            opaque_sgpr(ld4);
                            col_store(rd2, 128 * (v / 16) + acc_row(v % 16, 0), ld4, off, h2[v / 16][v % 16]);
                        }
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    fa[q] = fn[q];
                    fn[q] = fb[q];
                }
            }
            lds_fence();
#pragma unroll
            for (int r = 0; r < 16; r++) T[acc_row(r, h)][col] = acc[r] * activation_derivative<ACT>(a1own[k1][r]);
            lds_fence();
            float bs = 0.0f;   // db1 of unit col of this tile: samples 16h .. 16h + 15, then both halves
#pragma unroll
            for (int s = 0; s < 16; s++) bs += T[col][16 * h + s];
            bs += __shfl_xor(bs, 32, 64);
            db1r[k1] += bs;
#pragma unroll
            for (int kk = 0; kk < 8; kk++)
#pragma unroll
                for (int c = 0; c < 2; c++)
                    dw1acc[2 * k1 + c] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[kk], T[16 * c + l16][4 * kk + q16],
                                                                            dw1acc[2 * k1 + c], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // ---- partials: the own tiles' entries into row 2b + (w >> 1), zeros at the same entries of the other row
    constexpr int64_t PF = grad_part_floats(NT1, NT2);
    const bool accm = a.part_accum != 0;
    float* out = a.part + (size_t)(2u * blockIdx.x + (uint32_t)(w >> 1)) * PF;
    float* oth = a.part + (size_t)(2u * blockIdx.x + 1u - (uint32_t)(w >> 1)) * PF;
    const auto put = [&](int64_t idx, float v) {
        out[idx] = (accm ? out[idx] : 0.0f) + v;
        if (!accm) oth[idx] = 0.0f;
    };
#pragma unroll
    for (int k1 = 0; k1 < KO1; k1++)
#pragma unroll
        for (int c = 0; c < 2; c++)   // block 2 o1 + c: units 16 (2 o1 + c) + l16, feature rows 4 q16 + r
#pragma unroll
            for (int r = 0; r < 4; r++) put((int64_t)(4 * q16 + r) * H1p + 16 * (2 * (w + 4 * k1) + c) + l16, dw1acc[2 * k1 + c][r]);
    if (h == 0) {
#pragma unroll
        for (int k1 = 0; k1 < KO1; k1++) put(16 * H1p + 32 * (w + 4 * k1) + col, db1r[k1]);
    }
    if (q16 == 0) {                     // rows 0..3 = actions
#pragma unroll
        for (int k2 = 0; k2 < KO2; k2++)
#pragma unroll
            for (int c = 0; c < 2; c++)
#pragma unroll
                for (int r = 0; r < 4; r++) put(17 * H1p + (16 * (2 * (w + 4 * k2) + c) + l16) * 4 + r, dw3acc[2 * k2 + c][r]);
    }
    if (w == 0) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            float v = h == 0 ? gsum[k] : 0.0f;
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
            if (lane == 0) put(17 * H1p + 4 * H2p + k, v);
        }
    }
}

template <int ACT, int OBS, int FAC>
void launch_coop(const GradArgs& a, int grid, hipStream_t s) {
    constexpr int kBytes = CoopLds<8, 8>::kBytes;
    // the dynamic-LDS attribute is per kernel and device: one bit per device id, set on the first launch there (two
    // threads racing both set it, harmlessly).  A failure skips the launch and stays the last HIP error, which the
    // caller's hipGetLastError check reports.
    static std::atomic<uint64_t> attr_set{0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    const uint64_t bit = 1ull << (dev & 63);
    if (!(attr_set.load(std::memory_order_acquire) & bit)) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&grad_coop_kernel<8, 8, ACT, OBS, FAC>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kBytes) != hipSuccess)
            return;
        attr_set.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL((grad_coop_kernel<8, 8, ACT, OBS, FAC>), dim3(grid), dim3(kPolBlock), (unsigned)kBytes, s, a);
}

template <int ACT, int FAC>
void launch_coop_obs(const GradArgs& a, int obs, int grid, hipStream_t s) {
    if (obs == G2048_OBS_LOG2) launch_coop<ACT, G2048_OBS_LOG2, FAC>(a, grid, s);
    else launch_coop<ACT, G2048_OBS_RAW, FAC>(a, grid, s);
}

// grid = one workgroup per CU for grad_kernel (every wave one partial row); the cooperative kernel runs two per CU
// with two rows per workgroup, the same row count
template <int NT1, int NT2>
void launch_grad(const GradArgs& a, int act, int obs, int grid, hipStream_t s) {
    if constexpr (NT1 == 8 && NT2 == 8) {   // 256 x 256: the cooperative kernel (round 4: 0.78 of the fp32 MFMA peak
                                            // against grad_kernel's 0.68, profiles/round4/r4c6/)
        if (act == G2048_ACT_RELU && a.d2_form == 1) launch_coop_obs<0, 1>(a, obs, 2 * grid, s);
        else if (act == G2048_ACT_RELU && a.d2_form == 2) launch_coop_obs<0, 2>(a, obs, 2 * grid, s);
        else if (act == G2048_ACT_RELU) launch_coop_obs<0, 0>(a, obs, 2 * grid, s);
        else launch_coop_obs<1, 0>(a, obs, 2 * grid, s);
    } else if (act == G2048_ACT_RELU && a.d2_form == 1) {
        if (obs == G2048_OBS_LOG2) hipLaunchKernelGGL((grad_kernel<NT1, NT2, 0, G2048_OBS_LOG2, 1>), dim3(grid), dim3(kPolBlock), 0, s, a);
        else hipLaunchKernelGGL((grad_kernel<NT1, NT2, 0, G2048_OBS_RAW, 1>), dim3(grid), dim3(kPolBlock), 0, s, a);
    } else if (act == G2048_ACT_RELU && a.d2_form == 2) {
        if (obs == G2048_OBS_LOG2) hipLaunchKernelGGL((grad_kernel<NT1, NT2, 0, G2048_OBS_LOG2, 2>), dim3(grid), dim3(kPolBlock), 0, s, a);
        else hipLaunchKernelGGL((grad_kernel<NT1, NT2, 0, G2048_OBS_RAW, 2>), dim3(grid), dim3(kPolBlock), 0, s, a);
    } else if (act == G2048_ACT_RELU) {
        if (obs == G2048_OBS_LOG2) hipLaunchKernelGGL((grad_kernel<NT1, NT2, 0, G2048_OBS_LOG2>), dim3(grid), dim3(kPolBlock), 0, s, a);
        else hipLaunchKernelGGL((grad_kernel<NT1, NT2, 0, G2048_OBS_RAW>), dim3(grid), dim3(kPolBlock), 0, s, a);
    } else {
        if (obs == G2048_OBS_LOG2) hipLaunchKernelGGL((grad_kernel<NT1, NT2, 1, G2048_OBS_LOG2>), dim3(grid), dim3(kPolBlock), 0, s, a);
        else hipLaunchKernelGGL((grad_kernel<NT1, NT2, 1, G2048_OBS_RAW>), dim3(grid), dim3(kPolBlock), 0, s, a);
    }
}

template <int NT1>
void launch_grad_nt2(const GradArgs& a, int nt2, int act, int obs, int grid, hipStream_t s) {
    switch (nt2) {
        case 1: launch_grad<NT1, 1>(a, act, obs, grid, s); break;
        case 2: launch_grad<NT1, 2>(a, act, obs, grid, s); break;
        case 4: launch_grad<NT1, 4>(a, act, obs, grid, s); break;
        default: launch_grad<NT1, 8>(a, act, obs, grid, s); break;
    }
}

template <int NT1, int NT2, int ACT>
void launch_roll_obs(const RolloutArgs& a, int obs, int grid, hipStream_t s) {
    if (obs == G2048_OBS_LOG2) hipLaunchKernelGGL((rollout_kernel<NT1, NT2, ACT, G2048_OBS_LOG2>), dim3(grid), dim3(kPolBlock), 0, s, a);
    else hipLaunchKernelGGL((rollout_kernel<NT1, NT2, ACT, G2048_OBS_RAW>), dim3(grid), dim3(kPolBlock), 0, s, a);
}

template <int NT1, int NT2>
void launch_roll_act(const RolloutArgs& a, int act, int obs, int grid, hipStream_t s) {
    if (act == G2048_ACT_RELU) launch_roll_obs<NT1, NT2, 0>(a, obs, grid, s);
    else launch_roll_obs<NT1, NT2, 1>(a, obs, grid, s);
}

template <int NT1>
void launch_roll_nt2(const RolloutArgs& a, int nt2, int act, int obs, int grid, hipStream_t s) {
    switch (nt2) {
        case 1: launch_roll_act<NT1, 1>(a, act, obs, grid, s); break;
        case 2: launch_roll_act<NT1, 2>(a, act, obs, grid, s); break;
        case 4: launch_roll_act<NT1, 4>(a, act, obs, grid, s); break;
        default: launch_roll_act<NT1, 8>(a, act, obs, grid, s); break;
    }
}

int tiles_for(int hsize) {   // hidden units -> 32-unit tiles, rounded up to 1, 2, 4 or 8
    const int t = (hsize + 31) / 32;
    return t <= 1 ? 1 : t <= 2 ? 2 : t <= 4 ? 4 : 8;
}

}  // namespace

namespace g2048_internal {   // g2048.hip
int set_error(int code, const char* msg);   // the g2048_last_error() string
int device_tables(const uint8_t*& tab, int& cus);
int check_env_cfg(const g2048_env_cfg* c);
g2048::RewardCfg reward_cfg_of(const g2048_env_cfg& c);
}  // namespace g2048_internal

namespace {
int pfail(int code, const char* msg) { return g2048_internal::set_error(code, msg); }
}  // namespace

extern "C" {

#if G2048_DIAG
int g2048_diag_rollout_phases(unsigned long long* out, int blocks) {
    if (blocks > kRollDiagBlocks) blocks = kRollDiagBlocks;
    if (hipDeviceSynchronize() != hipSuccess) return G2048_EHIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_roll_ph), sizeof(unsigned long long) * 5 * blocks, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return G2048_EHIP;
    return blocks;
}
int g2048_diag_grad_phases(unsigned long long* out, int blocks) {
    if (blocks > kRollDiagBlocks) blocks = kRollDiagBlocks;
    if (hipDeviceSynchronize() != hipSuccess) return G2048_EHIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_grad_ph), sizeof(unsigned long long) * 6 * blocks, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return G2048_EHIP;
    return blocks;
}
#endif

int64_t g2048_policy_packed_size(int h1, int h2) {
    if (h1 < 1 || h1 > 256 || h2 < 1 || h2 > 256) return -1;
    return pol_layout(tiles_for(h1), tiles_for(h2)).total;
}

int g2048_policy_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                      const float* b3, int in_dim, int h1, int h2, float* packed, int64_t packed_len, void* stream) {
    if (in_dim != 16) return pfail(G2048_EINVAL, "fused policy: obs width must be 16 (log2 / raw obs)");
    const int64_t need = g2048_policy_packed_size(h1, h2);
    if (need < 0) return pfail(G2048_EINVAL, "fused policy: hidden sizes must be in 1..256");
    if (!W1 || !b1 || !W2 || !b2 || !W3 || !b3 || !packed) return pfail(G2048_EINVAL, "fused policy: NULL weight");
    if (packed_len < need) return pfail(G2048_EINVAL, "fused policy: packed buffer too small");
    PackArgs a{W1, b1, W2, b2, W3, b3, h1, h2, tiles_for(h1), tiles_for(h2), packed, need};
    const int grid = (int)((need + 255) / 256 < 4096 ? (need + 255) / 256 : 4096);
    hipLaunchKernelGGL(pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return pfail(G2048_EHIP, hipGetErrorString(e));
    return G2048_OK;
}

int g2048_policy(const float* packed, int h1, int h2, int activation, const uint64_t* boards,
                 const uint32_t* lane_state, const int32_t* lane_index, int obs_mode, float obs_scale, int use_mask,
                 int greedy, int rng_mode, uint64_t* rng_state, const uint64_t* rng_inc, const uint64_t* rng_buf,
                 uint64_t philox_key, const uint64_t* lane_seed, float* probs_out, float* logits_out,
                 uint8_t* actions, int64_t n, void* stream) {
    if (n < 0 || n > (int64_t)0xFFFFFFE0) return pfail(G2048_EINVAL, "n out of range");
    if (n == 0) return G2048_OK;
    if (!packed || !boards || !actions) return pfail(G2048_EINVAL, "packed / boards / actions is NULL");
    if (g2048_policy_packed_size(h1, h2) < 0) return pfail(G2048_EINVAL, "fused policy: hidden sizes must be in 1..256");
    if (activation != G2048_ACT_RELU && activation != G2048_ACT_SIGMOID)
        return pfail(G2048_EINVAL, "Unsupported activation");
    if (obs_mode != G2048_OBS_LOG2 && obs_mode != G2048_OBS_RAW)
        return pfail(G2048_EINVAL, "fused policy: obs_mode must be log2 or raw");
    if (rng_mode != G2048_RNG_PCG64 && rng_mode != G2048_RNG_PHILOX) return pfail(G2048_EINVAL, "Unsupported rng_mode");
    if (!greedy && rng_mode == G2048_RNG_PCG64 && (!rng_state || !rng_inc || !rng_buf))
        return pfail(G2048_EINVAL, "PCG64 sampling needs rng_state / rng_inc / rng_buf");
    PolArgs a;
    a.net = packed;
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
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0) cus = c;
    }
    const int64_t groups = (n + 31) / 32, waves_per_block = kPolBlock / 64;
    int64_t grid = (groups + waves_per_block - 1) / waves_per_block;
    const int nt1 = tiles_for(h1), nt2 = tiles_for(h2);
    const int per_cu = nt1 >= 8 ? 1 : 2;   // pol_waves_per_simd
    if (grid > per_cu * cus) grid = per_cu * cus;   // persistent
    hipStream_t s = (hipStream_t)stream;
    switch (nt1) {
        case 1: launch_pol_nt2<1>(a, nt2, activation, obs_mode, rng_mode, (int)grid, s); break;
        case 2: launch_pol_nt2<2>(a, nt2, activation, obs_mode, rng_mode, (int)grid, s); break;
        case 4: launch_pol_nt2<4>(a, nt2, activation, obs_mode, rng_mode, (int)grid, s); break;
        default: launch_pol_nt2<8>(a, nt2, activation, obs_mode, rng_mode, (int)grid, s); break;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return pfail(G2048_EHIP, hipGetErrorString(e));
    return G2048_OK;
}

int64_t g2048_grad_packed_size(int h1, int h2) {
    if (h1 < 1 || h1 > 256 || h2 < 1 || h2 > 256) return -1;
    return (int64_t)tiles_for(h1) * tiles_for(h2) * 1024;
}

int64_t g2048_grad_partial_size(int h1, int h2) {
    if (h1 < 1 || h1 > 256 || h2 < 1 || h2 > 256) return -1;
    return grad_part_floats(tiles_for(h1), tiles_for(h2));
}

int g2048_grad_pack(const float* W2, int h1, int h2, float* packed, int64_t packed_len, void* stream) {
    const int64_t need = g2048_grad_packed_size(h1, h2);
    if (need < 0) return pfail(G2048_EINVAL, "fused gradient: hidden sizes must be in 1..256");
    if (!W2 || !packed) return pfail(G2048_EINVAL, "fused gradient: NULL buffer");
    if (packed_len < need) return pfail(G2048_EINVAL, "fused gradient: packed buffer too small");
    GradPackArgs a{W2, h1, h2, tiles_for(h1), tiles_for(h2), packed, need};
    const int grid = (int)((need + 255) / 256 < 4096 ? (need + 255) / 256 : 4096);
    hipLaunchKernelGGL(grad_pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return pfail(G2048_EHIP, hipGetErrorString(e));
    return G2048_OK;
}

int g2048_actor_grad_waves(void) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0) cus = c;
    }
    return cus * (kPolBlock / 64);
}

// the actor and critic entry points share one kernel (GradArgs::critic selects the loss gradient)
static int actor_or_critic_grad(const float* packed, const float* grad_packed, int h1, int h2, int activation, int obs_mode,
                         float obs_scale, int use_mask, const uint64_t* boards, const uint8_t* actions,
                         const float* coef, int64_t n, int64_t ld, int64_t col_off, int64_t ncols, float* a1t, float* d2t,
                         float* partials, int accumulate, int64_t waves, void* stream, int critic, int huber,
                         float huber_delta, const float* target, float* delta_out, float* v_out, int d2_form = 0,
                         const g2048_td_rows* td = nullptr) {
    if (n < 0 || ld < n || (ld & 31) || ld > ((int64_t)1 << 21)) return pfail(G2048_EINVAL, "fused gradient: bad n / ld");
    if (col_off < 0 || (col_off & 31) || ncols < n || (ncols & 31) || col_off + ncols > ld)
        return pfail(G2048_EINVAL, "fused gradient: bad column window (col_off / ncols multiples of 32, n <= ncols, "
                                   "col_off + ncols <= ld)");
    if (g2048_grad_packed_size(h1, h2) < 0) return pfail(G2048_EINVAL, "fused gradient: hidden sizes must be in 1..256");
    if (activation != G2048_ACT_RELU && activation != G2048_ACT_SIGMOID)
        return pfail(G2048_EINVAL, "Unsupported activation");
    if (obs_mode != G2048_OBS_LOG2 && obs_mode != G2048_OBS_RAW)
        return pfail(G2048_EINVAL, "fused gradient: obs_mode must be log2 or raw");
    if (!packed || !grad_packed || !a1t || !d2t || !partials || (n > 0 && (!boards || !coef)))
        return pfail(G2048_EINVAL, "fused gradient: NULL buffer");
    if (waves != g2048_actor_grad_waves()) return pfail(G2048_EINVAL, "fused gradient: waves != g2048_actor_grad_waves()");
    if (d2_form != 0 && (d2_form != (critic ? 1 : 2) || activation != G2048_ACT_RELU))
        return pfail(G2048_EINVAL, "fused gradient: the factored d2 records are d2_form 1 for the ReLU critic, 2 for "
                                   "the ReLU actor");
    GradArgs a;
    a.net = packed;
    a.w2b = grad_packed;
    a.boards = boards;
    a.actions = actions;
    a.coef = coef;
    a.a1t = a1t;
    a.d2t = d2t;
    a.part = partials;
    a.n = (uint32_t)n;
    a.ld = (uint32_t)ld;
    a.obs_scale = obs_scale;
    a.use_mask = use_mask;
    a.critic = critic;
    a.huber = huber;
    a.huber_delta = huber_delta;
    a.target = target;
    a.delta_out = delta_out;
    a.v_out = v_out;
    a.has_td = td != nullptr;
    a.td = td ? *td : g2048_td_rows{};
    a.col_off = (uint32_t)col_off;
    a.ngroups = (uint32_t)(ncols >> 5);
    a.part_accum = accumulate;
    a.d2_form = d2_form;
    const int grid = (int)(waves / (kPolBlock / 64));   // one workgroup per CU; every wave writes its partial row
    const int nt1 = tiles_for(h1), nt2 = tiles_for(h2);
    hipStream_t s = (hipStream_t)stream;
    switch (nt1) {
        case 1: launch_grad_nt2<1>(a, nt2, activation, obs_mode, grid, s); break;
        case 2: launch_grad_nt2<2>(a, nt2, activation, obs_mode, grid, s); break;
        case 4: launch_grad_nt2<4>(a, nt2, activation, obs_mode, grid, s); break;
        default: launch_grad_nt2<8>(a, nt2, activation, obs_mode, grid, s); break;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return pfail(G2048_EHIP, hipGetErrorString(e));
    return G2048_OK;
}

int g2048_actor_grad(const float* packed, const float* grad_packed, int h1, int h2, int activation, int obs_mode,
                     float obs_scale, int use_mask, const uint64_t* boards, const uint8_t* actions, const float* coef,
                     int64_t n, int64_t ld, float* a1t, float* d2t, float* partials, int64_t waves, int d2_form,
                     void* stream) {
    if (n > 0 && !actions) return pfail(G2048_EINVAL, "fused gradient: NULL buffer");
    return actor_or_critic_grad(packed, grad_packed, h1, h2, activation, obs_mode, obs_scale, use_mask, boards, actions,
                                coef, n, ld, 0, ld, a1t, d2t, partials, 0, waves, stream, 0, 0, 0.0f, nullptr, nullptr,
                                nullptr, d2_form);
}

int g2048_critic_grad(const float* packed, const float* grad_packed, int h1, int h2, int activation, int obs_mode,
                      float obs_scale, int loss, float huber_delta, const uint64_t* boards, const float* target,
                      const float* weight, float* delta_out, float* value_out, int64_t n, int64_t ld, int64_t col_off,
                      int64_t ncols, float* a1t, float* d2t, float* partials, int accumulate, int64_t waves,
                      int d2_form, const g2048_td_rows* td, void* stream) {
    if (loss != 0 && loss != 1) return pfail(G2048_EINVAL, "Unknown critic loss type");
    if (n > 0 && !target && !td) return pfail(G2048_EINVAL, "fused gradient: NULL buffer");
    if (td && n > 0 && (!td->lane || !td->reward || !td->has_next || !td->v_next || !td->v_out))
        return pfail(G2048_EINVAL, "fused gradient: NULL TD-row buffer");
    return actor_or_critic_grad(packed, grad_packed, h1, h2, activation, obs_mode, obs_scale, 0, boards, nullptr, weight,
                                n, ld, col_off, ncols, a1t, d2t, partials, accumulate, waves, stream, 1, loss,
                                huber_delta, target, delta_out, value_out, d2_form, td);
}

int g2048_rollout(const float* packed, int h1, int h2, int activation, const g2048_env_cfg* cfg, int greedy,
                  const uint64_t* env_state, const uint64_t* env_inc, const uint64_t* env_buf, const uint64_t* pol_state,
                  const uint64_t* pol_inc, const uint64_t* pol_buf, uint32_t* queue, int64_t n, int64_t cap,
                  uint64_t* boards, uint8_t* actions, double* rewards, uint8_t* flags, float* probs, int32_t* lengths,
                  double* totals, uint8_t* max_tile, uint64_t* final_board, void* stream) {
    int rc = g2048_internal::check_env_cfg(cfg);
    if (rc) return rc;
    if (n < 0 || n > (int64_t)0x7FFFFFFF) return pfail(G2048_EINVAL, "n out of range");
    if (n == 0) return G2048_OK;
    if (cfg->obs_mode != G2048_OBS_LOG2 && cfg->obs_mode != G2048_OBS_RAW)
        return pfail(G2048_EINVAL, "fused rollout: obs_mode must be log2 or raw");
    if (cfg->max_steps < 0) return pfail(G2048_EINVAL, "fused rollout: max_steps must be set (>= 0)");
    if (cap < (cfg->max_steps > 1 ? cfg->max_steps : 1) || cap > (int64_t)0x7FFFFFFF)
        return pfail(G2048_EINVAL, "fused rollout: cap must be >= max(max_steps, 1)");
    if (g2048_policy_packed_size(h1, h2) < 0) return pfail(G2048_EINVAL, "fused policy: hidden sizes must be in 1..256");
    if (activation != G2048_ACT_RELU && activation != G2048_ACT_SIGMOID)
        return pfail(G2048_EINVAL, "Unsupported activation");
    if (!packed || !env_state || !env_inc || !env_buf || !pol_state || !pol_inc || !pol_buf || !queue || !boards ||
        !actions || !rewards || !flags || !lengths || !totals || !max_tile || !final_board)
        return pfail(G2048_EINVAL, "fused rollout: a required buffer is NULL");
    const uint8_t* tab = nullptr;
    int cus = 256;
    if ((rc = g2048_internal::device_tables(tab, cus))) return rc;
    RolloutArgs a;
    a.net = packed;
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
    a.boards = boards;
    a.actions = actions;
    a.rewards = rewards;
    a.flags = flags;
    a.probs = probs;
    a.lengths = lengths;
    a.totals = totals;
    a.max_tile = max_tile;
    a.final_board = final_board;
    a.n = (uint32_t)n;
    a.cap = (uint32_t)cap;
    const int nt1 = tiles_for(h1), nt2 = tiles_for(h2);
    int64_t grid = (n + 31) / 32;                  // one workgroup per 32 episode slots
    if (grid > kRollBlocksPerCU * cus) grid = kRollBlocksPerCU * cus;   // persistent; the slots refill from the queue
    hipStream_t s = (hipStream_t)stream;
    switch (nt1) {
        case 1: launch_roll_nt2<1>(a, nt2, activation, cfg->obs_mode, (int)grid, s); break;
        case 2: launch_roll_nt2<2>(a, nt2, activation, cfg->obs_mode, (int)grid, s); break;
        case 4: launch_roll_nt2<4>(a, nt2, activation, cfg->obs_mode, (int)grid, s); break;
        default: launch_roll_nt2<8>(a, nt2, activation, cfg->obs_mode, (int)grid, s); break;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return pfail(G2048_EHIP, hipGetErrorString(e));
    return G2048_OK;
}

}  // extern "C"
