// g2048.hip -- gfx950 (MI355X / CDNA4) kernels and the C ABI of libg2048.so (declared in include/g2048.h).
//
// One board per lane, uint64 bitboard (nibble r*4+c = log2 tile).  The hot kernel is g2048_step:
//   * integer/indexing work, no MFMA: the HBM stream of lane state is the roofline ("Kernels");
//   * the 65,536-entry move-left line table (uint16, 128 KiB) is staged once per workgroup into LDS and each
//     move is 4 LDS lookups (one per line of the move-left frame);
//   * action mask / done are 64-bit SWAR expressions (no table);
//   * the spawn draws the k-th empty cell with popcount bisection on the nibble-empty mask (numpy PCG64
//     stream in parity mode, Philox4x32-10 in throughput mode);
//   * observations are written wave-cooperatively: every store instruction covers 1 KiB of contiguous obs,
//     the owning board is fetched from its lane with a cross-lane shuffle.
// Workgroups are persistent over the board array (grid <= one 1024-thread workgroup per CU, limited by the
// 128 KiB LDS table), so the table fill is paid once per CU per launch.
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>

#include "g2048.h"
#include "g2048_core.h"

using namespace g2048;

namespace {

thread_local std::string g_err;
std::mutex g_mu;
constexpr int kMaxDev = 64;
uint16_t* g_lut[kMaxDev] = {};
int g_cus[kMaxDev] = {};

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define G2048_HIP(x)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) return fail(G2048_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kBlock = 1024;         // 16 waves per CU; one workgroup per CU (LDS table)
constexpr int kLutEntries = 65536;
constexpr int kLutSmallN = 16384;    // below this many lanes the table is read from L2 instead of LDS

struct LutFn {
    const uint16_t* t;
    __device__ uint32_t operator()(uint32_t i) const { return t[i]; }
};

__device__ inline uint64_t shfl64(uint64_t v, int src) {
    uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// Write obs for the 64 boards [w0, w0+64) held one per lane in `b` (lanes whose bit in `wmask` is clear
// write nothing).  Every store instruction covers a contiguous 1 KiB slice of the wave's obs region.
template <int OBS>
__device__ inline void write_obs_wave(float* __restrict__ obs, int64_t w0, uint64_t b, uint64_t wmask, int lane,
                                      float scale) {
    if constexpr (OBS == G2048_OBS_ONEHOT) {
        float4* dst = reinterpret_cast<float4*>(obs + w0 * 272);
#pragma unroll 4
        for (int k = 0; k < 68; k++) {
            const int q = k * 64 + lane;       // float4 index in the wave's region
            const int src = q / 68;            // owning board (lane)
            const int j = (q - src * 68) * 4;  // first float index inside the board's 272
            const uint64_t bb = shfl64(b, src);
            if ((wmask >> src) & 1ull) {
                float v[4];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const int idx = j + t;
                    const int cell = idx / 17;
                    const int ch = idx - cell * 17;
                    v[t] = ((int)((bb >> (4 * cell)) & 15u) == ch) ? 1.0f : 0.0f;
                }
                dst[q] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    } else if constexpr (OBS == G2048_OBS_LOG2 || OBS == G2048_OBS_RAW) {
        float4* dst = reinterpret_cast<float4*>(obs + w0 * 16);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int q = k * 64 + lane;
            const int src = q >> 2;
            const int row = q & 3;
            const uint64_t bb = shfl64(b, src);
            if ((wmask >> src) & 1ull) {
                float v[4];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const uint32_t e = (uint32_t)(bb >> (16 * row + 4 * t)) & 15u;
                    if constexpr (OBS == G2048_OBS_LOG2) v[t] = (float)e * scale;
                    else v[t] = e ? (float)(1u << e) : 0.0f;
                }
                dst[q] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    }
}

__device__ inline void store_mask(int8_t* mask, int64_t i, uint32_t m) {
    // int8[4] per board, one 32-bit store: byte a = bit a
    const uint32_t w = (m & 1u) | ((m & 2u) << 7) | ((m & 4u) << 14) | ((m & 8u) << 21);
    reinterpret_cast<uint32_t*>(mask)[i] = w;
}

__device__ inline Pcg64 load_pcg(const g2048_lanes& L, int64_t i) {
    Pcg64 g;
    const ulonglong2 s = reinterpret_cast<const ulonglong2*>(L.rng_state)[i];
    const ulonglong2 c = reinterpret_cast<const ulonglong2*>(L.rng_inc)[i];
    const uint64_t buf = L.rng_buf[i];
    g.s_lo = s.x;
    g.s_hi = s.y;
    g.i_lo = c.x;
    g.i_hi = c.y;
    g.has_uint32 = (uint32_t)(buf >> 32);
    g.uinteger = (uint32_t)buf;
    return g;
}

__device__ inline void store_pcg(const g2048_lanes& L, int64_t i, const Pcg64& g, bool with_inc) {
    reinterpret_cast<ulonglong2*>(L.rng_state)[i] = make_ulonglong2(g.s_lo, g.s_hi);
    if (with_inc) reinterpret_cast<ulonglong2*>(L.rng_inc)[i] = make_ulonglong2(g.i_lo, g.i_hi);
    L.rng_buf[i] = ((uint64_t)g.has_uint32 << 32) | g.uinteger;
}

__device__ inline U4 philox_ctr(uint64_t key, uint64_t seed, uint32_t ctr, uint32_t tag) {
    U4 c{(uint32_t)seed, (uint32_t)(seed >> 32), ctr, tag};
    return philox4x32(c, (uint32_t)key, (uint32_t)(key >> 32));
}

// Game2048.reset (src/game2048.py:26-34): empty board, two spawns from a fresh stream.
template <int RNG>
__device__ inline uint64_t fresh_board(uint64_t seed, uint64_t key, Pcg64& g) {
    uint64_t b = 0;
    if constexpr (RNG == G2048_RNG_PCG64) {
        g = pcg_seed(seed);
        b = spawn_pcg(b, g);
        b = spawn_pcg(b, g);
    } else {
        b = spawn_philox(b, philox_ctr(key, seed, 0u, 1u));
        b = spawn_philox(b, philox_ctr(key, seed, 0u, 2u));
    }
    return b;
}

struct StepArgs {
    g2048_lanes L;
    const uint8_t* actions;
    g2048_step_out out;
    RewardCfg rc;
    float obs_scale;
    int auto_reset;
    int64_t max_steps;
    uint64_t stride, key;
    const uint16_t* lut;
    int64_t n;
};

// One lane of Game2048Env.step (src/env.py:264-302).  Returns the board the obs/mask describe and whether
// this lane writes obs.
template <int RNG>
__device__ inline uint64_t step_lane(const StepArgs& a, int64_t i, const uint16_t* lut, bool& wobs) {
    const g2048_lanes& L = a.L;
    const uint64_t b = L.board[i];
    const uint8_t st = L.status[i];
    const uint32_t act = a.actions[i];
    if (a.out.prev_board) a.out.prev_board[i] = b;
    if (!(st & G2048_S_ACTIVE) || act > 3u) {
        a.out.reward[i] = 0.0f;
        a.out.flags[i] = (st & G2048_S_ACTIVE) ? G2048_F_BADACTION : G2048_F_INACTIVE;
        if (a.out.merged) a.out.merged[i] = 0u;
        wobs = false;
        return b;
    }
    uint32_t sc = L.step_count[i] + 1u;
    uint32_t mt = L.max_tile[i];
    uint32_t score = L.score[i];
    uint64_t seed = 0;
    if constexpr (RNG == G2048_RNG_PHILOX) seed = L.seed[i];  // PCG64 mode reads it only on auto-reset
    Pcg64 g;
    if constexpr (RNG == G2048_RNG_PCG64) g = load_pcg(L, i);

    // Game2048.step (src/game2048.py:40-70): move, score, spawn only if changed, done of the final board
    MoveSummary s;
    uint64_t m = board_move(b, act, LutFn{lut}, s);
    const bool changed = m != b;
    score += s.score;
    if (changed) {
        if constexpr (RNG == G2048_RNG_PCG64) m = spawn_pcg(m, g);
        else m = spawn_philox(m, philox_ctr(a.key, seed, sc, 0u));
    }
    const bool done = is_done(m);
    const bool invalid = !changed && !done;
    const double r = env_reward(a.rc, s, m, done, invalid, mt);
    const bool trunc = a.max_steps >= 0 && (int64_t)sc >= a.max_steps && !done;
    uint32_t fl = (changed ? G2048_F_CHANGED : 0u) | (done ? G2048_F_TERMINATED : 0u) |
                  (trunc ? G2048_F_TRUNCATED : 0u) | (invalid ? G2048_F_INVALID : 0u) |
                  (s.overflow ? G2048_F_OVERFLOW : 0u);
    uint8_t nst = st;
    bool new_inc = false;
    if (done || trunc) {
        if (a.auto_reset) {
            if constexpr (RNG == G2048_RNG_PCG64) seed = L.seed[i];
            seed += a.stride;
            m = fresh_board<RNG>(seed, a.key, g);
            new_inc = true;
            sc = 0u;
            score = 0u;
            mt = 2u;
            fl |= G2048_F_RESET;
            L.seed[i] = seed;
        } else {
            nst = (uint8_t)(st & ~G2048_S_ACTIVE);
            L.status[i] = nst;
        }
    }
    L.board[i] = m;
    L.step_count[i] = sc;
    L.score[i] = score;
    L.max_tile[i] = (uint8_t)mt;
    if constexpr (RNG == G2048_RNG_PCG64) store_pcg(L, i, g, new_inc);
    a.out.reward[i] = (float)r;
    a.out.flags[i] = (uint8_t)fl;
    if (a.out.merged) a.out.merged[i] = s.list;
    wobs = true;
    return m;
}

template <int OBS, int RNG, bool LDS>
__global__ void __launch_bounds__(kBlock) step_kernel(StepArgs a) {
    __shared__ uint4 lut_lds[LDS ? kLutEntries / 8 : 1];
    const uint16_t* lut = a.lut;
    if constexpr (LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(a.lut);
#pragma unroll 8
        for (int k = threadIdx.x; k < kLutEntries / 8; k += kBlock) lut_lds[k] = src[k];
        __syncthreads();
        lut = reinterpret_cast<const uint16_t*>(lut_lds);
    }
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t wstride = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t w0 = wave * 64; w0 < a.n; w0 += wstride * 64) {
        const int64_t i = w0 + lane;
        bool wobs = false;
        uint64_t b = 0;
        if (i < a.n) b = step_lane<RNG>(a, i, lut, wobs);
        if (wobs && a.out.mask) store_mask(a.out.mask, i, action_mask(b));
        if constexpr (OBS != G2048_OBS_NONE) {
            const uint64_t wm = __ballot(wobs);
            if (a.out.obs && wm) write_obs_wave<OBS>(a.out.obs, w0, b, wm, lane, a.obs_scale);
        }
    }
}

struct ResetArgs {
    g2048_lanes L;
    const uint64_t* seeds;
    const uint8_t* reset_mask;
    int8_t* mask_out;
    float* obs_out;
    float obs_scale;
    uint64_t key;
    int64_t n;
};

template <int OBS, int RNG>
__global__ void __launch_bounds__(256) reset_kernel(ResetArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t wstride = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t w0 = wave * 64; w0 < a.n; w0 += wstride * 64) {
        const int64_t i = w0 + lane;
        bool w = false;
        uint64_t b = 0;
        if (i < a.n && (!a.reset_mask || a.reset_mask[i])) {
            const uint64_t seed = a.seeds ? a.seeds[i] : a.L.seed[i];
            Pcg64 g;
            b = fresh_board<RNG>(seed, a.key, g);
            a.L.seed[i] = seed;
            a.L.board[i] = b;
            a.L.step_count[i] = 0u;
            a.L.score[i] = 0u;
            a.L.max_tile[i] = 2u;  // Game2048Env.max_tile_seen = 4 (src/env.py:183)
            a.L.status[i] = G2048_S_ACTIVE;
            if constexpr (RNG == G2048_RNG_PCG64) store_pcg(a.L, i, g, true);
            w = true;
            if (a.mask_out) store_mask(a.mask_out, i, action_mask(b));
        }
        if constexpr (OBS != G2048_OBS_NONE) {
            const uint64_t wm = __ballot(w);
            if (a.obs_out && wm) write_obs_wave<OBS>(a.obs_out, w0, b, wm, lane, a.obs_scale);
        }
    }
}

template <int OBS>
__global__ void __launch_bounds__(256) obs_kernel(const uint64_t* __restrict__ boards, float* obs, int8_t* mask,
                                                  float scale, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t wstride = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t w0 = wave * 64; w0 < n; w0 += wstride * 64) {
        const int64_t i = w0 + lane;
        const bool v = i < n;
        const uint64_t b = v ? boards[i] : 0ull;
        if (v && mask) store_mask(mask, i, action_mask(b));
        if constexpr (OBS != G2048_OBS_NONE) {
            const uint64_t wm = __ballot(v);
            if (obs) write_obs_wave<OBS>(obs, w0, b, wm, lane, scale);
        }
    }
}

__global__ void __launch_bounds__(256) move_kernel(const uint64_t* __restrict__ boards, const uint8_t* __restrict__ actions,
                                                   const uint16_t* __restrict__ lut, uint64_t* out, uint32_t* merged,
                                                   uint8_t* flags, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t b = boards[i];
        const uint32_t act = actions[i];
        if (act > 3u) {
            out[i] = b;
            if (merged) merged[i] = 0u;
            if (flags) flags[i] = G2048_F_BADACTION;
            continue;
        }
        MoveSummary s;
        const uint64_t m = board_move(b, act, LutFn{lut}, s);
        out[i] = m;
        if (merged) merged[i] = s.list;
        if (flags) flags[i] = (uint8_t)((m != b ? G2048_F_CHANGED : 0u) | (s.overflow ? G2048_F_OVERFLOW : 0u));
    }
}

__global__ void __launch_bounds__(256) seed_kernel(const uint64_t* __restrict__ seeds, uint64_t* st, uint64_t* inc,
                                                   uint64_t* buf, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const Pcg64 g = pcg_seed(seeds[i]);
        reinterpret_cast<ulonglong2*>(st)[i] = make_ulonglong2(g.s_lo, g.s_hi);
        reinterpret_cast<ulonglong2*>(inc)[i] = make_ulonglong2(g.i_lo, g.i_hi);
        buf[i] = 0ull;
    }
}

struct SampleArgs {
    const float* logits;
    const int8_t* mask;
    const uint8_t* active;
    uint64_t *st, *inc, *buf;
    uint64_t key;
    const uint64_t* lane_seed;
    const uint32_t* counter;
    float* probs_out;
    uint8_t* actions;
    int64_t n;
    int greedy;
};

// logits_to_probs (src/MLP.py:139-156) + select_action (src/reinforce_agent.py:178-190)
template <int RNG>
__global__ void __launch_bounds__(256) sample_kernel(SampleArgs a) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
        if (a.active && !a.active[i]) continue;
        const float4 lg = reinterpret_cast<const float4*>(a.logits)[i];
        uint32_t mw = 0x01010101u;
        if (a.mask) mw = reinterpret_cast<const uint32_t*>(a.mask)[i];
        const bool m0 = mw & 0xFFu, m1 = (mw >> 8) & 0xFFu, m2 = (mw >> 16) & 0xFFu, m3 = mw >> 24;
        const float l0 = m0 ? lg.x : -1e9f, l1 = m1 ? lg.y : -1e9f, l2 = m2 ? lg.z : -1e9f, l3 = m3 ? lg.w : -1e9f;
        const float mx = fmaxf(fmaxf(l0, l1), fmaxf(l2, l3));
        const float e0 = expf(l0 - mx), e1 = expf(l1 - mx), e2 = expf(l2 - mx), e3 = expf(l3 - mx);
        const float s = ((e0 + e1) + e2) + e3;
        const float p[4] = {e0 / s, e1 / s, e2 / s, e3 / s};
        if (a.probs_out) reinterpret_cast<float4*>(a.probs_out)[i] = make_float4(p[0], p[1], p[2], p[3]);
        uint32_t act = 0;
        if (a.greedy) {
            // probs = probs * action_mask; argmax (first maximum)
            const float q[4] = {a.mask ? p[0] * (float)m0 : p[0], a.mask ? p[1] * (float)m1 : p[1],
                                a.mask ? p[2] * (float)m2 : p[2], a.mask ? p[3] * (float)m3 : p[3]};
            float best = q[0];
#pragma unroll
            for (int k = 1; k < 4; k++)
                if (q[k] > best) { best = q[k]; act = k; }
        } else {
            // Generator.choice(4, p): fp64 cdf, normalised by its last entry, searchsorted(side='right')
            double cdf[4], acc = 0.0;
#pragma unroll
            for (int k = 0; k < 4; k++) { acc += (double)p[k]; cdf[k] = acc; }
            double u;
            if constexpr (RNG == G2048_RNG_PCG64) {
                Pcg64 g;
                const ulonglong2 st = reinterpret_cast<const ulonglong2*>(a.st)[i];
                const ulonglong2 ic = reinterpret_cast<const ulonglong2*>(a.inc)[i];
                const uint64_t bf = a.buf[i];
                g.s_lo = st.x; g.s_hi = st.y; g.i_lo = ic.x; g.i_hi = ic.y;
                g.has_uint32 = (uint32_t)(bf >> 32); g.uinteger = (uint32_t)bf;
                u = pcg_random(g);
                reinterpret_cast<ulonglong2*>(a.st)[i] = make_ulonglong2(g.s_lo, g.s_hi);
            } else {
                const U4 r = philox_ctr(a.key, a.lane_seed ? a.lane_seed[i] : (uint64_t)i, a.counter ? a.counter[i] : 0u, 3u);
                const uint64_t x = ((uint64_t)r.x << 32) | r.y;
                u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
            }
#pragma unroll
            for (int k = 0; k < 4; k++) act += (cdf[k] / cdf[3] <= u) ? 1u : 0u;
        }
        a.actions[i] = (uint8_t)act;
    }
}

// compute_returns (src/reinforce_agent.py:255-273), time-major [T, n], fp64 accumulation
__global__ void __launch_bounds__(256) returns_kernel(const float* __restrict__ r, const int32_t* __restrict__ len,
                                                      double gamma, float* __restrict__ out, int64_t T, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t L = len[i];
        L = L > T ? T : L;
        double G = 0.0;
        for (int64_t t = L - 1; t >= 0; t--) {
            G = (double)r[t * n + i] + gamma * G;
            out[t * n + i] = (float)G;
        }
    }
}

__global__ void __launch_bounds__(256) sym_kernel(const uint64_t* __restrict__ b, const uint8_t* __restrict__ act,
                                                  uint64_t* ob, uint8_t* oa, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t x = b[i];
        const uint32_t a = act ? act[i] : 0u;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            ob[k * n + i] = symmetry_board(x, k);
            if (act && oa) oa[k * n + i] = (uint8_t)symmetry_action(a, k);
        }
    }
}

int current_device(int& dev) {
    G2048_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDev) return fail(G2048_EINVAL, "device ordinal out of range");
    return G2048_OK;
}

int lut_for_current(const uint16_t*& lut, int& cus) {
    int dev = 0;
    int rc = current_device(dev);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_lut[dev]) return fail(G2048_ENOINIT, "g2048_init() was not called for device " + std::to_string(dev));
    lut = g_lut[dev];
    cus = g_cus[dev];
    return G2048_OK;
}

int grid_for(int64_t n, int block, int cap_blocks) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap_blocks) g = cap_blocks;
    return (int)g;
}

RewardCfg reward_cfg(const g2048_env_cfg& c) {
    RewardCfg r;
    r.reward_mode = c.reward_mode;
    r.bonus_mode = c.bonus_mode;
    r.use_action_mask = c.use_action_mask;
    r.base_reward_scale = c.base_reward_scale;
    r.empty_tile_reward = c.empty_tile_reward;
    r.merge_reward = c.merge_reward;
    r.bonus_scale = c.bonus_scale;
    r.step_reward = c.step_reward;
    r.endgame_penalty = c.endgame_penalty;
    r.invalid_action_penalty = c.invalid_action_penalty;
    return r;
}

int check_cfg(const g2048_env_cfg* c) {
    if (!c) return fail(G2048_EINVAL, "cfg is NULL");
    if (c->obs_mode < G2048_OBS_NONE || c->obs_mode > G2048_OBS_ONEHOT)
        return fail(G2048_EINVAL, "Unsupported obs_mode: " + std::to_string(c->obs_mode));
    if (c->reward_mode < 0 || c->reward_mode > 1)
        return fail(G2048_EINVAL, "Unsupported reward mode: " + std::to_string(c->reward_mode));
    if (c->bonus_mode < 0 || c->bonus_mode > 2)
        return fail(G2048_EINVAL, "Unsupported bonus mode: " + std::to_string(c->bonus_mode));
    return G2048_OK;
}

int check_lanes(const g2048_lanes* L, int rng_mode) {
    if (!L || !L->board || !L->step_count || !L->score || !L->max_tile || !L->status || !L->seed)
        return fail(G2048_EINVAL, "lanes: a required buffer is NULL");
    if (rng_mode == G2048_RNG_PCG64 && (!L->rng_state || !L->rng_inc || !L->rng_buf))
        return fail(G2048_EINVAL, "lanes: PCG64 mode needs rng_state / rng_inc / rng_buf");
    if (rng_mode != G2048_RNG_PCG64 && rng_mode != G2048_RNG_PHILOX)
        return fail(G2048_EINVAL, "Unsupported rng_mode: " + std::to_string(rng_mode));
    return G2048_OK;
}

template <int OBS, int RNG>
void launch_step(const StepArgs& a, bool lds, int cus, hipStream_t s) {
    if (lds) {
        const int grid = grid_for(a.n, kBlock, cus);
        hipLaunchKernelGGL((step_kernel<OBS, RNG, true>), dim3(grid), dim3(kBlock), 0, s, a);
    } else {
        const int grid = grid_for(a.n, kBlock, cus * 2);
        hipLaunchKernelGGL((step_kernel<OBS, RNG, false>), dim3(grid), dim3(kBlock), 0, s, a);
    }
}

template <int RNG>
void launch_step_obs(const StepArgs& a, int obs, bool lds, int cus, hipStream_t s) {
    switch (obs) {
        case G2048_OBS_RAW: launch_step<G2048_OBS_RAW, RNG>(a, lds, cus, s); break;
        case G2048_OBS_LOG2: launch_step<G2048_OBS_LOG2, RNG>(a, lds, cus, s); break;
        case G2048_OBS_ONEHOT: launch_step<G2048_OBS_ONEHOT, RNG>(a, lds, cus, s); break;
        default: launch_step<G2048_OBS_NONE, RNG>(a, lds, cus, s); break;
    }
}

template <int RNG>
void launch_reset(const ResetArgs& a, int obs, int cus, hipStream_t s) {
    const int grid = grid_for(a.n, 256, cus * 8);
    switch (obs) {
        case G2048_OBS_RAW: hipLaunchKernelGGL((reset_kernel<G2048_OBS_RAW, RNG>), dim3(grid), dim3(256), 0, s, a); break;
        case G2048_OBS_LOG2: hipLaunchKernelGGL((reset_kernel<G2048_OBS_LOG2, RNG>), dim3(grid), dim3(256), 0, s, a); break;
        case G2048_OBS_ONEHOT: hipLaunchKernelGGL((reset_kernel<G2048_OBS_ONEHOT, RNG>), dim3(grid), dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL((reset_kernel<G2048_OBS_NONE, RNG>), dim3(grid), dim3(256), 0, s, a); break;
    }
}

int device_cus(int dev) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    return cus;
}

}  // namespace

extern "C" {

int g2048_abi_version(void) { return G2048_ABI_VERSION; }

const char* g2048_last_error(void) { return g_err.c_str(); }

int g2048_init(int device) {
    if (device < 0 || device >= kMaxDev) return fail(G2048_EINVAL, "device ordinal out of range");
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_lut[device]) return G2048_OK;
    int prev = 0;
    G2048_HIP(hipGetDevice(&prev));
    G2048_HIP(hipSetDevice(device));
    static uint16_t host[kLutEntries];
    for (uint32_t r = 0; r < (uint32_t)kLutEntries; r++) host[r] = (uint16_t)line_move_left(r);
    uint16_t* d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(host));
    if (e == hipSuccess) e = hipMemcpy(d, host, sizeof(host), hipMemcpyHostToDevice);
    const hipError_t e2 = hipSetDevice(prev);
    if (e != hipSuccess) {
        if (d) (void)hipFree(d);
        return fail(G2048_EHIP, std::string("g2048_init: ") + hipGetErrorString(e));
    }
    if (e2 != hipSuccess) return fail(G2048_EHIP, std::string("g2048_init: ") + hipGetErrorString(e2));
    g_lut[device] = d;
    g_cus[device] = device_cus(device);
    return G2048_OK;
}

int g2048_seed_pcg64(const uint64_t* seeds, uint64_t* rng_state, uint64_t* rng_inc, uint64_t* rng_buf, int64_t n,
                     void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (n == 0) return G2048_OK;
    if (!seeds || !rng_state || !rng_inc || !rng_buf) return fail(G2048_EINVAL, "NULL buffer");
    hipLaunchKernelGGL(seed_kernel, dim3(grid_for(n, 256, 2048)), dim3(256), 0, (hipStream_t)stream, seeds, rng_state,
                       rng_inc, rng_buf, n);
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_reset(const g2048_lanes* lanes, const uint64_t* seeds, const uint8_t* reset_mask, const g2048_env_cfg* cfg,
                int rng_mode, uint64_t philox_key, int8_t* mask_out, float* obs_out, int64_t n, void* stream) {
    int rc = check_cfg(cfg);
    if (!rc) rc = check_lanes(lanes, rng_mode);
    if (rc) return rc;
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (n == 0) return G2048_OK;
    const uint16_t* lut = nullptr;
    int cus = 256;
    if ((rc = lut_for_current(lut, cus))) return rc;
    ResetArgs a{*lanes, seeds, reset_mask, mask_out, obs_out, cfg->obs_log2_scale, philox_key, n};
    if (rng_mode == G2048_RNG_PCG64) launch_reset<G2048_RNG_PCG64>(a, obs_out ? cfg->obs_mode : G2048_OBS_NONE, cus, (hipStream_t)stream);
    else launch_reset<G2048_RNG_PHILOX>(a, obs_out ? cfg->obs_mode : G2048_OBS_NONE, cus, (hipStream_t)stream);
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_step(const g2048_lanes* lanes, const uint8_t* actions, const g2048_env_cfg* cfg, const g2048_step_out* out,
               int rng_mode, uint64_t philox_key, int auto_reset, uint64_t reset_stride, int64_t n, void* stream) {
    int rc = check_cfg(cfg);
    if (!rc) rc = check_lanes(lanes, rng_mode);
    if (rc) return rc;
    if (!actions) return fail(G2048_EINVAL, "actions is NULL");
    if (!out || !out->reward || !out->flags) return fail(G2048_EINVAL, "out.reward / out.flags are required");
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (n == 0) return G2048_OK;
    const uint16_t* lut = nullptr;
    int cus = 256;
    if ((rc = lut_for_current(lut, cus))) return rc;
    StepArgs a;
    a.L = *lanes;
    a.actions = actions;
    a.out = *out;
    a.rc = reward_cfg(*cfg);
    a.obs_scale = cfg->obs_log2_scale;
    a.auto_reset = auto_reset;
    a.max_steps = cfg->max_steps;
    a.stride = reset_stride;
    a.key = philox_key;
    a.lut = lut;
    a.n = n;
    const int obs = out->obs ? cfg->obs_mode : G2048_OBS_NONE;
    const bool lds = n >= kLutSmallN;
    if (rng_mode == G2048_RNG_PCG64) launch_step_obs<G2048_RNG_PCG64>(a, obs, lds, cus, (hipStream_t)stream);
    else launch_step_obs<G2048_RNG_PHILOX>(a, obs, lds, cus, (hipStream_t)stream);
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_obs(const uint64_t* boards, int obs_mode, float obs_log2_scale, float* obs, int8_t* mask, int64_t n,
              void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (!boards) return fail(G2048_EINVAL, "boards is NULL");
    if (obs_mode < G2048_OBS_NONE || obs_mode > G2048_OBS_ONEHOT)
        return fail(G2048_EINVAL, "Unsupported obs_mode: " + std::to_string(obs_mode));
    if (n == 0) return G2048_OK;
    const int grid = grid_for(n, 256, 2048);
    hipStream_t s = (hipStream_t)stream;
    switch (obs ? obs_mode : G2048_OBS_NONE) {
        case G2048_OBS_RAW: hipLaunchKernelGGL(obs_kernel<G2048_OBS_RAW>, dim3(grid), dim3(256), 0, s, boards, obs, mask, obs_log2_scale, n); break;
        case G2048_OBS_LOG2: hipLaunchKernelGGL(obs_kernel<G2048_OBS_LOG2>, dim3(grid), dim3(256), 0, s, boards, obs, mask, obs_log2_scale, n); break;
        case G2048_OBS_ONEHOT: hipLaunchKernelGGL(obs_kernel<G2048_OBS_ONEHOT>, dim3(grid), dim3(256), 0, s, boards, obs, mask, obs_log2_scale, n); break;
        default: hipLaunchKernelGGL(obs_kernel<G2048_OBS_NONE>, dim3(grid), dim3(256), 0, s, boards, obs, mask, obs_log2_scale, n); break;
    }
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_move(const uint64_t* boards, const uint8_t* actions, uint64_t* out_board, uint32_t* merged, uint8_t* flags,
               int64_t n, void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (!boards || !actions || !out_board) return fail(G2048_EINVAL, "NULL buffer");
    if (n == 0) return G2048_OK;
    const uint16_t* lut = nullptr;
    int cus = 256;
    int rc = lut_for_current(lut, cus);
    if (rc) return rc;
    hipLaunchKernelGGL(move_kernel, dim3(grid_for(n, 256, 2048)), dim3(256), 0, (hipStream_t)stream, boards, actions,
                       lut, out_board, merged, flags, n);
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_sample(const float* logits, const int8_t* mask, const uint8_t* active, int greedy, int rng_mode,
                 uint64_t* rng_state, uint64_t* rng_inc, uint64_t* rng_buf, uint64_t philox_key,
                 const uint64_t* lane_seed, const uint32_t* counter, float* probs_out, uint8_t* actions, int64_t n,
                 void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (!logits || !actions) return fail(G2048_EINVAL, "logits / actions are required");
    if (!greedy && rng_mode == G2048_RNG_PCG64 && (!rng_state || !rng_inc || !rng_buf))
        return fail(G2048_EINVAL, "PCG64 sampling needs rng_state / rng_inc / rng_buf");
    if (rng_mode != G2048_RNG_PCG64 && rng_mode != G2048_RNG_PHILOX)
        return fail(G2048_EINVAL, "Unsupported rng_mode: " + std::to_string(rng_mode));
    if (n == 0) return G2048_OK;
    SampleArgs a{logits, mask, active, rng_state, rng_inc, rng_buf, philox_key, lane_seed, counter, probs_out, actions, n, greedy};
    const int grid = grid_for(n, 256, 2048);
    if (rng_mode == G2048_RNG_PCG64) hipLaunchKernelGGL(sample_kernel<G2048_RNG_PCG64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    else hipLaunchKernelGGL(sample_kernel<G2048_RNG_PHILOX>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_returns(const float* rewards, const int32_t* lengths, double gamma, float* returns, int64_t T, int64_t n,
                  void* stream) {
    if (n < 0 || T < 0) return fail(G2048_EINVAL, "n < 0 or T < 0");
    if (!rewards || !lengths || !returns) return fail(G2048_EINVAL, "NULL buffer");
    if (n == 0 || T == 0) return G2048_OK;
    hipLaunchKernelGGL(returns_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, (hipStream_t)stream, rewards, lengths,
                       gamma, returns, T, n);
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_symmetries(const uint64_t* boards, const uint8_t* actions, uint64_t* out_boards, uint8_t* out_actions,
                     int64_t n, void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (!boards || !out_boards) return fail(G2048_EINVAL, "NULL buffer");
    if (n == 0) return G2048_OK;
    hipLaunchKernelGGL(sym_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, (hipStream_t)stream, boards, actions,
                       out_boards, out_actions, n);
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

}  // extern "C"
