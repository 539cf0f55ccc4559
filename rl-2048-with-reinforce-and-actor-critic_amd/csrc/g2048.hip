// g2048.hip -- gfx950 (MI355X / CDNA4) kernels and the C ABI of libg2048.so (declared in include/g2048.h).
//
// One board per lane, uint64 bitboard (nibble r*4+c = log2 tile).  The hot kernel is g2048_step
// (integer / indexing work, no MFMA; DESIGN.md "Kernels" has its roofline):
//   * two row tables are staged once per workgroup into LDS and fill it exactly (160 KiB): the move-left image
//     of every 4-nibble line (65,536 x uint16) and its 4-bit merge code (which output cells are merge results),
//     so a move is 4 x (one u16 + one nibble LDS lookup) with the merge summary read off the new line;
//   * action mask and done are 64-bit SWAR expressions sharing one set of neighbour masks;
//   * the spawn draws the k-th empty cell by popcount bisection (numpy-PCG64 stream in parity mode,
//     Philox4x32-10 in throughput mode);
//   * auto-resets (SeedSequence + two spawns) are deferred to the end of the wave's board loop and done in one
//     batch, so a rare reset costs one divergent pass per wave instead of one per board sweep;
//   * observations are written wave-cooperatively (every store instruction is 1 KiB of contiguous obs; the
//     owning board comes from its lane through a cross-lane shuffle);
//   * 32-bit byte offsets on SGPR bases (the launcher splits calls above kMaxLanesPerLaunch lanes).
// Workgroups are persistent (one 1024-thread workgroup per CU: the LDS tables allow one), so the table fill
// is paid once per CU per launch.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <string>

#include "g2048.h"
#include "g2048_core.h"

using namespace g2048;

static_assert(G2048_F_CHANGED == kFChanged && G2048_F_TERMINATED == kFTerminated && G2048_F_TRUNCATED == kFTruncated &&
                  G2048_F_INVALID == kFInvalid && G2048_F_OVERFLOW == kFOverflow,
              "g2048_core.h step flag bits == include/g2048.h");

namespace {

thread_local std::string g_err;
std::mutex g_mu;
constexpr int kMaxDev = 64;
uint8_t* g_tab[kMaxDev] = {};   // [65536 x u16 line table][32768 x u8 merge codes][32768 x u8 max-merge fields]
int g_cus[kMaxDev] = {};

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define G2048_HIP(x)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) return fail(G2048_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

// G2048_DIAG=1 (tools/diag_build.sh only; never the shipped library): G2048_DIAG_FLAGS in the environment
// removes pieces of the step kernel for timing attribution: 1 no LDS table fill, 2 no deferred resets,
// 4 no game compute (the board is xor'ed with the action, everything else stored as if computed),
// 8 one sweep per wave per launch-equivalent grid (grid = ceil(n / 1024)), 16 no obs writes.
#ifndef G2048_DIAG
#define G2048_DIAG 0
#endif
#if G2048_DIAG
// per-workgroup phase timestamps of the last step launch (s_memrealtime, 100 MHz): entry, tables filled,
// main loop done, reset list built, end
constexpr int kDiagSlots = 5, kDiagBlocks = 4096;
__device__ uint64_t g_diag_ts[kDiagBlocks * kDiagSlots];
#define G2048_TS(slot)                                                                          \
    do {                                                                                        \
        if (threadIdx.x == 0 && blockIdx.x < kDiagBlocks)                                       \
            g_diag_ts[blockIdx.x * kDiagSlots + (slot)] = __builtin_amdgcn_s_memrealtime();     \
    } while (0)
#else
#define G2048_TS(slot) \
    do {               \
    } while (0)
#endif

constexpr int kBlock = 1024;                  // 16 waves per CU; one workgroup per CU (160 KiB of LDS tables)
constexpr int kLines = 65536;
constexpr int kTabBytes = kLines * 2 + kLines / 2;   // 163,840 B = the whole LDS of a gfx950 CU
constexpr int kTabVec = kTabBytes / 16;
// the device table in global memory: the line table, the merge codes (board_move_coded: the general reward path,
// the move / rollout kernels) and the max-merge fields (board_move_lean: the log2-reward step path).  A step
// kernel stages the line table and ONE of the two 4-bit tables in LDS (160 KiB).
constexpr int kMxOff = kTabBytes;
constexpr int kDevTabBytes = kTabBytes + kLines / 2;
constexpr int kLutSmallN = 16384;             // below this many lanes the tables are read through L1/L2
constexpr int64_t kMaxLanesPerLaunch = int64_t(1) << 27;   // keeps every byte offset (<= 16 B/lane) in 32 bits

// ------------------------------------------------------------------------------------- addressing helpers
template <class T>
__device__ __forceinline__ T ld(const T* p, uint32_t idx) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(p) + idx * (uint32_t)sizeof(T));
}
template <class T>
__device__ __forceinline__ void st(T* p, uint32_t idx, T v) {
    *reinterpret_cast<T*>(reinterpret_cast<char*>(p) + idx * (uint32_t)sizeof(T)) = v;
}

// observation stores are non-temporal (streaming): measured on MI355X, onehot obs (1,088 B/board) 260 -> 241 us at
// 1M boards and 1050 -> 908 us at 4M; log2 obs unchanged (round 1, profiles/round1/ab_nt.log)
__device__ __forceinline__ void st_obs(float4* base, int q, float4 v) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(base + q));
}

struct LineFn {
    const uint16_t* line;
    __device__ uint32_t operator()(uint32_t o) const { return line[o]; }
};
struct CodeFn {   // a 4-bit-per-line table: merge codes or max-merge fields
    const uint8_t* code;
    __device__ uint32_t operator()(uint32_t o) const { return (code[o >> 1] >> ((o & 1u) << 2)) & 15u; }
};

__device__ inline uint64_t shfl64(uint64_t v, int src) {
    uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ inline uint32_t nib(uint64_t b, uint32_t cell) { return (uint32_t)(b >> (4u * cell)) & 15u; }

// ------------------------------------------------------------------------------------- observation writers
// Write obs for the 64 boards [w0, w0+64) held one per lane in `b` (lanes whose bit in `wmask` is clear write
// nothing).  Every store instruction covers a contiguous 1 KiB slice of the wave's obs region.
template <int OBS>
__device__ inline void write_obs_wave(float* __restrict__ obs, uint32_t w0, uint64_t b, uint64_t wmask, int lane,
                                      float scale) {
    if constexpr (OBS == G2048_OBS_ONEHOT) {
        float4* dst = reinterpret_cast<float4*>(obs) + (size_t)w0 * 68;
        // float4 q of the wave's region: board src = q / 68, floats j..j+3 of its 272 -- they touch at most two
        // cells, and each cell's one-hot 1 sits at 17 cell + e
        const auto value = [&](int q, int src, uint64_t bb) {
            const int j = (q - src * 68) * 4;
            const int c0 = j / 17;
            const int c1 = c0 + 1 < 16 ? c0 + 1 : 15;
            const int p0 = 17 * c0 + (int)nib(bb, c0);
            const int p1 = 17 * c1 + (int)nib(bb, c1);
            float4 v;
            v.x = (j == p0 || j == p1) ? 1.0f : 0.0f;
            v.y = (j + 1 == p0 || j + 1 == p1) ? 1.0f : 0.0f;
            v.z = (j + 2 == p0 || j + 2 == p1) ? 1.0f : 0.0f;
            v.w = (j + 3 == p0 || j + 3 == p1) ? 1.0f : 0.0f;
            return v;
        };
        if (wmask == ~0ull) {   // wave-uniform: every board of the chunk writes (no per-store lane test)
#pragma unroll 4
            for (int k = 0; k < 68; k++) {
                const int q = k * 64 + lane;
                const int src = q / 68;
                st_obs(dst, q, value(q, src, shfl64(b, src)));
            }
        } else {
#pragma unroll 4
            for (int k = 0; k < 68; k++) {
                const int q = k * 64 + lane;
                const int src = q / 68;
                const uint64_t bb = shfl64(b, src);
                if ((wmask >> src) & 1ull) st_obs(dst, q, value(q, src, bb));
            }
        }
    } else if constexpr (OBS == G2048_OBS_LOG2 || OBS == G2048_OBS_RAW) {
        float4* dst = reinterpret_cast<float4*>(obs) + (size_t)w0 * 4;
        const auto st_row = [&](int q, float4 v) { st_obs(dst, q, v); };
        const auto row_obs = [&](uint64_t bb, uint32_t row) {
            const uint32_t r16 = (uint32_t)(bb >> (16u * row));
            float v[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint32_t e = (r16 >> (4 * t)) & 15u;
                if constexpr (OBS == G2048_OBS_LOG2) v[t] = (float)e * scale;
                else v[t] = e ? (float)(1u << e) : 0.0f;
            }
            return make_float4(v[0], v[1], v[2], v[3]);
        };
        if (wmask == ~0ull) {   // wave-uniform: every board of the chunk writes (no per-store lane test)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int q = k * 64 + lane;
                st_row(q, row_obs(shfl64(b, q >> 2), (uint32_t)q & 3u));
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int q = k * 64 + lane;
                const int src = q >> 2;
                const uint64_t bb = shfl64(b, src);
                if ((wmask >> src) & 1ull) st_row(q, row_obs(bb, (uint32_t)q & 3u));
            }
        }
    }
}

// one lane's own obs (used for the rare deferred auto-resets)
template <int OBS>
__device__ inline void write_obs_lane(float* __restrict__ obs, uint32_t i, uint64_t b, float scale) {
    if constexpr (OBS == G2048_OBS_ONEHOT) {
        float4* dst = reinterpret_cast<float4*>(obs) + (size_t)i * 68;
        for (int k = 0; k < 68; k++) {
            const int j = 4 * k;
            const int c0 = j / 17;
            const int c1 = c0 + 1 < 16 ? c0 + 1 : 15;
            const int p0 = 17 * c0 + (int)nib(b, c0), p1 = 17 * c1 + (int)nib(b, c1);
            dst[k] = make_float4((j == p0 || j == p1) ? 1.f : 0.f, (j + 1 == p0 || j + 1 == p1) ? 1.f : 0.f,
                                 (j + 2 == p0 || j + 2 == p1) ? 1.f : 0.f, (j + 3 == p0 || j + 3 == p1) ? 1.f : 0.f);
        }
    } else if constexpr (OBS == G2048_OBS_LOG2 || OBS == G2048_OBS_RAW) {
        float4* dst = reinterpret_cast<float4*>(obs) + (size_t)i * 4;
        for (int r = 0; r < 4; r++) {
            float v[4];
            for (int t = 0; t < 4; t++) {
                const uint32_t e = nib(b, 4 * r + t);
                if constexpr (OBS == G2048_OBS_LOG2) v[t] = (float)e * scale;
                else v[t] = e ? (float)(1u << e) : 0.0f;
            }
            dst[r] = make_float4(v[0], v[1], v[2], v[3]);
        }
    }
}

__device__ inline uint32_t mask_word(uint32_t m) {
    // int8[4] per board as one 32-bit word: byte a = bit a
    return (m & 1u) | ((m & 2u) << 7) | ((m & 4u) << 14) | ((m & 8u) << 21);
}

// ------------------------------------------------------------------------------------- RNG state
// The lane's numpy PCG64 stream: state and increment (16 + 16 B) and the next_uint32 buffer value (4 B); the
// buffer's has_uint32 flag lives in the lane state word (G2048_LS_HAS_U32) and is set by the caller.
__device__ inline Pcg64 load_pcg(const g2048_lanes& L, uint32_t i) {
    Pcg64 g;
    const ulonglong2 s = ld(reinterpret_cast<const ulonglong2*>(L.rng_state), i);
    const ulonglong2 c = ld(reinterpret_cast<const ulonglong2*>(L.rng_inc), i);
    g.s_lo = s.x;
    g.s_hi = s.y;
    g.i_lo = c.x;
    g.i_hi = c.y;
    g.has_uint32 = 0u;
    g.uinteger = ld(L.rng_uint, i);
    return g;
}

__device__ inline void store_pcg(const g2048_lanes& L, uint32_t i, const Pcg64& g, bool with_inc) {
    st(reinterpret_cast<ulonglong2*>(L.rng_state), i, make_ulonglong2(g.s_lo, g.s_hi));
    if (with_inc) st(reinterpret_cast<ulonglong2*>(L.rng_inc), i, make_ulonglong2(g.i_lo, g.i_hi));
    st(L.rng_uint, i, g.uinteger);
}

// a fresh episode's state word: step 0, max_tile_seen 4 (src/env.py:183), active, the PCG64 buffer flag
__device__ inline uint32_t fresh_state(const Pcg64& g) {
    return (2u << G2048_LS_MAXT_SHIFT) | G2048_LS_ACTIVE | (g.has_uint32 ? G2048_LS_HAS_U32 : 0u);
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
        const U4 r = philox_ctr(key, seed, 0u, 1u);
        b = spawn_philox(b, U4{r.x, r.y, 0u, 0u});
        b = spawn_philox(b, U4{r.z, r.w, 0u, 0u});
    }
    return b;
}

// ------------------------------------------------------------------------------------- step
struct StepArgs {
    g2048_lanes L;
    const uint8_t* actions;
    g2048_step_out out;
    RewardCfg rc;
    float obs_scale;
    int auto_reset;
    int64_t max_steps;
    uint64_t stride, key;
    const uint8_t* tab;
    uint32_t n;
    int diag;
};

// Auto-reset of lane i (deferred to the end of the loop): Game2048Env.reset with seed = prev_seed + stride.
template <int OBS, int RNG>
__device__ inline void reset_lane(const StepArgs& a, uint32_t i, uint64_t prev_seed) {
    const g2048_lanes& L = a.L;
    const uint64_t seed = prev_seed + a.stride;
    Pcg64 g;
    g.has_uint32 = 0u;
    const uint64_t b = fresh_board<RNG>(seed, a.key, g);
    st(L.seed, i, seed);
    st(L.board, i, b);
    st(L.state, i, fresh_state(g));
    if constexpr (RNG == G2048_RNG_PCG64) store_pcg(L, i, g, true);
    if (a.out.mask) st(reinterpret_cast<uint32_t*>(a.out.mask), i, mask_word(action_mask(b)));
    if (a.out.mask_bits) st(a.out.mask_bits, i, (uint8_t)action_mask(b));
    if constexpr (OBS != G2048_OBS_NONE)
        if (a.out.obs) write_obs_lane<OBS>(a.out.obs, i, b, a.obs_scale);
}

// Everything one lane reads for one board's step (all boards of a sweep are loaded before any is computed).
struct LaneIn {
    uint64_t b, seed;
    uint32_t st, act;    // lane state word (G2048_LS_*), action
    Pcg64 g;
};

template <int RNG>
__device__ inline void load_lane(const StepArgs& a, uint32_t i, LaneIn& x) {
    const g2048_lanes& L = a.L;
    x.b = ld(L.board, i);
    x.st = ld(L.state, i);
    x.act = ld(a.actions, i);
    if constexpr (RNG == G2048_RNG_PCG64) x.g = load_pcg(L, i);   // PCG64 mode reads the seed only on reset
    else x.seed = ld(L.seed, i);
}

// One lane of Game2048Env.step (src/env.py:264-302).  Returns the final board; wobs = this lane's obs/mask are
// written by the wave; reset = the episode ended and an auto-reset is pending for this lane.
// XO (optional outputs, chosen by the launcher): 0 = none of prev_board / reward64 / score_add / merged (the
// rollout and bench path: no null-pointer tests in the loop, whose uniform conditions the compiler otherwise keeps
// as spilled 64-bit lane masks), 1 = any of the first three, 2 = the merged list too; 3 = as 0 with the action
// mask written packed (mask_bits) instead of as int8[4].
// RK (reward kind, chosen by the launcher): 0 = any config, `code` is the merge-code table (board_move_coded);
// 1 = reward_mode "log2" with XO 0 / 3, `code` is the max-merge field table (board_move_lean: no merge decode,
// no score, count and sum_e from board aggregates, the moved board's nz bits reused by the spawn and the masks).
template <int RNG, int XO, int RK>
__device__ inline uint64_t step_lane(const StepArgs& a, uint32_t i, LaneIn& x, const LineFn& lut,
                                     const CodeFn& code, bool& wobs, bool& reset, uint32_t& mbits) {
    static_assert(RK == 0 || XO == 0 || XO == 3, "the lean path writes no score / merged list");
    constexpr bool LIST = XO == 2, EXTRA = XO == 1 || XO == 2;
    const g2048_lanes& L = a.L;
    const uint64_t b = x.b;
    if (EXTRA && a.out.prev_board) st(a.out.prev_board, i, b);
    wobs = false;
    reset = false;
    if (!(x.st & G2048_LS_ACTIVE) || x.act > 3u) {
        st(a.out.reward, i, 0.0f);
        if (EXTRA && a.out.reward64) st(a.out.reward64, i, 0.0);
        st(a.out.flags, i, (uint8_t)((x.st & G2048_LS_ACTIVE) ? G2048_F_BADACTION : G2048_F_INACTIVE));
        if (LIST && a.out.merged) st(a.out.merged, i, 0u);
        if (EXTRA && a.out.score_add) st(a.out.score_add, i, 0u);
        return b;
    }
    const uint32_t sc0 = x.st & G2048_LS_STEP_MASK;
    const uint32_t sc = sc0 + (sc0 < G2048_LS_STEP_MASK ? 1u : 0u);   // saturating 20-bit step count
    uint32_t mt = (x.st >> G2048_LS_MAXT_SHIFT) & 31u;
    if constexpr (RNG == G2048_RNG_PCG64) x.g.has_uint32 = (x.st & G2048_LS_HAS_U32) ? 1u : 0u;

    // Game2048.step (src/game2048.py:40-70): move, score, spawn only if changed, done of the final board
    MoveSummary s;
    uint64_t m, nzm = 0;
    if (G2048_DIAG && (a.diag & 4)) {
        s = MoveSummary{0, 0, 0, 0, 0, 0};
        m = b ^ ((uint64_t)x.act << 60);
        nzm = nz_bits(m);
    } else if constexpr (RK == 1) {
        m = board_move_lean(b, x.act, lut, code, s, nzm);
    } else {
        m = board_move_coded<LIST>(b, x.act, lut, code, s);
    }
    const bool changed = m != b;
    if constexpr (RK == 1) {
        // nz bits of the final board: the moved board's, plus the spawned tile's
        if constexpr (RNG == G2048_RNG_PCG64) {
            if (!(G2048_DIAG && (a.diag & 4))) {
                // formed for every lane (a wave holds changed and unchanged boards), kept where the board changed
                Pcg64 g2 = x.g;
                uint64_t nzbit;
                const uint64_t m2 = spawn_pcg_lean(m, ~nzm & kNibLsb, g2, nzbit);
                m = changed ? m2 : m;
                nzm = changed ? nzm | nzbit : nzm;
                x.g.s_hi = changed ? g2.s_hi : x.g.s_hi;
                x.g.s_lo = changed ? g2.s_lo : x.g.s_lo;
                x.g.uinteger = changed ? g2.uinteger : x.g.uinteger;
                x.g.has_uint32 = changed ? g2.has_uint32 : x.g.has_uint32;
            }
        } else if (changed && !(G2048_DIAG && (a.diag & 4))) {
            uint64_t nzbit;
            m = spawn_philox_z(m, ~nzm & kNibLsb, philox_ctr(a.key, x.seed, sc, 0u), nzbit);
            nzm |= nzbit;
        }
    } else {
        if (changed && !(G2048_DIAG && (a.diag & 4))) {
            if constexpr (RNG == G2048_RNG_PCG64) m = spawn_pcg(m, x.g);
            else m = spawn_philox(m, philox_ctr(a.key, x.seed, sc, 0u));
        }
        nzm = nz_bits(m);
    }
    const BoardBits bits = board_bits_nz(m, nzm);
    const bool done = bits_done(bits);
    const bool invalid = !changed && !done;
    const double r = env_reward_nz<RK == 1>(a.rc, s, nzm, done, invalid, mt);
    const bool trunc = a.max_steps >= 0 && (int64_t)sc >= a.max_steps && !done;
    const uint32_t fl = (changed ? G2048_F_CHANGED : 0u) | (done ? G2048_F_TERMINATED : 0u) |
                        (trunc ? G2048_F_TRUNCATED : 0u) | (invalid ? G2048_F_INVALID : 0u) |
                        (s.overflow ? G2048_F_OVERFLOW : 0u);
    st(a.out.reward, i, (float)r);
    if (EXTRA && a.out.reward64) st(a.out.reward64, i, r);
    if (LIST && a.out.merged) st(a.out.merged, i, s.list);
    if (EXTRA && a.out.score_add) st(a.out.score_add, i, s.score);
    reset = (done || trunc) && a.auto_reset;   // board / lane state / obs are rewritten by reset_lane after the loop
    // A resetting lane stores this step's board / state / stream / mask / obs like any other lane (reset_lane
    // overwrites them after the loop): the sweep's stores then cover whole lines.  A hole left for the reset pass
    // is written back as a partial line, and filled later by another partial write; HBM3E has no byte mask, so
    // each partial line is a read-modify-write in the memory controller (measured: the first steps after the
    // synthetic start, 2-3 % of lanes resetting, ran 34 us against 29 us later; tools/step_launch_probe.py).
    uint32_t nst = sc | (mt << G2048_LS_MAXT_SHIFT) | ((done || trunc) ? 0u : G2048_LS_ACTIVE);
    if constexpr (RNG == G2048_RNG_PCG64) nst |= x.g.has_uint32 ? G2048_LS_HAS_U32 : 0u;
    st(a.out.flags, i, (uint8_t)(fl | (reset ? G2048_F_RESET : 0u)));
    st(L.board, i, m);
    st(L.state, i, nst);
    if constexpr (RNG == G2048_RNG_PCG64) store_pcg(L, i, x.g, false);
    wobs = true;
    mbits = bits_mask(bits);
    return m;
}

// One sweep of one wave: the step of board w0 + lane (inputs already in registers), its mask, the wave's obs.
// A lane's first pending reset has its seed read here (`pseed`), so the read is long complete at the tail.
template <int OBS, int RNG, int XO, int RK>
__device__ __forceinline__ void sweep(const StepArgs& a, uint32_t w0, int lane, LaneIn& x, const LineFn& lut,
                                      const CodeFn& code, uint64_t& pending, uint64_t& pseed, uint32_t k) {
    const uint32_t i = w0 + lane;
    bool wobs = false, reset = false;
    uint32_t mbits = 0;
    uint64_t b = 0;
    if (i < a.n) b = step_lane<RNG, XO, RK>(a, i, x, lut, code, wobs, reset, mbits);
    if (reset) {
        if (!pending) {
            if constexpr (RNG == G2048_RNG_PCG64) pseed = ld(a.L.seed, i);
            else pseed = x.seed;
        }
        pending |= 1ull << k;
    }
    if constexpr (XO == 3) {
        if (wobs) st(a.out.mask_bits, i, (uint8_t)mbits);
    } else {
        if (wobs && a.out.mask) st(reinterpret_cast<uint32_t*>(a.out.mask), i, mask_word(mbits));
        if (wobs && a.out.mask_bits) st(a.out.mask_bits, i, (uint8_t)mbits);
    }
    if constexpr (OBS != G2048_OBS_NONE) {
        const uint64_t wm = __ballot(wobs);
        if (G2048_DIAG && (a.diag & 16)) return;
        if (a.out.obs && wm) write_obs_wave<OBS>(a.out.obs, w0, b, wm, lane, a.obs_scale);
    }
}

// LDS reuse after the last sweep: the block's reset list (counter, lane indices, previous seeds)
constexpr int kStepLdsBytes = kTabBytes;    // the row tables, then (after the last sweep) the reset list
constexpr int kStepLdsVec = kStepLdsBytes / 16;
constexpr int kResetCap = (kStepLdsBytes - 16) / 12;
static_assert(16 + kResetCap * 4 + kResetCap * 8 <= kStepLdsBytes, "reset list fits the LDS area");
static_assert(kTabVec % kBlock == 0, "table fill: whole chunks per thread");

// Persistent over the board array, one board per lane per sweep (wave g of W takes the chunks of 64 boards
// g, g + W, g + 2W, ...), software-pipelined with three register buffers A / B / C (no back-edge copy, which
// would force a wait on in-flight loads): the loads of the next two sweeps are in flight while one computes.
// Prefetch loads are issued unconditionally from a clamped lane index (lanes past n re-read lane n-1 and compute
// nothing): a load skipped on some path would make the compiler's vmcnt accounting assume that path and wait for
// every load in flight, including those of the sweeps being prefetched.
// LDS: stage the two row tables in LDS, else read them through L1/L2 (small batches).  The first two sweeps'
// loads are issued before the table fill; each workgroup fills its 10 chunks starting at a different one
// (blockIdx % 10), so the CUs sharing an L2 do not read the same lines at once.  Sweeps per wave <= 64
// (launcher): the `pending` reset bitmask.
// Auto-resets are deferred to the end.  With the LDS tables dead after the last sweep, the block compacts its
// pending resets into an LDS list and runs them densely (thread t takes entries t, t + 1024, ...): ~30 resets
// of a 1M-board step per CU cost one pass of one wave instead of one divergent pass in most of the 16 waves.
// (A dynamic schedule -- chunks claimed with device-scope atomics -- measured slower on MI355X: under this
// kernel's streaming load an atomic's return takes microseconds, and same-address atomics serialize.)
// (Round 4: an XCD-aware static partition -- contiguous chunk ranges, larger for the early-dispatched XCD groups --
// measured no gain against this strided one, profiles/round4/r4c10/ab_xcd.log.)
template <int OBS, int RNG, bool LDS, int XO, int U, int RK>
__global__ void __launch_bounds__(kBlock) step_kernel(StepArgs a) {
    static_assert(U == 1, "one board per lane per sweep");
    __shared__ uint4 tab_lds[LDS ? kStepLdsVec : 1];
    const int lane = threadIdx.x & 63;
    const uint32_t w_first = (blockIdx.x * kBlock + threadIdx.x) & ~63u;
    const uint32_t wstride = gridDim.x * kBlock;
    const uint32_t wend = a.n;
    const uint32_t last = a.n - 1u;           // n >= 1 (the launcher never launches n == 0)
    const auto lane_at = [&](uint32_t w) { return w + lane < last ? w + lane : last; };
    G2048_TS(0);
    LaneIn A, B, C;
    uint32_t w0 = w_first, w1 = w_first + wstride;
    load_lane<RNG>(a, lane_at(w0), A);
    load_lane<RNG>(a, lane_at(w1), B);
    const uint8_t* tab = a.tab;
    if constexpr (LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(a.tab);
        if (!(G2048_DIAG && (a.diag & 1))) {
            constexpr uint32_t kChunks = kTabVec / kBlock;
            const uint32_t rot = blockIdx.x % kChunks;
#pragma unroll
            for (uint32_t j = 0; j < kChunks; j++) {
                uint32_t c = j + rot;
                c -= c >= kChunks ? kChunks : 0u;
                const uint32_t k = c * kBlock + threadIdx.x;
                // chunks 8, 9 = the 4-bit table: merge codes (RK 0) or max-merge fields (RK 1, kMxOff)
                tab_lds[k] = src[k + (RK == 1 && c >= 8u ? (uint32_t)((kMxOff - 2 * kLines) / 16) : 0u)];
            }
        }
        __syncthreads();
        tab = reinterpret_cast<const uint8_t*>(tab_lds);
    }
    G2048_TS(1);
    const LineFn lut{reinterpret_cast<const uint16_t*>(tab)};
    const CodeFn code{tab + (LDS || RK == 0 ? 2 * kLines : kMxOff)};
    uint64_t pending = 0, pseed = 0;
    uint32_t k = 0;
    while (w0 < wend) {                        // wave-uniform
        const uint32_t w2 = w1 + wstride;
        load_lane<RNG>(a, lane_at(w2), C);
        sweep<OBS, RNG, XO, RK>(a, w0, lane, A, lut, code, pending, pseed, k);
        if (w1 >= wend) break;
        const uint32_t w3 = w2 + wstride;
        load_lane<RNG>(a, lane_at(w3), A);
        sweep<OBS, RNG, XO, RK>(a, w1, lane, B, lut, code, pending, pseed, k + 1);
        if (w2 >= wend) break;
        const uint32_t w4 = w3 + wstride;
        load_lane<RNG>(a, lane_at(w4), B);
        sweep<OBS, RNG, XO, RK>(a, w2, lane, C, lut, code, pending, pseed, k + 2);
        w0 = w3;
        w1 = w4;
        k += 3;
    }
    if (G2048_DIAG && (a.diag & 2)) pending = 0;
    if constexpr (LDS) {
        uint32_t* cnt = reinterpret_cast<uint32_t*>(tab_lds);
        uint32_t* ridx = cnt + 4;
        uint64_t* rseed = reinterpret_cast<uint64_t*>(ridx + kResetCap + (kResetCap & 1));
        __syncthreads();                       // every wave is past its last table read
        G2048_TS(2);
        if (threadIdx.x == 0) *cnt = 0u;
        __syncthreads();
        bool first = true;
        while (__ballot(pending != 0ull)) {    // wave-uniform; one round per pending board of the busiest lane
            const bool has = pending != 0ull;
            const uint32_t kk = has ? (uint32_t)__builtin_ctzll(pending) : 0u;
            const uint32_t i = w_first + kk * wstride + lane;
            const uint64_t sd = first ? pseed : (has ? ld(a.L.seed, i) : 0ull);
            const uint64_t bal = __ballot(has);
            const int leader = __builtin_ctzll(bal);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(cnt, (uint32_t)__popcll(bal));
            base = (uint32_t)__shfl((int)base, leader, 64);
            const uint32_t slot =
                base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            if (has) {
                if (slot < (uint32_t)kResetCap) {
                    ridx[slot] = i;
                    rseed[slot] = sd;
                } else {
                    reset_lane<OBS, RNG>(a, i, sd);   // list full (mass reset): the lane does its own
                }
                pending &= pending - 1ull;
            }
            first = false;
        }
        __syncthreads();
        G2048_TS(3);
        const uint32_t R = *cnt < (uint32_t)kResetCap ? *cnt : (uint32_t)kResetCap;
        for (uint32_t r = threadIdx.x; r < R; r += kBlock) reset_lane<OBS, RNG>(a, ridx[r], rseed[r]);
    } else {
        bool first = true;
        while (pending) {   // deferred auto-resets of this lane, one pass per pending board
            const uint32_t kk = (uint32_t)__builtin_ctzll(pending);
            pending &= pending - 1ull;
            const uint32_t i = w_first + kk * wstride + lane;
            reset_lane<OBS, RNG>(a, i, first ? pseed : ld(a.L.seed, i));
            first = false;
        }
    }
#if G2048_DIAG
    __syncthreads();
    G2048_TS(4);
#endif
}

// ------------------------------------------------------------------------------------- other kernels
struct ResetArgs {
    g2048_lanes L;
    const uint64_t* seeds;
    const uint8_t* reset_mask;
    int8_t* mask_out;
    float* obs_out;
    float obs_scale;
    uint64_t key;
    uint32_t n;
};

template <int OBS, int RNG>
__global__ void __launch_bounds__(256) reset_kernel(ResetArgs a) {
    const int lane = threadIdx.x & 63;
    const uint32_t w_first = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u;
    const uint32_t wstride = gridDim.x * blockDim.x;
    for (uint32_t w0 = w_first; w0 < a.n; w0 += wstride) {
        const uint32_t i = w0 + lane;
        bool w = false;
        uint64_t b = 0;
        if (i < a.n && (!a.reset_mask || ld(a.reset_mask, i))) {
            const uint64_t seed = a.seeds ? ld(a.seeds, i) : ld(a.L.seed, i);
            Pcg64 g;
            g.has_uint32 = 0u;
            b = fresh_board<RNG>(seed, a.key, g);
            st(a.L.seed, i, seed);
            st(a.L.board, i, b);
            st(a.L.state, i, fresh_state(g));   // step 0, max_tile_seen 4 (src/env.py:182-183), active
            if constexpr (RNG == G2048_RNG_PCG64) store_pcg(a.L, i, g, true);
            w = true;
            if (a.mask_out) st(reinterpret_cast<uint32_t*>(a.mask_out), i, mask_word(action_mask(b)));
        }
        if constexpr (OBS != G2048_OBS_NONE) {
            const uint64_t wm = __ballot(w);
            if (a.obs_out && wm) write_obs_wave<OBS>(a.obs_out, w0, b, wm, lane, a.obs_scale);
        }
    }
}

template <int OBS>
__global__ void __launch_bounds__(256) obs_kernel(const uint64_t* __restrict__ boards, float* obs, int8_t* mask,
                                                  float scale, uint32_t n) {
    const int lane = threadIdx.x & 63;
    const uint32_t w_first = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u;
    const uint32_t wstride = gridDim.x * blockDim.x;
    for (uint32_t w0 = w_first; w0 < n; w0 += wstride) {
        const uint32_t i = w0 + lane;
        const bool v = i < n;
        const uint64_t b = v ? ld(boards, i) : 0ull;
        if (v && mask) st(reinterpret_cast<uint32_t*>(mask), i, mask_word(action_mask(b)));
        if constexpr (OBS != G2048_OBS_NONE) {
            const uint64_t wm = __ballot(v);
            if (obs) write_obs_wave<OBS>(obs, w0, b, wm, lane, scale);
        }
    }
}

__global__ void __launch_bounds__(256) move_kernel(const uint64_t* __restrict__ boards, const uint8_t* __restrict__ actions,
                                                   const uint8_t* __restrict__ tab, uint64_t* out, uint32_t* merged,
                                                   uint8_t* flags, uint32_t n) {
    const LineFn lut{reinterpret_cast<const uint16_t*>(tab)};
    const CodeFn code{tab + 2 * kLines};
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t b = ld(boards, i);
        const uint32_t act = ld(actions, i);
        if (act > 3u) {
            st(out, i, b);
            if (merged) st(merged, i, 0u);
            if (flags) st(flags, i, (uint8_t)G2048_F_BADACTION);
            continue;
        }
        MoveSummary s;
        const uint64_t m = board_move_coded<true>(b, act, lut, code, s);
        st(out, i, m);
        if (merged) st(merged, i, s.list);
        if (flags) st(flags, i, (uint8_t)((m != b ? G2048_F_CHANGED : 0u) | (s.overflow ? G2048_F_OVERFLOW : 0u)));
    }
}

__global__ void __launch_bounds__(256) seed_kernel(const uint64_t* __restrict__ seeds, uint64_t* rs, uint64_t* inc,
                                                   uint64_t* buf, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const Pcg64 g = pcg_seed(ld(seeds, i));
        st(reinterpret_cast<ulonglong2*>(rs), i, make_ulonglong2(g.s_lo, g.s_hi));
        st(reinterpret_cast<ulonglong2*>(inc), i, make_ulonglong2(g.i_lo, g.i_hi));
        st(buf, i, (uint64_t)0);
    }
}

struct SampleArgs {
    const float* logits;
    const int8_t* mask;
    const uint32_t* lane_state;
    uint64_t *rs, *inc, *buf;
    uint64_t key;
    const uint64_t* lane_seed;
    float* probs_out;
    uint8_t* actions;
    uint32_t n;
    int greedy;
};

// logits_to_probs (src/MLP.py:139-156) + select_action (src/reinforce_agent.py:178-190)
template <int RNG>
__global__ void __launch_bounds__(256) sample_kernel(SampleArgs a) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
        const uint32_t ls = a.lane_state ? ld(a.lane_state, i) : G2048_LS_ACTIVE;
        if (!(ls & G2048_LS_ACTIVE)) continue;
        const float4 lg4 = ld(reinterpret_cast<const float4*>(a.logits), i);
        const float lg[4] = {lg4.x, lg4.y, lg4.z, lg4.w};
        const uint32_t mw = a.mask ? ld(reinterpret_cast<const uint32_t*>(a.mask), i) : 0x01010101u;
        double u = 0.0;
        if (!a.greedy) {
            if constexpr (RNG == G2048_RNG_PCG64) {
                Pcg64 g;
                const ulonglong2 sv = ld(reinterpret_cast<const ulonglong2*>(a.rs), i);
                const ulonglong2 ic = ld(reinterpret_cast<const ulonglong2*>(a.inc), i);
                const uint64_t bf = ld(a.buf, i);
                g.s_lo = sv.x; g.s_hi = sv.y; g.i_lo = ic.x; g.i_hi = ic.y;
                g.has_uint32 = (uint32_t)(bf >> 32); g.uinteger = (uint32_t)bf;
                u = pcg_random(g);
                st(reinterpret_cast<ulonglong2*>(a.rs), i, make_ulonglong2(g.s_lo, g.s_hi));
            } else {
                const U4 r = philox_ctr(a.key, a.lane_seed ? ld(a.lane_seed, i) : (uint64_t)i,
                                        ls & G2048_LS_STEP_MASK, 3u);
                const uint64_t x = ((uint64_t)r.x << 32) | r.y;
                u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
            }
        }
        float p[4];
        const uint32_t act = softmax_select(lg, mw, a.mask != nullptr, a.greedy != 0, u, p);
        if (a.probs_out) st(reinterpret_cast<float4*>(a.probs_out), i, make_float4(p[0], p[1], p[2], p[3]));
        st(a.actions, i, (uint8_t)act);
    }
}

// compute_returns (src/reinforce_agent.py:255-273), time-major [T, n], fp64 accumulation
__global__ void __launch_bounds__(256) returns_kernel(const double* __restrict__ r, const int32_t* __restrict__ len,
                                                      double gamma, float* __restrict__ out, int64_t T, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t Li = len[i];
        Li = Li > T ? T : Li;
        double G = 0.0;
        for (int64_t t = Li - 1; t >= 0; t--) {
            G = r[t * n + i] + gamma * G;
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

// ------------------------------------------------------------------------------------- host helpers
int current_device(int& dev) {
    G2048_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDev) return fail(G2048_EINVAL, "device ordinal out of range");
    return G2048_OK;
}

int tab_for_current(const uint8_t*& tab, int& cus) {
    int dev = 0;
    int rc = current_device(dev);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_tab[dev]) return fail(G2048_ENOINIT, "g2048_init() was not called for device " + std::to_string(dev));
    tab = g_tab[dev];
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
    r.terms = reward_terms(r);
    return r;
}

int check_cfg(const g2048_env_cfg* c) {
    if (!c) return fail(G2048_EINVAL, "cfg is NULL");
    if (c->max_steps > G2048_MAX_STEPS_LIMIT)
        return fail(G2048_EINVAL, "max_steps must be <= " + std::to_string(G2048_MAX_STEPS_LIMIT) +
                                      " (the lane step count is 20 bits) or None");
    if (c->obs_mode < G2048_OBS_NONE || c->obs_mode > G2048_OBS_ONEHOT)
        return fail(G2048_EINVAL, "Unsupported obs_mode: " + std::to_string(c->obs_mode));
    if (c->reward_mode < 0 || c->reward_mode > 1)
        return fail(G2048_EINVAL, "Unsupported reward mode: " + std::to_string(c->reward_mode));
    if (c->bonus_mode < 0 || c->bonus_mode > 2)
        return fail(G2048_EINVAL, "Unsupported bonus mode: " + std::to_string(c->bonus_mode));
    return G2048_OK;
}

int check_lanes(const g2048_lanes* L, int rng_mode) {
    if (!L || !L->board || !L->state || !L->seed) return fail(G2048_EINVAL, "lanes: a required buffer is NULL");
    if (rng_mode == G2048_RNG_PCG64 && (!L->rng_state || !L->rng_inc || !L->rng_uint))
        return fail(G2048_EINVAL, "lanes: PCG64 mode needs rng_state / rng_inc / rng_uint");
    if (rng_mode != G2048_RNG_PCG64 && rng_mode != G2048_RNG_PHILOX)
        return fail(G2048_EINVAL, "Unsupported rng_mode: " + std::to_string(rng_mode));
    return G2048_OK;
}

// offset every per-lane buffer by `off` lanes (for launches split at kMaxLanesPerLaunch)
g2048_lanes shift_lanes(const g2048_lanes& L, int64_t off) {
    g2048_lanes r = L;
    r.board += off;
    r.state += off;
    r.seed += off;
    if (r.rng_state) r.rng_state += 2 * off;
    if (r.rng_inc) r.rng_inc += 2 * off;
    if (r.rng_uint) r.rng_uint += off;
    return r;
}

// boards per lane per sweep.  U = 2 measured equal or slower on MI355X at 1M boards (and 4 spills past the
// 128-VGPR budget of 4 waves/SIMD), so one board per lane per sweep.
constexpr int kStepU = 1;

template <int OBS, int RNG, bool LDS, int U>
void launch_step3(const StepArgs& a, int grid, int xo, int rk, hipStream_t s) {
    if (rk == 1 && xo == 3) hipLaunchKernelGGL((step_kernel<OBS, RNG, LDS, 3, U, 1>), dim3(grid), dim3(kBlock), 0, s, a);
    else if (rk == 1 && xo == 0) hipLaunchKernelGGL((step_kernel<OBS, RNG, LDS, 0, U, 1>), dim3(grid), dim3(kBlock), 0, s, a);
    else if (xo == 3) hipLaunchKernelGGL((step_kernel<OBS, RNG, LDS, 3, U, 0>), dim3(grid), dim3(kBlock), 0, s, a);
    else if (xo == 2) hipLaunchKernelGGL((step_kernel<OBS, RNG, LDS, 2, U, 0>), dim3(grid), dim3(kBlock), 0, s, a);
    else if (xo == 1) hipLaunchKernelGGL((step_kernel<OBS, RNG, LDS, 1, U, 0>), dim3(grid), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((step_kernel<OBS, RNG, LDS, 0, U, 0>), dim3(grid), dim3(kBlock), 0, s, a);
}

template <int OBS, int RNG, int kU>
void launch_step_u(const StepArgs& a, int cus, hipStream_t s) {
    const bool lds = a.n >= (uint32_t)kLutSmallN;
    // persistent grid: <= one workgroup per CU (LDS), but enough workgroups that sweeps * kU <= 64 (the per-lane
    // pending-reset bitmask)
    const int64_t per_block_sweep = (int64_t)kBlock * kU;
    const int64_t min_blocks = ((int64_t)a.n + per_block_sweep * (64 / kU) - 1) / (per_block_sweep * (64 / kU));
    int grid = grid_for((a.n + kU - 1) / kU, kBlock, lds ? cus : cus * 2);
    if (grid < min_blocks) grid = (int)min_blocks;
    if (G2048_DIAG && (a.diag & 8)) grid = grid_for(a.n, kBlock, 1 << 30);
    int xo = a.out.merged ? 2 : (a.out.prev_board || a.out.reward64 || a.out.score_add) ? 1 : 0;
    if (xo == 0 && a.out.mask_bits && !a.out.mask) xo = 3;
    // the lean summary path: log2 rewards, no score / merged-list outputs
    const int rk = a.rc.reward_mode == 1 && (xo == 0 || xo == 3) ? 1 : 0;
    if (lds) launch_step3<OBS, RNG, true, kU>(a, grid, xo, rk, s);
    else launch_step3<OBS, RNG, false, kU>(a, grid, xo, rk, s);
}

template <int OBS, int RNG>
void launch_step(const StepArgs& a, int cus, hipStream_t s) {
    launch_step_u<OBS, RNG, kStepU>(a, cus, s);
}

template <int RNG>
void launch_step_obs(const StepArgs& a, int obs, int cus, hipStream_t s) {
    switch (obs) {
        case G2048_OBS_RAW: launch_step<G2048_OBS_RAW, RNG>(a, cus, s); break;
        case G2048_OBS_LOG2: launch_step<G2048_OBS_LOG2, RNG>(a, cus, s); break;
        case G2048_OBS_ONEHOT: launch_step<G2048_OBS_ONEHOT, RNG>(a, cus, s); break;
        default: launch_step<G2048_OBS_NONE, RNG>(a, cus, s); break;
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

// shared with the other translation unit of the library (g2048_policy.hip): the error string, the current
// device's row tables, env-config validation / reward config
namespace g2048_internal {
int set_error(int code, const char* msg) { return fail(code, msg); }
int device_tables(const uint8_t*& tab, int& cus) { return tab_for_current(tab, cus); }
int check_env_cfg(const g2048_env_cfg* c) { return check_cfg(c); }
RewardCfg reward_cfg_of(const g2048_env_cfg& c) { return reward_cfg(c); }
}  // namespace g2048_internal

extern "C" {

int g2048_abi_version(void) { return G2048_ABI_VERSION; }

#if G2048_DIAG
// diag build only: copy the phase timestamps of the last step launch (blocks x 5 u64) to host memory
int g2048_diag_times(uint64_t* out, int blocks) {
    if (blocks > kDiagBlocks) blocks = kDiagBlocks;
    G2048_HIP(hipDeviceSynchronize());
    G2048_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_ts), sizeof(uint64_t) * kDiagSlots * blocks, 0,
                                  hipMemcpyDeviceToHost));
    return blocks;
}
#endif

const char* g2048_last_error(void) { return g_err.c_str(); }

int g2048_init(int device) {
    if (device < 0 || device >= kMaxDev) return fail(G2048_EINVAL, "device ordinal out of range");
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_tab[device]) return G2048_OK;
    int prev = 0;
    G2048_HIP(hipGetDevice(&prev));
    G2048_HIP(hipSetDevice(device));
    static uint8_t host[kDevTabBytes];
    uint16_t* line = reinterpret_cast<uint16_t*>(host);
    uint8_t* code = host + 2 * kLines;
    uint8_t* mx = host + kMxOff;
    for (uint32_t r = 0; r < (uint32_t)kLines; r++) {
        line[r] = (uint16_t)line_move_left(r);
        const uint32_t c = line_merge_code(r), f = line_max_merge_field(r);
        if (r & 1u) {
            code[r >> 1] = (uint8_t)(code[r >> 1] | (c << 4));
            mx[r >> 1] = (uint8_t)(mx[r >> 1] | (f << 4));
        } else {
            code[r >> 1] = (uint8_t)c;
            mx[r >> 1] = (uint8_t)f;
        }
    }
    uint8_t* d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(host));
    if (e == hipSuccess) e = hipMemcpy(d, host, sizeof(host), hipMemcpyHostToDevice);
    const hipError_t e2 = hipSetDevice(prev);
    if (e != hipSuccess) {
        if (d) (void)hipFree(d);
        return fail(G2048_EHIP, std::string("g2048_init: ") + hipGetErrorString(e));
    }
    if (e2 != hipSuccess) return fail(G2048_EHIP, std::string("g2048_init: ") + hipGetErrorString(e2));
    g_tab[device] = d;
    g_cus[device] = device_cus(device);
    return G2048_OK;
}

int g2048_seed_pcg64(const uint64_t* seeds, uint64_t* rng_state, uint64_t* rng_inc, uint64_t* rng_buf, int64_t n,
                     void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (!seeds || !rng_state || !rng_inc || !rng_buf) return fail(G2048_EINVAL, "NULL buffer");
    for (int64_t off = 0; off < n; off += kMaxLanesPerLaunch) {
        const uint32_t m = (uint32_t)(n - off < kMaxLanesPerLaunch ? n - off : kMaxLanesPerLaunch);
        hipLaunchKernelGGL(seed_kernel, dim3(grid_for(m, 256, 2048)), dim3(256), 0, (hipStream_t)stream, seeds + off,
                           rng_state + 2 * off, rng_inc + 2 * off, rng_buf + off, m);
    }
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_reset(const g2048_lanes* lanes, const uint64_t* seeds, const uint8_t* reset_mask, const g2048_env_cfg* cfg,
                int rng_mode, uint64_t philox_key, int8_t* mask_out, float* obs_out, int64_t n, void* stream) {
    int rc = check_cfg(cfg);
    if (!rc) rc = check_lanes(lanes, rng_mode);
    if (rc) return rc;
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    const uint8_t* tab = nullptr;
    int cus = 256;
    if ((rc = tab_for_current(tab, cus))) return rc;
    const int obs = obs_out ? cfg->obs_mode : G2048_OBS_NONE;
    const int width = cfg->obs_mode == G2048_OBS_ONEHOT ? 272 : 16;
    for (int64_t off = 0; off < n; off += kMaxLanesPerLaunch) {
        const uint32_t m = (uint32_t)(n - off < kMaxLanesPerLaunch ? n - off : kMaxLanesPerLaunch);
        ResetArgs a{shift_lanes(*lanes, off), seeds ? seeds + off : nullptr, reset_mask ? reset_mask + off : nullptr,
                    mask_out ? mask_out + 4 * off : nullptr, obs_out ? obs_out + width * off : nullptr,
                    cfg->obs_log2_scale, philox_key, m};
        if (rng_mode == G2048_RNG_PCG64) launch_reset<G2048_RNG_PCG64>(a, obs, cus, (hipStream_t)stream);
        else launch_reset<G2048_RNG_PHILOX>(a, obs, cus, (hipStream_t)stream);
    }
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
    if (rng_mode == G2048_RNG_PHILOX && cfg->max_steps < 0)
        return fail(G2048_EINVAL, "Philox mode needs a finite max_steps: its draw counter is the 20-bit lane step count");
    const uint8_t* tab = nullptr;
    int cus = 256;
    if ((rc = tab_for_current(tab, cus))) return rc;
    const int obs = out->obs ? cfg->obs_mode : G2048_OBS_NONE;
    const int width = cfg->obs_mode == G2048_OBS_ONEHOT ? 272 : 16;
    for (int64_t off = 0; off < n; off += kMaxLanesPerLaunch) {
        const uint32_t m = (uint32_t)(n - off < kMaxLanesPerLaunch ? n - off : kMaxLanesPerLaunch);
        StepArgs a;
        a.L = shift_lanes(*lanes, off);
        a.actions = actions + off;
        a.out = *out;
        a.out.reward += off;
        a.out.flags += off;
        if (a.out.mask) a.out.mask += 4 * off;
        if (a.out.obs) a.out.obs += width * off;
        if (a.out.merged) a.out.merged += off;
        if (a.out.prev_board) a.out.prev_board += off;
        if (a.out.reward64) a.out.reward64 += off;
        if (a.out.score_add) a.out.score_add += off;
        if (a.out.mask_bits) a.out.mask_bits += off;
        a.rc = reward_cfg(*cfg);
        a.obs_scale = cfg->obs_log2_scale;
        a.auto_reset = auto_reset;
        a.max_steps = cfg->max_steps;
        a.stride = reset_stride;
        a.key = philox_key;
        a.tab = tab;
        a.n = m;
        a.diag = 0;
        if (G2048_DIAG) {
            static const int diag_flags = std::getenv("G2048_DIAG_FLAGS") ? std::atoi(std::getenv("G2048_DIAG_FLAGS")) : 0;
            a.diag = diag_flags;
        }
        if (rng_mode == G2048_RNG_PCG64) launch_step_obs<G2048_RNG_PCG64>(a, obs, cus, (hipStream_t)stream);
        else launch_step_obs<G2048_RNG_PHILOX>(a, obs, cus, (hipStream_t)stream);
    }
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_obs(const uint64_t* boards, int obs_mode, float obs_log2_scale, float* obs, int8_t* mask, int64_t n,
              void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (!boards) return fail(G2048_EINVAL, "boards is NULL");
    if (obs_mode < G2048_OBS_NONE || obs_mode > G2048_OBS_ONEHOT)
        return fail(G2048_EINVAL, "Unsupported obs_mode: " + std::to_string(obs_mode));
    const int width = obs_mode == G2048_OBS_ONEHOT ? 272 : 16;
    hipStream_t s = (hipStream_t)stream;
    for (int64_t off = 0; off < n; off += kMaxLanesPerLaunch) {
        const uint32_t m = (uint32_t)(n - off < kMaxLanesPerLaunch ? n - off : kMaxLanesPerLaunch);
        const uint64_t* b = boards + off;
        float* o = obs ? obs + width * off : nullptr;
        int8_t* mk = mask ? mask + 4 * off : nullptr;
        const int grid = grid_for(m, 256, 2048);
        switch (o ? obs_mode : G2048_OBS_NONE) {
            case G2048_OBS_RAW: hipLaunchKernelGGL(obs_kernel<G2048_OBS_RAW>, dim3(grid), dim3(256), 0, s, b, o, mk, obs_log2_scale, m); break;
            case G2048_OBS_LOG2: hipLaunchKernelGGL(obs_kernel<G2048_OBS_LOG2>, dim3(grid), dim3(256), 0, s, b, o, mk, obs_log2_scale, m); break;
            case G2048_OBS_ONEHOT: hipLaunchKernelGGL(obs_kernel<G2048_OBS_ONEHOT>, dim3(grid), dim3(256), 0, s, b, o, mk, obs_log2_scale, m); break;
            default: hipLaunchKernelGGL(obs_kernel<G2048_OBS_NONE>, dim3(grid), dim3(256), 0, s, b, o, mk, obs_log2_scale, m); break;
        }
    }
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_move(const uint64_t* boards, const uint8_t* actions, uint64_t* out_board, uint32_t* merged, uint8_t* flags,
               int64_t n, void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (!boards || !actions || !out_board) return fail(G2048_EINVAL, "NULL buffer");
    const uint8_t* tab = nullptr;
    int cus = 256;
    int rc = tab_for_current(tab, cus);
    if (rc) return rc;
    for (int64_t off = 0; off < n; off += kMaxLanesPerLaunch) {
        const uint32_t m = (uint32_t)(n - off < kMaxLanesPerLaunch ? n - off : kMaxLanesPerLaunch);
        hipLaunchKernelGGL(move_kernel, dim3(grid_for(m, 256, 2048)), dim3(256), 0, (hipStream_t)stream, boards + off,
                           actions + off, tab, out_board + off, merged ? merged + off : nullptr,
                           flags ? flags + off : nullptr, m);
    }
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_sample(const float* logits, const int8_t* mask, const uint32_t* lane_state, int greedy, int rng_mode,
                 uint64_t* rng_state, uint64_t* rng_inc, uint64_t* rng_buf, uint64_t philox_key,
                 const uint64_t* lane_seed, float* probs_out, uint8_t* actions, int64_t n, void* stream) {
    if (n < 0) return fail(G2048_EINVAL, "n < 0");
    if (!logits || !actions) return fail(G2048_EINVAL, "logits / actions are required");
    if (!greedy && rng_mode == G2048_RNG_PCG64 && (!rng_state || !rng_inc || !rng_buf))
        return fail(G2048_EINVAL, "PCG64 sampling needs rng_state / rng_inc / rng_buf");
    if (rng_mode != G2048_RNG_PCG64 && rng_mode != G2048_RNG_PHILOX)
        return fail(G2048_EINVAL, "Unsupported rng_mode: " + std::to_string(rng_mode));
    for (int64_t off = 0; off < n; off += kMaxLanesPerLaunch) {
        const uint32_t m = (uint32_t)(n - off < kMaxLanesPerLaunch ? n - off : kMaxLanesPerLaunch);
        SampleArgs a{logits + 4 * off, mask ? mask + 4 * off : nullptr, lane_state ? lane_state + off : nullptr,
                     rng_state ? rng_state + 2 * off : nullptr, rng_inc ? rng_inc + 2 * off : nullptr,
                     rng_buf ? rng_buf + off : nullptr, philox_key, lane_seed ? lane_seed + off : nullptr,
                     probs_out ? probs_out + 4 * off : nullptr, actions + off, m, greedy};
        const int grid = grid_for(m, 256, 2048);
        if (rng_mode == G2048_RNG_PCG64) hipLaunchKernelGGL(sample_kernel<G2048_RNG_PCG64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
        else hipLaunchKernelGGL(sample_kernel<G2048_RNG_PHILOX>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    }
    G2048_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_returns(const double* rewards, const int32_t* lengths, double gamma, float* returns, int64_t T, int64_t n,
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
