/*
 * g2048.h -- C ABI of libg2048.so, the MI355X (gfx950) HIP implementation of the 2048 hot path of
 * pqpeqr/RL-2048-with-Reinforce-and-Actor-Critic.
 *
 * The reference is pure Python/NumPy and exposes no FFI; its boundary for this path is its Python API.  Each
 * entry point below replaces the reference interface cited next to it, batched over n boards ("lanes").
 * The Python host layer (rl-2048-with-reinforce-and-actor-critic_amd/) binds these with ctypes and mirrors
 * the reference's classes and error behaviour on top (INTEGRATION.md shows the binding).
 *
 * Conventions (all entry points):
 *   - Every pointer argument that names a buffer is a DEVICE pointer owned by the caller (torch tensors in
 *     practice).  The library never allocates caller buffers; it owns only its row lookup table.
 *   - Calls are asynchronous and ordered on `stream` (a hipStream_t; NULL = the default stream).  Nothing
 *     synchronises the host.  Calls on different streams are independent (reentrant).
 *   - Return value: G2048_OK or an error code; g2048_last_error() gives a thread-local message.  Bad
 *     arguments are rejected before any launch (the Python layer turns them into ValueError /
 *     AssertionError exactly where the reference raises).  Per-lane conditions (invalid action, tile
 *     overflow) never abort: they are reported in the per-lane flags.
 *   - Board encoding ("bitboard"): one uint64 per board, nibble (r*4+c) holds log2(tile) (0 = empty).
 *     A tile of 2**15 merging with another 2**15 (the reference's int64 board would hold 65536) saturates
 *     at 2**15 and raises G2048_F_OVERFLOW; rewards/score still use the true merged value.
 *   - Actions: 0 up, 1 right, 2 down, 3 left (src/game2048.py:9).
 */
#ifndef G2048_H
#define G2048_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define G2048_ABI_VERSION 16

/* status codes */
#define G2048_OK 0
#define G2048_EINVAL 1   /* bad argument (null required buffer, bad mode, n < 0) */
#define G2048_EHIP 2     /* HIP runtime error (message in g2048_last_error) */
#define G2048_ENOINIT 3  /* g2048_init() not called for the current device */

/* observation encodings: Game2048EnvConfig.obs_mode (src/env.py:23, :131-150) */
#define G2048_OBS_NONE (-1)
#define G2048_OBS_RAW 0
#define G2048_OBS_LOG2 1
#define G2048_OBS_ONEHOT 2     /* 17 channels per cell, index (r*4+c)*17 + log2(tile) */

/* spawn / policy random streams */
#define G2048_RNG_PCG64 0      /* numpy default_rng(seed) bit-exact (parity mode) */
#define G2048_RNG_PHILOX 1     /* Philox4x32-10, counter = (lane seed, step, tag): throughput mode */

/* per-lane step flags (uint8) */
#define G2048_F_CHANGED 0x01     /* Game2048.step is_changed */
#define G2048_F_TERMINATED 0x02  /* is_done -> Game2048Env.step terminated */
#define G2048_F_TRUNCATED 0x04   /* step_count >= max_steps and not terminated */
#define G2048_F_INVALID 0x08     /* Game2048Env.step info["invalid_action"] = not changed and not done */
#define G2048_F_OVERFLOW 0x10    /* a 2**15 + 2**15 merge saturated (see encoding note) */
#define G2048_F_RESET 0x20       /* lane finished and was auto-reset in this call */
#define G2048_F_INACTIVE 0x40    /* lane was already finished (no auto-reset): nothing happened */
#define G2048_F_BADACTION 0x80   /* action outside 0..3: lane untouched (reference raises) */

/* Per-lane state word (g2048_lanes.state, one uint32 per lane; read and written once per step):
 *   bits  0..19  Game2048Env._step_count (== Game2048.step_count); saturates at 2^20 - 1, so cfg->max_steps must
 *                be < 2^20 (checked; max_steps None only stops counting step_index past 1,048,575 steps)
 *   bits 20..24  log2(Game2048Env.max_tile_seen)
 *   bit  25      the lane is in an episode (G2048_LS_ACTIVE)
 *   bit  26      numpy PCG64's next_uint32 buffer is full (has_uint32; the value is g2048_lanes.rng_uint) */
#define G2048_LS_STEP_MASK 0x000FFFFFu
#define G2048_LS_MAXT_SHIFT 20
#define G2048_LS_MAXT_MASK 0x01F00000u
#define G2048_LS_ACTIVE 0x02000000u
#define G2048_LS_HAS_U32 0x04000000u
#define G2048_MAX_STEPS_LIMIT 0x000FFFFF

/* Game2048EnvConfig (src/env.py:19-40).  size is fixed at 4. */
typedef struct g2048_env_cfg {
    int32_t obs_mode;              /* G2048_OBS_* */
    int32_t reward_mode;           /* 0 "sum", 1 "log2" */
    int32_t bonus_mode;            /* 0 "off", 1 "raw", 2 "log2" */
    int32_t use_action_mask;       /* bool */
    float obs_log2_scale;
    int32_t _pad0;
    double base_reward_scale;
    double empty_tile_reward;
    double merge_reward;
    double bonus_scale;
    double step_reward;
    double endgame_penalty;
    double invalid_action_penalty;
    int64_t max_steps;             /* < 0 means None; otherwise <= G2048_MAX_STEPS_LIMIT */
} g2048_env_cfg;

/* Per-lane environment state, structure-of-arrays, each array of length n (rng_state / rng_inc of length 2n).
 * 49 B read + 33 B written per lane per step in PCG64 mode (board, state word, RNG), 20 / 12 B with Philox. */
typedef struct g2048_lanes {
    uint64_t* board;       /* Game2048.board as a bitboard */
    uint32_t* state;       /* the lane state word (G2048_LS_*) */
    uint64_t* seed;        /* seed of the lane's current episode (Game2048.reset(seed)); read every step only in
                              Philox mode (PCG64 mode reads it when an episode ends and auto-resets) */
    uint64_t* rng_state;   /* PCG64 128-bit state, (lo, hi) per lane            [PCG64 mode only] */
    uint64_t* rng_inc;     /* PCG64 128-bit increment, (lo, hi) per lane        [PCG64 mode only] */
    uint32_t* rng_uint;    /* PCG64 next_uint32 buffer value (its flag: G2048_LS_HAS_U32) [PCG64 mode only] */
} g2048_lanes;

/* Outputs of one step.  reward and flags are required; the others may be NULL. */
typedef struct g2048_step_out {
    float* reward;         /* [n] Game2048Env._compute_reward (computed in fp64, stored fp32) */
    uint8_t* flags;        /* [n] G2048_F_* */
    int8_t* mask;          /* [n*4] obs["action_mask"] of the resulting board (src/env.py:154-156) */
    float* obs;            /* [n*16] or [n*272] obs["board"] of the resulting board, cfg.obs_mode */
    uint32_t* merged;      /* [n] merged tiles of this step in the reference's list order, as nibbles
                              (log2(v) - 1), first merge in the lowest nibble, 0-terminated (<= 8) */
    uint64_t* prev_board;  /* [n] the board before the step (trajectory record) */
    double* reward64;      /* [n] the same reward in fp64 -- the Python float src/env.py:261 returns (may be NULL) */
    uint32_t* score_add;   /* [n] sum of this step's merged tiles: Game2048.score's increment (src/game2048.py:54);
                              the caller keeps the running score when it needs one (may be NULL) */
    uint8_t* mask_bits;    /* [n] the same action mask packed: bit a set = action a changes the board (may be NULL;
                              1 B per board-step instead of the 4 of `mask`) */
} g2048_step_out;

/* ---------------------------------------------------------------------------------------------------- */

int g2048_abi_version(void);
const char* g2048_last_error(void);

/* Build the 65,536-entry row table (move-left of every 4-nibble line) in the memory of `device`.
 * Idempotent and thread-safe.  Replaces the per-row Python loop of Game2048._row_move_left
 * (src/game2048.py:120-137). */
int g2048_init(int device);

/* Seed PCG64 streams exactly like np.random.default_rng(seed[i]) (numpy SeedSequence -> PCG64).
 * Replaces Game2048._set_seed (src/game2048.py:102-106) and default_rng(policy_seed)
 * (src/reinforce_agent.py:211).  rng_state / rng_inc: [2n] (lo, hi); rng_buf: [n]. */
int g2048_seed_pcg64(const uint64_t* seeds, uint64_t* rng_state, uint64_t* rng_inc, uint64_t* rng_buf,
                     int64_t n, void* stream);

/* Reset lanes: Game2048Env.reset(seed=...) (src/env.py:174-194) -> Game2048.reset (src/game2048.py:26-34).
 * seeds: [n] or NULL (NULL keeps lanes->seed); reset_mask: [n] (nonzero = reset this lane) or NULL (all).
 * mask_out [n*4] / obs_out (cfg->obs_mode) may be NULL. */
int g2048_reset(const g2048_lanes* lanes, const uint64_t* seeds, const uint8_t* reset_mask,
                const g2048_env_cfg* cfg, int rng_mode, uint64_t philox_key, int8_t* mask_out, float* obs_out,
                int64_t n, void* stream);

/* One environment step of every lane: Game2048Env.step(action) (src/env.py:264-302) with
 * Game2048.step (src/game2048.py:40-70) and the reward of _compute_reward (src/env.py:197-261).
 * actions: [n] uint8.  auto_reset != 0: a lane that terminates or truncates is reset in the same call with
 * seed += reset_stride (flag G2048_F_RESET; obs/mask then describe the new episode).  auto_reset == 0: the
 * lane is marked inactive and later calls leave it untouched (G2048_F_INACTIVE).  Outputs are the same for every
 * combination of `out` fields; a log2-reward config that asks for none of merged / prev_board / reward64 /
 * score_add runs a leaner kernel (no merge decode or score: the reward reads only sum and max of the merges). */
int g2048_step(const g2048_lanes* lanes, const uint8_t* actions, const g2048_env_cfg* cfg,
               const g2048_step_out* out, int rng_mode, uint64_t philox_key, int auto_reset,
               uint64_t reset_stride, int64_t n, void* stream);

/* Observation + action mask of a board array (src/env.py:131-159 with src/MLP.py:22-43 flattening and
 * Game2048.get_action_mask src/game2048.py:95-99).  obs may be NULL (mask only), mask may be NULL. */
int g2048_obs(const uint64_t* boards, int obs_mode, float obs_log2_scale, float* obs, int8_t* mask, int64_t n,
              void* stream);

/* Pre-spawn move only: Game2048._move (src/game2048.py:158-165) for KATs.  out_board [n]; merged [n] as
 * in g2048_step_out; flags [n] gets G2048_F_CHANGED / G2048_F_OVERFLOW / G2048_F_BADACTION. */
int g2048_move(const uint64_t* boards, const uint8_t* actions, uint64_t* out_board, uint32_t* merged,
               uint8_t* flags, int64_t n, void* stream);

/* Policy head: logits_to_probs (src/MLP.py:139-156) + action choice of ReinforceAgent.select_action
 * (src/reinforce_agent.py:178-190).  logits [n*4] fp32, mask [n*4] int8 (NULL = no mask).
 * greedy != 0: argmax(probs * mask).  Otherwise rng_mode PCG64: Generator.choice(4, p=probs) on the lane's
 * stream (rng_* as in g2048_seed_pcg64); PHILOX: inverse-CDF on a Philox draw keyed (philox_key, lane_seed[i],
 * the lane's step count).  lane_state: the env lanes' state words [n] (g2048_lanes.state: the active bit and, for
 * Philox, the step count; NULL = all active, count 0); inactive lanes are left untouched.  probs_out [n*4] may
 * be NULL. */
int g2048_sample(const float* logits, const int8_t* mask, const uint32_t* lane_state, int greedy, int rng_mode,
                 uint64_t* rng_state, uint64_t* rng_inc, uint64_t* rng_buf, uint64_t philox_key,
                 const uint64_t* lane_seed, float* probs_out, uint8_t* actions, int64_t n, void* stream);

/* Discounted returns per episode (ReinforceAgent.compute_returns src/reinforce_agent.py:255-273):
 * rewards [T, n] fp64 (the Python floats Game2048Env.step returns) and returns [T, n] fp32, both time-major (lane
 * i's episode occupies rows 0..lengths[i]-1); the scan is accumulated in fp64 like the reference's Python float
 * and stored as fp32. */
int g2048_returns(const double* rewards, const int32_t* lengths, double gamma, float* returns, int64_t T,
                  int64_t n, void* stream);

/* The 8 dihedral symmetries of Game2048Env.get_symmetries (src/env.py:317-398) on bitboards:
 * boards [n] -> out_boards [8n] (symmetry-major: out[k*n + i]); actions [n] -> out_actions [8n] (NULL ok);
 * masks are recomputed from the transformed boards by g2048_obs. */
int g2048_symmetries(const uint64_t* boards, const uint8_t* actions, uint64_t* out_boards, uint8_t* out_actions,
                     int64_t n, void* stream);

/* ---- fused policy (rollout / evaluation forward) ----------------------------------------------------------
 * One kernel for forward_logits (src/MLP.py:159-196) + logits_to_probs (:139-156) + the action choice of
 * select_action (src/reinforce_agent.py:178-190), for the reference's MLP with two hidden layers of 1..256 units
 * (MLPConfig.hidden_sizes, src/MLP.py:45-94), obs width 16 ("log2" / "raw" obs built from the bitboards in the
 * kernel), ReLU or Sigmoid, 4 actions.  fp32 throughout (MFMA f32: a k-ordered fmaf chain), so it agrees with the
 * GEMM path up to fp32 summation order; the choice is the g2048_sample code on the resulting probabilities. */
#define G2048_ACT_RELU 0
#define G2048_ACT_SIGMOID 1

/* floats of the packed net for hidden sizes (h1, h2); -1 if unsupported */
int64_t g2048_policy_packed_size(int h1, int h2);

/* Pack W1 [in_dim x h1], b1 [h1], W2 [h1 x h2], b2 [h2], W3 [h2 x 4], b3 [4] (row-major, x @ W layout of
 * src/MLP.py) into `packed` (g2048_policy_packed_size floats, device memory).  Re-pack after every update. */
int g2048_policy_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                      const float* b3, int in_dim, int h1, int h2, float* packed, int64_t packed_len, void* stream);

/* boards / lane_state / rng / outputs are per lane; the call covers n entries: entry j is lane
 * lane_index[j] (int32, NULL = lane j), so a rollout can run the net on its still-active lanes only;
 * lane_state: the env lanes' state words (G2048_LS_ACTIVE; NULL = all active) -- inactive lanes are left
 * untouched;
 * use_mask: mask the logits with the boards' action masks (Game2048.get_action_mask, src/game2048.py:95-99);
 * greedy / rng_mode / rng_* / philox_key / lane_seed / probs_out / actions as in g2048_sample;
 * logits_out [n*4] may be NULL. */
int g2048_policy(const float* packed, int h1, int h2, int activation, const uint64_t* boards,
                 const uint32_t* lane_state, const int32_t* lane_index, int obs_mode, float obs_scale, int use_mask,
                 int greedy, int rng_mode, uint64_t* rng_state, const uint64_t* rng_inc, const uint64_t* rng_buf,
                 uint64_t philox_key, const uint64_t* lane_seed, float* probs_out, float* logits_out,
                 uint8_t* actions, int64_t n, void* stream);

/* ---- fused actor gradient (update_batch's actor branch) ---------------------------------------------------
 * For the same nets as g2048_policy: ReinforceAgent.update_batch's actor gradient (src/reinforce_agent.py:502-555:
 * _policy_gradient_step :328-354, _backpropagation :639-678, _activation_derivative :624-636) over n samples
 * (valid steps): forward from the boards, masked softmax (use_mask: the boards' action masks, as
 * logits_to_probs src/MLP.py:139-156), g = (onehot(action) - p) * coef[i] (coef = advantage * step weight),
 * the output and input deltas and the small weight gradients, all in one kernel.  Outputs:
 *   a1t, d2t [R x ld] fp32, R = max(H1p, H2p), stored in 16-column blocks: element (row, col) at
 *                         ((col >> 4) R + row) 16 + (col & 15).  Column i < n of a1t holds sample i's first hidden
 *                         layer activations a1 (rows < H1p), of d2t its second hidden layer deltas d2 (rows < H2p);
 *                         columns n..ld-1 are written as padding with coefficient 0 (d2 = 0), so g2048_dw2 over
 *                         all ld columns gives the layer-2 weight gradient a1^T d2 and bias gradient sum d2;
 *   partials [waves x g2048_grad_partial_size]  per-wave sums: dW1 [16][H1p], db1 [H1p], dW3 [H2p][4], db3 [4].
 * H1p / H2p = hidden sizes rounded up to 32, 64, 128 or 256; ld a multiple of 32, n <= ld < 2^26;
 * waves = g2048_actor_grad_waves() (every wave writes its row); ld < 2^21 (< 2 GB column buffers). */
int64_t g2048_grad_packed_size(int h1, int h2);
int64_t g2048_grad_partial_size(int h1, int h2);
/* Pack W2 [h1 x h2] (src/MLP.py layout) for the input-delta product; re-pack after every update. */
int g2048_grad_pack(const float* W2, int h1, int h2, float* packed, int64_t packed_len, void* stream);
int g2048_actor_grad_waves(void);
/* d2_form 2 (ReLU actor): instead of d2 columns, d2t receives one 1 KiB record per 16-column block c: bytes
 * [0, 2 H2p) the mask words as for the critic's d2_form 1, bytes [512, 768) the 4 values of g (the logit gradient)
 * of each of the block's 16 columns (float4 per column); g2048_dw2_actor rebuilds d2 from it bit for bit. */
int g2048_actor_grad(const float* packed, const float* grad_packed, int h1, int h2, int activation, int obs_mode,
                     float obs_scale, int use_mask, const uint64_t* boards, const uint8_t* actions, const float* coef,
                     int64_t n, int64_t ld, float* a1t, float* d2t, float* partials, int64_t waves, int d2_form,
                     void* stream);
/* ABI 14: the per-row critic pass's TD targets inside the gradient kernels (g2048_critic_grad, g2048_deep_grad).
 * With td != NULL the kernels ignore `target` / `value_out` and compute target_j =
 * ((v_next[lane[j]] * gamma) * has_next[j]) + reward[j] in fp32 (the host's operation order), writing the launch's
 * V(s_j) to v_out[lane[j]]: the time rows of the critic branch (src/reinforce_agent.py:423-443, V(s') = the next
 * step's value) run one launch each, last row first, with two lane-indexed value buffers alternating and no
 * host-side gather or scatter between launches.  v_next must be finite for every lane read (rows with
 * has_next = 0 multiply it by 0). */
typedef struct g2048_td_rows {
    const int64_t* lane;     /* sample j -> its episode (batch column) */
    const float* reward;     /* r_j (fp32, the critic's rewards) */
    const float* has_next;   /* 1.0 when step j has a successor in its episode, else 0.0 */
    const float* v_next;     /* by lane: V of the next time row */
    float* v_out;            /* by lane: this launch's V(s) */
    float gamma;
    int32_t reserved;
} g2048_td_rows;
/* The critic branch of update_batch (src/reinforce_agent.py:403-498, _get_grad_logits_critic :884-910) on the same
 * kernel: the critic packed like the actor with its value head [h2 x 1] / [1] as output 0 of a 4-wide layer (outputs
 * 1..3 zero); per sample the value V(s), the TD error delta_out = target - V (target = r + gamma V(s') m from the
 * host, or from td: g2048_td_rows), and dL/dV = (V - target) (loss 0, MSE) or its Huber clip at huber_delta (loss 1), times weight[i];
 * the outputs as for g2048_actor_grad (only column / entry 0 of dW3 / db3 is the value head's), plus V(s) per
 * sample in value_out (NULL ok).  Column window: sample i's a1^T / d2^T column is col_off + i, and the columns
 * col_off .. col_off + ncols - 1 are written (those past n as zero-coefficient padding; col_off, ncols multiples
 * of 32, n <= ncols, col_off + ncols <= ld) -- so consecutive launches (one per time row of a batch, whose V(s)
 * is the previous row's V(s')) can fill one column buffer before one layer-2 GEMM.  accumulate != 0 adds this
 * launch's per-wave partials into `partials` instead of overwriting them.
 * d2_form 1 (factored; ReLU only): the critic's d2 is m * (W3[:, 0] g) with m = [a2 > 0] and g = dL/dV * weight per
 * sample, so instead of d2 columns d2t receives one 1 KiB record per 16-column block c (ld / 16 records): bytes
 * [0, 2 H2p) the mask, one uint16 per second-layer unit j (bit k = column 16 c + k has a2_j > 0); bytes [512, 576)
 * g of the block's 16 columns (fp32); the rest unused.  g2048_dw2_factored reads that form (64 B per sample
 * instead of 1 KiB).  d2_form 0: d2 columns as for the actor. */
int g2048_critic_grad(const float* packed, const float* grad_packed, int h1, int h2, int activation, int obs_mode,
                      float obs_scale, int loss, float huber_delta, const uint64_t* boards, const float* target,
                      const float* weight, float* delta_out, float* value_out, int64_t n, int64_t ld, int64_t col_off,
                      int64_t ncols, float* a1t, float* d2t, float* partials, int accumulate, int64_t waves,
                      int d2_form, const g2048_td_rows* td, void* stream);

/* The layer-2 weight / bias gradient of the fused update (the a1 d2^T outer products of _backpropagation,
 * src/reinforce_agent.py:639-678, summed over samples): over the columns [col0, col0 + ncols) of the column
 * buffers g2048_actor_grad / g2048_critic_grad write (a1t, d2t: see there), partials[p] [H1p + 1][H2p] fp32 = sum
 * over the columns [col0 + p cols_per_part, ...) of a1 d2^T (rows 0..H1p-1, dW2) and of d2 (row H1p, db2); the
 * caller sums the nparts = ceil(ncols / cols_per_part) slabs.  Columns where no sample is must hold zeros in d2t
 * (padding).  ld, col0, ncols, cols_per_part multiples of 16.  fp32-accurate: each operand split exactly into three
 * bf16 planes, six plane products on the bf16 MFMA. */
int g2048_dw2(const float* a1t, const float* d2t, int h1, int h2, int64_t ld, int64_t col0, int64_t ncols,
              int64_t cols_per_part, float* partials, int64_t nparts, void* stream);
/* g2048_dw2 for the ReLU critic's factored form (g2048_critic_grad d2_form 1; records: see there): partials[p] rows
 * i < H1p = W3[j] * sum over the slab's columns of fl(a1_i g) m_j, row H1p = W3[j] * sum g m_j; w3 = W3[:, 0]
 * padded with zeros to H2p.  The mask is exact in one bf16 plane, so three plane products per step. */
int g2048_dw2_factored(const float* a1t, const float* records, const float* w3, int h1, int h2, int64_t ld,
                       int64_t col0, int64_t ncols, int64_t cols_per_part, float* partials, int64_t nparts,
                       void* stream);
/* g2048_dw2 for the ReLU actor's records (g2048_actor_grad d2_form 2): d2 of column k, unit j is rebuilt as
 * fl(fl(fl(fl(g0 W3[j,0]) + g1 W3[j,1]) + g2 W3[j,2]) + g3 W3[j,3]) (fused multiply-adds) times the mask bit --
 * bit for bit the d2 g2048_actor_grad computes -- then summed as g2048_dw2 sums d2 columns; w3 = W3 [H2p][4]
 * zero-padded (64 B per sample read instead of 1 KiB). */
int g2048_dw2_actor(const float* a1t, const float* records, const float* w3, int h1, int h2, int64_t ld, int64_t col0,
                    int64_t ncols, int64_t cols_per_part, float* partials, int64_t nparts, void* stream);
/* acc[i] += sum over p < nparts of partials[p * slab + i] (i < slab), the sum taken in fp64 in a fixed order: folds
 * g2048_dw2's slabs (slab = (H1p + 1) H2p) or any per-wave fp32 partials into an fp64 accumulator on the device
 * (the fp64 chunk sums of update_from_batch; no fp32 -> fp64 conversion pass). */
int g2048_fold_partials(const float* partials, int64_t nparts, int64_t slab, double* acc, void* stream);

/* The whole batched rollout in one launch: ReinforceAgent.run_episode (src/reinforce_agent.py:195-252) for n
 * (env_seed, policy_seed) pairs -- select_action (the fused policy above) + Game2048Env.step until terminated or
 * truncated, per episode.  env_* / pol_*: the PCG64 streams of default_rng(env_seed) / default_rng(policy_seed)
 * per episode (g2048_seed_pcg64); queue: one uint32, zero before the call (episode work queue).
 * Trajectory rows are time-major [cap, n]: boards (pre-step), actions, rewards (fp64, the Python floats
 * run_episode records), flags (G2048_F_*), probs [cap, n, 4] (NULL ok); rows at or past an episode's length are
 * not written.  Per episode: lengths, totals (fp64 running sum in step order, src/reinforce_agent.py:233),
 * max_tile (log2 of max_tile_seen), final_board.
 * Requires obs_mode log2 / raw, cfg->max_steps >= 0 and cap >= max(max_steps, 1) (episodes end by then). */
int g2048_rollout(const float* packed, int h1, int h2, int activation, const g2048_env_cfg* cfg, int greedy,
                  const uint64_t* env_state, const uint64_t* env_inc, const uint64_t* env_buf, const uint64_t* pol_state,
                  const uint64_t* pol_inc, const uint64_t* pol_buf, uint32_t* queue, int64_t n, int64_t cap,
                  uint64_t* boards, uint8_t* actions, double* rewards, uint8_t* flags, float* probs, int32_t* lengths,
                  double* totals, uint8_t* max_tile, uint64_t* final_board, void* stream);

/* ---- nets of any depth and one-hot first layers (g2048_deep.hip; ABI 13) ----------------------------------------
 * forward_logits (src/MLP.py:159-196) for 1..G2048_DEEP_MAX_HIDDEN hidden layers of 1..256 units, ReLU / Sigmoid,
 * on log2 / raw obs (16 features) or one-hot obs (272: the first layer is a gather of W1's rows 17 c + e_c, the
 * one-hot encoding of src/env.py:143-150 read off the bitboard -- no obs buffer).  Packed layout: g2048_deep.hip.
 * ABI 15: a one-hot net's packed form also holds W1 split exactly into three bf16 planes in MFMA fragment order
 * (g2048_deep_packed_size grows by 12,288 floats per 32-unit tile of layer 0), and every one-hot forward -- policy,
 * rollout, pattern probe, the update's layer 0 -- computes x W1 as one exact bf16 product per cell and plane,
 * accumulated hi plane / mid + lo planes, so all of them produce the same bits. */
#define G2048_DEEP_MAX_HIDDEN 4
/* floats of the packed net, or -1 if the shape is not covered (hidden: n_hidden sizes) */
int64_t g2048_deep_packed_size(int obs_mode, int n_hidden, const int32_t* hidden);
/* W[l] / b[l] (l = 0..n_hidden): device pointers of the reference-layout fp32 parameters, W_l [in, out] row-major
 * (params["W"], params["b"] of src/MLP.py:45-94); out_dim 4 (actor) or 1 (critic value head, packed as output 0). */
int g2048_deep_pack(const float* const* W, const float* const* b, int obs_mode, int n_hidden, const int32_t* hidden,
                    int out_dim, float* packed, int64_t packed_len, void* stream);
/* g2048_policy's contract for a packed deep net: forward from boards[lane_index ? lane_index[j] : j] (j < n), then
 * (actions != NULL) logits_to_probs + select_action's choice (src/reinforce_agent.py:126-192) on the lane's stream;
 * actions == NULL: forward only (logits_out, e.g. a critic's V(s) in component 0). */
int g2048_deep_policy(const float* packed, int n_hidden, const int32_t* hidden, int activation, const uint64_t* boards,
                      const uint32_t* lane_state, const int32_t* lane_index, int obs_mode, float obs_scale, int use_mask,
                      int greedy, int rng_mode, uint64_t* rng_state, const uint64_t* rng_inc, const uint64_t* rng_buf,
                      uint64_t philox_key, const uint64_t* lane_seed, float* probs_out, float* logits_out,
                      uint8_t* actions, int64_t n, void* stream);
/* Trajectory buffers of a batched rollout: rows are time-major [cap, n] (row t of episode e at t n + e); boards
 * (pre-step), actions, rewards (fp64, the Python floats run_episode records), flags (G2048_F_*), probs [cap, n, 4]
 * (NULL ok); per episode: lengths, totals (fp64 running sum in step order), max_tile (log2 of max_tile_seen),
 * final_board.  Rows at or past an episode's length are not written. */
typedef struct g2048_traj {
    uint64_t* boards;
    uint8_t* actions;
    double* rewards;
    uint8_t* flags;
    float* probs;
    int32_t* lengths;
    double* totals;
    uint8_t* max_tile;
    uint64_t* final_board;
} g2048_traj;
/* Episodes suspended at row cap (g2048_deep_rollout): per episode board, meta {rows so far, step count, max tile
 * exponent} (3 x uint32), running total; list[0 .. *count) = the suspended episodes (count zero before the call). */
typedef struct g2048_suspend {
    uint64_t* board;
    uint32_t* meta;
    double* total;
    int32_t* list;
    uint32_t* count;
} g2048_suspend;
/* g2048_rollout for a packed deep net (any depth, one-hot obs included) and for unbounded episodes: episodes
 * order[0 .. n_order) (NULL: 0 .. n-1, n_order = n) run to their end inside one persistent launch; one that reaches
 * row cap without ending (max_steps None, or cap < max_steps) is suspended -- streams written back into env_* /
 * pol_*, its state into *sus -- and is resumed by a later call with resume = 1, order = the suspended list and the
 * trajectory buffers grown (same n, larger cap; rows below the old cap kept).  queue: one uint32, zero before each
 * call. */
int g2048_deep_rollout(const float* packed, int n_hidden, const int32_t* hidden, int activation, const g2048_env_cfg* cfg,
                       int greedy, uint64_t* env_state, const uint64_t* env_inc, uint64_t* env_buf, uint64_t* pol_state,
                       const uint64_t* pol_inc, uint64_t* pol_buf, uint32_t* queue, const int32_t* order,
                       int64_t n_order, int resume, const g2048_suspend* sus, int64_t n, int64_t cap,
                       const g2048_traj* traj, void* stream);
/* The activations of hidden layer `layer` as g2048_deep_grad computes them (in its 32-sample instantiations -- log2 /
 * raw nets, one-hot nets of 41..64 dense tiles -- a layer with fewer than 8 output tiles and at least 2 k-tiles sums
 * two half-k chains; the 64-sample one and g2048_deep_policy / g2048_deep_rollout keep one chain):
 * out[j * ld + u], u < its padded width (tests and diagnostics: the gradient kernel's own activation pattern). */
int g2048_deep_hidden(const float* packed, int n_hidden, const int32_t* hidden, int activation, int obs_mode,
                      float obs_scale, const uint64_t* boards, int64_t n, int layer, float* out, int64_t ld,
                      void* stream);
/* update_batch's actor or critic gradient (src/reinforce_agent.py:403-555, _backpropagation :639-678) fused for a
 * packed deep net (forward + loss gradient + backward in one kernel, 32 or 64 samples per workgroup step), covered when
 * g2048_deep_grad_slab() >= 0 (1..4 hidden layers of 1..256 units).  Nets of at most 64 dense 32x32 weight-gradient
 * tiles on one-hot obs (48 on log2 / raw: [256, 256], [256, 128, 64] and smaller) take one launch; larger ones one
 * launch per range of tiles, each redoing the forward and delta chains (g2048_deep_grad_passes()).  The workgroup
 * count depends on the instantiation (ABI 14; one per CU since round 6) -- pass nparts = g2048_deep_grad_parts()
 * (any nparts >= 1 is correct; that one fills the chip).
 * grad_packed: g2048_deep_grad_pack (the dense layers' weights in backward-fragment order; re-pack after every
 * update).  Actor: coef = advantage x step weight, actions; critic (critic = 1): coef = step weight, target =
 * r + gamma V(s') m, loss 0 MSE / 1 Huber, delta_out = target - V, value_out = V (NULL ok).  partials [nparts][slab]
 * (nparts = one per workgroup, e.g. the CU count): per workgroup, in floats -- for l = 0 .. n_hidden - 1: dW_l
 * (l = 0: [16][H0p] on log2 / raw obs, nothing on one-hot obs; l >= 1: [H_{l-1}p][H_lp]) then db_l [H_lp]; then
 * dW_out [H_{L-1}p][4] and db_out [4] (Hp = units rounded up to 32).  One-hot obs: d0_out [n][H0p] receives the
 * first layer's deltas for g2048_onehot_dw1 (ld = H0p). */
int64_t g2048_deep_grad_pack_size(int obs_mode, int n_hidden, const int32_t* hidden);
int64_t g2048_deep_grad_slab(int obs_mode, int n_hidden, const int32_t* hidden);
/* the workgroup count that fills the current device for this net (ABI 14; -1 when g2048_deep_grad_slab() < 0) */
int g2048_deep_grad_parts(int obs_mode, int n_hidden, const int32_t* hidden);
/* launches per g2048_deep_grad call for this net: 1 within one launch's accumulator budget, more past it (ABI 16;
 * -1 when g2048_deep_grad_slab() < 0) */
int g2048_deep_grad_passes(int obs_mode, int n_hidden, const int32_t* hidden);
int g2048_deep_grad_pack(const float* const* W, int obs_mode, int n_hidden, const int32_t* hidden, float* packed,
                         int64_t packed_len, void* stream);
int g2048_deep_grad(const float* packed, const float* grad_packed, int n_hidden, const int32_t* hidden,
                    int activation, int obs_mode, float obs_scale, int use_mask, const uint64_t* boards,
                    const uint8_t* actions, const float* coef, int critic, int loss, float huber_delta,
                    const float* target, float* delta_out, float* value_out, float* d0_out, int64_t n,
                    float* partials, int64_t nparts, const g2048_td_rows* td, void* stream);
/* The update's one-hot first layer: out[s * ld + j] = act(b1[j] + sum_c W1[17 c + e_c(s), j]) for s < m, j < h1
 * (W1 the [272, h1] parameter) -- the kept layer-1 activations of _backpropagation (src/reinforce_agent.py:639-678)
 * without the [m, 272] one-hot obs. */
int g2048_onehot_layer1(const float* W1, const float* b1, int h1, int activation, const uint64_t* boards, int64_t m,
                        int64_t ld, float* out, void* stream);
/* floats of one g2048_onehot_dw1 partial slab: 272 h1 (dW1) + h1 (db1) */
int64_t g2048_onehot_dw1_slab(int h1);
/* dW1 = X^T D1 and db1 = sum D1 of a one-hot first layer (X one-hot, D1 = d1[s * ld + j] the layer-1 deltas): slab
 * p of partials (nparts = ceil(m / per)) holds the sums over samples [p per, (p + 1) per) -- ABI 14: an fp32
 * accumulation on the bf16 MFMA of the exact products of the one-hot with each delta's three bf16 planes
 * (deterministic, one 8-wave workgroup per slab: pick per so that nparts ~ the CU count); fold them with
 * g2048_fold_partials.  Rows on 16-byte boundaries (d1 16-byte aligned, ld % 4 == 0, h1 % 4 == 0) stream through an LDS ring
 * (round 5), any other stride through registers: the same bits either way. */
int g2048_onehot_dw1(const uint64_t* boards, const float* d1, int h1, int64_t m, int64_t ld, int64_t per,
                     float* partials, int64_t nparts, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* G2048_H */
