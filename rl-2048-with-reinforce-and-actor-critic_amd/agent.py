"""ReinforceAgent (src/reinforce_agent.py) on the MI355X path.

Two faces over one implementation:

* the reference's API, unchanged in names / arguments / results -- ``select_action``, ``run_episode``,
  ``compute_returns``, ``update_batch(trajectories: list[dict])``, ``load_model`` / ``save_model``,
  ``clip_grads_global_norm``;
* the batched hot path -- ``rollout_batch(env_seeds, policy_seeds)`` plays every episode of a batch in its own
  device lane (VecGame2048Env + the fused masked-softmax/choice kernel) and records a time-major device
  trajectory buffer; ``update_from_batch(batch)`` applies exactly the update of ``update_batch`` to it.

The update is the reference's per-timestep manual backprop (src/reinforce_agent.py:502-555, :639-678) restated
as one batched manual backprop over all valid steps (mlp.mlp_backward_): the actor's logit gradient is
A_t * (onehot(a_t) - pi(.|s_t)) scaled by rank_w / (T_i * n) and back-propagated through the MLP (identical to
summing the reference's per-step outer products; the weight gradients are split-K batched GEMMs); the critic's is
the (MSE or Huber) TD gradient with the same weights.  Gradient clipping, SGD ascent /
descent and Adam follow :558-582, :719-770, :835-861.

Data parallel: when torch.distributed is initialised each rank holds a shard of the batch's episodes; rank
weights all-gather the episode totals, the batch baselines all-reduce three scalars, and the actor+critic
gradients travel in ONE fused all-reduce (RCCL over xGMI on MI355X) before clipping, so every rank applies the
update of the concatenated batch.
"""
from __future__ import annotations

import ctypes
import logging
import os
from dataclasses import dataclass
from typing import Any, Callable, Literal

import numpy as np
import torch
from . import _lib as L
from . import dp
from .config import Game2048EnvConfig, obs_width
from .mlp import (MLPConfig, encode_observation, forward_logits, init_model_params, load_model_params, mlp_backward_,
                  mlp_forward_kept,
                  logits_to_probs, save_model_params)
from .vec_env import VecGame2048Env

BaselineMode = Literal["off", "each", "batch", "batch_norm"]
OptimizerType = Literal["sgd", "adam"]
CriticLossType = Literal["mse", "huber"]

_OBS_CODE = {"raw": L.OBS_RAW, "log2": L.OBS_LOG2, "onehot": L.OBS_ONEHOT}


@dataclass
class ReinforceAgentConfig:
    gamma: float = 1
    learning_rate: float = 1e-3
    baseline_mode: BaselineMode = "off"
    model_seed: int = 0
    reward_rank_weights: list[float] | None = None
    optimizer: OptimizerType = "sgd"
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    augmentation: bool = False
    use_critic: bool = False
    critic_learning_rate: float = 1e-3
    max_grad_norm: float = 1.0
    critic_loss_type: CriticLossType = "mse"
    huber_delta: float = 1.0


@dataclass
class TrajectoryBatch:
    """Device trajectory buffer of one batch of episodes, time-major: row t, column = episode (lane).
    boards[t, i] is the board BEFORE action actions[t, i]; rewards[t, i] its reward; valid iff t < lengths[i]."""
    boards: torch.Tensor       # [T, n] int64 bitboards
    actions: torch.Tensor      # [T, n] uint8
    rewards: torch.Tensor      # [T, n] float64 (the Python float Game2048Env.step returns)
    flags: torch.Tensor        # [T, n] uint8 (G2048_F_*)
    lengths: torch.Tensor      # [n] int32
    total_reward: torch.Tensor  # [n] float64
    max_tile: torch.Tensor     # [n] int64 (Game2048Env.max_tile_seen at the end of the episode)
    final_boards: torch.Tensor  # [n] int64
    probs: torch.Tensor | None = None  # [T, n, 4] policy probabilities used for each draw (record_probs=True)
    # data parallel: the episode count of every rank's shard of the global batch (dp.shard_sizes), set by whoever
    # sharded it; lets the rank-weight all-gather run without a host synchronisation
    shard_sizes: tuple[int, ...] | None = None

    @property
    def n(self) -> int:
        return int(self.lengths.numel())

    @property
    def T(self) -> int:
        return int(self.boards.shape[0])


def _seed_seq(seeds):
    """A batch of episode seeds as a tensor / numpy array (kept: the fast conversion path) or a list."""
    return seeds if isinstance(seeds, (torch.Tensor, np.ndarray)) else list(seeds)


def _render_values(vals: np.ndarray) -> str:
    from .env import _render

    return _render(vals.tolist())


def _board_values(b: int) -> np.ndarray:
    e = np.array([(b >> (4 * i)) & 15 for i in range(16)], dtype=np.int64).reshape(4, 4)
    return np.where(e > 0, np.left_shift(np.int64(1), e), 0).astype(np.int64)


def _unrecord(rec: torch.Tensor, w3: torch.Tensor, c0: int, m: int) -> torch.Tensor:
    """The d2 columns [c0, c0 + m) that the factored block records (g2048_critic_grad d2_form 1) stand for, [H2p, m]:
    fl(g * W3[j]) where unit j's mask bit is set -- bit for bit the d2 the unfactored kernel computes (its
    d2 = (g W3[j] + 0 ...) * 1 or * 0)."""
    H2p = w3.numel()
    blocks = rec.view(-1, 256)
    words = blocks.view(torch.int16).view(-1, 512)[:, :H2p].to(torch.int32) & 0xFFFF   # [blocks, H2p]
    g = blocks[:, 128:144].reshape(-1)                                                   # [blocks * 16]
    cols = torch.arange(c0, c0 + m, device=rec.device)
    bits = (words[cols >> 4] >> (cols & 15)[:, None]) & 1                                 # [m, H2p]
    return ((g[cols][:, None] * w3[None, :]) * bits.to(torch.float32)).t()


def _unrecord_actor(rec: torch.Tensor, w3: torch.Tensor, c0: int, m: int) -> torch.Tensor:
    """The d2 columns [c0, c0 + m) that the actor's block records (g2048_actor_grad d2_form 2) stand for, [H2p, m]:
    fl(fl(fl(fl(g0 W3[j,0]) + g1 W3[j,1]) + g2 W3[j,2]) + g3 W3[j,3]) where unit j's mask bit is set (w3: [H2p, 4])."""
    H2p = w3.shape[0]
    blocks = rec.view(-1, 256)
    words = blocks.view(torch.int16).view(-1, 512)[:, :H2p].to(torch.int32) & 0xFFFF   # [blocks, H2p]
    g = blocks[:, 128:192].reshape(-1, 4)                                                # [blocks * 16, 4]
    cols = torch.arange(c0, c0 + m, device=rec.device)
    bits = (words[cols >> 4] >> (cols & 15)[:, None]) & 1                                 # [m, H2p]
    gc = g[cols]
    # the kernel's operation order, one rounding per step.  fmaf = fl32(g w + dh): the product is exact in fp64, the
    # fp64 sum s may round (a 48-bit product plus dh), and rounding s to fp32 could then round twice; the exact
    # error e of the fp64 sum (TwoSum) settles the one case that matters -- s exactly halfway between two floats,
    # where fp32's tie-to-even picked the neighbour on the wrong side of the true value s + e.
    dh = (gc[:, 0:1] * w3[None, :, 0])
    for k in (1, 2, 3):
        p = gc[:, k:k + 1].double() * w3[None, :, k].double()
        d = dh.double()
        s = p + d
        bb = s - p
        e = (p - (s - bb)) + (d - bb)
        r = s.to(torch.float32)
        diff = s - r.double()
        nxt = torch.nextafter(r, torch.where(diff > 0, torch.full_like(r, float("inf")), torch.full_like(r, float("-inf"))))
        tie = (diff != 0) & (2.0 * diff.abs() == (nxt.double() - r.double()).abs())
        dh = torch.where(tie & (e * diff > 0), nxt, r)
    return (dh * bits.to(torch.float32)).t()


def _unblock(buf: torch.Tensor, rows: int, c0: int, m: int) -> torch.Tensor:
    """Rows [0, rows) x columns [c0, c0 + m) of a column buffer stored in 16-column blocks (include/g2048.h) as a
    row-major copy (diagnostics: ReinforceAgent.grad_probe)."""
    R, ld = buf.shape
    return buf.reshape(ld // 16, R, 16).permute(1, 0, 2).reshape(R, ld)[:rows, c0:c0 + m]


def _round32(h: int) -> int:
    """Hidden units as the any-depth kernels pad them (g2048_deep.hip): whole 32-unit tiles."""
    return 32 * ((h + 31) // 32)


def _padded_units(h: int) -> int:
    """Hidden units as the fused kernels pad them: whole 32-unit MFMA tiles, 1, 2, 4 or 8 of them (tiles_for in
    csrc/g2048_policy.hip)."""
    t = (h + 31) // 32
    return 32 * (1 if t <= 1 else 2 if t <= 2 else 4 if t <= 4 else 8)


class _Steps:
    """The valid steps of a batch in time-major order plus how to build their MLP inputs.

    Feature source is either bitboards (batched path: obs / mask built on the fly by g2048_obs, symmetries by
    g2048_symmetries) or host-provided features (drop-in update_batch on reference trajectories)."""

    def __init__(self, agent: "ReinforceAgent", lengths: torch.Tensor, actions: torch.Tensor, rewards: torch.Tensor,
                 boards: torch.Tensor | None = None, X: torch.Tensor | None = None, M: torch.Tensor | None = None):
        dev = agent.device
        self.agent = agent
        self.T, self.n = rewards.shape
        self.lengths = lengths.to(dev, torch.int64)
        t_idx = torch.arange(self.T, device=dev).unsqueeze(1)
        valid = t_idx < self.lengths.unsqueeze(0)                     # [T, n]
        self.vidx = valid.reshape(-1).nonzero().squeeze(1)             # flat t*n + lane, time-major
        self.lane = self.vidx % self.n
        self.t = self.vidx // self.n
        self.has_next = (self.t + 1) < self.lengths[self.lane]
        self.actions = actions.reshape(-1)[self.vidx].to(torch.int64)
        # fp32 per valid step for the critic (np.array(rewards, float32), src/reinforce_agent.py:420); the fp64
        # time-major rows for compute_returns (fp64 scan of the Python floats, :263-271)
        self.rewards = rewards.reshape(-1)[self.vidx].to(torch.float32)
        self.rewards_tm = rewards.to(torch.float64)
        self.boards = boards
        self.X = X
        self.M = M
        self.N = int(self.vidx.numel())

    # ---------------------------------------------------------------- features of flat time-major indices
    def _board_obs(self, flat: torch.Tensor, k: int):
        b = self.boards.reshape(-1)[flat].contiguous()
        if k:
            b = self.agent._symmetry_boards(b, k)
        return self.agent._obs_from_boards(b)

    def features(self, sel: torch.Tensor, k: int = 0, nxt: bool = False):
        """(x [m, D] f32, mask [m, 4] int8) of the valid steps `sel` (indices into vidx), symmetry k, or of
        their successor step (nxt=True; a step without one -- its episode's last -- gives itself, masked by the
        caller, like the reference's padding src/reinforce_agent.py:423)."""
        flat = self.vidx[sel]
        if nxt:
            flat = torch.where(self.has_next[sel], flat + self.n, flat)
        if self.boards is not None:
            return self._board_obs(flat, k)
        x = self.X.reshape(self.T * self.n, -1)[flat]
        m = self.M.reshape(self.T * self.n, 4)[flat] if self.M is not None else None
        if k:
            x, m = self.agent._symmetry_features(x, m, k)
        return x, m

    def boards_at(self, sel: torch.Tensor, k: int = 0, nxt: bool = False) -> torch.Tensor:
        """The bitboards of the valid steps `sel` (or of their successors, as features(nxt=True)), symmetry k."""
        flat = self.vidx[sel]
        if nxt:
            flat = torch.where(self.has_next[sel], flat + self.n, flat)
        b = self.boards.reshape(-1)[flat].contiguous()
        return self.agent._symmetry_boards(b, k) if k else b

    def actions_k(self, sel: torch.Tensor, k: int) -> torch.Tensor:
        a = self.actions[sel]
        if k == 0:
            return a
        if k >= 4:
            a = torch.where(a == 1, 3, torch.where(a == 3, 1, a))
        return (a - (k & 3)) % 4


class ReinforceAgent:
    def __init__(self, env, mlp_config: MLPConfig, agent_config: ReinforceAgentConfig | None = None,
                 initial_params_path: str | None = None, device=None, chunk_steps: int = 1 << 18):
        """env: a Game2048Env (drop-in, src/reinforce_agent.py:51-105) or a Game2048EnvConfig."""
        if isinstance(env, Game2048EnvConfig):
            self.env = None
            self.env_config = env
        else:
            self.env = env
            self.env_config = env.config
        self.mlp_config = mlp_config
        self.agent_config = agent_config or ReinforceAgentConfig()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        L.ensure_device(self.device)
        self.rng = np.random.default_rng(self.agent_config.model_seed)
        self._logger = logging.getLogger(__name__ + ".ReinforceAgent")
        if not self._logger.handlers:
            self._logger.addHandler(logging.NullHandler())
        if self.env is not None:
            self.env.reset(seed=0)       # the reference probes input_dim this way (src/reinforce_agent.py:70)
        self.input_dim = obs_width(self.env_config.obs_mode)
        self.n_actions = 4
        if initial_params_path is None:
            self.params = init_model_params(self.input_dim, self.mlp_config.hidden_sizes, self.n_actions, self.rng,
                                            self.mlp_config.init_distribution, self.mlp_config.last_init_normal,
                                            device=self.device)
        else:
            self.params = load_model_params(initial_params_path, device=self.device)
        self._init_adam(self.params, prefix="actor")
        self._adam_t = 0
        self.critic_params = None
        if self.agent_config.use_critic:
            self.critic_params = init_model_params(self.input_dim, self.mlp_config.hidden_sizes, 1, self.rng,
                                                   self.mlp_config.init_distribution,
                                                   self.mlp_config.last_init_normal, device=self.device)
            self._init_adam(self.critic_params, prefix="critic")
            self._adam_t_c = 0
        self.chunk_steps = int(chunk_steps)
        # rollout / evaluation forward through the fused g2048_policy kernel when the net fits it
        self.use_fused_policy = True
        # ... and the whole rollout in one launch (g2048_rollout) when the episodes are bounded (max_steps set)
        self.use_fused_rollout = True
        # update_batch's actor gradient through the fused g2048_actor_grad kernel when the net fits it (batched path)
        self.use_fused_grad = True
        # two-layer log2 / raw nets through the cooperative g2048_actor_grad / g2048_critic_grad kernels (+ g2048_dw2);
        # False routes them to g2048_deep_grad where it covers the net (tools/bench_update.py --deep-grad A/B)
        self.use_two_layer_grad = True
        # nets past g2048_deep_grad's one-launch tile budget through it anyway, one launch per tile range (tests);
        # off: they take the gather + hipBLASLt path, which measured faster for them (_deep_grad_spec)
        self.deep_grad_multi_launch = False
        # ... and the fused critic per time row, V(s') taken from the next row's pass (large batches)
        self.use_critic_rows = True
        self.critic_factored_d2 = True   # ReLU critic rows: the factored d2 records + g2048_dw2_factored
        # ReLU actor: d2 block records (mask + g) + g2048_dw2_actor instead of d2 columns + g2048_dw2.  Off: the
        # rebuild of d2 from 4 values of g adds VALU work to the MFMA-bound g2048_dw2 (configs[2] update 0.817-0.823
        # against 0.789-0.794 s with the columns, profiles/round4/r4c6/), more than the 1 KiB / sample of HBM saved
        self.actor_d2_records = False
        self.grad_chunk_steps = 1 << 20
        # diagnostics (tests): called as grad_probe(slot, k, sample_idx, a1_cols, d2_cols) with the column buffers
        # of every fused-gradient launch before they are reused -- sample_idx indexes the batch's valid steps
        # (time-major), a1_cols [H1p, m] holds the layer-1 activations the kernel computed, d2_cols [H2p, m] its
        # layer-2 deltas (row-major copies) -- so a checker can evaluate the formula under the kernel's own
        # activation pattern
        self.grad_probe: Callable | None = None
        self._pack_cache: dict[str, list] = {}
        self._params_version = 0
        self._vec_cache: dict = {}
        self._lib = L.lib()
        self.last_stats: dict = {}
        self._paths: dict[str, str] = {}   # which implementation ran each phase last (last_paths)

    # ============================================================================================ model I/O
    def load_model(self, file_path: str = "params.npz") -> None:
        """src/reinforce_agent.py:108-116"""
        self.params = load_model_params(file_path, device=self.device)
        self.mlp_config.hidden_sizes = [int(W.shape[1]) for W in self.params["W"][:-1]]
        self._params_version += 1
        self._logger.info(f"Model parameters loaded from {file_path}")

    def save_model(self, file_path: str = "params.npz") -> None:
        """src/reinforce_agent.py:119-123"""
        save_model_params(self.params, file_path)

    # ============================================================================================ checkpoints
    # Resume-capable checkpoints (the reference's model_*.npz holds the actor only,
    # runner.py:642-660).  One npz, no pickle: the actor under the reference's keys (n_layers, W_i, b_i -- so a
    # checkpoint also loads with load_model / src/MLP.py:97-107), then Adam moments and step counters, the critic
    # and its Adam state, and caller state under "extra_<name>".
    def checkpoint_state(self) -> dict[str, np.ndarray]:
        def host(t):
            return t.detach().to("cpu").numpy()

        st: dict[str, np.ndarray] = {"n_layers": np.array(len(self.params["W"]), dtype=np.int64),
                                     "adam_t": np.array(self._adam_t, dtype=np.int64)}
        for i, (W, b) in enumerate(zip(self.params["W"], self.params["b"])):
            st[f"W_{i}"], st[f"b_{i}"] = host(W), host(b)
            st[f"adam_mW_{i}"], st[f"adam_vW_{i}"] = host(self._adam_m_W[i]), host(self._adam_v_W[i])
            st[f"adam_mb_{i}"], st[f"adam_vb_{i}"] = host(self._adam_m_B[i]), host(self._adam_v_B[i])
        if self.critic_params is not None:
            st["critic_n_layers"] = np.array(len(self.critic_params["W"]), dtype=np.int64)
            st["critic_adam_t"] = np.array(self._adam_t_c, dtype=np.int64)
            for i, (W, b) in enumerate(zip(self.critic_params["W"], self.critic_params["b"])):
                st[f"critic_W_{i}"], st[f"critic_b_{i}"] = host(W), host(b)
                st[f"critic_adam_mW_{i}"], st[f"critic_adam_vW_{i}"] = host(self._adam_m_W_c[i]), host(self._adam_v_W_c[i])
                st[f"critic_adam_mb_{i}"], st[f"critic_adam_vb_{i}"] = host(self._adam_m_B_c[i]), host(self._adam_v_B_c[i])
        return st

    def load_checkpoint_state(self, st) -> None:
        def dev(a):
            return torch.as_tensor(np.asarray(a, dtype=np.float32), device=self.device).contiguous()

        n = int(st["n_layers"])
        self.params = {"W": [dev(st[f"W_{i}"]) for i in range(n)], "b": [dev(st[f"b_{i}"]) for i in range(n)]}
        self.mlp_config.hidden_sizes = [int(W.shape[1]) for W in self.params["W"][:-1]]
        self._params_version += 1
        self._adam_m_W = [dev(st[f"adam_mW_{i}"]) for i in range(n)]
        self._adam_v_W = [dev(st[f"adam_vW_{i}"]) for i in range(n)]
        self._adam_m_B = [dev(st[f"adam_mb_{i}"]) for i in range(n)]
        self._adam_v_B = [dev(st[f"adam_vb_{i}"]) for i in range(n)]
        self._adam_t = int(st["adam_t"])
        if (self.critic_params is not None) != ("critic_n_layers" in st):
            raise ValueError("checkpoint critic does not match agent_config.use_critic")
        if self.critic_params is not None:
            m = int(st["critic_n_layers"])
            self.critic_params = {"W": [dev(st[f"critic_W_{i}"]) for i in range(m)],
                                  "b": [dev(st[f"critic_b_{i}"]) for i in range(m)]}
            self._adam_m_W_c = [dev(st[f"critic_adam_mW_{i}"]) for i in range(m)]
            self._adam_v_W_c = [dev(st[f"critic_adam_vW_{i}"]) for i in range(m)]
            self._adam_m_B_c = [dev(st[f"critic_adam_mb_{i}"]) for i in range(m)]
            self._adam_v_B_c = [dev(st[f"critic_adam_vb_{i}"]) for i in range(m)]
            self._adam_t_c = int(st["critic_adam_t"])

    def save_checkpoint(self, file_path: str, extra: dict | None = None) -> None:
        st = self.checkpoint_state()
        for k, v in (extra or {}).items():
            st[f"extra_{k}"] = np.asarray(v)
        tmp = str(file_path) + ".tmp.npz"
        np.savez(tmp, **st)
        os.replace(tmp, file_path)

    def load_checkpoint(self, file_path: str) -> dict:
        """Restores what save_checkpoint wrote; returns the extra_* entries (numpy scalars / arrays)."""
        with np.load(file_path, allow_pickle=False) as z:
            st = {k: z[k] for k in z.files}
        self.load_checkpoint_state(st)
        self._logger.info(f"Checkpoint loaded from {file_path}")
        return {k[len("extra_"):]: v for k, v in st.items() if k.startswith("extra_")}

    def last_paths(self) -> dict[str, str]:
        """Which implementation ran the last rollout / actor gradient / critic gradient (bench and test
        reporting)."""
        return dict(self._paths)

    # ============================================================================================ helpers
    @property
    def _stream(self) -> int:
        return L.stream_handle(self.device)

    def _obs_from_boards(self, boards: torch.Tensor):
        m = boards.numel()
        x = torch.empty(m, self.input_dim, dtype=torch.float32, device=self.device)
        mk = torch.empty(m, 4, dtype=torch.int8, device=self.device)
        L.check(self._lib.g2048_obs(L.ptr(boards), _OBS_CODE[self.env_config.obs_mode],
                                    float(self.env_config.obs_log2_scale), L.ptr(x), L.ptr(mk), m, self._stream))
        return x, mk

    def _symmetry_boards(self, boards: torch.Tensor, k: int) -> torch.Tensor:
        m = boards.numel()
        out = torch.empty(8 * m, dtype=torch.int64, device=self.device)
        L.check(self._lib.g2048_symmetries(L.ptr(boards), None, L.ptr(out), None, m, self._stream))
        return out[k * m:(k + 1) * m]

    def _symmetry_features(self, x: torch.Tensor, m: torch.Tensor | None, k: int):
        """get_symmetries (src/env.py:317-398) on host-provided features: board [.,4,4(,17)] and mask."""
        onehot = x.shape[1] == 272
        b = x.view(-1, 4, 4, 17) if onehot else x.view(-1, 4, 4)
        if k >= 4:
            b = torch.flip(b, dims=[2])
            if m is not None:
                m = m[:, [0, 3, 2, 1]]
        for _ in range(k & 3):
            b = torch.rot90(b, k=1, dims=(1, 2))
            if m is not None:
                m = torch.roll(m, shifts=-1, dims=1)
        return b.reshape(x.shape[0], -1).contiguous(), m

    def _vec_env(self, n: int, rng: str) -> VecGame2048Env:
        key = (n, rng)
        if key not in self._vec_cache:
            self._vec_cache.clear()
            self._vec_cache[key] = VecGame2048Env(n, self.env_config, device=self.device, rng=rng, track_score=False)
        return self._vec_cache[key]

    def _policy_logits(self, x: torch.Tensor) -> torch.Tensor:
        return forward_logits(self.params, x, self.mlp_config.activation, keep_cache=False)[0]

    def _fused_policy_spec(self):
        """(h1, h2, activation code) when g2048_policy covers the actor (obs width 16, two hidden layers of
        1..256 units, ReLU / Sigmoid, fp32), else None (the GEMM path + g2048_sample then runs)."""
        return self._net_spec() if self.use_fused_policy else None

    def _fused_grad_spec(self):
        """The same net check for g2048_actor_grad (else the batched torch backprop runs)."""
        return self._net_spec() if self.use_fused_grad and self.use_two_layer_grad else None

    def _fused_critic_spec(self):
        """... and for the critic (value head of width 1) through g2048_critic_grad."""
        if not self.use_fused_grad or not self.use_two_layer_grad or self.critic_params is None:
            return None
        return self._net_spec(self.critic_params, 1)

    def _net_spec(self, params=None, out_dim: int = 4):
        if self.env_config.obs_mode not in ("log2", "raw"):
            return None
        params = self.params if params is None else params
        Ws, bs = params["W"], params["b"]
        if len(Ws) != 3 or len(bs) != 3 or tuple(Ws[0].shape)[0] != 16 or tuple(Ws[2].shape)[1] != out_dim:
            return None
        h1, h2 = int(Ws[0].shape[1]), int(Ws[1].shape[1])
        act = {"ReLU": L.ACT_RELU, "Sigmoid": L.ACT_SIGMOID}.get(self.mlp_config.activation)
        if act is None or not (1 <= h1 <= 256 and 1 <= h2 <= 256) or tuple(Ws[1].shape)[0] != h1 or \
                tuple(Ws[2].shape)[0] != h2:
            return None
        if any(t.dtype != torch.float32 or t.device != self.device for t in Ws + bs):
            return None
        return h1, h2, act

    def _deep_spec(self, params=None, out_dim: int = 4):
        """(obs code, hidden sizes, activation code, int32 ctypes array of the sizes) when the net is covered by the
        any-depth kernels of g2048_deep.hip (1..4 hidden layers of 1..256 units, ReLU / Sigmoid, fp32 on this
        device, log2 / raw / one-hot obs), else None."""
        params = self.params if params is None else params
        Ws, bs = params["W"], params["b"]
        nh = len(Ws) - 1
        act = {"ReLU": L.ACT_RELU, "Sigmoid": L.ACT_SIGMOID}.get(self.mlp_config.activation)
        if act is None or not (1 <= nh <= L.DEEP_MAX_HIDDEN) or len(bs) != len(Ws):
            return None
        hidden = tuple(int(W.shape[1]) for W in Ws[:-1])
        if tuple(Ws[0].shape)[0] != self.input_dim or tuple(Ws[-1].shape)[1] != out_dim or \
                not all(1 <= h <= 256 for h in hidden):
            return None
        if any(tuple(Ws[l].shape)[0] != hidden[l - 1] for l in range(1, nh + 1)):
            return None
        if any(t.dtype != torch.float32 or t.device != self.device for t in Ws + bs):
            return None
        return (_OBS_CODE[self.env_config.obs_mode], hidden, act, (ctypes.c_int32 * nh)(*hidden))

    def _pack_deep(self, params, dspec, slot: str, out_dim: int) -> torch.Tensor:
        """g2048_deep_pack of a net, cached per slot until a parameter tensor changes."""
        Ws, bs = params["W"], params["b"]
        key = (self._params_version,) + tuple((t.data_ptr(), t._version) for t in Ws + bs)
        entry = self._pack_cache.setdefault(slot + "/deep", [None, None, None])
        if key != entry[1]:
            obs_code, hidden, _, harr = dspec
            size = int(self._lib.g2048_deep_packed_size(obs_code, len(hidden), harr))
            if entry[0] is None or entry[0].numel() < size:
                entry[0] = torch.empty(size, dtype=torch.float32, device=self.device)
            ws = [t.contiguous() for t in Ws]
            bb = [t.contiguous() for t in bs]
            wp = (ctypes.c_void_p * len(ws))(*[t.data_ptr() for t in ws])
            bp = (ctypes.c_void_p * len(bb))(*[t.data_ptr() for t in bb])
            L.check(self._lib.g2048_deep_pack(wp, bp, obs_code, len(hidden), harr, out_dim, L.ptr(entry[0]), size,
                                              self._stream))
            entry[1] = key
            entry[2] = (ws, bb)      # keep the contiguous copies alive until the (stream-ordered) pack has run
        return entry[0]

    def _deep_forward(self, params, dspec, slot: str, boards: torch.Tensor, out_dim: int) -> torch.Tensor:
        """forward_logits of the boards through g2048_deep_policy (forward only): [m, 4] (a value head in column 0)."""
        m = boards.numel()
        out = torch.empty(m, 4, dtype=torch.float32, device=self.device)
        if m == 0:
            return out
        packed = self._pack_deep(params, dspec, slot, out_dim)
        obs_code, hidden, act, harr = dspec
        L.check(self._lib.g2048_deep_policy(L.ptr(packed), len(hidden), harr, act, L.ptr(boards.contiguous()), None,
                                            None, obs_code, float(self.env_config.obs_log2_scale), 0, 1, L.RNG_PCG64,
                                            None, None, None, 0, None, None, L.ptr(out), None, m, self._stream))
        return out

    def _onehot_first_layer(self, steps: "_Steps") -> bool:
        """The batched update gathers the one-hot first layer from the bitboards (g2048_onehot_layer1 /
        g2048_onehot_dw1) instead of materialising [m, 272] one-hot obs for 272-wide GEMMs."""
        return steps.boards is not None and self.env_config.obs_mode == "onehot"

    def _mask_from_boards(self, boards: torch.Tensor) -> torch.Tensor:
        m = boards.numel()
        mk = torch.empty(m, 4, dtype=torch.int8, device=self.device)
        L.check(self._lib.g2048_obs(L.ptr(boards), L.OBS_NONE, 1.0, None, L.ptr(mk), m, self._stream))
        return mk

    def _forward_kept_steps(self, params, steps: "_Steps", sel: torch.Tensor, k: int, want_mask: bool = False):
        """mlp_forward_kept of the valid steps `sel` (symmetry k): (output, kept activations, boards or None, action
        mask or None).  On one-hot obs the first layer is g2048_onehot_layer1's gather from the boards (returned for
        the dW1 scatter)."""
        act = self.mlp_config.activation
        if self._onehot_first_layer(steps):
            b = steps.boards_at(sel, k)
            W1, b1 = params["W"][0].contiguous(), params["b"][0].contiguous()
            h1 = int(W1.shape[1])
            a1 = torch.empty(b.numel(), h1, dtype=torch.float32, device=self.device)
            L.check(self._lib.g2048_onehot_layer1(L.ptr(W1), L.ptr(b1), h1,
                                                  {"ReLU": L.ACT_RELU, "Sigmoid": L.ACT_SIGMOID}[act], L.ptr(b),
                                                  b.numel(), h1, L.ptr(a1), self._stream))
            out, kept = mlp_forward_kept(params, None, act, a1=a1)
            return out, kept, b, (self._mask_from_boards(b) if want_mask else None)
        x, mk = steps.features(sel, k)
        out, kept = mlp_forward_kept(params, x, act)
        return out, kept, None, mk

    def _onehot_dw1_into(self, boards: torch.Tensor, d1: torch.Tensor, acc: torch.Tensor, h1: int | None = None) -> None:
        """acc (fp64 [273 h1]: dW1 rows, then db1) += the one-hot first layer's weight / bias gradient of the deltas
        d1 [m, ld] (units < h1, default ld; g2048_onehot_dw1 partial slabs folded in fp64)."""
        m, ld = d1.shape
        h1 = ld if h1 is None else h1
        if m == 0:
            return
        d1 = d1.contiguous()
        cus = int(self._lib.g2048_actor_grad_waves()) // 4
        per = max(512, -(-m // (16 * cus)) * 16)         # one 8-wave MFMA workgroup per CU, whole 16-sample steps
        nparts = -(-m // per)
        part = torch.empty(nparts, int(self._lib.g2048_onehot_dw1_slab(h1)), dtype=torch.float32, device=self.device)
        L.check(self._lib.g2048_onehot_dw1(L.ptr(boards), L.ptr(d1), h1, m, ld, per, L.ptr(part), nparts,
                                           self._stream))
        self._fold(part, acc)

    def _deep_grad_spec(self, params, out_dim: int):
        """_deep_spec when g2048_deep_grad covers the net in one launch per chunk (g2048_deep_grad_passes() == 1:
        at most 64 dense 32x32 weight-gradient tiles on one-hot obs, 48 on log2 / raw), else None.  Larger nets run
        it as one launch per range of tiles (each redoing the forward and delta chains) only with
        deep_grad_multi_launch: measured slower than the gather + hipBLASLt path for one-hot [256, 256, 256] (update
        1.31 s against 1.14 s at 262,144 episodes, profiles/round5/r6w/)."""
        if not self.use_fused_grad:
            return None
        d = self._deep_spec(params, out_dim)
        if d is None:
            return None
        passes = int(self._lib.g2048_deep_grad_passes(d[0], len(d[1]), d[3]))
        if passes < 1 or (passes > 1 and not self.deep_grad_multi_launch):
            return None
        return d

    def _pack_deep_grad(self, params, dspec, slot: str) -> torch.Tensor:
        """g2048_deep_grad_pack (the dense layers' backward fragments), cached per slot until a parameter changes."""
        Ws = params["W"]
        key = (self._params_version,) + tuple((t.data_ptr(), t._version) for t in Ws)
        entry = self._pack_cache.setdefault(slot + "/deepgrad", [None, None, None])
        if key != entry[1]:
            obs_code, hidden, _, harr = dspec
            size = int(self._lib.g2048_deep_grad_pack_size(obs_code, len(hidden), harr))
            if entry[0] is None or entry[0].numel() < size:
                entry[0] = torch.empty(size, dtype=torch.float32, device=self.device)
            ws = [t.contiguous() for t in Ws]
            wp = (ctypes.c_void_p * len(ws))(*[t.data_ptr() for t in ws])
            L.check(self._lib.g2048_deep_grad_pack(wp, obs_code, len(hidden), harr, L.ptr(entry[0]), size,
                                                   self._stream))
            entry[1] = key
            entry[2] = ws
        return entry[0]

    @staticmethod
    def _deep_slab_layout(hidden, onehot: bool):
        """(pw, pb) float offsets of g2048_deep_grad's partial slab (include/g2048.h)."""
        Hp = [_round32(h) for h in hidden]
        pw, pb, off = [], [], 0
        for l in range(len(hidden)):
            pw.append(off)
            off += (0 if onehot else 16 * Hp[0]) if l == 0 else Hp[l - 1] * Hp[l]
            pb.append(off)
            off += Hp[l]
        pw.append(off)
        off += Hp[-1] * 4
        pb.append(off)
        return pw, pb

    def _deep_grad_fused(self, params, slot: str, dspec, steps: "_Steps", K: int, gW: list[torch.Tensor],
                         gb: list[torch.Tensor], out_dim: int, adv=None, step_w=None, deltas=None) -> None:
        """update_batch's actor (adv given) or critic (deltas given) branch for a deep / one-hot net through
        g2048_deep_grad (forward + loss gradient + backward fused, dense weight gradients in registers), chunked;
        the critic's V(s') by g2048_deep_policy's forward; one-hot first layers by the g2048_onehot_dw1 scatter of
        the kernel's layer-0 deltas.  Accumulates into gW / gb like mlp_backward_."""
        c = self.agent_config
        obs_code, hidden, act, harr = dspec
        onehot = obs_code == L.OBS_ONEHOT
        critic = deltas is not None
        packed = self._pack_deep(params, dspec, slot, out_dim)
        bpacked = self._pack_deep_grad(params, dspec, slot)
        nparts = int(self._lib.g2048_deep_grad_parts(obs_code, len(hidden), harr))   # fills the chip
        slab = int(self._lib.g2048_deep_grad_slab(obs_code, len(hidden), harr))
        part = torch.empty(nparts, slab, dtype=torch.float32, device=self.device)
        acc = torch.zeros(slab, dtype=torch.float64, device=self.device)
        h0, H0p = hidden[0], _round32(hidden[0])
        acc1 = torch.zeros(273 * h0, dtype=torch.float64, device=self.device) if onehot else None
        use_mask = int(bool(self.env_config.use_action_mask))
        loss = {"mse": 0, "huber": 1}[c.critic_loss_type] if critic else 0
        scale = float(self.env_config.obs_log2_scale)
        for k in range(K):
            for s0 in range(0, steps.N, self.grad_chunk_steps):
                m = min(self.grad_chunk_steps, steps.N - s0)
                sel = torch.arange(s0, s0 + m, device=self.device)
                b = steps.boards_at(sel, k)
                acts = tgt = None
                if critic:
                    hn = steps.has_next[sel]
                    vn = self._deep_forward(params, dspec, slot, steps.boards_at(sel, k, nxt=True), 1)[:, 0]
                    tgt = (steps.rewards[sel] + (float(c.gamma) * vn) * hn.to(torch.float32)).contiguous()
                    coef = step_w[sel].contiguous()
                else:
                    acts = steps.actions_k(sel, k).to(torch.uint8).contiguous()
                    coef = (adv[k, sel] * step_w[sel]).contiguous()
                d0 = torch.empty(m, H0p, dtype=torch.float32, device=self.device) if onehot else None
                L.check(self._lib.g2048_deep_grad(L.ptr(packed), L.ptr(bpacked), len(hidden), harr, act, obs_code,
                                                  scale, use_mask, L.ptr(b), L.ptr(acts), L.ptr(coef), int(critic),
                                                  loss, float(c.huber_delta), L.ptr(tgt),
                                                  L.ptr(deltas[k, s0:s0 + m]) if critic else None, None, L.ptr(d0),
                                                  m, L.ptr(part), nparts, None, self._stream))
                self._fold(part, acc)
                if onehot:
                    self._onehot_dw1_into(b, d0, acc1, h1=h0)
        pw, pb = self._deep_slab_layout(hidden, onehot)
        Hp = [_round32(h) for h in hidden]
        acc = acc.to(torch.float32)
        nh = len(hidden)
        if onehot:
            gW[0] += acc1[:272 * h0].view(272, h0).to(torch.float32)
        else:
            gW[0] += acc[pw[0]:pw[0] + 16 * Hp[0]].view(16, Hp[0])[:, :h0]
        gb[0] += acc[pb[0]:pb[0] + Hp[0]][:h0]
        for l in range(1, nh):
            gW[l] += acc[pw[l]:pw[l] + Hp[l - 1] * Hp[l]].view(Hp[l - 1], Hp[l])[:hidden[l - 1], :hidden[l]]
            gb[l] += acc[pb[l]:pb[l] + Hp[l]][:hidden[l]]
        gW[nh] += acc[pw[nh]:pw[nh] + Hp[-1] * 4].view(Hp[-1], 4)[:hidden[-1], :out_dim]
        gb[nh] += acc[pb[nh]:pb[nh] + 4][:out_dim]

    def _td_rows(self, steps: "_Steps", hn_f: torch.Tensor, s0: int, cnt: int, v_next: torch.Tensor,
                 v_out: torch.Tensor):
        """g2048_td_rows of time row [s0, s0 + cnt): the kernel forms r + (gamma V(s')) m from the later row's
        lane-indexed values v_next and writes this row's V(s) by lane into v_out (src/reinforce_agent.py:423-443)."""
        return L.TdRows(L.ptr(steps.lane[s0:s0 + cnt]), L.ptr(steps.rewards[s0:s0 + cnt]), L.ptr(hn_f[s0:s0 + cnt]),
                        L.ptr(v_next), L.ptr(v_out), float(self.agent_config.gamma), 0)

    def _deep_critic_rows(self, params, dspec, steps: "_Steps", K: int, gW: list[torch.Tensor],
                          gb: list[torch.Tensor], step_w: torch.Tensor, deltas: torch.Tensor) -> None:
        """The critic branch through g2048_deep_grad without a separate V(s') forward (as _critic_grad_rows for the
        two-layer kernels): the time rows of the time-major valid steps run LAST first, one launch each, and each
        launch's V(s) (v_out) is the V(s') of the previous row's TD targets (src/reinforce_agent.py:423-443).  The
        trailing short rows run first as one launch with their own V(s') forward (g2048_deep_policy), handing V(s)
        of their first row to the chain.  One-hot first layers: each launch's layer-0 deltas collect in one buffer
        (with their boards) that g2048_onehot_dw1 scatters whenever it is full."""
        c = self.agent_config
        obs_code, hidden, act, harr = dspec
        onehot = obs_code == L.OBS_ONEHOT
        loss = {"mse": 0, "huber": 1}[c.critic_loss_type]
        packed = self._pack_deep(params, dspec, "critic", 1)
        bpacked = self._pack_deep_grad(params, dspec, "critic")
        nparts = int(self._lib.g2048_deep_grad_parts(obs_code, len(hidden), harr))
        slab = int(self._lib.g2048_deep_grad_slab(obs_code, len(hidden), harr))
        part = torch.empty(nparts, slab, dtype=torch.float32, device=self.device)
        acc = torch.zeros(slab, dtype=torch.float64, device=self.device)
        h0, H0p = hidden[0], _round32(hidden[0])
        acc1 = torch.zeros(273 * h0, dtype=torch.float64, device=self.device) if onehot else None
        scale = float(self.env_config.obs_log2_scale)
        gamma = float(c.gamma)
        n = steps.n
        counts = torch.bincount(steps.t, minlength=steps.T).tolist()      # samples per time row (one host sync)
        starts = [0] * len(counts)
        for t in range(1, len(counts)):
            starts[t] = starts[t - 1] + counts[t - 1]
        t_tail, tail_m = len(counts), 0
        while t_tail > 0 and counts[t_tail - 1] < self.critic_tail_row_max:
            t_tail -= 1
            tail_m += counts[t_tail]
        vout = torch.empty(max(max(counts), tail_m, 1), dtype=torch.float32, device=self.device)
        ldb = max(self.grad_chunk_steps, max(counts), tail_m)
        d0buf = torch.empty(ldb, H0p, dtype=torch.float32, device=self.device) if onehot else None
        bbuf = torch.empty(ldb, dtype=torch.int64, device=self.device) if onehot else None
        used = 0

        def flush_d0() -> None:
            nonlocal used
            if onehot and used:
                self._onehot_dw1_into(bbuf[:used], d0buf[:used], acc1, h1=h0)
            used = 0

        allb = steps.boards.reshape(-1)[steps.vidx].contiguous()     # the steps' boards, gathered once
        hn_f = steps.has_next.to(torch.float32)

        def launch(s0: int, cnt: int, tgt, k: int, td=None) -> None:
            nonlocal used
            b = allb[s0:s0 + cnt]
            if k:
                b = self._symmetry_boards(b, k)
            if onehot and used + cnt > ldb:
                flush_d0()
            d0 = d0buf[used:used + cnt] if onehot else None
            L.check(self._lib.g2048_deep_grad(L.ptr(packed), L.ptr(bpacked), len(hidden), harr, act, obs_code, scale,
                                              0, L.ptr(b), None, L.ptr(step_w[s0:s0 + cnt]), 1, loss,
                                              float(c.huber_delta), L.ptr(tgt), L.ptr(deltas[k, s0:s0 + cnt]),
                                              L.ptr(vout), L.ptr(d0), cnt, L.ptr(part), nparts,
                                              ctypes.byref(td) if td is not None else None, self._stream))
            self._fold(part, acc)
            if onehot:
                bbuf[used:used + cnt] = b
                used += cnt

        for k in range(K):
            vb = [torch.zeros(n, dtype=torch.float32, device=self.device) for _ in range(2)]
            if tail_m:
                s0 = starts[t_tail]
                sel = torch.arange(s0, s0 + tail_m, device=self.device)
                hn = steps.has_next[sel]
                vn = self._deep_forward(params, dspec, "critic", steps.boards_at(sel, k, nxt=True), 1)[:, 0]
                launch(s0, tail_m, (steps.rewards[sel] + (gamma * vn) * hn.to(torch.float32)).contiguous(), k)
                if t_tail > 0:
                    vb[t_tail & 1].index_copy_(0, steps.lane[s0:s0 + counts[t_tail]], vout[:counts[t_tail]])
            for t in range(t_tail - 1, -1, -1):
                cnt = counts[t]
                if cnt == 0:
                    continue
                s0 = starts[t]
                launch(s0, cnt, None, k, td=self._td_rows(steps, hn_f, s0, cnt, vb[(t + 1) & 1], vb[t & 1]))
        flush_d0()
        pw, pb = self._deep_slab_layout(hidden, onehot)
        Hp = [_round32(h) for h in hidden]
        acc = acc.to(torch.float32)
        nh = len(hidden)
        if onehot:
            gW[0] += acc1[:272 * h0].view(272, h0).to(torch.float32)
            gb[0] += acc[pb[0]:pb[0] + Hp[0]][:h0]
        else:
            gW[0] += acc[pw[0]:pw[0] + 16 * Hp[0]].view(16, Hp[0])[:, :h0]
            gb[0] += acc[pb[0]:pb[0] + Hp[0]][:h0]
        for l in range(1, nh):
            gW[l] += acc[pw[l]:pw[l] + Hp[l - 1] * Hp[l]].view(Hp[l - 1], Hp[l])[:hidden[l - 1], :hidden[l]]
            gb[l] += acc[pb[l]:pb[l] + Hp[l]][:hidden[l]]
        gW[nh] += acc[pw[nh]:pw[nh] + Hp[-1] * 4].view(Hp[-1], 4)[:hidden[-1], :1]
        gb[nh] += acc[pb[nh]:pb[nh] + 4][:1]

    def _packed_policy(self, spec) -> torch.Tensor:
        """The actor packed in MFMA fragment order (g2048_policy_pack), re-packed whenever a parameter tensor is
        replaced or modified in place (or after an update / load)."""
        return self._pack_net(self.params, spec, "actor")

    def _pack_net(self, params, spec, slot: str, grad: bool = False) -> torch.Tensor:
        """g2048_policy_pack (grad=False) or g2048_grad_pack of W[1] (grad=True) of a two-hidden-layer net, cached
        per slot until a parameter tensor changes; a value head [h2, 1] / [1] is packed as output 0 of 4."""
        Ws, bs = params["W"], params["b"]
        key = (self._params_version,) + tuple((t.data_ptr(), t._version) for t in Ws + bs)
        entry = self._pack_cache.setdefault(slot + ("/grad" if grad else ""), [None, None])
        if key != entry[1]:
            h1, h2, _ = spec
            size = int(self._lib.g2048_grad_packed_size(h1, h2) if grad else self._lib.g2048_policy_packed_size(h1, h2))
            if entry[0] is None or entry[0].numel() < size:
                entry[0] = torch.empty(size, dtype=torch.float32, device=self.device)
            if grad:
                L.check(self._lib.g2048_grad_pack(L.ptr(Ws[1].contiguous()), h1, h2, L.ptr(entry[0]), size, self._stream))
            else:
                W3, b3 = Ws[2], bs[2]
                if W3.shape[1] != 4:
                    W3 = torch.nn.functional.pad(W3, (0, 4 - W3.shape[1]))
                    b3 = torch.nn.functional.pad(b3, (0, 4 - b3.shape[0]))
                w = [t.contiguous() for t in (Ws[0], bs[0], Ws[1], bs[1], W3, b3)]
                L.check(self._lib.g2048_policy_pack(*[L.ptr(t) for t in w], 16, h1, h2, L.ptr(entry[0]), size,
                                                    self._stream))
            entry[1] = key
        return entry[0]

    # columns per g2048_dw2 workgroup: one workgroup per CU at 2^20 columns, never fewer than this many columns each
    dw2_min_cols_per_part = 2048

    def _dw2_parts(self, ncols: int, h2: int) -> tuple[int, int]:
        """(columns per part, parts) of a g2048_dw2* call: one workgroup per part, about one per CU (a 256-wide
        second layer runs one 8-wave workgroup per part)."""
        cus = int(self._lib.g2048_actor_grad_waves()) // 4
        cpp = max(self.dw2_min_cols_per_part, -(-ncols // (16 * max(cus, 1))) * 16)
        return cpp, -(-ncols // cpp)

    def _fold(self, part: torch.Tensor, acc: torch.Tensor) -> None:
        """acc (fp64, contiguous) += the sum of part's rows, taken in fp64 on the device (g2048_fold_partials)."""
        assert acc.dtype == torch.float64 and acc.is_contiguous() and part.is_contiguous()
        slab = acc.numel()
        assert part.numel() % slab == 0
        L.check(self._lib.g2048_fold_partials(L.ptr(part), part.numel() // slab, slab, L.ptr(acc), self._stream))

    def _dw2(self, a1t: torch.Tensor, d2t: torch.Tensor, h1: int, h2: int, ncols: int, acc: torch.Tensor) -> None:
        """acc [H1p + 1, H2p] fp64 += dW2 / db2 of the columns [0, ncols) of the fused kernels' column buffers
        (g2048_dw2: the a1 d2^T outer products on the bf16 MFMA with three-plane fp32-accurate operands, one
        workgroup per CU; its fp32 slabs folded into acc in fp64; row H1p = db2)."""
        H1p, H2p = _padded_units(h1), _padded_units(h2)
        if ncols == 0:
            return
        assert a1t.numel() == d2t.numel() and a1t.shape[0] == max(H1p, H2p)
        assert acc.shape == (H1p + 1, H2p)
        cpp, nparts = self._dw2_parts(ncols, h2)
        part = torch.empty(nparts, H1p + 1, H2p, dtype=torch.float32, device=self.device)
        L.check(self._lib.g2048_dw2(L.ptr(a1t), L.ptr(d2t), h1, h2, int(a1t.shape[1]), 0, ncols, cpp, L.ptr(part),
                                    nparts, self._stream))
        self._fold(part, acc)

    def _dw2_factored(self, a1t: torch.Tensor, rec: torch.Tensor, w3: torch.Tensor, h1: int, h2: int, ncols: int,
                      acc: torch.Tensor) -> None:
        """_dw2 for the ReLU critic's factored d2 form (g2048_critic_grad d2_form 1): the 1 KiB block records (mask
        words + g) instead of d2 columns; g2048_dw2_factored scales by W3[:, 0] (w3, padded to H2p)."""
        H1p, H2p = _padded_units(h1), _padded_units(h2)
        if ncols == 0:
            return
        assert rec.numel() * 4 >= (ncols // 16) * 1024 and w3.numel() == H2p and acc.shape == (H1p + 1, H2p)
        cpp, nparts = self._dw2_parts(ncols, h2)
        part = torch.empty(nparts, H1p + 1, H2p, dtype=torch.float32, device=self.device)
        L.check(self._lib.g2048_dw2_factored(L.ptr(a1t), L.ptr(rec), L.ptr(w3), h1, h2, int(a1t.shape[1]), 0, ncols,
                                             cpp, L.ptr(part), nparts, self._stream))
        self._fold(part, acc)

    def _dw2_actor(self, a1t: torch.Tensor, rec: torch.Tensor, w3: torch.Tensor, h1: int, h2: int, ncols: int,
                   acc: torch.Tensor) -> None:
        """_dw2 for the ReLU actor's d2 block records (g2048_actor_grad d2_form 2): g2048_dw2_actor rebuilds d2 from
        the mask words and g with W3 (w3: [H2p, 4] padded) bit for bit, then sums as g2048_dw2."""
        H1p, H2p = _padded_units(h1), _padded_units(h2)
        if ncols == 0:
            return
        assert rec.numel() * 4 >= (ncols // 16) * 1024 and tuple(w3.shape) == (H2p, 4) and acc.shape == (H1p + 1, H2p)
        cpp, nparts = self._dw2_parts(ncols, h2)
        part = torch.empty(nparts, H1p + 1, H2p, dtype=torch.float32, device=self.device)
        L.check(self._lib.g2048_dw2_actor(L.ptr(a1t), L.ptr(rec), L.ptr(w3), h1, h2, int(a1t.shape[1]), 0, ncols, cpp,
                                          L.ptr(part), nparts, self._stream))
        self._fold(part, acc)

    def _actor_grad_fused(self, steps: "_Steps", adv: torch.Tensor, step_w: torch.Tensor, K: int,
                          gW: list[torch.Tensor], gb: list[torch.Tensor], spec) -> None:
        """The actor branch of update_batch (src/reinforce_agent.py:502-555) for every valid step and symmetry k:
        g2048_actor_grad (forward from the bitboards, masked softmax, deltas, dW1 / db1 / dW3 / db3 per wave)
        plus g2048_dw2 for the layer-2 weight and bias gradient over the a1^T / d2^T columns the kernel writes.
        Accumulates into gW / gb like mlp_backward_."""
        use_mask = int(bool(self.env_config.use_action_mask))
        records = spec[2] == L.ACT_RELU and self.actor_d2_records

        def launch(k, s0, sel, b, m, ld, a1t, d2t, part, waves, packed, gpacked, h1, h2, act, obs_code, scale):
            a = steps.actions_k(sel, k).to(torch.uint8).contiguous()
            coef = (adv[k, sel] * step_w[sel]).contiguous()
            L.check(self._lib.g2048_actor_grad(L.ptr(packed), L.ptr(gpacked), h1, h2, act, obs_code, scale, use_mask,
                                               L.ptr(b), L.ptr(a), L.ptr(coef), m, ld, L.ptr(a1t), L.ptr(d2t),
                                               L.ptr(part), waves, 2 if records else 0, self._stream))

        self._fused_grad(self.params, "actor", spec, steps, K, gW, gb, 4, launch, records=records)

    def _critic_grad_fused(self, steps: "_Steps", step_w: torch.Tensor, K: int, gW: list[torch.Tensor],
                           gb: list[torch.Tensor], deltas: torch.Tensor, spec) -> None:
        """The critic branch of update_batch (src/reinforce_agent.py:403-498, _get_grad_logits_critic :884-910):
        V(s') of every step with a successor by the fused forward (g2048_policy, logits only), the TD target
        r + gamma V(s') m on the device, then g2048_critic_grad (value, TD error into `deltas`, loss gradient and
        backprop) and the same g2048_dw2 pass as the actor."""
        c = self.agent_config
        loss = {"mse": 0, "huber": 1}[c.critic_loss_type]
        flat = steps.boards.reshape(-1)

        def launch(k, s0, sel, b, m, ld, a1t, d2t, part, waves, packed, gpacked, h1, h2, act, obs_code, scale):
            fi, hn = steps.vidx[sel], steps.has_next[sel]
            bn = flat[torch.where(hn, fi + steps.n, fi)].contiguous()
            if k:
                bn = self._symmetry_boards(bn, k)
            lg = torch.empty(m, 4, dtype=torch.float32, device=self.device)
            dummy = torch.empty(m, dtype=torch.uint8, device=self.device)
            L.check(self._lib.g2048_policy(L.ptr(packed), h1, h2, act, L.ptr(bn), None, None, obs_code, scale, 0, 1,
                                           L.RNG_PCG64, None, None, None, 0, None, None, L.ptr(lg), L.ptr(dummy),
                                           m, self._stream))
            tgt = (steps.rewards[sel] + (float(c.gamma) * lg[:, 0]) * hn.to(torch.float32)).contiguous()
            w = step_w[sel].contiguous()
            L.check(self._lib.g2048_critic_grad(L.ptr(packed), L.ptr(gpacked), h1, h2, act, obs_code, scale, loss,
                                                float(c.huber_delta), L.ptr(b), L.ptr(tgt), L.ptr(w),
                                                L.ptr(deltas[k, s0:s0 + m]), None, m, ld, 0, ld, L.ptr(a1t),
                                                L.ptr(d2t), L.ptr(part), 0, waves, 0, None, self._stream))

        if self._critic_by_rows(steps):
            self._critic_grad_rows(steps, step_w, K, gW, gb, deltas, spec)
            return
        self._fused_grad(self.critic_params, "critic", spec, steps, K, gW, gb, 1, launch)

    # the per-row critic pass pays ~7 small launches per time row; worth it from this many samples per row
    critic_rows_min_avg = 16384
    # trailing rows below this many samples run as one "tail" launch with their own V(s') forward: a row launch
    # costs at least one 32-sample group's latency (~115 us on MI355X) however few samples it has, while the tail
    # pays ~1.5x the flops per sample (the extra forward) at full occupancy -- break-even near 28k samples
    critic_tail_row_max = 24576

    def _critic_by_rows(self, steps: "_Steps") -> bool:
        if not self.use_critic_rows or steps.N == 0:
            return False
        T_used = int(steps.lengths.max())
        return steps.N >= self.critic_rows_min_avg * max(T_used, 1) and steps.n + 32 <= (1 << 21) - 2048

    def _critic_grad_rows(self, steps: "_Steps", step_w: torch.Tensor, K: int, gW: list[torch.Tensor],
                          gb: list[torch.Tensor], deltas: torch.Tensor, spec) -> None:
        """The critic branch without a separate V(s') forward: the valid steps are time-major, so the steps of one
        time row are a contiguous range; rows run LAST first, one g2048_critic_grad launch each, and every launch
        returns V(s) of its row (value_out) -- which is the V(s') the previous row's TD targets r + gamma V(s') m need
        (src/reinforce_agent.py:423-443: X_next = the next step's obs).  The launches fill one a1^T / d2^T column
        buffer (column window per row) and accumulate their per-wave partials; the layer-2 GEMM runs once per full
        buffer.  Saves the ~141 kflop / sample V(s') forward of the chunked path.  The trailing short rows (fewer
        than critic_tail_row_max samples each -- episodes have ended) run first as one launch with their own V(s')
        forward, which then hands V(s) of its first row to the per-row chain."""
        c = self.agent_config
        loss = {"mse": 0, "huber": 1}[c.critic_loss_type]
        h1, h2, act = spec
        H1p, H2p = _padded_units(h1), _padded_units(h2)
        params = self.critic_params
        packed, gpacked = self._pack_net(params, spec, "critic"), self._pack_net(params, spec, "critic", grad=True)
        waves = int(self._lib.g2048_actor_grad_waves())
        pf = int(self._lib.g2048_grad_partial_size(h1, h2))
        part = torch.zeros(waves, pf, dtype=torch.float32, device=self.device)
        big = torch.zeros(H1p + 1, H2p, dtype=torch.float64, device=self.device)
        obs_code, scale = _OBS_CODE[self.env_config.obs_mode], float(self.env_config.obs_log2_scale)
        flat = steps.boards.reshape(-1)
        n = steps.n
        counts = torch.bincount(steps.t, minlength=steps.T).tolist()      # samples per time row (one host sync)
        starts = [0] * len(counts)
        for t in range(1, len(counts)):
            starts[t] = starts[t - 1] + counts[t - 1]
        # column-buffer width: a multiple of 2048 columns, so the buffer splits into whole g2048_dw2 parts
        # (dw2_min_cols_per_part) and every row launch's 32-column groups stay inside it
        blk = 2048
        ld = -(-max(self.grad_chunk_steps, max(counts) + 32) // blk) * blk
        # the tail: trailing rows t_tail.. with fewer than critic_tail_row_max samples each, at most ld - 32 in all
        t_tail, tail_m = len(counts), 0
        while t_tail > 0 and counts[t_tail - 1] < self.critic_tail_row_max and tail_m + counts[t_tail - 1] <= ld - 32:
            t_tail -= 1
            tail_m += counts[t_tail]
        R = max(H1p, H2p)
        a1t = torch.empty(R, ld, dtype=torch.float32, device=self.device)     # 16-column blocks (include/g2048.h)
        # ReLU: the factored d2 form -- one 1 KiB record (mask words + g) per 16 columns instead of d2 columns
        fac = act == L.ACT_RELU and self.critic_factored_d2
        if fac:
            d2t = torch.empty(ld // 16 * 256, dtype=torch.float32, device=self.device)
            w3 = torch.zeros(H2p, dtype=torch.float32, device=self.device)
            w3[:h2] = params["W"][2][:, 0]
        else:
            d2t = torch.empty(R, ld, dtype=torch.float32, device=self.device)
        vout = torch.empty(max(max(counts), tail_m), dtype=torch.float32, device=self.device)
        gamma = float(c.gamma)

        small = torch.zeros(pf, dtype=torch.float64, device=self.device)
        launched: list[tuple[int, int, int, int]] = []     # (k, s0, cnt, column) of the launches in the buffer

        def fold() -> None:
            # the per-wave partials accumulate in fp32 across row launches; fold them into fp64 every so often
            self._fold(part, small)
            part.zero_()

        def flush(used: int) -> None:
            nonlocal big
            if used == 0:
                return
            if self.grad_probe is not None:
                for k_, s0_, cnt_, c0 in launched:
                    d2c = _unrecord(d2t, w3, c0, cnt_) if fac else _unblock(d2t, H2p, c0, cnt_)
                    self.grad_probe("critic", k_, torch.arange(s0_, s0_ + cnt_, device=self.device),
                                    _unblock(a1t, H1p, c0, cnt_), d2c)
            launched.clear()
            fold()
            if fac:   # every column < used was written by a row launch
                self._dw2_factored(a1t, d2t, w3, h1, h2, used, big)
            else:
                self._dw2(a1t, d2t, h1, h2, used, big)

        # the steps' boards gathered once (k = 0) instead of per row launch
        allb = flat[steps.vidx].contiguous()
        hn_f = steps.has_next.to(torch.float32)

        def grad_launch(s0: int, cnt: int, tgt, k: int, td=None) -> None:
            nonlocal col, since_fold
            b = allb[s0:s0 + cnt]
            if k:
                b = self._symmetry_boards(b, k)
            ncols = -(-cnt // 32) * 32
            if col + ncols > ld:
                flush(col)
                col = 0
            L.check(self._lib.g2048_critic_grad(L.ptr(packed), L.ptr(gpacked), h1, h2, act, obs_code, scale, loss,
                                                float(c.huber_delta), L.ptr(b), L.ptr(tgt), L.ptr(step_w[s0:s0 + cnt]),
                                                L.ptr(deltas[k, s0:s0 + cnt]), L.ptr(vout), cnt, ld, col, ncols,
                                                L.ptr(a1t), L.ptr(d2t), L.ptr(part), 1, waves, int(fac),
                                                ctypes.byref(td) if td is not None else None, self._stream))
            launched.append((k, s0, cnt, col))
            col += ncols
            since_fold += 1
            if since_fold == 64:
                fold()
                since_fold = 0

        col = 0
        since_fold = 0
        for k in range(K):
            vb = [torch.zeros(n, dtype=torch.float32, device=self.device) for _ in range(2)]
            if tail_m:
                # the tail rows in one launch: V(s') by the fused forward (the successor is the same lane's next
                # row, flat index + n), then V(s) of row t_tail hands over to the per-row chain below
                s0 = starts[t_tail]
                fi, hn = steps.vidx[s0:s0 + tail_m], steps.has_next[s0:s0 + tail_m]
                bn = flat[torch.where(hn, fi + n, fi)].contiguous()
                if k:
                    bn = self._symmetry_boards(bn, k)
                lg = torch.empty(tail_m, 4, dtype=torch.float32, device=self.device)
                dummy = torch.empty(tail_m, dtype=torch.uint8, device=self.device)
                L.check(self._lib.g2048_policy(L.ptr(packed), h1, h2, act, L.ptr(bn), None, None, obs_code, scale, 0,
                                               1, L.RNG_PCG64, None, None, None, 0, None, None, L.ptr(lg),
                                               L.ptr(dummy), tail_m, self._stream))
                tgt = (steps.rewards[s0:s0 + tail_m] + (gamma * lg[:, 0]) * hn.to(torch.float32)).contiguous()
                grad_launch(s0, tail_m, tgt, k)
                if t_tail > 0:
                    vb[t_tail & 1].index_copy_(0, steps.lane[s0:s0 + counts[t_tail]], vout[:counts[t_tail]])
            for t in range(t_tail - 1, -1, -1):
                cnt = counts[t]
                if cnt == 0:
                    continue
                s0 = starts[t]
                # r + (gamma V(s')) m in the kernel from the lane-indexed values of row t + 1 (g2048_td_rows; the
                # same roundings as the chunked path), its V(s) written by lane for row t - 1
                grad_launch(s0, cnt, None, k, td=self._td_rows(steps, hn_f, s0, cnt, vb[(t + 1) & 1], vb[t & 1]))
        flush(col)
        small = small.to(torch.float32)
        big = big.to(torch.float32)
        gW[0] += small[:16 * H1p].view(16, H1p)[:, :h1]
        gb[0] += small[16 * H1p:17 * H1p][:h1]
        gW[1] += big[:h1, :h2]
        gb[1] += big[H1p, :h2]
        gW[2] += small[17 * H1p:17 * H1p + 4 * H2p].view(H2p, 4)[:h2, :1]
        gb[2] += small[17 * H1p + 4 * H2p:][:1]

    def _fused_grad(self, params, slot: str, spec, steps: "_Steps", K: int, gW: list[torch.Tensor],
                    gb: list[torch.Tensor], out_dim: int, launch, records: bool = False) -> None:
        """Chunked driver of the fused gradient kernels: per chunk of valid steps (symmetry k) `launch` runs the
        kernel, then the layer-2 weight + bias gradient a1^T d2 over the kernel's column buffers is g2048_dw2
        (_dw2: bf16 three-plane MFMA, one fp32 slab per workgroup folded into fp64) and the per-wave partials are
        folded into fp64 (g2048_fold_partials); the padded gradients are cut to the net's shapes at the end."""
        h1, h2, act = spec
        H1p, H2p = _padded_units(h1), _padded_units(h2)
        R = max(H1p, H2p)
        packed, gpacked = self._pack_net(params, spec, slot), self._pack_net(params, spec, slot, grad=True)
        waves = int(self._lib.g2048_actor_grad_waves())
        pf = int(self._lib.g2048_grad_partial_size(h1, h2))
        part = torch.empty(waves, pf, dtype=torch.float32, device=self.device)
        # cross-chunk sums in fp64 (the per-chunk results are added into these as fp32 tensors)
        small = torch.zeros(pf, dtype=torch.float64, device=self.device)
        big = torch.zeros(H1p + 1, H2p, dtype=torch.float64, device=self.device)
        obs_code, scale = _OBS_CODE[self.env_config.obs_mode], float(self.env_config.obs_log2_scale)
        flat = steps.boards.reshape(-1)
        if records:   # W3 [H2p, 4] zero-padded: g2048_dw2_actor rebuilds d2 with it
            w3 = torch.zeros(H2p, 4, dtype=torch.float32, device=self.device)
            w3[:h2, :out_dim] = params["W"][2]
        for k in range(K):
            for s0 in range(0, steps.N, self.grad_chunk_steps):
                m = min(self.grad_chunk_steps, steps.N - s0)
                sel = torch.arange(s0, s0 + m, device=self.device)
                b = flat[steps.vidx[sel]].contiguous()
                if k:
                    b = self._symmetry_boards(b, k)
                # column buffers: the kernel writes every column < ld (those past m as zero-coefficient padding)
                ld = -(-m // 32) * 32
                a1t = torch.empty(R, ld, dtype=torch.float32, device=self.device)     # 16-column blocks
                if records:   # one 1 KiB record per 16 columns instead of d2 columns
                    d2t = torch.empty(ld // 16 * 256, dtype=torch.float32, device=self.device)
                else:
                    d2t = torch.empty(R, ld, dtype=torch.float32, device=self.device)
                launch(k, s0, sel, b, m, ld, a1t, d2t, part, waves, packed, gpacked, h1, h2, act, obs_code, scale)
                if self.grad_probe is not None:
                    d2c = _unrecord_actor(d2t, w3, 0, m) if records else _unblock(d2t, H2p, 0, m)
                    self.grad_probe(slot, k, sel, _unblock(a1t, H1p, 0, m), d2c)
                # layer-2 weight + bias gradient, chunks summed in fp64
                if records:
                    self._dw2_actor(a1t, d2t, w3, h1, h2, ld, big)
                else:
                    self._dw2(a1t, d2t, h1, h2, ld, big)
                self._fold(part, small)
        big, small = big.to(torch.float32), small.to(torch.float32)
        gW[0] += small[:16 * H1p].view(16, H1p)[:, :h1]
        gb[0] += small[16 * H1p:17 * H1p][:h1]
        gW[1] += big[:h1, :h2]
        gb[1] += big[H1p, :h2]
        gW[2] += small[17 * H1p:17 * H1p + 4 * H2p].view(H2p, 4)[:h2, :out_dim]
        gb[2] += small[17 * H1p + 4 * H2p:][:out_dim]

    # ============================================================================================ acting
    def select_action(self, obs, rng: np.random.Generator, action_fn: Callable | None = None,
                      use_greedy: bool = False):
        """src/reinforce_agent.py:126-192 for one observation (numpy obs from Game2048Env).  The forward runs on
        the device; the draw uses the caller's numpy Generator exactly like the reference."""
        x, action_mask = encode_observation(obs)
        xt = torch.as_tensor(np.asarray(x, dtype=np.float32), device=self.device).unsqueeze(0)
        logits, acts, pres = forward_logits(self.params, xt, self.mlp_config.activation)
        mk = None if action_mask is None else torch.as_tensor(np.asarray(action_mask), device=self.device).unsqueeze(0)
        probs = logits_to_probs(logits, mk)[0].cpu().numpy()
        action = None
        if action_fn is not None:
            try:
                candidate = int(action_fn(self.env.state if self.env is not None else None, action_mask))
            except Exception as e:  # noqa: BLE001 (same fallback as the reference)
                self._logger.exception(f"action_fn raised an exception: {e}. Falling back to policy.")
            else:
                if not (0 <= candidate < len(probs)):
                    self._logger.warning(f"action_fn returned out-of-range action {candidate}, falling back to policy.")
                elif action_mask is not None and not bool(action_mask[candidate]):
                    self._logger.warning(f"action_fn returned masked-out action {candidate}, falling back to policy.")
                else:
                    action = candidate
        if action is None:
            if use_greedy:
                p = probs * action_mask if action_mask is not None else probs
                action = int(np.argmax(p))
            else:
                action = int(rng.choice(len(probs), p=probs))
        return action, probs, [a[0] for a in acts], [p[0] for p in pres]

    @torch.no_grad()
    def rollout_batch(self, env_seeds, policy_seeds, use_greedy: bool = False, rng: str = "pcg64",
                      check_every: int = 8, record_probs: bool = False) -> TrajectoryBatch:
        """Play one episode per lane (env.reset(seed=env_seeds[i]), policy stream default_rng(policy_seeds[i]))
        until every lane terminates or truncates -- the batched equivalent of calling run_episode for each
        (env_seed, policy_seed) pair (runner.py:587-591).  Everything stays on the device."""
        n = len(env_seeds)
        if len(policy_seeds) != n:
            raise ValueError("env_seeds and policy_seeds must have the same length")
        spec = self._fused_policy_spec()
        if spec is not None and rng == "pcg64" and self.env_config.max_steps is not None and self.use_fused_rollout:
            self._paths["rollout"] = "g2048_rollout (one persistent launch)"
            return self._rollout_fused(env_seeds, policy_seeds, spec, use_greedy, record_probs)
        dspec = self._deep_spec() if self.use_fused_policy else None
        if dspec is not None and rng == "pcg64" and self.use_fused_rollout:
            self._paths["rollout"] = "g2048_deep_rollout (persistent launches, suspended episodes resumed)"
            return self._rollout_deep(env_seeds, policy_seeds, dspec, use_greedy, record_probs)
        if spec is not None:
            dspec = None
        self._paths["rollout"] = ("g2048_policy + g2048_step per step (active lanes)" if spec is not None else
                                  "g2048_deep_policy + g2048_step per step (active lanes)" if dspec is not None else
                                  "hipBLASLt forward (active lanes) + g2048_sample + g2048_step per step")
        env = self._vec_env(n, rng)
        env.reset(seed=_seed_seq(env_seeds))
        dev = self.device
        from .vec_env import _as_u64_seeds

        pseeds = _as_u64_seeds(_seed_seq(policy_seeds), n, 0, dev)
        pst = torch.empty(2 * n, dtype=torch.int64, device=dev)
        pinc = torch.empty(2 * n, dtype=torch.int64, device=dev)
        pbuf = torch.empty(n, dtype=torch.int64, device=dev)
        rng_mode = L.RNG_PCG64 if rng == "pcg64" else L.RNG_PHILOX
        if rng_mode == L.RNG_PCG64:
            L.check(self._lib.g2048_seed_pcg64(L.ptr(pseeds), L.ptr(pst), L.ptr(pinc), L.ptr(pbuf), n, self._stream))
        ms = self.env_config.max_steps
        cap = int(ms) if (ms is not None and ms > 0) else 1024
        cap = max(cap, 1)
        boards = torch.empty(cap, n, dtype=torch.int64, device=dev)
        actions = torch.empty(cap, n, dtype=torch.uint8, device=dev)
        rewards = torch.zeros(cap, n, dtype=torch.float64, device=dev)
        flags = torch.empty(cap, n, dtype=torch.uint8, device=dev)
        probs = torch.zeros(cap, n, 4, dtype=torch.float32, device=dev) if record_probs else None
        # total_reward += float(reward) in step order (src/reinforce_agent.py:233); finished lanes add 0.0
        total = torch.zeros(n, dtype=torch.float64, device=dev)
        # the reference masks the logits only when the obs carries an action mask (encode_observation,
        # src/MLP.py:22-43 -> select_action src/reinforce_agent.py:138-145)
        use_mask = bool(self.env_config.use_action_mask)
        packed = self._packed_policy(spec) if spec is not None else None
        dpacked = self._pack_deep(self.params, dspec, "actor", 4) if dspec is not None else None
        logits_buf = None
        active_idx = None
        t = 0
        while True:
            if t == cap:
                grow = cap
                boards = torch.cat([boards, torch.empty(grow, n, dtype=torch.int64, device=dev)])
                actions = torch.cat([actions, torch.empty(grow, n, dtype=torch.uint8, device=dev)])
                rewards = torch.cat([rewards, torch.zeros(grow, n, dtype=torch.float64, device=dev)])
                flags = torch.cat([flags, torch.empty(grow, n, dtype=torch.uint8, device=dev)])
                if probs is not None:
                    probs = torch.cat([probs, torch.zeros(grow, n, 4, dtype=torch.float32, device=dev)])
                cap += grow
            # the lanes still active at the last check (compacted every check_every steps)
            if active_idx is None or t % check_every == 0:
                active_idx = torch.nonzero(env.active).view(-1).to(torch.int32)
            m = int(active_idx.numel())
            if spec is not None or dspec is not None:
                # fused forward + choice straight from the boards; the step then skips the obs buffer
                common = (L.ptr(env.board), L.ptr(env.state), L.ptr(active_idx) if m < n else None,
                          _OBS_CODE[self.env_config.obs_mode], float(self.env_config.obs_log2_scale), int(use_mask),
                          int(use_greedy), rng_mode, L.ptr(pst), L.ptr(pinc), L.ptr(pbuf), env.philox_key ^ 0x5A5A,
                          L.ptr(pseeds), L.ptr(probs[t]) if probs is not None else None, None, L.ptr(actions[t]),
                          m if m < n else n, self._stream)
                if spec is not None:
                    L.check(self._lib.g2048_policy(L.ptr(packed), spec[0], spec[1], spec[2], *common))
                else:
                    L.check(self._lib.g2048_deep_policy(L.ptr(dpacked), len(dspec[1]), dspec[3], dspec[2], *common))
                env.step_into(actions[t], reward=env.reward, flags=flags[t], prev_board=boards[t], write_obs=False,
                              reward64=rewards[t])
            else:
                if m < n:
                    # forward only the active lanes; finished lanes are skipped by g2048_sample (lane state)
                    if logits_buf is None:
                        logits_buf = torch.zeros(n, 4, dtype=torch.float32, device=dev)
                    ai = active_idx.long()
                    logits_buf.index_copy_(0, ai, self._policy_logits(env.obs.index_select(0, ai)))
                    logits = logits_buf
                else:
                    logits = self._policy_logits(env.obs)
                L.check(self._lib.g2048_sample(L.ptr(logits), L.ptr(env.mask) if use_mask else None,
                                               L.ptr(env.state), int(use_greedy), rng_mode, L.ptr(pst),
                                               L.ptr(pinc), L.ptr(pbuf), env.philox_key ^ 0x5A5A, L.ptr(pseeds),
                                               L.ptr(probs[t]) if probs is not None else None,
                                               L.ptr(actions[t]), n, self._stream))
                env.step_into(actions[t], reward=env.reward, flags=flags[t], prev_board=boards[t],
                              reward64=rewards[t])
            total += rewards[t]      # inactive lanes got reward 0.0
            t += 1
            if t % check_every == 0 and not bool(env.active.any()):
                break
        fl = flags[:t]
        lengths = ((fl & L.F_INACTIVE) == 0).sum(0).to(torch.int32)
        T = int(lengths.max().item()) if n else 0
        return TrajectoryBatch(boards=boards[:T], actions=actions[:T], rewards=rewards[:T],
                               flags=fl[:T], lengths=lengths, total_reward=total,
                               max_tile=env.max_tile_seen.clone(), final_boards=env.board.clone(),
                               probs=probs[:T] if probs is not None else None)

    def _rollout_fused(self, env_seeds, policy_seeds, spec, use_greedy: bool, record_probs: bool) -> TrajectoryBatch:
        """rollout_batch in ONE launch (g2048_rollout): every episode runs to its end inside a persistent kernel
        (fused policy + env step per step, episode slots refilled from a work queue)."""
        from .config import env_cfg_struct
        from .vec_env import _as_u64_seeds

        n = len(env_seeds)
        dev = self.device
        es = _as_u64_seeds(_seed_seq(env_seeds), n, 0, dev)
        ps = _as_u64_seeds(_seed_seq(policy_seeds), n, 0, dev)
        streams = []
        for seeds in (es, ps):
            st = torch.empty(2 * n, dtype=torch.int64, device=dev)
            inc = torch.empty(2 * n, dtype=torch.int64, device=dev)
            buf = torch.empty(n, dtype=torch.int64, device=dev)
            L.check(self._lib.g2048_seed_pcg64(L.ptr(seeds), L.ptr(st), L.ptr(inc), L.ptr(buf), n, self._stream))
            streams += [st, inc, buf]
        cap = max(int(self.env_config.max_steps), 1)
        boards = torch.empty(cap, n, dtype=torch.int64, device=dev)
        actions = torch.zeros(cap, n, dtype=torch.uint8, device=dev)
        rewards = torch.zeros(cap, n, dtype=torch.float64, device=dev)
        flags = torch.full((cap, n), L.F_INACTIVE, dtype=torch.uint8, device=dev)
        probs = torch.zeros(cap, n, 4, dtype=torch.float32, device=dev) if record_probs else None
        lengths = torch.empty(n, dtype=torch.int32, device=dev)
        totals = torch.empty(n, dtype=torch.float64, device=dev)
        max_e = torch.empty(n, dtype=torch.uint8, device=dev)
        final = torch.empty(n, dtype=torch.int64, device=dev)
        queue = torch.zeros(1, dtype=torch.int32, device=dev)
        cfg = env_cfg_struct(self.env_config)
        packed = self._packed_policy(spec)
        L.check(self._lib.g2048_rollout(L.ptr(packed), spec[0], spec[1], spec[2], ctypes.byref(cfg), int(use_greedy),
                                        *[L.ptr(t) for t in streams], L.ptr(queue), n, cap, L.ptr(boards),
                                        L.ptr(actions), L.ptr(rewards), L.ptr(flags),
                                        L.ptr(probs) if probs is not None else None, L.ptr(lengths), L.ptr(totals),
                                        L.ptr(max_e), L.ptr(final), self._stream))
        T = int(lengths.max().item()) if n else 0
        return TrajectoryBatch(boards=boards[:T], actions=actions[:T], rewards=rewards[:T], flags=flags[:T],
                               lengths=lengths, total_reward=totals,
                               max_tile=torch.ones(n, dtype=torch.int64, device=dev) << max_e.to(torch.int64),
                               final_boards=final, probs=probs[:T] if probs is not None else None)

    # first trajectory capacity of g2048_deep_rollout when max_steps is None (doubled while episodes run past it), and
    # the most rows it may grow to (an episode that never ends raises instead of exhausting device memory)
    deep_rollout_cap0 = 512
    deep_rollout_max_rows = 1 << 24

    def _rollout_deep(self, env_seeds, policy_seeds, dspec, use_greedy: bool, record_probs: bool) -> TrajectoryBatch:
        """rollout_batch through g2048_deep_rollout (any depth, one-hot obs, max_steps None): every episode runs
        inside a persistent launch until it ends or fills the trajectory buffer's `cap` rows; the episodes that
        filled it are suspended by the kernel, the buffer grows (x2) and one more launch resumes just those."""
        from .config import env_cfg_struct
        from .vec_env import _as_u64_seeds

        n = len(env_seeds)
        dev = self.device
        es = _as_u64_seeds(_seed_seq(env_seeds), n, 0, dev)
        ps = _as_u64_seeds(_seed_seq(policy_seeds), n, 0, dev)
        streams = []
        for seeds in (es, ps):
            st = torch.empty(2 * n, dtype=torch.int64, device=dev)
            inc = torch.empty(2 * n, dtype=torch.int64, device=dev)
            buf = torch.empty(n, dtype=torch.int64, device=dev)
            L.check(self._lib.g2048_seed_pcg64(L.ptr(seeds), L.ptr(st), L.ptr(inc), L.ptr(buf), n, self._stream))
            streams += [st, inc, buf]
        ms = self.env_config.max_steps
        cap = max(int(ms) if ms is not None else self.deep_rollout_cap0, 1)
        boards = torch.empty(cap, n, dtype=torch.int64, device=dev)
        actions = torch.zeros(cap, n, dtype=torch.uint8, device=dev)
        rewards = torch.zeros(cap, n, dtype=torch.float64, device=dev)
        flags = torch.full((cap, n), L.F_INACTIVE, dtype=torch.uint8, device=dev)
        probs = torch.zeros(cap, n, 4, dtype=torch.float32, device=dev) if record_probs else None
        lengths = torch.empty(n, dtype=torch.int32, device=dev)
        totals = torch.empty(n, dtype=torch.float64, device=dev)
        max_e = torch.empty(n, dtype=torch.uint8, device=dev)
        final = torch.empty(n, dtype=torch.int64, device=dev)
        sus_board = torch.empty(n, dtype=torch.int64, device=dev)
        sus_meta = torch.empty(3 * n, dtype=torch.int32, device=dev)
        sus_total = torch.empty(n, dtype=torch.float64, device=dev)
        sus_list = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        sus_count = torch.zeros(1, dtype=torch.int32, device=dev)
        sus = L.Suspend(*[L.ptr(t) for t in (sus_board, sus_meta, sus_total, sus_list, sus_count)])
        queue = torch.zeros(1, dtype=torch.int32, device=dev)
        cfg = env_cfg_struct(self.env_config)
        packed = self._pack_deep(self.params, dspec, "actor", 4)
        obs_code, hidden, act, harr = dspec
        order, n_order, resume = None, n, 0
        while True:
            traj = L.Traj(*[L.ptr(t) for t in (boards, actions, rewards, flags, probs, lengths, totals, max_e, final)])
            L.check(self._lib.g2048_deep_rollout(L.ptr(packed), len(hidden), harr, act, ctypes.byref(cfg),
                                                 int(use_greedy), *[L.ptr(t) for t in streams], L.ptr(queue),
                                                 L.ptr(order), n_order, resume, ctypes.byref(sus), n, cap,
                                                 ctypes.byref(traj), self._stream))
            k = int(sus_count.item())          # one host sync per launch
            if k == 0:
                break
            order, n_order, resume = sus_list[:k].clone(), k, 1
            queue.zero_()
            sus_count.zero_()
            grow = cap
            # The batch is time-major [T, n] for all n episodes (the update's layout), so a few long episodes grow
            # every lane's rows.  An episode that never ends (max_steps None with invalid actions allowed, where the
            # reference itself would loop forever) must not run the device out of memory: refuse past the rows the
            # free memory holds, or past deep_rollout_max_rows.
            row_bytes = n * (8 + 1 + 8 + 1 + (16 if probs is not None else 0))
            free_b = 1 << 62
            if dev.type == "cuda":
                # free device memory plus what torch's caching allocator holds reserved but unused (torch.cat below
                # reuses or releases that cache before it would fail)
                free_b = (torch.cuda.mem_get_info(dev)[0] + torch.cuda.memory_reserved(dev) -
                          torch.cuda.memory_allocated(dev))
            if cap + grow > self.deep_rollout_max_rows or (cap + grow) * row_bytes > free_b + cap * row_bytes // 2:
                hint = "set max_steps" + ("" if self.env_config.use_action_mask else " or use_action_mask=True")
                raise RuntimeError(
                    f"rollout_batch (max_steps=None): {k} episode(s) still running after {cap} steps; growing the "
                    f"[T, n] trajectory buffer to {cap + grow} rows needs {(cap + grow) * row_bytes / 2**30:.1f} GiB "
                    f"(free: {free_b / 2**30:.1f} GiB, row limit {self.deep_rollout_max_rows}) -- {hint}")
            boards = torch.cat([boards, torch.empty(grow, n, dtype=torch.int64, device=dev)])
            actions = torch.cat([actions, torch.zeros(grow, n, dtype=torch.uint8, device=dev)])
            rewards = torch.cat([rewards, torch.zeros(grow, n, dtype=torch.float64, device=dev)])
            flags = torch.cat([flags, torch.full((grow, n), L.F_INACTIVE, dtype=torch.uint8, device=dev)])
            if probs is not None:
                probs = torch.cat([probs, torch.zeros(grow, n, 4, dtype=torch.float32, device=dev)])
            cap += grow
        T = int(lengths.max().item()) if n else 0
        return TrajectoryBatch(boards=boards[:T], actions=actions[:T], rewards=rewards[:T], flags=flags[:T],
                               lengths=lengths, total_reward=totals,
                               max_tile=torch.ones(n, dtype=torch.int64, device=dev) << max_e.to(torch.int64),
                               final_boards=final, probs=probs[:T] if probs is not None else None)

    def trajectories_from_batch(self, batch: TrajectoryBatch, with_states: bool = True) -> list[dict[str, Any]]:
        """Convert a device batch to the reference's trajectory dicts (src/reinforce_agent.py:240-247)."""
        n, T = batch.n, batch.T
        x, mk = self._obs_from_boards(batch.boards.reshape(-1).contiguous())
        x = x.view(T, n, -1).cpu().numpy()
        mk = mk.view(T, n, 4).cpu().numpy()
        boards = batch.boards.cpu().numpy().view(np.uint64)
        acts = batch.actions.cpu().numpy()
        rews = batch.rewards.cpu().numpy()
        lens = batch.lengths.cpu().numpy()
        tot = batch.total_reward.cpu().numpy()
        mt = batch.max_tile.cpu().numpy()
        shape = (4, 4, 17) if self.input_dim == 272 else (4, 4)
        out = []
        for i in range(n):
            Ti = int(lens[i])
            obs = []
            for t in range(Ti):
                board = x[t, i].reshape(shape).copy()
                obs.append({"board": board, "action_mask": mk[t, i].copy()} if self.env_config.use_action_mask
                           else board)
            traj = {"obs": obs, "actions": [int(a) for a in acts[:Ti, i]],
                    "rewards": [float(r) for r in rews[:Ti, i]], "total_reward": float(tot[i]),
                    "states": [_render_values(_board_values(int(b))) for b in boards[:Ti, i]] if with_states else [],
                    "max_tile": int(mt[i])}
            out.append(traj)
        return out

    def run_episode(self, env_seed: int, policy_seed: int, action_gen: Callable | None = None,
                    use_greedy: bool = False) -> dict[str, Any]:
        """src/reinforce_agent.py:195-252.  Without action_gen the episode runs on the device lane path (same
        spawn and policy streams as the reference); with action_gen it steps the drop-in env from the host."""
        if action_gen is None:
            return self.trajectories_from_batch(self.rollout_batch([env_seed], [policy_seed], use_greedy))[0]
        from .env import Game2048Env

        env = self.env if self.env is not None else Game2048Env(self.env_config, device=self.device)
        saved = self.env
        self.env = env
        try:
            obs, _ = env.reset(seed=env_seed)
            state = env.render(mode="ansi")
            prng = np.random.default_rng(policy_seed)
            traj = {"obs": [], "actions": [], "rewards": [], "states": []}
            total, done = 0.0, False
            while not done:
                a, _, _, _ = self.select_action(obs, prng, action_gen, use_greedy=use_greedy)
                nobs, r, te, tr, _ = env.step(a)
                traj["obs"].append(obs)
                traj["actions"].append(a)
                traj["rewards"].append(float(r))
                traj["states"].append(state)
                total += float(r)
                obs = nobs
                done = te or tr
                state = env.render(mode="ansi")
            traj["total_reward"] = total
            traj["max_tile"] = env.max_tile_seen
            return traj
        finally:
            self.env = saved

    # ============================================================================================ returns
    def compute_returns(self, rewards) -> np.ndarray:
        """src/reinforce_agent.py:255-273 (fp64 scan of the fp64 rewards, fp32 result) on the device."""
        r = torch.as_tensor(np.asarray(rewards, dtype=np.float64), device=self.device).view(-1, 1).contiguous()
        T = r.shape[0]
        out = torch.zeros(T, 1, dtype=torch.float32, device=self.device)
        ln = torch.full((1,), T, dtype=torch.int32, device=self.device)
        L.check(self._lib.g2048_returns(L.ptr(r), L.ptr(ln), float(self.agent_config.gamma), L.ptr(out), T, 1,
                                        self._stream))
        return out.view(-1).cpu().numpy()

    def _returns_tm(self, rewards_tm: torch.Tensor, lengths: torch.Tensor) -> torch.Tensor:
        T, n = rewards_tm.shape
        out = torch.zeros(T, n, dtype=torch.float32, device=self.device)
        ln = lengths.to(torch.int32).contiguous()
        L.check(self._lib.g2048_returns(L.ptr(rewards_tm.to(torch.float64).contiguous()), L.ptr(ln), float(self.agent_config.gamma),
                                        L.ptr(out), T, n, self._stream))
        return out

    # ============================================================================================ weights & baselines
    def _compute_episode_rank_weights(self, totals: torch.Tensor, sizes=None) -> torch.Tensor:
        """src/reinforce_agent.py:681-716 on the global batch (dp.rank_weights; `sizes` = every rank's episode
        count when known, else one host-synchronising size exchange under data parallelism)."""
        return dp.rank_weights(totals, self.agent_config.reward_rank_weights, sizes=sizes)

    def _advantages(self, values: torch.Tensor, lane: torch.Tensor, n_lanes: int, step_rank_w: torch.Tensor) -> torch.Tensor:
        """_compute_advantages (src/reinforce_agent.py:276-325) + _compute_weighted_stats (:864-881) over flat
        steps, on the device; 'batch' statistics are global across ranks (dp.batch_mean_std: one tiny
        all-reduce, no host sync).  As in the reference, mean and std are applied in fp32."""
        mode = self.agent_config.baseline_mode
        if mode == "off":
            return values
        if mode == "each":
            s = torch.zeros(n_lanes, dtype=torch.float64, device=self.device).index_add_(0, lane, values.double())
            c = torch.zeros(n_lanes, dtype=torch.float64, device=self.device).index_add_(
                0, lane, torch.ones_like(values, dtype=torch.float64))
            mean = (s / c.clamp(min=1)).to(torch.float32)
            return values - mean[lane]
        if mode not in ("batch", "batch_norm"):
            raise ValueError(f"Unknown baseline mode: {mode}")
        mean, std = dp.batch_mean_std(values, step_rank_w)
        if mode == "batch":
            return values - mean.to(torch.float32)
        return (values - mean.to(torch.float32)) / std.clamp(min=1e-8).to(torch.float32)

    # ============================================================================================ optimiser
    def _init_adam(self, params, prefix="actor"):
        """src/reinforce_agent.py:811-832"""
        z = lambda ts: [torch.zeros_like(t) for t in ts]  # noqa: E731
        if prefix == "actor":
            self._adam_m_W, self._adam_v_W = z(params["W"]), z(params["W"])
            self._adam_m_B, self._adam_v_B = z(params["b"]), z(params["b"])
        else:
            self._adam_m_W_c, self._adam_v_W_c = z(params["W"]), z(params["W"])
            self._adam_m_B_c, self._adam_v_B_c = z(params["b"]), z(params["b"])

    def _clip_(self, grads: list[torch.Tensor]) -> torch.Tensor:
        """clip_grads_global_norm on the device: fp32 L2 over all W then all b, scaled in place by
        max_norm / norm when that is < 1 (a multiply by exactly 1.0 otherwise).  Returns the norm as a device
        scalar -- no host synchronisation."""
        max_norm = self.agent_config.max_grad_norm
        sq = torch.zeros((), dtype=torch.float32, device=self.device)
        for g in grads:
            sq = sq + torch.linalg.vector_norm(g.float()) ** 2
        total = torch.sqrt(sq)
        coef = torch.tensor(np.float32(max_norm), device=self.device) / total.clamp(min=1e-8)
        coef = torch.where(coef < 1.0, coef, torch.ones_like(coef))
        for g in grads:
            g.mul_(coef)
        return total

    def clip_grads_global_norm(self, grad_W_list, grad_b_list):
        """src/reinforce_agent.py:835-861: scale the gradients in place if their global norm exceeds max_grad_norm;
        returns the (pre-clip) norm as a Python float like the reference."""
        return float(self._clip_(list(grad_W_list) + list(grad_b_list)))

    def _adam_update(self, grad_W_list, grad_b_list, prefix="actor") -> None:
        """src/reinforce_agent.py:719-770 (fp32, eps outside the sqrt, separate step counters)."""
        c = self.agent_config
        if prefix == "actor":
            P, mW, vW, mB, vB = self.params, self._adam_m_W, self._adam_v_W, self._adam_m_B, self._adam_v_B
            self._adam_t += 1
            t, lr, sign = self._adam_t, c.learning_rate, 1.0
        else:
            P, mW, vW, mB, vB = (self.critic_params, self._adam_m_W_c, self._adam_v_W_c, self._adam_m_B_c,
                                 self._adam_v_B_c)
            self._adam_t_c += 1
            t, lr, sign = self._adam_t_c, c.critic_learning_rate, -1.0
        b1, b2, eps = c.adam_beta1, c.adam_beta2, 1e-8
        bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
        for key, m, v, G in (("W", mW, vW, grad_W_list), ("b", mB, vB, grad_b_list)):
            for l in range(len(P[key])):
                m[l].mul_(b1).add_(G[l] * (1.0 - b1))
                v[l].mul_(b2).add_((G[l] * G[l]) * (1.0 - b2))
                P[key][l] = P[key][l] + sign * lr * (m[l] / bc1) / (torch.sqrt(v[l] / bc2) + eps)

    # ============================================================================================ update
    def update_batch(self, trajectories: list[dict[str, Any]]) -> None:
        """src/reinforce_agent.py:357-620 on reference-format trajectories (obs as numpy dicts/arrays)."""
        n = len(trajectories)
        lens = [len(tr["obs"]) for tr in trajectories]
        if n == 0:
            return
        T = max(lens) if lens else 0
        D = self.input_dim
        X = np.zeros((T, n, D), dtype=np.float32)
        M = np.ones((T, n, 4), dtype=np.int8)
        A = np.zeros((T, n), dtype=np.uint8)
        R = np.zeros((T, n), dtype=np.float64)     # the trajectories' Python floats
        for i, tr in enumerate(trajectories):
            for t, o in enumerate(tr["obs"]):
                x, m = encode_observation(o)
                X[t, i] = x
                if m is not None:
                    M[t, i] = m
            A[:lens[i], i] = tr["actions"]
            R[:lens[i], i] = tr["rewards"]
        dev = self.device
        totals = torch.tensor([float(tr["total_reward"]) for tr in trajectories], dtype=torch.float64, device=dev)
        steps = _Steps(self, torch.tensor(lens, device=dev), torch.from_numpy(A).to(dev), torch.from_numpy(R).to(dev),
                       X=torch.from_numpy(X).to(dev), M=torch.from_numpy(M).to(dev))
        self._update(steps, totals)

    def update_from_batch(self, batch: TrajectoryBatch) -> dict:
        """update_batch on a device TrajectoryBatch (the hot path: no host round trip)."""
        steps = _Steps(self, batch.lengths, batch.actions, batch.rewards, boards=batch.boards)
        return self._update(steps, batch.total_reward, batch.shard_sizes)

    def _chunks(self, N: int, size: int | None = None):
        size = size or self.chunk_steps
        for s in range(0, N, size):
            yield torch.arange(s, min(N, s + size), device=self.device)

    def _update(self, steps: _Steps, totals: torch.Tensor, shard_sizes=None) -> dict:
        """update_batch (src/reinforce_agent.py:357-620) on a batch of valid steps.  Per-step weights are
        rank_w / T_i; the 1 / n_traj factor is applied after the gradient all-reduce (dp.reduce_gradients_), so the
        data-parallel update needs ONE gradient collective and nothing synchronises the host before the final
        statistics."""
        c = self.agent_config
        n_local = steps.n
        K = 8 if c.augmentation else 1
        rank_w = self._compute_episode_rank_weights(totals, shard_sizes)  # [n_local]
        lane = steps.lane
        lens_f = steps.lengths.to(torch.float64)
        step_w = (rank_w[lane].double() / lens_f[lane]).to(torch.float32)   # rank_w / T_i (1 / n: after the reduce)

        actor_g = [torch.zeros_like(p) for p in self.params["W"] + self.params["b"]]
        critic_g = None
        if c.use_critic:
            critic_g = [torch.zeros_like(p) for p in self.critic_params["W"] + self.critic_params["b"]]
            deltas = torch.empty(K, steps.N, dtype=torch.float32, device=self.device)
            ncW = len(self.critic_params["W"])
            cspec = (self._fused_critic_spec() if steps.boards is not None and c.critic_loss_type in ("mse", "huber")
                     else None)
            self._paths["critic_grad"] = "g2048_critic_grad + g2048_dw2" if cspec is not None else "hipBLASLt backprop"
            if cspec is not None:
                with torch.no_grad():
                    self._critic_grad_fused(steps, step_w, K, critic_g[:ncW], critic_g[ncW:], deltas, cspec)
            cdg = (self._deep_grad_spec(self.critic_params, 1) if cspec is None and steps.boards is not None and
                   c.critic_loss_type in ("mse", "huber") else None)
            if cdg is not None:
                self._paths["critic_grad"] = "g2048_deep_grad" + (" + g2048_onehot_dw1" if
                                                                 cdg[0] == L.OBS_ONEHOT else "")
                with torch.no_grad():
                    if self._critic_by_rows(steps):
                        self._paths["critic_grad"] += " (time rows, last first)"
                        self._deep_critic_rows(self.critic_params, cdg, steps, K, critic_g[:ncW], critic_g[ncW:],
                                               step_w, deltas)
                    else:
                        self._deep_grad_fused(self.critic_params, "critic", cdg, steps, K, critic_g[:ncW],
                                              critic_g[ncW:], 1, step_w=step_w, deltas=deltas)
                cspec = cdg      # handled: skip the torch loop below
            cdspec = self._deep_spec(self.critic_params, 1) if cspec is None and steps.boards is not None else None
            oh1 = self._onehot_first_layer(steps) and cspec is None
            acc1c = torch.zeros(273 * int(self.critic_params["W"][0].shape[1]), dtype=torch.float64,
                                device=self.device) if oh1 else None
            if cspec is None:
                self._paths["critic_grad"] = (("g2048_onehot_layer1 + hipBLASLt backprop + g2048_onehot_dw1"
                                               if oh1 else "hipBLASLt backprop") +
                                              ("; V(s') by g2048_deep_policy" if cdspec is not None else ""))
            for k in range(K if cspec is None else 0):
                for sel in self._chunks(steps.N):
                    with torch.no_grad():
                        v, kept, bsel, _ = self._forward_kept_steps(self.critic_params, steps, sel, k)
                        v = v.view(-1)
                        hn = steps.has_next[sel]
                        # V(s'): the step itself where there is no successor (masked below)
                        if cdspec is not None:
                            vn = self._deep_forward(self.critic_params, cdspec, "critic",
                                                    steps.boards_at(sel, k, nxt=True), 1)[:, 0]
                        else:
                            xn, _ = steps.features(sel, k, nxt=True)
                            vn = forward_logits(self.critic_params, xn, self.mlp_config.activation,
                                                keep_cache=False)[0].view(-1)
                        r = steps.rewards[sel]
                        tgt = r + (float(c.gamma) * vn) * hn.to(torch.float32)
                        deltas[k, sel] = tgt - v
                        diff = v - tgt
                        if c.critic_loss_type == "mse":
                            g = diff
                        elif c.critic_loss_type == "huber":
                            g = torch.where(diff.abs() <= c.huber_delta, diff,
                                            float(c.huber_delta) * torch.sign(diff))
                        else:
                            raise ValueError(f"Unknown critic loss type: {c.critic_loss_type}")
                        g = g * step_w[sel]
                        fl = (lambda d, b_=bsel: self._onehot_dw1_into(b_, d, acc1c)) if bsel is not None else None
                        mlp_backward_(self.critic_params, kept, self.mlp_config.activation, g.unsqueeze(1),
                                      critic_g[:ncW], critic_g[ncW:], first_layer_grad=fl)
            if acc1c is not None:
                h1c = int(self.critic_params["W"][0].shape[1])
                critic_g[0] += acc1c[:272 * h1c].view(272, h1c).to(torch.float32)
                critic_g[ncW] += acc1c[272 * h1c:].to(torch.float32)
            # advantages from TD errors, over all K x n "episodes"
            lane_k = (torch.arange(K, device=self.device).unsqueeze(1) * n_local + lane.unsqueeze(0)).reshape(-1)
            adv = self._advantages(deltas.reshape(-1), lane_k, K * n_local,
                                   rank_w[lane].repeat(K)).view(K, steps.N)
        else:
            G = self._returns_tm(steps.rewards_tm, steps.lengths).reshape(-1)[steps.vidx]
            adv1 = self._advantages(G, lane, n_local, rank_w[lane])
            adv = adv1.unsqueeze(0).expand(K, -1)

        nW = len(self.params["W"])
        gspec = self._fused_grad_spec() if steps.boards is not None else None
        self._paths["actor_grad"] = "g2048_actor_grad + g2048_dw2" if gspec is not None else "hipBLASLt backprop"
        adg = self._deep_grad_spec(self.params, 4) if gspec is None and steps.boards is not None else None
        with torch.no_grad():
            if gspec is not None:
                self._actor_grad_fused(steps, adv, step_w, K, actor_g[:nW], actor_g[nW:], gspec)
            elif adg is not None:
                self._paths["actor_grad"] = "g2048_deep_grad" + (" + g2048_onehot_dw1" if adg[0] == L.OBS_ONEHOT
                                                                 else "")
                self._deep_grad_fused(self.params, "actor", adg, steps, K, actor_g[:nW], actor_g[nW:], 4, adv=adv,
                                      step_w=step_w)
                gspec = adg      # handled: skip the torch loop below
            oh1 = gspec is None and self._onehot_first_layer(steps)
            acc1 = torch.zeros(273 * int(self.params["W"][0].shape[1]), dtype=torch.float64,
                               device=self.device) if oh1 else None
            if gspec is None and oh1:
                self._paths["actor_grad"] = "g2048_onehot_layer1 + hipBLASLt backprop + g2048_onehot_dw1"
            for k in range(K if gspec is None else 0):
                for sel in self._chunks(steps.N):
                    logits, kept, bsel, mk = self._forward_kept_steps(self.params, steps, sel, k, want_mask=True)
                    if steps.boards is not None and not self.env_config.use_action_mask:
                        mk = None   # bare-board obs: unmasked probabilities, as select_action used them
                    p = logits_to_probs(logits, mk)
                    onehot = torch.nn.functional.one_hot(steps.actions_k(sel, k), 4).to(torch.float32)
                    g = (onehot - p) * (adv[k, sel] * step_w[sel]).unsqueeze(1)
                    fl = (lambda d, b_=bsel: self._onehot_dw1_into(b_, d, acc1)) if bsel is not None else None
                    mlp_backward_(self.params, kept, self.mlp_config.activation, g, actor_g[:nW], actor_g[nW:],
                                  first_layer_grad=fl)
            if acc1 is not None:
                h1 = int(self.params["W"][0].shape[1])
                actor_g[0] += acc1[:272 * h1].view(272, h1).to(torch.float32)
                actor_g[nW] += acc1[272 * h1:].to(torch.float32)

            # ONE collective: actor + critic gradients and the episode count; then the 1 / n_traj weight
            dp.reduce_gradients_(actor_g + (critic_g or []), n_local * K)
            self.last_grads = {"actor": [g.clone() for g in actor_g],
                               "critic": [g.clone() for g in critic_g] if critic_g else None}
            gW, gb = actor_g[:nW], actor_g[nW:]
            norms = [self._clip_(actor_g)]
            if c.use_critic:
                ncW = len(self.critic_params["W"])
                gWc, gbc = critic_g[:ncW], critic_g[ncW:]
                norms.append(self._clip_(critic_g))
            if c.optimizer == "sgd":
                for l in range(nW):
                    self.params["W"][l] = self.params["W"][l] + c.learning_rate * gW[l]
                    self.params["b"][l] = self.params["b"][l] + c.learning_rate * gb[l]
                if c.use_critic:
                    for l in range(ncW):
                        self.critic_params["W"][l] = self.critic_params["W"][l] - c.critic_learning_rate * gWc[l]
                        self.critic_params["b"][l] = self.critic_params["b"][l] - c.critic_learning_rate * gbc[l]
            elif c.optimizer == "adam":
                self._adam_update(gW, gb)
                if c.use_critic:
                    self._adam_update(gWc, gbc, prefix="critic")
            else:
                raise ValueError(f"Unknown optimizer: {c.optimizer}")
        self._params_version += 1
        vals = torch.stack(norms).tolist()          # the update's only host synchronisation
        stats = {"actor_grad_norm": vals[0]}
        if c.use_critic:
            stats["critic_grad_norm"] = vals[1]
        if self._logger.isEnabledFor(logging.INFO):
            self._log_update(stats, adv.reshape(-1))   # the augmented list when augmentation is on (:596)
        self.last_stats = stats
        return stats

    def _log_update(self, stats: dict, adv: torch.Tensor) -> None:
        """The INFO log lines of src/reinforce_agent.py:585-620 (gradient norms, advantage statistics)."""
        self._logger.info(f"Global Grad Norms: Actor: {stats['actor_grad_norm']:.4f}")
        if "critic_grad_norm" in stats:
            self._logger.info(f"Global Grad Norms: Critic: {stats['critic_grad_norm']:.4f}")
        if adv.numel() == 0:
            return
        a = adv.float()
        k = min(5, a.numel())
        top = a[torch.topk(a.abs(), k).indices].tolist()
        self._logger.info("Advantages stats: mean=%.6f, std=%.6f, min=%.6f, max=%.6f, pos=%d, neg=%d, total=%d, "
                          "top|A|=%s", float(a.mean()), float(a.std(unbiased=False)), float(a.min()), float(a.max()),
                          int((a > 0).sum()), int((a < 0).sum()), a.numel(), ", ".join(f"{v:.4f}" for v in top))
