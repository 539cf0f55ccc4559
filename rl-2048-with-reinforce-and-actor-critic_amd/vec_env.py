"""VecGame2048Env: n 2048 boards stepped together on one HIP device by libg2048.so.

The batched form of Game2048Env (src/env.py:44-302) and Game2048 (src/game2048.py:11-237).  Per-lane state
lives in device tensors (structure of arrays, see include/g2048.h ``g2048_lanes``); every call is one kernel
launch on the current torch stream and never synchronises the host.

Observations follow src/env.py:131-159 (+ the flattening of src/MLP.py:22-43): ``obs["board"]`` is
float32 [n,4,4] (raw / log2) or [n,4,4,17] (onehot) and ``obs["action_mask"]`` int8 [n,4].  The returned tensors
are the env's own buffers and are overwritten by the next step (clone to keep them).  Lanes that finished
(without auto-reset) keep their final obs and report ``F_INACTIVE`` until reset.
"""
from __future__ import annotations

import ctypes
import secrets

import numpy as np
import torch

from . import _lib as L
from .config import Game2048EnvConfig, env_cfg_struct, obs_width


def _signed64(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= 1 << 63 else v


def _as_u64_seeds(seed, n: int, offset: int, device) -> torch.Tensor:
    """seed: None (fresh entropy, like Game2048._set_seed src/game2048.py:103-104), int (lane i gets
    seed + offset + i, mod 2**64), or a sequence / tensor of n seeds (python ints in [0, 2**64)).
    Returned as int64 tensors holding the uint64 bit patterns."""
    if seed is None:
        seed = secrets.randbits(63)
    if isinstance(seed, int):
        if seed < 0:
            raise ValueError("expected non-negative integer")  # numpy SeedSequence raises the same
        return torch.arange(n, dtype=torch.int64, device=device) + _signed64(seed + offset)
    if isinstance(seed, torch.Tensor):
        if seed.numel() != n:
            raise ValueError(f"expected {n} seeds, got {seed.numel()}")
        return seed.to(device=device, dtype=torch.int64).contiguous()
    # fast path: numpy range-checks a list of python ints in C (negative or >= 2**64 raise OverflowError);
    # integer arrays are checked for negatives here (numpy casts arrays with wraparound)
    try:
        if isinstance(seed, np.ndarray):
            arr = None
            if seed.dtype.kind in "iu" and seed.ndim == 1 and not (seed.dtype.kind == "i" and bool((seed < 0).any())):
                arr = seed.astype(np.uint64, copy=False)
        elif isinstance(seed, (list, tuple)) and all(type(v) is int for v in seed[:8]):
            arr = np.array(seed, dtype=np.uint64)
        else:
            arr = None
        if arr is not None and arr.ndim == 1 and arr.size == n:
            return torch.from_numpy(np.ascontiguousarray(arr).view(np.int64)).to(device)
    except (OverflowError, TypeError, ValueError):
        pass   # the checks below produce the reference's error messages
    vals = [int(s) for s in seed]
    if len(vals) != n:
        raise ValueError(f"expected {n} seeds, got {len(vals)}")
    for v in vals:
        if v < 0:
            raise ValueError("expected non-negative integer")
        if v >= 1 << 64:
            raise ValueError("seeds >= 2**64 are not supported by the device SeedSequence")
    return torch.tensor([_signed64(v) for v in vals], dtype=torch.int64, device=device)


class VecGame2048Env:
    """n independent Game2048Env lanes on one device.

    rng="pcg64": every lane's spawn stream is numpy's default_rng(seed) (bit-exact with the reference).
    rng="philox": Philox4x32-10 keyed by (philox_key, lane seed, step) -- same distribution, no RNG state traffic.
    auto_reset: a lane that terminates/truncates restarts in the same call with seed += reset_stride.
    lane_offset: global index of lane 0 (for sharding a global board batch across ranks).
    track_score: keep Game2048.score per lane (info["score"]) from the step's score increment (one small torch op
    per step); off for pure throughput runs.
    Lane state lives in one uint32 word per lane (include/g2048.h G2048_LS_*): ``step_count``, ``max_tile``,
    ``status`` and ``active`` are views computed from it.
    packed_mask: the steps write the action mask as one byte per lane (``mask_bits``, bit a = action a) instead
    of int8[4] -- 3 B less per board-step; ``obs["action_mask"]`` is then unpacked from it on access.
    """

    def __init__(self, num_envs: int, config: Game2048EnvConfig | None = None, device=None, rng: str = "pcg64",
                 auto_reset: bool = False, reset_stride: int | None = None, philox_key: int = 0x2048,
                 lane_offset: int = 0, record_merged: bool = False, record_prev_board: bool = False,
                 record_reward64: bool = False, track_score: bool = True, packed_mask: bool = False):
        if num_envs <= 0:
            raise ValueError("num_envs must be positive")
        self.config = config or Game2048EnvConfig()
        self._cfg = env_cfg_struct(self.config)          # validates modes (ValueError like src/env.py:110,223,249)
        self.n = int(num_envs)
        if rng not in ("pcg64", "philox"):
            raise ValueError(f"Unsupported rng: {rng}")
        if rng == "philox" and self.config.max_steps is None:
            # the Philox counter of the spawn / policy draws is the lane's 20-bit step count: past 2**20 - 1 steps
            # of one episode the draws would repeat (and a lane repeating an unmasked invalid action never ends)
            raise ValueError("rng='philox' needs a finite max_steps (<= "
                             f"{L.MAX_STEPS_LIMIT}): its draw counter is the 20-bit lane step count")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        L.ensure_device(self.device)
        self.rng_mode = L.RNG_PCG64 if rng == "pcg64" else L.RNG_PHILOX
        self.auto_reset = bool(auto_reset)
        self.reset_stride = int(reset_stride if reset_stride is not None else num_envs)
        self.philox_key = int(philox_key) & 0xFFFFFFFFFFFFFFFF
        self.lane_offset = int(lane_offset)
        n, dev = self.n, self.device
        z = lambda dt, *s: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        # lane state (g2048_lanes)
        self.board = z(torch.int64, n)
        self.state = z(torch.int32, n)                   # G2048_LS_* word (uint32 bits in an int32 tensor)
        self.seed = z(torch.int64, n)
        pcg = self.rng_mode == L.RNG_PCG64
        self.rng_state = z(torch.int64, 2 * n) if pcg else None
        self.rng_inc = z(torch.int64, 2 * n) if pcg else None
        self.rng_uint = z(torch.int32, n) if pcg else None
        self.score = z(torch.int64, n) if track_score else None
        self._score_add = z(torch.int32, n) if track_score else None
        # outputs (g2048_step_out)
        self.reward = z(torch.float32, n)
        # the fp64 reward (the Python float src/env.py:261 returns); off by default: +8 B per board-step
        self.reward64 = z(torch.float64, n) if record_reward64 else None
        self.flags = z(torch.uint8, n)
        self.mask = z(torch.int8, n, 4)                  # written by reset (and by steps unless packed_mask)
        self.mask_bits = z(torch.uint8, n) if packed_mask else None
        self.obs_width = obs_width(self.config.obs_mode)
        self.obs = z(torch.float32, n, self.obs_width)
        self.merged = z(torch.int32, n) if record_merged else None
        self.prev_board = z(torch.int64, n) if record_prev_board else None
        self._lanes = L.Lanes(*[L.ptr(t) for t in (self.board, self.state, self.seed, self.rng_state, self.rng_inc,
                                                   self.rng_uint)])
        self._out = L.StepOut(L.ptr(self.reward), L.ptr(self.flags), self._mask_ptr(), L.ptr(self.obs),
                              L.ptr(self.merged), L.ptr(self.prev_board), L.ptr(self.reward64), L.ptr(self._score_add),
                              L.ptr(self.mask_bits))
        self._lib = L.lib()
        self._stream = L.stream_handle(self.device)

    # ------------------------------------------------------------------------------------------------------
    def _mask_ptr(self):
        return None if self.mask_bits is not None else L.ptr(self.mask)

    @property
    def action_mask(self) -> torch.Tensor:
        """int8 [n, 4]: the action mask of every lane's current board."""
        if self.mask_bits is None:
            return self.mask
        bits = torch.tensor([1, 2, 4, 8], dtype=torch.uint8, device=self.device)
        return ((self.mask_bits.unsqueeze(1) & bits) != 0).to(torch.int8)

    def _obs_view(self):
        board = self.obs.view(self.n, 4, 4, 17) if self.obs_width == 272 else self.obs.view(self.n, 4, 4)
        if self.config.use_action_mask:
            return {"board": board, "action_mask": self.action_mask}
        return board

    def reset(self, *, seed=None, options=None, mask: torch.Tensor | None = None):
        """Game2048Env.reset (src/env.py:174-194) for every lane (or the lanes where ``mask`` is nonzero).
        Returns (obs, info) with info = {"score", "board"}."""
        seeds = _as_u64_seeds(seed, self.n, self.lane_offset, self.device)
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            L.check(self._lib.g2048_reset(ctypes.byref(self._lanes), L.ptr(seeds), L.ptr(m), ctypes.byref(self._cfg),
                                          self.rng_mode, self.philox_key, L.ptr(self.mask), L.ptr(self.obs), self.n,
                                          L.stream_handle(self.device)))
        if self.score is not None:
            if m is None:
                self.score.zero_()
            else:
                self.score.masked_fill_(m != 0, 0)
        if self.mask_bits is not None:
            # reset writes the int8[4] form for the lanes it resets; steps write only the packed form, so
            # self.mask is stale on every other lane: repack the reset lanes only
            w = torch.tensor([1, 2, 4, 8], dtype=torch.int32, device=self.device)
            packed = ((self.mask != 0).to(torch.int32) * w).sum(1).to(torch.uint8)
            if m is None:
                self.mask_bits.copy_(packed)
            else:
                self.mask_bits.copy_(torch.where(m != 0, packed, self.mask_bits))
        return self._obs_view(), {"score": self.score, "board": self.board}

    def step_into(self, actions: torch.Tensor, reward: torch.Tensor | None = None, flags: torch.Tensor | None = None,
                  prev_board: torch.Tensor | None = None, write_obs: bool = True,
                  reward64: torch.Tensor | None = None) -> None:
        """Launch one step writing reward/flags (and the pre-step board, the fp64 reward) into caller tensors
        (trajectory rows).  write_obs=False skips the obs buffer (its consumer reads the boards itself, e.g.
        g2048_policy)."""
        if actions.dtype != torch.uint8 or actions.device != self.device or actions.numel() != self.n:
            raise ValueError("actions must be a uint8 tensor of num_envs elements on the env device")
        out = self._out
        if reward is not None or flags is not None or prev_board is not None or not write_obs or reward64 is not None:
            out = L.StepOut(L.ptr(reward if reward is not None else self.reward),
                            L.ptr(flags if flags is not None else self.flags), self._mask_ptr(),
                            L.ptr(self.obs) if write_obs else None,
                            L.ptr(self.merged), L.ptr(prev_board if prev_board is not None else self.prev_board),
                            L.ptr(reward64 if reward64 is not None else self.reward64), L.ptr(self._score_add),
                            L.ptr(self.mask_bits))
        if torch.cuda.current_device() != self.device.index:
            with torch.cuda.device(self.device):
                return self.step_into(actions, reward, flags, prev_board, write_obs, reward64)
        L.check(self._lib.g2048_step(ctypes.byref(self._lanes), L.ptr(actions), ctypes.byref(self._cfg),
                                     ctypes.byref(out), self.rng_mode, self.philox_key, int(self.auto_reset),
                                     self.reset_stride, self.n, L.stream_handle(self.device)))
        if self.score is not None:   # Game2048.score += sum(merged); an auto-reset lane starts its new game at 0
            fl = flags if flags is not None else self.flags
            self.score.add_(self._score_add).masked_fill_((fl & L.F_RESET) != 0, 0)

    def step(self, actions):
        """Game2048Env.step (src/env.py:264-302) for every lane.  actions: int tensor/sequence of n in 0..3.
        Returns (obs, reward[n], terminated[n] bool, truncated[n] bool, info); reward is fp64 when the env records
        it (record_reward64=True), else its fp32 rounding."""
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(actions)
        if a.dtype.is_floating_point:
            raise AssertionError("Invalid action dtype")
        a = a.to(device=self.device, dtype=torch.uint8 if a.dtype == torch.uint8 else torch.int64)
        if a.dtype != torch.uint8:
            if bool(((a < 0) | (a > 3)).any()):
                raise AssertionError("Invalid action: outside 0..3")
            a = a.to(torch.uint8)
        self.step_into(a.contiguous())
        f = self.flags
        info = {"score": self.score, "flags": f, "changed": (f & L.F_CHANGED) != 0,
                "invalid_action": (f & L.F_INVALID) != 0, "step_index": self.step_count,
                "reset": (f & L.F_RESET) != 0, "overflow": (f & L.F_OVERFLOW) != 0}
        if self.merged is not None:
            info["merged_packed"] = self.merged
        rew = self.reward64 if self.reward64 is not None else self.reward
        return (self._obs_view(), rew, (f & L.F_TERMINATED) != 0, (f & L.F_TRUNCATED) != 0, info)

    # ---- views of the lane state word
    @property
    def step_count(self) -> torch.Tensor:
        """Game2048Env._step_count per lane (int32)."""
        return self.state & L.LS_STEP_MASK

    @property
    def max_tile(self) -> torch.Tensor:
        """log2(Game2048Env.max_tile_seen) per lane (int32)."""
        return (self.state >> L.LS_MAXT_SHIFT) & 31

    @property
    def status(self) -> torch.Tensor:
        """1 where the lane is in an episode, else 0 (uint8)."""
        return ((self.state & L.LS_ACTIVE) != 0).to(torch.uint8)

    @property
    def active(self) -> torch.Tensor:
        return (self.state & L.LS_ACTIVE) != 0

    def set_active(self, lanes: torch.Tensor | None = None) -> None:
        """Mark lanes (all, or a bool mask) as in-episode again (the single-board drop-ins keep stepping a finished
        game, as the reference allows)."""
        on = self.state | L.LS_ACTIVE
        if lanes is None:
            self.state.copy_(on)
        else:
            self.state.copy_(torch.where(lanes, on, self.state))

    def set_lane_state(self, step_count=None, max_tile_exp=None, active=None) -> None:
        """Overwrite fields of every lane's state word (synthetic workloads / tests)."""
        st = self.state
        if step_count is not None:
            st = (st & ~L.LS_STEP_MASK) | (torch.as_tensor(step_count, device=self.device).to(torch.int32) & L.LS_STEP_MASK)
        if max_tile_exp is not None:
            st = (st & ~(31 << L.LS_MAXT_SHIFT)) | ((torch.as_tensor(max_tile_exp, device=self.device).to(torch.int32)
                                                     & 31) << L.LS_MAXT_SHIFT)
        if active is not None:
            a = torch.as_tensor(active, device=self.device).to(torch.bool)
            st = torch.where(a, st | L.LS_ACTIVE, st & ~L.LS_ACTIVE)
        self.state.copy_(st)

    @property
    def max_tile_seen(self) -> torch.Tensor:
        """Game2048Env.max_tile_seen per lane (4 at reset; raised by merges >= 8, src/env.py:238-250)."""
        return torch.ones_like(self.state, dtype=torch.int64) << self.max_tile.to(torch.int64)

    def boards_exponents(self) -> torch.Tensor:
        """[n,4,4] int64 exponents (0 = empty) of the current boards."""
        b = self.board
        shifts = torch.arange(0, 64, 4, device=self.device, dtype=torch.int64)
        return ((b.unsqueeze(1) >> shifts) & 15).view(self.n, 4, 4)

    def boards_values(self) -> torch.Tensor:
        e = self.boards_exponents()
        return torch.where(e > 0, torch.ones_like(e) << e, torch.zeros_like(e))


def decode_merged(word: int) -> list[int]:
    """g2048_step_out.merged -> the reference's merged list (tile values, src/game2048.py:131)."""
    out = []
    w = int(word) & 0xFFFFFFFF
    for k in range(8):
        nib = (w >> (4 * k)) & 15
        if nib == 0:
            break
        out.append(1 << (nib + 1))
    return out
