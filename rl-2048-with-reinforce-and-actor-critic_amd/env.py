"""Drop-in single-board classes with the reference's API, running on the HIP path (B = 1 lane).

* ``Game2048``  -- src/game2048.py:11-237 (reset / step / get_action_mask / render / state / score)
* ``Game2048Env`` -- src/env.py:44-398 (reset / step / render / get_symmetries / state / max_tile_seen)

Each call is one kernel launch plus a small device->host copy: convenient for code written against the
reference, not the fast path (use VecGame2048Env / the batched agent for throughput).
"""
from __future__ import annotations

from typing import Any

import numpy as np
import torch

from . import _lib as L
from .config import Game2048EnvConfig
from .vec_env import VecGame2048Env, decode_merged

Action = int  # 0:up, 1: right, 2: down, 3: left


class Discrete:
    """The slice of gymnasium.spaces.Discrete the reference uses (src/env.py:70, :265)."""

    def __init__(self, n: int):
        self.n = n

    def contains(self, x) -> bool:
        # gymnasium's Discrete.contains: a Python int (bool included) or an integer numpy scalar / 0-d array
        if isinstance(x, int) or (isinstance(x, (np.generic, np.ndarray)) and x.shape == () and
                                  np.issubdtype(x.dtype, np.integer)):
            return 0 <= int(x) < self.n
        return False


def _render(state: list[list[int]]) -> str:
    """Game2048.render (src/game2048.py:73-93) output format."""
    width = max(4, max((len(str(x)) for row in state for x in row), default=1))
    sep = "+" + "+".join(["-" * width] * len(state)) + "+"
    lines = [sep]
    for row in state:
        lines.append("|" + "|".join(f"{x}".rjust(width) if x else " ".rjust(width) for x in row) + "|")
        lines.append(sep)
    return "\n".join(lines)


def _values(b: int) -> np.ndarray:
    e = np.array([(b >> (4 * i)) & 15 for i in range(16)], dtype=np.int64).reshape(4, 4)
    return np.where(e > 0, np.left_shift(np.int64(1), e), 0).astype(np.int64)


class Game2048:
    """src/game2048.py:Game2048 on one device lane.  Tile values are exact up to 2**15; a 2**15+2**15
    merge saturates on the board (``overflow`` becomes True) while step()'s merged list and score stay exact."""

    def __init__(self, size: int = 4, device=None):
        if size != 4:
            raise ValueError("only size=4 boards are supported")
        self.size = size
        self._vec = VecGame2048Env(1, Game2048EnvConfig(max_steps=None), device=device, record_merged=True)
        self._host_board = np.zeros((4, 4), dtype=np.int64)
        self.step_count = 0
        self.score = 0
        self.overflow = False

    def _pull(self) -> None:
        vals = torch.stack([self._vec.board, self._vec.score.to(torch.int64),
                            self._vec.flags.to(torch.int64), self._vec.merged.to(torch.int64)]).cpu().tolist()
        b, score, flags, merged = [int(v[0]) for v in vals]
        self._host_board = _values(b & 0xFFFFFFFFFFFFFFFF)
        self.score = score
        return flags, merged

    @property
    def board(self) -> np.ndarray:
        return self._host_board.copy()

    @property
    def state(self) -> list[list[int]]:
        return self._host_board.tolist()

    def reset(self, seed: int | None = None) -> list[list[int]]:
        self._vec.reset(seed=seed)
        self._pull()
        self.step_count = 0
        self.overflow = False
        return self.state

    def step(self, action: Action) -> tuple[bool, list[list[int]], list[int], bool]:
        if action not in (0, 1, 2, 3):
            raise ValueError("invalid action")
        self._vec.step_into(torch.full((1,), int(action), dtype=torch.uint8, device=self._vec.device))
        self.step_count += 1
        flags, merged = self._pull()
        self.overflow |= bool(flags & L.F_OVERFLOW)
        # the vectorised env deactivates a lane once it is done; Game2048 keeps accepting steps (the
        # reference never stops a finished game), so re-activate it
        if flags & L.F_TERMINATED:
            self._vec.set_active()
        return bool(flags & L.F_CHANGED), self.state, decode_merged(merged), bool(flags & L.F_TERMINATED)

    def get_action_mask(self) -> list[int]:
        return [int(x) for x in self._vec.mask[0].cpu().tolist()]

    def render(self) -> str:
        return _render(self.state)


class Game2048Env:
    """src/env.py:Game2048Env on one device lane: same config, obs (numpy), reward (python float), flags."""

    metadata = {"render_modes": ["human", "ansi"]}

    def __init__(self, config: Game2048EnvConfig | None = None, device=None) -> None:
        self.config = config or Game2048EnvConfig()
        self._vec = VecGame2048Env(1, self.config, device=device, record_merged=True, record_reward64=True)
        self._max_num = 16.0
        self.action_space = Discrete(4)
        self._step_count = 0
        self.max_tile_seen = 4
        self._board = np.zeros((4, 4), dtype=np.int64)
        self._score = 0

    # -------------------------------------------------------------------------------------------- helpers
    @property
    def state(self) -> list[list[int]]:
        return self._board.tolist()

    def _sync(self):
        v = self._vec
        ints = torch.stack([v.board, v.score.to(torch.int64), v.flags.to(torch.int64), v.merged.to(torch.int64),
                            v.max_tile.to(torch.int64), v.step_count.to(torch.int64)]).cpu()
        b, score, flags, merged, mt, sc = [int(x) for x in ints[:, 0].tolist()]
        obs = v.obs[0].cpu().numpy().copy()
        mask = v.mask[0].cpu().numpy().copy()
        reward = float(v.reward64[0].item())    # fp64, as src/env.py:261 returns it
        self._board = _values(b & 0xFFFFFFFFFFFFFFFF)
        self._score = score
        self.max_tile_seen = 1 << mt
        return obs, mask, reward, flags, merged

    def _obs(self, obs: np.ndarray, mask: np.ndarray):
        board = obs.reshape(4, 4, 17) if obs.size == 272 else obs.reshape(4, 4)
        if self.config.use_action_mask:
            return {"board": board, "action_mask": mask.astype(np.int8)}
        return board

    # ------------------------------------------------------------------------------------------------ API
    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        self._vec.reset(seed=seed)
        self._step_count = 0
        obs, mask, _, _, _ = self._sync()
        self.max_tile_seen = 4
        return self._obs(obs, mask), {"score": self._score, "raw_state": self.state}

    def step(self, action: Action):
        assert self.action_space.contains(action), f"Invalid action: {action}"
        self._step_count += 1
        self._vec.step_into(torch.full((1,), int(action), dtype=torch.uint8, device=self._vec.device))
        obs, mask, reward, flags, merged = self._sync()
        terminated = bool(flags & L.F_TERMINATED)
        truncated = bool(flags & L.F_TRUNCATED)
        invalid = bool(flags & L.F_INVALID)
        if terminated or truncated:
            self._vec.set_active()  # the reference env keeps stepping after the end if asked to
        info = {"score": self._score, "raw_state": self.state, "merged": decode_merged(merged),
                "invalid_action": invalid, "step_index": self._step_count}
        return self._obs(obs, mask), float(reward), terminated, truncated, info

    def render(self, mode: str = "human") -> str | None:
        text = _render(self.state)
        if mode == "human":
            print(text)
            return None
        if mode == "ansi":
            return text
        raise NotImplementedError(f"Unsupported render mode: {mode}")

    @staticmethod
    def get_symmetries(obs, action: Action):
        """src/env.py:317-398: the 8 dihedral copies of one (obs, action) pair (host-side utility)."""
        def rot_a(a):
            return (a - 1) % 4

        def flip_a(a):
            return {1: 3, 3: 1}.get(a, a)

        if isinstance(obs, dict):
            board, mask = obs["board"], obs["action_mask"]
        else:
            board, mask = obs, None
        out = []
        for start_board, start_a, start_m in ((board.copy(), action, None if mask is None else mask.copy()),
                                              (np.fliplr(board.copy()), flip_a(action),
                                               None if mask is None else mask[[0, 3, 2, 1]])):
            b, a, m = start_board, start_a, start_m
            for _ in range(4):
                out.append(({"board": b, "action_mask": m}, a) if m is not None else (b, a))
                b = np.rot90(b, k=1, axes=(0, 1))
                a = rot_a(a)
                m = np.roll(m, shift=-1) if m is not None else None
        return out
