"""Game2048EnvConfig (src/env.py:19-40) with the same field names and defaults, and its C-ABI image."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Literal

from . import _lib as L

ObsMode = Literal["raw", "log2", "onehot"]
RewardMode = Literal["sum", "log2"]
BonusMode = Literal["off", "raw", "log2"]

_OBS = {"raw": L.OBS_RAW, "log2": L.OBS_LOG2, "onehot": L.OBS_ONEHOT}
_REWARD = {"sum": 0, "log2": 1}
_BONUS = {"off": 0, "raw": 1, "log2": 2}


@dataclass
class Game2048EnvConfig:
    size: int = 4
    # obs
    obs_mode: ObsMode = "raw"
    obs_log2_scale: float = 1.0
    # basic reward
    reward_mode: RewardMode = "sum"
    base_reward_scale: float = 1.0
    # additional rewards
    empty_tile_reward: float = 0.0
    merge_reward: float = 0.0
    # record bonus
    bonus_mode: BonusMode = "off"
    bonus_scale: float = 1.0
    # step and endgame rewards
    step_reward: float = 0.0
    endgame_penalty: float = 0.0
    # action mask
    use_action_mask: bool = True
    invalid_action_penalty: float = -1.0
    max_steps: int | None = 1024


def obs_width(obs_mode: str) -> int:
    if obs_mode not in _OBS:
        raise ValueError(f"Unsupported obs_mode: {obs_mode}")
    return 272 if obs_mode == "onehot" else 16


def env_cfg_struct(cfg: Game2048EnvConfig) -> L.EnvCfg:
    """Validate and convert.  Raises ValueError with the reference's messages (src/env.py:110,223,249);
    the reference raises the reward/bonus ones lazily at the first step, this build at construction."""
    if cfg.size != 4:
        raise ValueError("only size=4 boards are supported (uint64 bitboard)")
    if cfg.obs_mode not in _OBS:
        raise ValueError(f"Unsupported obs_mode: {cfg.obs_mode}")
    if cfg.reward_mode not in _REWARD:
        raise ValueError(f"Unsupported reward mode: {cfg.reward_mode}")
    if cfg.bonus_mode not in _BONUS:
        raise ValueError(f"Unsupported bonus mode: {cfg.bonus_mode}")
    c = L.EnvCfg()
    c.obs_mode = _OBS[cfg.obs_mode]
    c.reward_mode = _REWARD[cfg.reward_mode]
    c.bonus_mode = _BONUS[cfg.bonus_mode]
    c.use_action_mask = int(bool(cfg.use_action_mask))
    c.obs_log2_scale = float(cfg.obs_log2_scale)
    for k in ("base_reward_scale", "empty_tile_reward", "merge_reward", "bonus_scale", "step_reward",
              "endgame_penalty", "invalid_action_penalty"):
        setattr(c, k, float(getattr(cfg, k)))
    # None -> -1 (never truncate); any int n truncates once _step_count >= n (n <= 0: at the first step)
    c.max_steps = -1 if cfg.max_steps is None else max(int(cfg.max_steps), 0)
    if c.max_steps > L.MAX_STEPS_LIMIT:
        raise ValueError(f"max_steps must be <= {L.MAX_STEPS_LIMIT} on the device (20-bit lane step count) or None")
    return c
