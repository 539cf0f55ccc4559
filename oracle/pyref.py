"""CPU ORACLE -- test infrastructure and bench.py's cpu_baseline leg only (never imported by the product).

A pure-Python + NumPy restatement of the reference's CPU step loop, Game2048 (src/game2048.py) driven by
Game2048Env (src/env.py), kept in the reference's own representation and cost model so that its speed on a host
core stands in for the reference on the GPU box (where /root/reference does not exist):
  * the board is an int64 4x4 array of tile values;
  * a move rotates the board clockwise 3 - action times with np.rot90, slides every row left with a Python
    loop over its tiles, and rotates back (src/game2048.py:120-165);
  * the spawn draws from numpy's Generator(PCG64): integers(#empty) over np.argwhere's row-major order, then
    random() < 0.9 for a 2 (src/game2048.py:108-118);
  * done / action mask / reward / obs / truncation follow src/game2048.py:95-99, :172-237 and src/env.py:131-302.
It is pinned bit for bit (boards, fp64 rewards, flags, obs, masks) to the real src/env.py outputs in
tests/golden/env_steps.npz by tests/test_oracle_ref_fixtures.py; tools/pyref_ratio.py measures its speed against
the real reference in the build container (profiles/round2/pyref_ratio.txt).
"""
from __future__ import annotations

import os
import time

import numpy as np

OBS_WIDTH = {"raw": 16, "log2": 16, "onehot": 272}


class PyGame:
    """Game2048 (src/game2048.py:11-237) restated."""

    def __init__(self):
        self.board = np.zeros((4, 4), dtype=np.int64)
        self.score = 0
        self.step_count = 0
        self.rng = np.random.default_rng(0)

    def reset(self, seed: int) -> None:
        self.rng = np.random.default_rng(seed)
        self.board = np.zeros((4, 4), dtype=np.int64)
        self.score = 0
        self.step_count = 0
        self.spawn()
        self.spawn()

    def spawn(self) -> None:
        free = np.argwhere(self.board == 0)
        if len(free):
            r, c = free[self.rng.integers(len(free))]
            self.board[r, c] = 2 if self.rng.random() < 0.9 else 4

    @staticmethod
    def slide_left(row, merged: list | None) -> list[int]:
        """One row pushed left, equal neighbours merged once, left to right."""
        tiles = [int(v) for v in row if v]
        out, i = [], 0
        while i < len(tiles):
            if i + 1 < len(tiles) and tiles[i] == tiles[i + 1]:
                out.append(tiles[i] * 2)
                if merged is not None:
                    merged.append(tiles[i] * 2)
                i += 2
            else:
                out.append(tiles[i])
                i += 1
        return out + [0] * (4 - len(out))

    def moved(self, action: int, merged: list | None) -> tuple[np.ndarray, bool]:
        turns = 3 - action                                   # clockwise quarter turns into the move-left frame
        frame = np.rot90(self.board, -turns)
        slid = np.array([self.slide_left(r, merged) for r in frame], dtype=np.int64)
        return np.rot90(slid, turns), not np.array_equal(slid, frame)

    def done(self) -> bool:
        b = self.board
        if (b == 0).any():
            return False
        return not ((b[:, 1:] == b[:, :-1]).any() or (b[1:, :] == b[:-1, :]).any())

    def step(self, action: int):
        if action not in (0, 1, 2, 3):
            raise ValueError("invalid action")
        self.step_count += 1
        merged: list[int] = []
        nb, changed = self.moved(action, merged)
        self.board = np.ascontiguousarray(nb)
        self.score += sum(merged)
        if changed:
            self.spawn()
        return changed, merged, self.done()

    def action_mask(self) -> list[int]:
        return [int(self.moved(a, None)[1]) for a in range(4)]


class PyEnv:
    """Game2048Env (src/env.py:44-302) over PyGame: reward, truncation, obs and mask."""

    def __init__(self, obs_mode="raw", obs_log2_scale=1.0, reward_mode="sum", base_reward_scale=1.0,
                 empty_tile_reward=0.0, merge_reward=0.0, bonus_mode="off", bonus_scale=1.0, step_reward=0.0,
                 endgame_penalty=0.0, use_action_mask=True, invalid_action_penalty=-1.0, max_steps=1024, size=4):
        self.c = dict(obs_mode=obs_mode, obs_log2_scale=obs_log2_scale, reward_mode=reward_mode,
                      base_reward_scale=base_reward_scale, empty_tile_reward=empty_tile_reward,
                      merge_reward=merge_reward, bonus_mode=bonus_mode, bonus_scale=bonus_scale,
                      step_reward=step_reward, endgame_penalty=endgame_penalty, use_action_mask=use_action_mask,
                      invalid_action_penalty=invalid_action_penalty, max_steps=max_steps)
        self.game = PyGame()
        self.steps = 0
        self.max_tile_seen = 4

    def reset(self, seed: int):
        self.steps = 0
        self.max_tile_seen = 4
        self.game.reset(seed)
        return self.obs()

    def reward(self, merged: list[int], done: bool, invalid: bool) -> float:
        c = self.c
        if not c["use_action_mask"] and invalid:
            return c["invalid_action_penalty"]
        if c["reward_mode"] == "sum":
            r = float(sum(merged))
        elif c["reward_mode"] == "log2":
            r = 0.0
            for v in merged:
                r += float(np.log2(v))
        else:
            raise ValueError(f"Unsupported reward mode: {c['reward_mode']}")
        r *= c["base_reward_scale"]
        if c["empty_tile_reward"] != 0.0:
            r += c["empty_tile_reward"] * float(np.sum(self.game.board == 0))
        if c["merge_reward"] != 0.0:
            r += c["merge_reward"] * float(len(merged))
        top = max(merged, default=0)
        if top >= 8 and top > self.max_tile_seen:
            bonus = {"off": 0.0, "raw": float(top), "log2": float(np.log2(top))}[c["bonus_mode"]]
            self.max_tile_seen = top
            r += bonus * c["bonus_scale"]
        r += c["step_reward"]
        if done and c["endgame_penalty"] != 0.0:
            r += c["endgame_penalty"]
        return r

    def obs(self) -> np.ndarray:
        """_preprocess_board flattened (src/env.py:131-150, src/MLP.py:41)."""
        b = self.game.board.astype(np.float32)
        mode = self.c["obs_mode"]
        if mode == "raw":
            return b.reshape(-1)
        nz = b > 0
        if mode == "log2":
            out = np.zeros_like(b)
            out[nz] = np.log2(b[nz])
            return (out * self.c["obs_log2_scale"]).reshape(-1)
        e = np.zeros((4, 4), dtype=np.int64)
        e[nz] = np.log2(b[nz]).astype(np.int64)
        return np.eye(17, dtype=np.float32)[e].reshape(-1)

    def step(self, action: int):
        self.steps += 1
        changed, merged, done = self.game.step(action)
        invalid = not changed and not done
        r = self.reward(merged, done, invalid)
        ms = self.c["max_steps"]
        truncated = ms is not None and self.steps >= ms and not done
        return r, done, truncated, invalid


def _bench_worker(args) -> int:
    """One process: `boards` envs stepped round-robin with uniform random actions (invalid moves included), obs +
    action mask materialised every step, auto-reset on termination / truncation; stops after `seconds`."""
    wid, boards, seconds, cfg = args
    rng = np.random.default_rng(wid)
    envs = [PyEnv(**cfg) for _ in range(boards)]
    seeds = [1000 + wid * boards + i for i in range(boards)]
    for e, s in zip(envs, seeds):
        e.reset(s)
    steps = 0
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        for i, e in enumerate(envs):
            r, done, trunc, _ = e.step(int(rng.integers(4)))
            e.obs()
            e.game.action_mask()
            steps += 1
            if done or trunc:
                seeds[i] += 1 << 20
                e.reset(seeds[i])
    return steps


def bench(cores: int, seconds: float, cfg: dict, boards_per_core: int = 64) -> tuple[int, float]:
    """CPU baseline: one process per core (OMP/OPENBLAS threads 1), each running its own boards for `seconds`.
    Returns (env steps, wall seconds)."""
    import multiprocessing as mp

    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        steps = sum(pool.map(_bench_worker, [(w, boards_per_core, seconds, cfg) for w in range(cores)]))
    return steps, time.perf_counter() - t0
