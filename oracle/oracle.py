"""CPU ORACLE -- test infrastructure only.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module,
and only as the checker (or the reported CPU baseline).  The product package never imports it.

ctypes front-end for ``oracle/g2048_oracle.c`` (the literal CPU restatement of src/game2048.py and
src/env.py plus numpy's PCG64 stream) and small helpers to pack/unpack boards.  The numpy restatement of
the agent's update math lives in ``oracle/agent_oracle.py``.  Pinning status: see the C file's header and
DESIGN.md "Oracle".
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    """Compile liboracle.so with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class PCG64State(ctypes.Structure):
    _fields_ = [("state_lo", ctypes.c_uint64), ("state_hi", ctypes.c_uint64),
                ("inc_lo", ctypes.c_uint64), ("inc_hi", ctypes.c_uint64),
                ("has_uint32", ctypes.c_uint32), ("uinteger", ctypes.c_uint32)]


class GameState(ctypes.Structure):
    _fields_ = [("board", ctypes.c_int64 * 16), ("step_count", ctypes.c_int64), ("score", ctypes.c_int64),
                ("rng", PCG64State), ("merged", ctypes.c_int64 * 8), ("n_merged", ctypes.c_int32),
                ("_pad", ctypes.c_int32)]


class EnvCfg(ctypes.Structure):
    _fields_ = [("obs_mode", ctypes.c_int32), ("reward_mode", ctypes.c_int32), ("bonus_mode", ctypes.c_int32),
                ("use_action_mask", ctypes.c_int32), ("obs_log2_scale", ctypes.c_double),
                ("base_reward_scale", ctypes.c_double), ("empty_tile_reward", ctypes.c_double),
                ("merge_reward", ctypes.c_double), ("bonus_scale", ctypes.c_double),
                ("step_reward", ctypes.c_double), ("endgame_penalty", ctypes.c_double),
                ("invalid_action_penalty", ctypes.c_double), ("max_steps", ctypes.c_int64)]


class EnvState(ctypes.Structure):
    _fields_ = [("game", GameState), ("step_count", ctypes.c_int64), ("max_tile_seen", ctypes.c_int64)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        L.or_seedseq_state4.argtypes = [ctypes.c_uint64, P(ctypes.c_uint64)]
        L.or_pcg64_seed.argtypes = [ctypes.c_uint64, P(PCG64State)]
        L.or_pcg64_next64.argtypes = [P(PCG64State)]
        L.or_pcg64_next64.restype = ctypes.c_uint64
        L.or_pcg64_next32.argtypes = [P(PCG64State)]
        L.or_pcg64_next32.restype = ctypes.c_uint32
        L.or_pcg64_random.argtypes = [P(PCG64State)]
        L.or_pcg64_random.restype = ctypes.c_double
        L.or_pcg64_integers.argtypes = [P(PCG64State), ctypes.c_int64]
        L.or_pcg64_integers.restype = ctypes.c_int64
        L.or_choice4.argtypes = [P(PCG64State), P(ctypes.c_float)]
        L.or_choice4.restype = ctypes.c_int
        L.or_game_reset.argtypes = [P(GameState), ctypes.c_uint64]
        L.or_game_step.argtypes = [P(GameState), ctypes.c_int, P(ctypes.c_int32), P(ctypes.c_int32)]
        L.or_game_step.restype = ctypes.c_int
        L.or_game_mask.argtypes = [P(GameState), P(ctypes.c_int8)]
        L.or_game_is_done.argtypes = [P(GameState)]
        L.or_game_is_done.restype = ctypes.c_int
        L.or_env_reset.argtypes = [P(EnvState), ctypes.c_uint64]
        L.or_env_step.argtypes = [P(EnvState), P(EnvCfg), ctypes.c_int, P(ctypes.c_double), P(ctypes.c_int32),
                                  P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_int32)]
        L.or_env_step.restype = ctypes.c_int
        L.or_env_obs.argtypes = [P(EnvState), P(EnvCfg), P(ctypes.c_float)]
        L.or_env_obs.restype = ctypes.c_int
        L.or_pack_board.argtypes = [P(ctypes.c_int64), P(ctypes.c_uint64)]
        L.or_pack_board.restype = ctypes.c_int
        L.or_unpack_board.argtypes = [ctypes.c_uint64, P(ctypes.c_int64)]
        L.or_move_packed.argtypes = [ctypes.c_uint64, ctypes.c_int, P(ctypes.c_uint64), P(ctypes.c_int64),
                                     P(ctypes.c_int32), P(ctypes.c_int32)]
        L.or_move_packed.restype = ctypes.c_int
        L.or_philox4x32_10.argtypes = [P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32)]
        L.or_env_reset_philox.argtypes = [P(EnvState), ctypes.c_uint64, ctypes.c_uint64]
        L.or_env_step_philox.argtypes = [P(EnvState), P(EnvCfg), ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                         P(ctypes.c_double), P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_int32),
                                         P(ctypes.c_int32)]
        L.or_env_step_philox.restype = ctypes.c_int
        L.or_bench_env_steps.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, P(EnvCfg),
                                         P(ctypes.c_double)]
        L.or_bench_env_steps.restype = ctypes.c_int64
        for name, T in (("or_sizeof_game", GameState), ("or_sizeof_env", EnvState), ("or_sizeof_env_cfg", EnvCfg)):
            fn = getattr(L, name)
            fn.restype = ctypes.c_int
            assert fn() == ctypes.sizeof(T), f"struct layout mismatch for {T.__name__}"
        _lib = L
    return _lib


# ---------------------------------------------------------------------------------------------- RNG
class PCG64:
    """numpy ``default_rng(seed)`` stream restated in C (see g2048_oracle.c)."""

    def __init__(self, seed: int):
        self.st = PCG64State()
        lib().or_pcg64_seed(ctypes.c_uint64(seed), ctypes.byref(self.st))

    @property
    def state128(self) -> tuple[int, int]:
        return ((self.st.state_hi << 64) | self.st.state_lo, (self.st.inc_hi << 64) | self.st.inc_lo)

    def next64(self) -> int:
        return lib().or_pcg64_next64(ctypes.byref(self.st))

    def next32(self) -> int:
        return lib().or_pcg64_next32(ctypes.byref(self.st))

    def random(self) -> float:
        return lib().or_pcg64_random(ctypes.byref(self.st))

    def integers(self, n: int) -> int:
        return lib().or_pcg64_integers(ctypes.byref(self.st), n)

    def choice4(self, probs) -> int:
        p = (ctypes.c_float * 4)(*[float(x) for x in np.asarray(probs, dtype=np.float32)])
        return lib().or_choice4(ctypes.byref(self.st), p)


# ---------------------------------------------------------------------------------------------- boards
def pack_exponents(exps) -> int:
    """16 exponents (row-major, nibble r*4+c) -> uint64 bitboard."""
    x = 0
    for i, e in enumerate(np.asarray(exps).reshape(16)):
        x |= int(e) << (4 * i)
    return x


def unpack_exponents(x: int) -> np.ndarray:
    return np.array([(int(x) >> (4 * i)) & 15 for i in range(16)], dtype=np.int64).reshape(4, 4)


def values_to_exponents(vals) -> np.ndarray:
    v = np.asarray(vals, dtype=np.int64)
    out = np.zeros_like(v)
    nz = v > 0
    out[nz] = np.round(np.log2(v[nz])).astype(np.int64)
    return out


def move_packed(board: int, action: int):
    """Pre-spawn move of a packed board (src/game2048.py:158-165). Returns (board', merged list, changed, ok)."""
    out = ctypes.c_uint64()
    merged = (ctypes.c_int64 * 8)()
    nm = ctypes.c_int32()
    ch = ctypes.c_int32()
    rc = lib().or_move_packed(ctypes.c_uint64(board), action, ctypes.byref(out), merged, ctypes.byref(nm), ctypes.byref(ch))
    return int(out.value), [int(merged[i]) for i in range(nm.value)], bool(ch.value), rc == 0


# ---------------------------------------------------------------------------------------------- game / env
class Game:
    """Oracle twin of src/game2048.py:Game2048 (values, not exponents)."""

    def __init__(self):
        self.g = GameState()

    def reset(self, seed: int):
        lib().or_game_reset(ctypes.byref(self.g), ctypes.c_uint64(seed))
        return self.board

    @property
    def board(self) -> np.ndarray:
        return np.array(self.g.board[:], dtype=np.int64).reshape(4, 4)

    @board.setter
    def board(self, vals):
        for i, v in enumerate(np.asarray(vals, dtype=np.int64).reshape(16)):
            self.g.board[i] = int(v)

    def step(self, action: int):
        ch = ctypes.c_int32()
        dn = ctypes.c_int32()
        rc = lib().or_game_step(ctypes.byref(self.g), action, ctypes.byref(ch), ctypes.byref(dn))
        if rc != 0:
            raise ValueError("invalid action")
        merged = [int(self.g.merged[i]) for i in range(self.g.n_merged)]
        return bool(ch.value), self.board, merged, bool(dn.value)

    def mask(self) -> np.ndarray:
        m = (ctypes.c_int8 * 4)()
        lib().or_game_mask(ctypes.byref(self.g), m)
        return np.array(m[:], dtype=np.int8)

    @property
    def score(self) -> int:
        return int(self.g.score)


OBS_MODES = {"raw": 0, "log2": 1, "onehot": 2}
REWARD_MODES = {"sum": 0, "log2": 1}
BONUS_MODES = {"off": 0, "raw": 1, "log2": 2}


def make_env_cfg(**kw) -> EnvCfg:
    """Build the C config from Game2048EnvConfig field names (src/env.py:19-40)."""
    d = dict(obs_mode="raw", obs_log2_scale=1.0, reward_mode="sum", base_reward_scale=1.0, empty_tile_reward=0.0,
             merge_reward=0.0, bonus_mode="off", bonus_scale=1.0, step_reward=0.0, endgame_penalty=0.0,
             use_action_mask=True, invalid_action_penalty=-1.0, max_steps=1024)
    d.update(kw)
    c = EnvCfg()
    c.obs_mode = OBS_MODES[d["obs_mode"]]
    c.reward_mode = REWARD_MODES[d["reward_mode"]]
    c.bonus_mode = BONUS_MODES[d["bonus_mode"]]
    c.use_action_mask = int(bool(d["use_action_mask"]))
    for k in ("obs_log2_scale", "base_reward_scale", "empty_tile_reward", "merge_reward", "bonus_scale",
              "step_reward", "endgame_penalty", "invalid_action_penalty"):
        setattr(c, k, float(d[k]))
    c.max_steps = -1 if d["max_steps"] is None else max(int(d["max_steps"]), 0)
    return c


def philox4x32_10(ctr, key) -> list[int]:
    c = (ctypes.c_uint32 * 4)(*[int(x) & 0xFFFFFFFF for x in ctr])
    k = (ctypes.c_uint32 * 2)(*[int(x) & 0xFFFFFFFF for x in key])
    out = (ctypes.c_uint32 * 4)()
    lib().or_philox4x32_10(c, k, out)
    return list(out)


class Env:
    """Oracle twin of src/env.py:Game2048Env (reset/step/obs/mask).  rng="philox" replays the build's Philox
    throughput-mode spawn stream (key `philox_key`, the current episode's seed) instead of numpy's PCG64."""

    def __init__(self, rng: str = "pcg64", philox_key: int = 0x2048, **cfg):
        self.cfg = make_env_cfg(**cfg)
        self.e = EnvState()
        self.rng = rng
        self.key = int(philox_key) & 0xFFFFFFFFFFFFFFFF
        self.seed = 0

    def reset(self, seed: int):
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        if self.rng == "philox":
            lib().or_env_reset_philox(ctypes.byref(self.e), ctypes.c_uint64(self.seed), ctypes.c_uint64(self.key))
        else:
            lib().or_env_reset(ctypes.byref(self.e), ctypes.c_uint64(seed))
        return self.obs(), self.mask()

    def step(self, action: int):
        r = ctypes.c_double()
        ch, te, tr, inv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        if self.rng == "philox":
            rc = lib().or_env_step_philox(ctypes.byref(self.e), ctypes.byref(self.cfg), action,
                                          ctypes.c_uint64(self.seed), ctypes.c_uint64(self.key), ctypes.byref(r),
                                          ctypes.byref(ch), ctypes.byref(te), ctypes.byref(tr), ctypes.byref(inv))
        else:
            rc = lib().or_env_step(ctypes.byref(self.e), ctypes.byref(self.cfg), action, ctypes.byref(r),
                                   ctypes.byref(ch), ctypes.byref(te), ctypes.byref(tr), ctypes.byref(inv))
        if rc != 0:
            raise AssertionError(f"Invalid action: {action}")
        return dict(reward=r.value, changed=bool(ch.value), terminated=bool(te.value), truncated=bool(tr.value),
                    invalid=bool(inv.value))

    def obs(self) -> np.ndarray:
        n = 272 if self.cfg.obs_mode == 2 else 16
        buf = (ctypes.c_float * n)()
        if lib().or_env_obs(ctypes.byref(self.e), ctypes.byref(self.cfg), buf) != 0:
            raise IndexError("tile exponent > 16 cannot be one-hot encoded")
        return np.array(buf[:], dtype=np.float32)

    def mask(self) -> np.ndarray:
        m = (ctypes.c_int8 * 4)()
        lib().or_game_mask(ctypes.byref(self.e.game), m)
        return np.array(m[:], dtype=np.int8)

    @property
    def board(self) -> np.ndarray:
        return np.array(self.e.game.board[:], dtype=np.int64).reshape(4, 4)

    @property
    def max_tile_seen(self) -> int:
        return int(self.e.max_tile_seen)

    @property
    def score(self) -> int:
        return int(self.e.game.score)

    @property
    def step_count(self) -> int:
        return int(self.e.step_count)


def obs_of_values(vals, **cfg) -> tuple[np.ndarray, np.ndarray]:
    """(obs["board"] flattened float32, action mask int8) of a board given as tile values, under an env config:
    src/env.py:131-159 restated (``or_env_obs``) + the game's mask."""
    e = Env(**cfg)
    for i, v in enumerate(np.asarray(vals, dtype=np.int64).reshape(16)):
        e.e.game.board[i] = int(v)
    return e.obs(), e.mask()


def obs_of_bitboard(board: int, **cfg) -> tuple[np.ndarray, np.ndarray]:
    e = unpack_exponents(board)
    return obs_of_values(np.where(e > 0, np.left_shift(np.int64(1), e), 0), **cfg)


def bench_env_steps(n_boards: int, n_rounds: int, seed0: int = 1000, **cfg) -> tuple[int, float]:
    """CPU baseline leg: run the oracle env step loop (OpenMP over boards). Returns (steps, reward_sum)."""
    c = make_env_cfg(**cfg)
    rs = ctypes.c_double()
    steps = lib().or_bench_env_steps(n_boards, n_rounds, ctypes.c_uint64(seed0), ctypes.byref(c), ctypes.byref(rs))
    return int(steps), float(rs.value)
