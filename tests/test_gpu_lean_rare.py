"""GPU parity of the LEAN step kernel (RK 1 -- the bench's headline kernel: log2 reward, no score output, packed or
int8 mask) on its rare branches, which random play at bench size practically never reaches:

* high-tile merges: 2^14 + 2^14 -> 2^15, the saturated 2^15 + 2^15 (the 65536 of the reference: overflow flag,
  max-merge field 15 -> the exact per-line sum, log2 reward term 16, raw bonus 2^16) and boards holding several
  of them in one move;
* the Lemire-rejection fallback of spawn_pcg_lean: lanes whose next_uint32 is a chosen buffered value (0, or
  ceil(2^32 / n_empty)) so the bounded draw's low word is < n_empty -- accepted or rejected (then redrawn);
* the reference's crafted boards (crafted.npz, from src/game2048.py) through the lean kernel.

Every lane is replayed by the oracle (oracle/g2048_oracle.c, pinned to src/game2048.py + src/env.py) from the same
board and PCG64 state: fp64 rewards rounded once to fp32, flags, boards, log2 obs, masks and max_tile_seen,
bit-exact, over several steps.  A lane whose step saturated (2^15 + 2^15) is compared on that step's reward and
flags, then dropped (its nibble board holds 2^15 where the reference holds 65536 -- DESIGN.md section 7).
Both table paths run: LDS tables (>= 16,384 lanes) and L1/L2 tables (small batches).
Reference: src/game2048.py:108-137 (spawn, row move), src/env.py:197-261 (reward)."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
HAS_U32 = 0x04000000


def _high_tile_boards(rng, n):
    """n boards (exponent arrays [n, 16]) rich in 2^12..2^15 tiles, plus explicit 14+14 / 15+15 lines."""
    p = np.array([0.30] + [0.10 / 11] * 11 + [0.15, 0.15, 0.15, 0.15])
    e = rng.choice(16, size=(n, 16), p=p / p.sum())
    lines = ([14, 14, 0, 0], [15, 15, 0, 0], [15, 15, 15, 15], [14, 14, 15, 15], [15, 0, 15, 3], [0, 15, 0, 15],
             [13, 13, 14, 14], [14, 0, 14, 15])
    for k in range(0, n, 3):                        # every third board: an explicit line in a random slot / frame
        ln = np.array(lines[rng.integers(len(lines))])
        r = int(rng.integers(4))
        b = e[k].reshape(4, 4)
        if rng.integers(2):
            b[r, :] = ln if rng.integers(2) else ln[::-1]
        else:
            b[:, r] = ln if rng.integers(2) else ln[::-1]
    return e


def _lemire_value(moved_board: int, rng) -> int | None:
    """A buffered next_uint32 value that sends the spawn's bounded draw (Lemire, n = empty cells of the moved
    board) to its low-word fallback: 0 (low word 0 < n; rejected unless n is a power of two) or ceil(2^32 / n)
    (low word n - 2^32 mod n < n)."""
    ne = sum(((moved_board >> (4 * c)) & 15) == 0 for c in range(16))
    if ne == 0:
        return None
    if ne & (ne - 1) == 0 or rng.integers(2):
        return 0
    return -(-(1 << 32) // ne)


@pytest.mark.parametrize("n,packed,bonus", [(20000 + 37, True, "raw"), (20000 + 37, False, "log2"), (3001, True, "raw")])
def test_lean_kernel_high_tiles_and_lemire_fallback(n, packed, bonus):
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    cfg = dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5,
               empty_tile_reward=0.1, merge_reward=0.25, bonus_mode=bonus, bonus_scale=0.01, step_reward=-0.003,
               endgame_penalty=-7.5, max_steps=1024)
    env = VecGame2048Env(n, Game2048EnvConfig(**cfg), device=DEV, track_score=False, packed_mask=packed)
    seeds = [900_001 + 7 * i for i in range(n)]
    env.reset(seed=seeds)
    rng = np.random.default_rng(0x1EA7 + n)
    exps = _high_tile_boards(rng, n)
    packed_b = np.array([O.pack_exponents(x) for x in exps], dtype=np.uint64)
    env.board.copy_(torch.from_numpy(packed_b.view(np.int64)).to(DEV))
    T = 6
    acts = rng.integers(0, 4, size=(T, n)).astype(np.uint8)
    # lanes forced onto the Lemire fallback at their first step
    uint = env.rng_uint.cpu().numpy().view(np.uint32).copy()
    state = env.state.cpu().numpy().view(np.uint32).copy()
    forced = {}
    for i in range(0, n, 2):
        mv, _, ch, ok = O.move_packed(int(packed_b[i]), int(acts[0, i]))
        if ch and ok:
            x = _lemire_value(mv, rng)
            if x is not None:
                forced[i] = x
                uint[i] = x
                state[i] |= HAS_U32
    env.rng_uint.copy_(torch.from_numpy(uint.view(np.int32)).to(DEV))
    env.state.copy_(torch.from_numpy(state.view(np.int32)).to(DEV))
    # the oracle's twin of every lane
    ref = []
    for i in range(n):
        e = O.Env(**cfg)
        e.reset(seeds[i])
        for c in range(16):
            e.e.game.board[c] = (1 << int(exps[i, c])) if exps[i, c] else 0
        if i in forced:
            e.e.game.rng.has_uint32, e.e.game.rng.uinteger = 1, forced[i]
        ref.append(e)
    live = np.ones(n, dtype=bool)
    n_sat = n_1415 = n_reject = 0
    for t in range(T):
        env.step_into(torch.from_numpy(acts[t]).to(DEV))
        rw, fl = env.reward.cpu().numpy(), env.flags.cpu().numpy()
        bd, ob = env.board.cpu().numpy().view(np.uint64), env.obs.cpu().numpy()
        mk, mt = env.action_mask.cpu().numpy(), env.max_tile_seen.cpu().numpy()
        for i in np.nonzero(live)[0]:
            before = ref[i].board.max()
            r = ref[i].step(int(acts[t, i]))
            sat = ref[i].board.max() == 65536 and before < 65536
            if not sat or bool(fl[i] & 0x02) == r["terminated"]:
                # (on a saturating step the nibble board may keep two mergeable 2^15 tiles where the reference's
                # 65536 cannot merge, so done -- hence the endgame term -- may differ there: DESIGN.md section 7)
                assert rw[i] == np.float32(r["reward"]), (t, i, rw[i], r["reward"])
            assert bool(fl[i] & 0x01) == r["changed"] and bool(fl[i] & 0x08) == r["invalid"], (t, i)
            assert bool(fl[i] & 0x04) == r["truncated"] or sat, (t, i)
            assert bool(fl[i] & 0x10) == sat, (t, i)
            if sat:                                      # the nibble board saturates here
                n_sat += 1
                assert mt[i] == ref[i].max_tile_seen == 65536, (t, i)
                live[i] = False
                continue
            n_1415 += ref[i].board.max() == 32768 and before < 32768
            assert bool(fl[i] & 0x02) == r["terminated"], (t, i)
            assert bd[i] == O.pack_exponents(O.values_to_exponents(ref[i].board)), (t, i)
            np.testing.assert_array_equal(ob[i], ref[i].obs())
            np.testing.assert_array_equal(mk[i], ref[i].mask())
            assert mt[i] == ref[i].max_tile_seen, (t, i)
            if r["terminated"]:
                live[i] = False
    for i, x in forced.items():
        ne = sum(1 for c in range(16) if not (O.move_packed(int(packed_b[i]), int(acts[0, i]))[0] >> (4 * c)) & 15)
        n_reject += x == 0 and (1 << 32) % ne != 0
    assert n_sat > 50 and n_1415 > 50, (n_sat, n_1415)
    assert len(forced) > n // 8 and n_reject > 50, (len(forced), n_reject)


def test_lean_kernel_on_reference_crafted_boards(golden_dir):
    """crafted.npz (the real Game2048 on high-tile / full / terminal / empty boards with seeded spawns) through the
    lean kernel: boards, changed, done, mask and overflow against the reference's outputs; rewards, obs and
    max_tile_seen against the oracle (the fixture predates the env)."""
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    d = np.load(os.path.join(golden_dir, "crafted.npz"))
    m = len(d["board_in"])
    reps = -(-20000 // m)                           # tiled past 16,384 lanes: the LDS-table path
    n = m * reps
    cfg = dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5, bonus_mode="raw",
               bonus_scale=0.01, max_steps=None)
    env = VecGame2048Env(n, Game2048EnvConfig(**cfg), device=DEV, track_score=False, packed_mask=True)
    seeds = [int(s) for s in d["seed"]] * reps
    env.reset(seed=seeds)
    env.board.copy_(torch.from_numpy(np.tile(d["board_in"], reps).view(np.int64)).to(DEV))
    env.step_into(torch.from_numpy(np.tile(d["action"].astype(np.uint8), reps)).to(DEV))
    b = env.board.cpu().numpy().view(np.uint64)
    fl, rw, ob = env.flags.cpu().numpy(), env.reward.cpu().numpy(), env.obs.cpu().numpy()
    mk = (env.action_mask.cpu().numpy() * (1 << np.arange(4))).sum(1)
    mt = env.max_tile_seen.cpu().numpy()
    for i in range(n):
        j = i % m
        assert bool(fl[i] & 1) == d["changed"][j], i
        assert bool(fl[i] & 0x10) == d["overflow"][j], i
        e = O.Env(**cfg)
        e.reset(int(d["seed"][j]))
        for c in range(16):
            e.e.game.board[c] = (1 << ((int(d["board_in"][j]) >> (4 * c)) & 15)) if (int(d["board_in"][j]) >> (4 * c)) & 15 else 0
        r = e.step(int(d["action"][j]))
        assert rw[i] == np.float32(r["reward"]), (i, rw[i], r["reward"])
        assert mt[i] == e.max_tile_seen, i
        if not d["overflow"][j]:
            assert b[i] == d["board_out"][j], i
            assert bool(fl[i] & 2) == d["done"][j], i
            assert mk[i] == d["mask"][j], i
            np.testing.assert_array_equal(ob[i], e.obs())
