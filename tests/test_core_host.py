"""CPU check of the bitboard arithmetic the gfx950 kernels run (csrc/g2048_core.h), through a TEST-ONLY host
build (tests/native/core_host.cpp), against the golden fixtures of the real reference and the CPU oracle.

This is not a parity claim for the GPU path (those are the -m gpu tests); it localises logic bugs on CPU.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
CSRC = os.path.join(ROOT, "rl-2048-with-reinforce-and-actor-critic_amd", "csrc")


@pytest.fixture(scope="module")
def ch():
    so = os.path.join(NATIVE, "libcore_host.so")
    src = os.path.join(NATIVE, "core_host.cpp")
    hdr = os.path.join(CSRC, "g2048_core.h")
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        tmp = f"{so}.{os.getpid()}.tmp"   # build aside, then rename: parallel workers never load a partial file
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + CSRC, "-o", tmp, src], check=True)
        os.replace(tmp, so)
    L = ctypes.CDLL(so)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    L.ch_board_move.restype = ctypes.c_uint64
    L.ch_board_move.argtypes = [ctypes.c_uint64, ctypes.c_uint32] + [u32p] * 6
    L.ch_board_move_coded.restype = ctypes.c_uint64
    L.ch_board_move_coded.argtypes = [ctypes.c_uint64, ctypes.c_uint32] + [u32p] * 6
    L.ch_board_move_coded_nolist.restype = ctypes.c_uint64
    L.ch_board_move_coded_nolist.argtypes = [ctypes.c_uint64, ctypes.c_uint32] + [u32p] * 6
    L.ch_philox.argtypes = [u32p, u32p, u32p]
    L.ch_spawn_philox.restype = ctypes.c_uint64
    L.ch_spawn_philox.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
    L.ch_board_move_alu.restype = ctypes.c_uint64
    L.ch_board_move_alu.argtypes = [ctypes.c_uint64, ctypes.c_uint32] + [u32p] * 6
    L.ch_check_alu.restype = ctypes.c_int64
    L.ch_check_alu.argtypes = [ctypes.c_int64, ctypes.c_uint64]
    L.ch_check_lean.restype = ctypes.c_int64
    L.ch_check_lean.argtypes = [ctypes.c_int64, ctypes.c_uint64]
    L.ch_check_spawn_lean.restype = ctypes.c_int64
    L.ch_check_spawn_lean.argtypes = [ctypes.c_int64, ctypes.c_uint64]
    L.ch_check_frames.restype = ctypes.c_int64
    L.ch_check_frames.argtypes = [ctypes.c_int64, ctypes.c_uint64]
    L.ch_bits_mask.restype = ctypes.c_uint32
    L.ch_bits_mask.argtypes = [ctypes.c_uint64]
    L.ch_bits_done.argtypes = [ctypes.c_uint64]
    L.ch_action_mask.restype = ctypes.c_uint32
    L.ch_action_mask.argtypes = [ctypes.c_uint64]
    L.ch_is_done.argtypes = [ctypes.c_uint64]
    L.ch_transpose.restype = ctypes.c_uint64
    L.ch_transpose.argtypes = [ctypes.c_uint64]
    L.ch_symmetry.restype = ctypes.c_uint64
    L.ch_symmetry.argtypes = [ctypes.c_uint64, ctypes.c_int]
    L.ch_symmetry_action.restype = ctypes.c_uint32
    L.ch_symmetry_action.argtypes = [ctypes.c_uint32, ctypes.c_int]
    L.ch_pcg_seed.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.ch_episode.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    L.ch_reward.restype = ctypes.c_double
    L.ch_reward.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                            ctypes.c_int, ctypes.c_int, u32p]
    return L


def _move(ch, b, a, coded=False):
    vals = [ctypes.c_uint32() for _ in range(6)]
    fn = {False: ch.ch_board_move, True: ch.ch_board_move_coded, "nolist": ch.ch_board_move_coded_nolist,
          "alu": ch.ch_board_move_alu}[coded]
    m = fn(b, a, *[ctypes.byref(v) for v in vals])
    lst, cnt, score, sum_e, max_e, ovf = [v.value for v in vals]
    if coded == "nolist":
        # the list is not built; its length (the merge count) still is
        return m, cnt, score, sum_e, max_e, ovf
    merged = [((lst >> (4 * k)) & 15) + 1 for k in range(cnt)]
    return m, merged, score, sum_e, max_e, ovf


def _rand_boards(rng, n, p_empty=0.375, hi=15):
    e = rng.integers(1, hi + 1, size=(n, 16))
    e[rng.random((n, 16)) < p_empty] = 0
    return [O.pack_exponents(x) for x in e]


@pytest.mark.parametrize("coded", [False, True, "nolist", "alu"])
def test_board_move_vs_oracle(ch, coded):
    rng = np.random.default_rng(3)
    boards = _rand_boards(rng, 3000) + _rand_boards(rng, 2000, p_empty=0.0, hi=4) + _rand_boards(rng, 1000, 0.7)
    boards += _rand_boards(rng, 1500, p_empty=0.2, hi=15) + [O.pack_exponents([15] * 16), O.pack_exponents([15, 15, 14, 14] * 4),
                                                             O.pack_exponents([14, 14, 15, 15] * 4)]
    for b in boards:
        for a in range(4):
            m, merged, score, sum_e, max_e, ovf = _move(ch, b, a, coded)
            ob, omerged, ochanged, ok = O.move_packed(b, a)
            oe = [int(v).bit_length() - 1 for v in omerged]
            if coded == "nolist":
                assert merged == len(oe), (hex(b), a)
            else:
                assert merged == oe, (hex(b), a)
            assert score == sum(omerged) and sum_e == sum(oe) and max_e == max(oe, default=0)
            assert bool(ovf) == (not ok)
            if ok:
                assert m == ob, (hex(b), a)
            assert (m != b) == ochanged


def test_board_move_alu_equals_table_move(ch):
    """The table-free move (line_move_alu) against the two-table move: every 16-bit line in every line slot under
    all four actions (boards, merge summaries and merged lists equal), plus 200k random boards."""
    assert ch.ch_check_alu(200_000, 0x2048) == 0


def test_board_move_lean_equals_table_move(ch):
    """The step kernel's log2-reward move (board_move_lean: line table + max-merge field table, count and sum_e from
    board aggregates, an exact per-line fallback on saturated 15+15 merges) against the two-table move: every
    16-bit line in every line slot under all four actions, plus 200k random boards -- board, count, sum_e, max_e,
    overflow and the moved board's nz bits."""
    assert ch.ch_check_lean(200_000, 0x2049) == 0


def test_spawn_pcg_lean_equals_spawn(ch):
    """The lean step's branch-free PCG64 spawn (one- and two-step successors formed, next_uint32's buffer picks
    random()'s state; integer compare for random() < 0.9; exact fallback on a possible Lemire rejection) against
    spawn_pcg_z on 2M random boards and states, buffered values 0 and tiny included (the fallback path)."""
    assert ch.ch_check_spawn_lean(2_000_000, 0x2050) == 0


def test_frame_transforms_match_definitions(ch):
    """transpose / reverse_rows (delta swap + byte permutes) against the cell-by-cell definitions, 2M boards."""
    assert ch.ch_check_frames(2_000_000, 0x2051) == 0


def test_mask_done_vs_oracle(ch):
    rng = np.random.default_rng(4)
    boards = _rand_boards(rng, 4000) + _rand_boards(rng, 4000, p_empty=0.0, hi=6) + _rand_boards(rng, 500, 0.0, 2)
    for b in boards:
        g = O.Game()
        g.board = np.where(O.unpack_exponents(b) > 0, np.left_shift(1, O.unpack_exponents(b)), 0)
        m = g.mask()
        assert ch.ch_action_mask(b) == sum(int(x) << i for i, x in enumerate(m)), hex(b)
        assert ch.ch_bits_mask(b) == ch.ch_action_mask(b)
        assert bool(ch.ch_is_done(b)) == bool(O.lib().or_game_is_done(ctypes.byref(g.g)))
        assert ch.ch_bits_done(b) == ch.ch_is_done(b)


def test_transpose_and_symmetries(ch):
    rng = np.random.default_rng(5)
    for b in _rand_boards(rng, 500, 0.3):
        B = O.unpack_exponents(b)
        assert O.unpack_exponents(ch.ch_transpose(b)).tolist() == B.T.tolist()
        # Game2048Env.get_symmetries order (src/env.py:355-396)
        expect = [np.rot90(B, k) for k in range(4)] + [np.rot90(np.fliplr(B), k) for k in range(4)]
        for k in range(8):
            assert O.unpack_exponents(ch.ch_symmetry(b, k)).tolist() == expect[k].tolist(), k
    for a in range(4):
        exp_a = []
        cur = a
        for _ in range(4):
            exp_a.append(cur)
            cur = (cur - 1) % 4
        cur = {1: 3, 3: 1}.get(a, a)
        for _ in range(4):
            exp_a.append(cur)
            cur = (cur - 1) % 4
        assert [ch.ch_symmetry_action(a, k) for k in range(8)] == exp_a


def test_pcg_seed_vs_golden(ch, golden_dir):
    d = np.load(os.path.join(golden_dir, "pcg64.npz"))
    out = (ctypes.c_uint64 * 4)()
    for s, st in zip(d["seeds"], d["state"]):
        ch.ch_pcg_seed(int(s), out)
        assert list(out) == [int(x) for x in st]


def test_episodes_vs_golden(ch, golden_dir):
    """Whole seeded episodes (spawn stream included) of the real Game2048 through the kernel arithmetic."""
    d = np.load(os.path.join(golden_dir, "episodes.npz"))
    for e in range(len(d["ep_seed"])):
        s0, n = int(d["ep_start"][e]), int(d["ep_len"][e])
        acts = np.ascontiguousarray(d["action"][s0:s0 + n])
        boards = np.zeros(n, np.uint64)
        changed = np.zeros(n, np.uint8)
        done = np.zeros(n, np.uint8)
        score = np.zeros(n, np.uint32)
        rb = ctypes.c_uint64()
        ch.ch_episode(int(d["ep_seed"][e]), acts.ctypes.data, n, boards.ctypes.data, changed.ctypes.data,
                      done.ctypes.data, score.ctypes.data, ctypes.byref(rb))
        assert rb.value == d["reset_board"][e]
        np.testing.assert_array_equal(boards, d["board"][s0:s0 + n])
        np.testing.assert_array_equal(changed.astype(bool), d["changed"][s0:s0 + n])
        np.testing.assert_array_equal(done.astype(bool), d["done"][s0:s0 + n])
        np.testing.assert_array_equal(score, d["score"][s0:s0 + n])


ENV_CFGS = [
    dict(),
    dict(reward_mode="log2", base_reward_scale=0.5),
    dict(reward_mode="log2", base_reward_scale=0.5, empty_tile_reward=0.1, merge_reward=0.25, bonus_mode="raw",
         bonus_scale=0.01, step_reward=-0.003, endgame_penalty=-7.5),
    dict(bonus_mode="log2", bonus_scale=2.0, use_action_mask=False, invalid_action_penalty=-1.5),
    dict(reward_mode="sum", base_reward_scale=1.0 / 3.0, empty_tile_reward=-0.07, max_steps=37),
]


@pytest.mark.parametrize("cfg", ENV_CFGS)
def test_reward_vs_oracle(ch, cfg):
    """Kernel reward arithmetic == oracle _compute_reward (src/env.py:197-261) bit-for-bit in fp64."""
    env = O.Env(**cfg)
    c = env.cfg
    scal = (ctypes.c_double * 7)(c.base_reward_scale, c.empty_tile_reward, c.merge_reward, c.bonus_scale,
                                 c.step_reward, c.endgame_penalty, c.invalid_action_penalty)
    rng = np.random.default_rng(11)
    for ep in range(25):
        env.reset(900 + ep)
        mt = ctypes.c_uint32(2)
        for t in range(400):
            b = O.pack_exponents(O.values_to_exponents(env.board))
            a = int(rng.integers(4))
            m, merged, score, sum_e, max_e, ovf = _move(ch, b, a)
            r = env.step(a)
            fb = O.pack_exponents(O.values_to_exponents(env.board))
            got = ch.ch_reward(c.reward_mode, c.bonus_mode, c.use_action_mask, scal, len(merged), sum_e, score, max_e,
                               fb, int(r["terminated"]), int(r["invalid"]), ctypes.byref(mt))
            assert got == r["reward"], (cfg, ep, t)
            assert (1 << mt.value) == env.max_tile_seen
            if r["terminated"] or r["truncated"]:
                break


# Random123 known-answer vectors for philox4x32 with 10 rounds (kat_vectors of the published library)
PHILOX_KAT = [([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
              ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
              ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
               [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1])]


def test_philox_kat_and_spawn_vs_oracle(ch):
    """The build's Philox4x32-10 (throughput mode) against Random123's known answers, and its spawn against the
    oracle's independent restatement of the same spec on random boards / draws."""
    u32x4, u32x2 = ctypes.c_uint32 * 4, ctypes.c_uint32 * 2
    for ctr, key, exp in PHILOX_KAT:
        out = u32x4()
        ch.ch_philox(u32x4(*ctr), u32x2(*key), out)
        assert list(out) == exp
        assert O.philox4x32_10(ctr, key) == exp
    rng = np.random.default_rng(9)
    for b in _rand_boards(rng, 2000):
        x, y = (int(v) for v in rng.integers(0, 2**32, size=2, dtype=np.uint64))
        got = ch.ch_spawn_philox(int(b), x, y)
        e = O.unpack_exponents(int(b)).reshape(16)
        empties = np.nonzero(e == 0)[0]
        if len(empties) == 0:
            assert got == int(b)
            continue
        cell = empties[(x * len(empties)) >> 32]
        assert got == int(b) | ((1 if y < 3865470566 else 2) << (4 * int(cell)))
