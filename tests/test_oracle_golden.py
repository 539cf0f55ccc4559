"""Pin the CPU oracle (oracle/g2048_oracle.c) against the reference's own outputs (tests/golden/*.npz, made by
tests/golden/make_golden.py from the real src/game2048.py and src/MLP.py) and against numpy's RNG.

CPU only.  These tests are what make the oracle trustworthy as the checker for the HIP path.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False)


def _unpack_merged(word, n):
    return [int((int(word) >> (5 * i)) & 31) for i in range(int(n))]


def _row_vals(exps):
    return [0 if e == 0 else 1 << int(e) for e in exps]


def test_row_table_exhaustive(golden_dir):
    """All 65,536 rows through Game2048._row_move_left (src/game2048.py:120-137) == oracle move-left."""
    d = _load(golden_dir, "row_table")
    out_exp, merged_exp, n_merged = d["out_exp"], d["merged_exp"], d["n_merged"]
    # the oracle moves whole boards; put each row in row 0 of an otherwise empty board, action 3 (left)
    rows = np.arange(65536)
    rng = np.random.default_rng(0)
    sample = np.concatenate([rows[:4096], rng.choice(65536, 4096, replace=False), rows[-256:]])
    for r in sample:
        r = int(r)
        exps = [(r >> (4 * k)) & 15 for k in range(4)]
        # overflow rows (two 2**15 merging) cannot be packed; checked through the merged list
        board_vals = np.zeros(16, dtype=np.int64)
        board_vals[:4] = _row_vals(exps)
        out, merged, changed, ok = O.move_packed(O.pack_exponents(O.values_to_exponents(board_vals)), 3)
        got_merged = [int(v).bit_length() - 1 for v in merged]
        assert got_merged == list(merged_exp[r][: n_merged[r]]), r
        if ok:
            got = O.unpack_exponents(out)[0]
            assert list(got) == list(out_exp[r]), r
        else:
            assert max(out_exp[r]) == 16, r
        assert changed == (list(out_exp[r]) != exps)


def test_row_table_full_hash(golden_dir):
    """Whole-table check through the 4-direction board move: each row placed in every row slot / column."""
    d = _load(golden_dir, "row_table")
    out_exp = d["out_exp"].astype(np.int64)
    rng = np.random.default_rng(1)
    for r in rng.choice(65536, 2000, replace=False):
        r = int(r)
        exps = [(r >> (4 * k)) & 15 for k in range(4)]
        if 16 in out_exp[r]:
            continue
        slot = int(rng.integers(4))
        # right move: row reversed in the move-left frame
        rev = exps[::-1]
        rr = sum(e << (4 * k) for k, e in enumerate(rev))
        b = np.zeros((4, 4), dtype=np.int64)
        b[slot] = exps
        out, _, _, ok = O.move_packed(O.pack_exponents(b), 1)
        if 16 in out_exp[rr]:
            continue
        assert list(O.unpack_exponents(out)[slot]) == list(out_exp[rr][::-1])
        # up move: the row as a column
        b = np.zeros((4, 4), dtype=np.int64)
        b[:, slot] = exps
        out, _, _, ok = O.move_packed(O.pack_exponents(b), 0)
        assert list(O.unpack_exponents(out)[:, slot]) == list(out_exp[r])


def test_pcg64_seeding_matches_numpy(golden_dir):
    d = _load(golden_dir, "pcg64")
    for s, st in zip(d["seeds"], d["state"]):
        p = O.PCG64(int(s))
        state, inc = p.state128
        assert state == (int(st[0]) << 64) | int(st[1])
        assert inc == (int(st[2]) << 64) | int(st[3])


def test_pcg64_streams(golden_dir):
    d = _load(golden_dir, "pcg64")
    for k, s in enumerate(d["seq_seeds"]):
        p = O.PCG64(int(s))
        for j in range(d["seq_ops"].shape[1]):
            if d["seq_ops"][k, j] == 0:
                assert p.integers(int(d["seq_n"][k, j])) == d["seq_int"][k, j]
            else:
                assert p.random() == d["seq_flt"][k, j]


def test_fixed_seed_iter_known_answers(golden_dir):
    """runner.py:244-261: first values of make_fixed_seed_iter(3) as recorded in SURVEY.md section 8c."""
    d = _load(golden_dir, "pcg64")
    assert list(d["fixed_seed_iter3"][:3]) == [789974133212406139, 2184191404571879930, 7390452496230446618]


def test_choice_matches_numpy(golden_dir):
    d = _load(golden_dir, "choice")
    for k, s in enumerate(d["seeds"]):
        p = O.PCG64(int(s))
        got = [p.choice4(pr) for pr in d["probs"]]
        assert got == list(d["idx"][k])


def test_episodes_bit_exact(golden_dir):
    """Seeded episodes of the real Game2048 (uniform incl. invalid moves, random-valid, two heuristics)."""
    d = _load(golden_dir, "episodes")
    for e in range(len(d["ep_seed"])):
        g = O.Game()
        g.reset(int(d["ep_seed"][e]))
        assert O.pack_exponents(O.values_to_exponents(g.board)) == d["reset_board"][e]
        m = g.mask()
        assert sum(int(b) << i for i, b in enumerate(m)) == d["reset_mask"][e]
        s0, n = int(d["ep_start"][e]), int(d["ep_len"][e])
        for t in range(s0, s0 + n):
            ch, b, mg, dn = g.step(int(d["action"][t]))
            assert ch == bool(d["changed"][t]) and dn == bool(d["done"][t]), (e, t)
            assert O.pack_exponents(O.values_to_exponents(b)) == d["board"][t], (e, t)
            assert [int(v).bit_length() - 1 for v in mg] == _unpack_merged(d["merged"][t], d["n_merged"][t])
            assert g.score == d["score"][t]
            m = g.mask()
            assert sum(int(bb) << i for i, bb in enumerate(m)) == d["mask"][t]


def test_crafted_boards(golden_dir):
    d = _load(golden_dir, "crafted")
    for i in range(len(d["board_in"])):
        g = O.Game()
        g.reset(int(d["seed"][i]))
        g.board = np.where(O.unpack_exponents(int(d["board_in"][i])) > 0,
                           np.left_shift(1, O.unpack_exponents(int(d["board_in"][i]))), 0)
        ch, b, mg, dn = g.step(int(d["action"][i]))
        assert ch == bool(d["changed"][i]) and dn == bool(d["done"][i]), i
        assert [int(v).bit_length() - 1 for v in mg] == _unpack_merged(d["merged"][i], d["n_merged"][i])
        if d["overflow"][i]:
            assert b.max() > 32768
        else:
            assert O.pack_exponents(O.values_to_exponents(b)) == d["board_out"][i], i
        assert sum(int(bb) << k for k, bb in enumerate(g.mask())) == d["mask"][i]


@pytest.mark.parametrize("kind,ref_avg", [(1, 1103.61), (2, 2266.07), (3, 2595.54)])
def test_statistical_kats(golden_dir, kind, ref_avg):
    """tools/simple_action_gen.py:10,19,27 published average scores, checked on the golden episodes'
    score under reward_mode='sum' (= final Game2048.score) and on fresh oracle env episodes."""
    policy = {1: "random_valid", 2: "urdl", 3: "urld"}[kind]
    rng = np.random.default_rng(10 + kind)
    totals = []
    n_ep = 150
    for ep in range(n_ep):
        env = O.Env(reward_mode="sum", max_steps=None)
        _, m = env.reset(5000 + ep)
        total = 0.0
        while True:
            valid = [i for i in range(4) if m[i]]
            if policy == "random_valid":
                a = valid[int(rng.integers(len(valid)))]
            elif policy == "urdl":
                a = valid[0]
            else:
                a = next(x for x in (0, 1, 3, 2) if m[x])
            r = env.step(a)
            total += r["reward"]
            m = env.mask()
            if r["terminated"] or r["truncated"]:
                break
        assert total == env.score
        totals.append(total)
    mean, sem = np.mean(totals), np.std(totals) / np.sqrt(n_ep)
    assert abs(mean - ref_avg) < 4.5 * sem, (mean, sem, ref_avg)
