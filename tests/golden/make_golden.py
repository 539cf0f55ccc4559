"""Generate the golden fixtures in tests/golden/ from the REAL reference (run in the build container only).

    python tests/golden/make_golden.py [--ref /root/reference]

Imports, by file path and without writing bytecode into the reference tree:
  * src/game2048.py  (needs only numpy/secrets/logging)  -> row table, seeded episodes, crafted boards, masks
  * src/MLP.py       (needs only numpy)                  -> init_model_params / forward_logits / logits_to_probs
numpy itself (2.2.6, where the reference's RNG lives) -> PCG64 seeding / streams / Generator.choice.

src/env.py and src/reinforce_agent.py import ``gymnasium``, which is not installed here; no stand-in is
written for it, so they are NOT imported (DESIGN.md "Oracle" records what that leaves unpinned).

Every fixture is data only: inputs and the reference's outputs.  Boards are stored as exponent bitboards
(uint64, nibble r*4+c = log2(tile), 0 = empty); merged lists as exponents.
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _load(path: str, name: str):
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def pack(board) -> int:
    x = 0
    for i, v in enumerate(np.asarray(board, dtype=np.int64).reshape(16)):
        v = int(v)
        e = 0 if v == 0 else v.bit_length() - 1
        assert e <= 15, "tile does not fit a nibble"
        x |= e << (4 * i)
    return x


def exps_of(values) -> list[int]:
    return [int(v).bit_length() - 1 for v in values]


def seed_iter(base: int):
    """runner.py:244-261 make_fixed_seed_iter (runner.py itself imports src.env -> gymnasium)."""
    rng = np.random.default_rng(base)
    hi = np.iinfo(np.int64).max
    while True:
        yield int(rng.integers(low=0, high=hi, dtype=np.int64))


def gen_row_table(G):
    g = G.Game2048()
    rows = np.arange(65536, dtype=np.int64)
    ex_in = np.stack([(rows >> (4 * k)) & 15 for k in range(4)], axis=1)
    out = np.zeros((65536, 4), dtype=np.uint8)
    merged = np.zeros((65536, 2), dtype=np.uint8)
    nmerged = np.zeros(65536, dtype=np.uint8)
    for r in range(65536):
        vals = np.where(ex_in[r] > 0, np.left_shift(1, ex_in[r]), 0).astype(np.int64)
        g._new_merged = []
        nr = g._row_move_left(vals)
        out[r] = [0 if int(v) == 0 else int(v).bit_length() - 1 for v in nr]
        m = exps_of(g._new_merged)
        nmerged[r] = len(m)
        merged[r, : len(m)] = m
    np.savez_compressed(os.path.join(HERE, "row_table.npz"), out_exp=out, merged_exp=merged, n_merged=nmerged)


def gen_pcg(_G):
    seeds = [0, 1, 2, 3, 7, 42, 12345, 54321, 2**32 - 1, 2**32, 2**32 + 1, 2**63 - 5, 2**64 - 1]
    it3, it7 = seed_iter(3), seed_iter(7)
    seeds += [next(it3) for _ in range(8)] + [next(it7) for _ in range(8)]
    r = np.random.default_rng(0x5EED)
    seeds += [int(x) for x in r.integers(0, 2**63 - 1, size=16, dtype=np.int64)]
    st = np.zeros((len(seeds), 4), dtype=np.uint64)  # state_hi, state_lo, inc_hi, inc_lo
    for i, s in enumerate(seeds):
        d = np.random.PCG64(s).state["state"]
        st[i] = [d["state"] >> 64, d["state"] & (2**64 - 1), d["inc"] >> 64, d["inc"] & (2**64 - 1)]
    # mixed draw streams: ops 0 = integers(n) with n in 1..16, 1 = random()
    n_seq = 4096
    ops = r.integers(0, 2, size=(4, n_seq)).astype(np.uint8)
    ns = r.integers(1, 17, size=(4, n_seq)).astype(np.int64)
    out_int = np.zeros((4, n_seq), dtype=np.int64)
    out_flt = np.zeros((4, n_seq), dtype=np.float64)
    for k, s in enumerate(seeds[:4]):
        g = np.random.default_rng(s)
        for j in range(n_seq):
            if ops[k, j] == 0:
                out_int[k, j] = int(g.integers(int(ns[k, j])))
            else:
                out_flt[k, j] = g.random()
    seq_seeds = np.array(seeds[:4], dtype=np.uint64)
    it = seed_iter(3)
    fixed3 = np.array([next(it) for _ in range(64)], dtype=np.int64)
    it = seed_iter(7)
    fixed7 = np.array([next(it) for _ in range(64)], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "pcg64.npz"), seeds=np.array(seeds, dtype=np.uint64), state=st,
                        seq_seeds=seq_seeds, seq_ops=ops, seq_n=ns, seq_int=out_int, seq_flt=out_flt,
                        fixed_seed_iter3=fixed3, fixed_seed_iter7=fixed7)


def _policy_actions(kind, mask, rng):
    valid = [i for i, v in enumerate(mask) if v]
    if kind == "uniform":            # uniformly random over 0..3 (includes invalid, no-change moves)
        return int(rng.integers(4))
    if kind == "random_valid":       # tools/simple_action_gen.py:7-13 restated with a seeded rng
        return int(valid[int(rng.integers(len(valid)))]) if valid else 0
    if kind == "urdl":               # tools/simple_action_gen.py:16-21
        return valid[0] if valid else 0
    if kind == "urld":               # tools/simple_action_gen.py:24-33
        for a in (0, 1, 3, 2):
            if mask[a]:
                return a
        return 0
    raise ValueError(kind)


def gen_episodes(G):
    """Seeded episodes through the real Game2048: reset(seed) then step(action) until done / cap."""
    rng = np.random.default_rng(2048)
    it = seed_iter(3)
    kinds = ["uniform"] * 48 + ["random_valid"] * 24 + ["urdl"] * 12 + ["urld"] * 12
    cap = 3000
    ep_seed, ep_kind, ep_start, ep_len = [], [], [], []
    reset_board, reset_mask = [], []
    act, board, changed, done, score, mask, merged_packed, n_merged = [], [], [], [], [], [], [], []
    for k, kind in enumerate(kinds):
        seed = next(it)
        g = G.Game2048()
        st = g.reset(seed=seed)
        ep_seed.append(seed)
        ep_kind.append(k)
        ep_start.append(len(act))
        reset_board.append(pack(st))
        m = g.get_action_mask()
        reset_mask.append(sum(b << i for i, b in enumerate(m)))
        t = 0
        while t < cap:
            a = _policy_actions(kind, m, rng)
            ch, s, mg, dn = g.step(a)
            m = g.get_action_mask()
            act.append(a)
            board.append(pack(s))
            changed.append(ch)
            done.append(dn)
            score.append(g.score)
            mask.append(sum(b << i for i, b in enumerate(m)))
            e = exps_of(mg)
            assert len(e) <= 8
            merged_packed.append(sum(x << (5 * i) for i, x in enumerate(e)))  # 5 bits per exponent, <= 8 merges
            n_merged.append(len(e))
            t += 1
            if dn:
                break
        ep_len.append(t)
    np.savez_compressed(
        os.path.join(HERE, "episodes.npz"), ep_seed=np.array(ep_seed, dtype=np.uint64),
        ep_kind=np.array([["uniform", "random_valid", "urdl", "urld"].index(k) for k in kinds], dtype=np.uint8),
        ep_start=np.array(ep_start, dtype=np.int64), ep_len=np.array(ep_len, dtype=np.int64),
        reset_board=np.array(reset_board, dtype=np.uint64), reset_mask=np.array(reset_mask, dtype=np.uint8),
        action=np.array(act, dtype=np.uint8), board=np.array(board, dtype=np.uint64),
        changed=np.array(changed, dtype=np.bool_), done=np.array(done, dtype=np.bool_),
        score=np.array(score, dtype=np.int64), mask=np.array(mask, dtype=np.uint8),
        merged=np.array(merged_packed, dtype=np.uint64), n_merged=np.array(n_merged, dtype=np.uint8))


def gen_crafted(G):
    """Crafted boards (high tiles incl. 2**14 / 2**15, full boards, near-terminal) x 4 actions with a fixed
    spawn stream: board after step, merged, changed, done, mask.  Exercises what random play rarely reaches."""
    rng = np.random.default_rng(77)
    boards = []
    for _ in range(400):
        p_empty = rng.choice([0.0, 0.1, 0.375, 0.7])
        e = rng.integers(1, 16, size=16)
        e[rng.random(16) < p_empty] = 0
        boards.append(e)
    # structured cases
    boards.append(np.array([15, 15, 0, 0] + [0] * 12))           # 32768+32768 merge (overflow of a nibble)
    boards.append(np.array([14, 14, 14, 14] + [1, 2, 3, 4] * 3))
    boards.append(np.array([1, 1, 1, 1] * 4))
    boards.append(np.array([1, 2, 1, 2, 2, 1, 2, 1] * 2))        # terminal checkerboard
    boards.append(np.zeros(16, dtype=np.int64))                  # empty board
    out = dict(board_in=[], action=[], seed=[], board_out=[], changed=[], done=[], mask=[], merged=[], n_merged=[],
               overflow=[])
    for i, e in enumerate(boards):
        for a in range(4):
            g = G.Game2048()
            seed = int(rng.integers(0, 2**62))
            g.reset(seed=seed)                                  # seeds g._rng, then we overwrite the board
            vals = np.where(e > 0, np.left_shift(1, e), 0).astype(np.int64).reshape(4, 4)
            g.board = vals.copy()
            ch, s, mg, dn = g.step(a)
            ovf = any(int(v) > 32768 for row in s for v in row)
            out["board_in"].append(pack(vals))
            out["action"].append(a)
            out["seed"].append(seed)
            out["board_out"].append(0 if ovf else pack(s))
            out["overflow"].append(ovf)
            out["changed"].append(ch)
            out["done"].append(dn)
            m = g.get_action_mask()
            out["mask"].append(sum(b << k for k, b in enumerate(m)))
            ex = exps_of(mg)
            out["merged"].append(sum(x << (5 * k) for k, x in enumerate(ex)))
            out["n_merged"].append(len(ex))
    np.savez_compressed(os.path.join(HERE, "crafted.npz"),
                        board_in=np.array(out["board_in"], dtype=np.uint64), action=np.array(out["action"], np.uint8),
                        seed=np.array(out["seed"], dtype=np.uint64), board_out=np.array(out["board_out"], np.uint64),
                        overflow=np.array(out["overflow"], np.bool_), changed=np.array(out["changed"], np.bool_),
                        done=np.array(out["done"], np.bool_), mask=np.array(out["mask"], np.uint8),
                        merged=np.array(out["merged"], np.uint64), n_merged=np.array(out["n_merged"], np.uint8))


def gen_mlp(M):
    cases = [
        ("he_relu_log2", 16, [256, 256], 4, "HeNormal", 0),
        ("xn_onehot", 272, [32, 16], 4, "XavierNormal", 5),
        ("xu_critic", 16, [8], 1, "XavierUniform", 9),
        ("normal_linear", 16, [], 4, "Normal", 3),
        ("he_onehot_critic", 272, [64, 32], 1, "HeNormal", 11),
    ]
    data = {}
    r = np.random.default_rng(99)
    for name, din, hid, dout, dist, seed in cases:
        rng = np.random.default_rng(seed)
        p = M.init_model_params(din, list(hid), dout, rng, dist, True)
        data[f"{name}__meta"] = np.array([din, dout, seed, len(hid)] + list(hid), dtype=np.int64)
        data[f"{name}__dist"] = np.array(dist)
        for i, (W, b) in enumerate(zip(p["W"], p["b"])):
            data[f"{name}__W{i}"] = W
            data[f"{name}__b{i}"] = b
        X = r.standard_normal((64, din)).astype(np.float32)
        for act in ("ReLU", "Sigmoid"):
            logits, acts, pres = M.forward_logits(p, X, act)
            data[f"{name}__X"] = X
            data[f"{name}__logits_{act}"] = logits
        if dout == 4:
            mask = (r.random((64, 4)) < 0.7).astype(np.int8)
            mask[mask.sum(1) == 0, 2] = 1
            data[f"{name}__mask"] = mask
            data[f"{name}__probs"] = M.logits_to_probs(data[f"{name}__logits_ReLU"], mask)
    # a second agent-style init: actor then critic from the SAME rng (src/reinforce_agent.py:62,77,95)
    rng = np.random.default_rng(0)
    pa = M.init_model_params(16, [256, 256], 4, rng, "HeNormal", True)
    pc = M.init_model_params(16, [256, 256], 1, rng, "HeNormal", True)
    assert all(np.array_equal(a, b) for a, b in zip(pa["W"], [data[f"he_relu_log2__W{i}"] for i in range(3)]))
    data["agent_critic__W0"] = pc["W"][0]
    data["agent_critic__W1_rows8"] = pc["W"][1][:8]
    data["agent_critic__W2"] = pc["W"][2]
    np.savez_compressed(os.path.join(HERE, "mlp.npz"), **data)


def gen_choice(_G):
    """Generator.choice(4, p) streams for masked-softmax probs (src/reinforce_agent.py:187)."""
    r = np.random.default_rng(4)
    n = 4000
    probs = np.zeros((n, 4), dtype=np.float32)
    for i in range(n):
        logits = r.standard_normal(4).astype(np.float32) * 3
        mask = r.random(4) < 0.75
        if not mask.any():
            mask[r.integers(4)] = True
        lg = np.where(mask, logits, -1e9)
        e = np.exp(lg - lg.max())
        probs[i] = (e / e.sum()).astype(np.float32)
    seeds = [3, 99, 2**40 + 17, 7390452496230446618]
    idx = np.zeros((len(seeds), n), dtype=np.int8)
    for k, s in enumerate(seeds):
        g = np.random.default_rng(s)
        for i in range(n):
            idx[k, i] = int(g.choice(4, p=probs[i]))
    np.savez_compressed(os.path.join(HERE, "choice.npz"), probs=probs, seeds=np.array(seeds, dtype=np.uint64), idx=idx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    G = _load(os.path.join(a.ref, "src", "game2048.py"), "ref_game2048")
    M = _load(os.path.join(a.ref, "src", "MLP.py"), "ref_mlp")
    jobs = dict(row_table=(gen_row_table, G), pcg64=(gen_pcg, G), episodes=(gen_episodes, G),
                crafted=(gen_crafted, G), mlp=(gen_mlp, M), choice=(gen_choice, G))
    for name, (fn, mod) in jobs.items():
        if a.only and name not in a.only.split(","):
            continue
        fn(mod)
        print("wrote", name)


if __name__ == "__main__":
    main()
