"""Generate env / agent / runner fixtures from the REAL reference (build container only).

    python tests/golden/make_golden_ref.py [--ref /root/reference] [--only env,obs,sym,update,small,runner]
                                           [--update-from K]   (append update cases K.. to update.npz)

Imports the reference's own modules -- src/env.py, src/reinforce_agent.py, src/MLP.py, src/utils/*, runner.py --
by package path from ``--ref`` with ``sys.dont_write_bytecode`` set (nothing is written into the reference tree).
``gymnasium`` is not installed in this image; tests/golden/gym_shim/ provides the behaviour-neutral stand-in that
SURVEY.md section 8(c) describes (Env.reset no-op, Discrete.contains, inert Box / Dict).  The reference's
computations are then run unchanged; the only instrumentation wraps methods to RECORD their inputs / outputs
(select_action, clip_grads_global_norm, _compute_advantages, _compute_episode_rank_weights) and forwards to the
original.

Fixtures written (data only: inputs and the reference's outputs; boards as exponent bitboards, nibble r*4+c):
  env_steps.npz   Game2048Env.reset / step under 8 Game2048EnvConfigs (src/env.py:174-302): reward (fp64),
                  terminated, truncated, invalid_action, max_tile_seen, score, step_index, obs, mask per step
  obs_enc.npz     _preprocess_board + _get_obs + encode_observation (src/env.py:131-171, src/MLP.py:22-43)
  symmetries.npz  Game2048Env.get_symmetries (src/env.py:317-398) on log2-dict / raw-bare / onehot-dict obs
  update.npz      ReinforceAgent.run_episode + update_batch (src/reinforce_agent.py:195-620): per case and update,
                  the trajectories (boards, actions, fp64 rewards, the probabilities select_action drew from),
                  rank weights, advantage inputs (returns / TD errors) and outputs, pre-clip gradients captured
                  at clip_grads_global_norm (:835), norms, post-update parameters
  small.npz       compute_returns (:255) on non-dyadic fp64 rewards; _compute_episode_rank_weights (:681) on
                  near-tied totals; _compute_weighted_stats (:864)
  runner.npz      runner.py training_loop (:495-679) CSV rows + final actor, evaluation_loop (:737-828) summaries
"""
from __future__ import annotations

import argparse
import csv
import json
import logging
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import pack, seed_iter  # noqa: E402  (same directory; board packing + runner seed stream)


def import_reference(ref: str):
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(HERE, "gym_shim"))
    sys.path.insert(0, ref)
    import src.env as E  # noqa: E402
    import src.MLP as M  # noqa: E402
    import src.reinforce_agent as RA  # noqa: E402
    return E, RA, M


def _mask_bits(m) -> int:
    return int(sum(int(b) << i for i, b in enumerate(m)))


# ================================================================================================== env steps
ENV_CFGS = [
    dict(),
    dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5),
    dict(obs_mode="log2", obs_log2_scale=0.1, reward_mode="sum", base_reward_scale=0.1, empty_tile_reward=0.05,
         merge_reward=0.3, bonus_mode="raw", bonus_scale=0.7, step_reward=-0.01, endgame_penalty=-10.0,
         max_steps=150),
    dict(obs_mode="onehot", reward_mode="log2", base_reward_scale=1 / 3, bonus_mode="log2", bonus_scale=1.5,
         use_action_mask=False, invalid_action_penalty=-0.25, max_steps=60),
    dict(obs_mode="raw", use_action_mask=False, reward_mode="sum", empty_tile_reward=0.1, max_steps=None),
    dict(obs_mode="log2", obs_log2_scale=1.0, reward_mode="sum", base_reward_scale=0.01, bonus_mode="raw",
         bonus_scale=0.01, endgame_penalty=-1.5, merge_reward=0.1, max_steps=40),
    dict(obs_mode="onehot", reward_mode="log2", max_steps=1),
    dict(obs_mode="log2", obs_log2_scale=0.3, use_action_mask=False, step_reward=0.1, reward_mode="log2",
         base_reward_scale=0.7, bonus_mode="log2", bonus_scale=0.3, endgame_penalty=-2.0, max_steps=300),
]


def _obs_flat(obs):
    board = obs["board"] if isinstance(obs, dict) else obs
    return np.asarray(board, dtype=np.float32).reshape(-1)


def gen_env(E, RA, M):
    rng = np.random.default_rng(20480)
    it = seed_iter(11)
    data = {"configs": np.array(json.dumps(ENV_CFGS))}
    for c, kw in enumerate(ENV_CFGS):
        cfg = E.Game2048EnvConfig(**kw)
        env = E.Game2048Env(cfg)
        cap = 600 if cfg.max_steps is None else cfg.max_steps + 5
        ep_seed, ep_start, ep_len, r_board, r_obs, r_mask, r_score = [], [], [], [], [], [], []
        st = {k: [] for k in ("action", "board_prev", "board", "reward", "terminated", "truncated", "invalid",
                              "max_tile_seen", "score", "step_index", "mask", "obs", "merged_sum")}
        for e in range(6):
            seed = next(it)
            obs, info = env.reset(seed=seed)
            ep_seed.append(seed)
            ep_start.append(len(st["action"]))
            r_board.append(pack(env.game.board))
            r_obs.append(_obs_flat(obs))
            r_mask.append(_mask_bits(env.game.get_action_mask()))
            r_score.append(info["score"])
            assert env.max_tile_seen == 4
            t = 0
            while t < cap:
                m = env.game.get_action_mask()
                valid = [i for i, v in enumerate(m) if v]
                a = int(rng.integers(4)) if (e < 3 or not valid) else int(valid[int(rng.integers(len(valid)))])
                bprev = pack(env.game.board)
                obs, r, term, trunc, info = env.step(a)
                assert isinstance(r, float)
                st["action"].append(a)
                st["board_prev"].append(bprev)
                st["board"].append(pack(env.game.board))
                st["reward"].append(r)
                st["terminated"].append(term)
                st["truncated"].append(trunc)
                st["invalid"].append(bool(info["invalid_action"]))
                st["max_tile_seen"].append(env.max_tile_seen)
                st["score"].append(info["score"])
                st["step_index"].append(info["step_index"])
                st["mask"].append(_mask_bits(env.game.get_action_mask()))
                st["obs"].append(_obs_flat(obs))
                st["merged_sum"].append(sum(info["merged"]))
                if isinstance(obs, dict):
                    assert _mask_bits(obs["action_mask"]) == st["mask"][-1]
                t += 1
                if term or trunc:
                    break
            ep_len.append(t)
        p = f"c{c}_"
        data[p + "ep_seed"] = np.array(ep_seed, dtype=np.uint64)
        data[p + "ep_start"] = np.array(ep_start, dtype=np.int64)
        data[p + "ep_len"] = np.array(ep_len, dtype=np.int64)
        data[p + "reset_board"] = np.array(r_board, dtype=np.uint64)
        data[p + "reset_obs"] = np.array(r_obs, dtype=np.float32)
        data[p + "reset_mask"] = np.array(r_mask, dtype=np.uint8)
        data[p + "reset_score"] = np.array(r_score, dtype=np.int64)
        dt = dict(action=np.uint8, board_prev=np.uint64, board=np.uint64, reward=np.float64, terminated=np.bool_,
                  truncated=np.bool_, invalid=np.bool_, max_tile_seen=np.int64, score=np.int64, step_index=np.int64,
                  mask=np.uint8, obs=np.float32, merged_sum=np.int64)
        for k, v in st.items():
            data[p + k] = np.array(v, dtype=dt[k])
        print(f"  env cfg {c}: {len(st['action'])} steps, "
              f"{int(np.sum(data[p + 'terminated']))} terminated, {int(np.sum(data[p + 'truncated']))} truncated, "
              f"{int(np.sum(data[p + 'invalid']))} invalid")
    np.savez_compressed(os.path.join(HERE, "env_steps.npz"), **data)


# ================================================================================================== obs encodings
OBS_CFGS = [("raw", 1.0), ("log2", 1.0), ("log2", 0.0625), ("log2", 0.1), ("log2", 1 / 3), ("onehot", 1.0)]


def gen_obs(E, RA, M):
    rng = np.random.default_rng(131)
    exps = []
    for _ in range(200):
        e = rng.integers(1, 16, size=16)
        e[rng.random(16) < rng.choice([0.0, 0.3, 0.7])] = 0
        exps.append(e)
    exps += [np.full(16, 15), np.zeros(16, dtype=np.int64), np.arange(16), np.arange(16)[::-1]]
    big = np.zeros(16, dtype=np.int64)
    big[5] = 16                                      # 65536: representable by the reference, not by a nibble
    exps.append(big)
    exps = np.array(exps, dtype=np.int64)
    vals = np.where(exps > 0, np.left_shift(np.int64(1), exps), 0).astype(np.int64)
    data = {"values": vals, "configs": np.array(json.dumps(OBS_CFGS))}
    for k, (mode, scale) in enumerate(OBS_CFGS):
        env = E.Game2048Env(E.Game2048EnvConfig(obs_mode=mode, obs_log2_scale=scale))
        env.reset(seed=0)
        xs, ms, pre = [], [], []
        for v in vals:
            env.game.board = v.reshape(4, 4).copy()
            obs = env._get_obs()
            x, m = M.encode_observation(obs)
            xs.append(x)
            ms.append(m)
            pre.append(env._preprocess_board(env.game.board).shape)
            assert np.array_equal(obs["board"].reshape(-1), x)
        data[f"k{k}_x"] = np.array(xs, dtype=np.float32)
        data[f"k{k}_mask"] = np.array(ms, dtype=np.int8)
        data[f"k{k}_shape"] = np.array(pre[0], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "obs_enc.npz"), **data)


# ================================================================================================== symmetries
def gen_sym(E, RA, M):
    rng = np.random.default_rng(8)
    data = {}
    kinds = [("log2", True), ("raw", False), ("onehot", True), ("log2", False)]
    for k, (mode, with_mask) in enumerate(kinds):
        env = E.Game2048Env(E.Game2048EnvConfig(obs_mode=mode, obs_log2_scale=0.25, use_action_mask=with_mask))
        env.reset(seed=0)
        b_in, m_in, a_in, b_out, m_out, a_out = [], [], [], [], [], []
        for i in range(24):
            e = rng.integers(0, 12, size=16)
            env.game.board = np.where(e > 0, np.left_shift(np.int64(1), e), 0).reshape(4, 4).astype(np.int64)
            obs = env._get_obs()
            for a in range(4):
                syms = E.Game2048Env.get_symmetries(obs, a)
                assert len(syms) == 8
                b_in.append(_obs_flat(obs))
                m_in.append(obs["action_mask"] if with_mask else np.zeros(4, np.int8))
                a_in.append(a)
                b_out.append([_obs_flat(s[0]) for s in syms])
                m_out.append([s[0]["action_mask"] if with_mask else np.zeros(4, np.int8) for s in syms])
                a_out.append([s[1] for s in syms])
        data[f"k{k}_board_in"] = np.array(b_in, dtype=np.float32)
        data[f"k{k}_mask_in"] = np.array(m_in, dtype=np.int8)
        data[f"k{k}_action_in"] = np.array(a_in, dtype=np.uint8)
        data[f"k{k}_board_out"] = np.array(b_out, dtype=np.float32)
        data[f"k{k}_mask_out"] = np.array(m_out, dtype=np.int8)
        data[f"k{k}_action_out"] = np.array(a_out, dtype=np.uint8)
        data[f"k{k}_kind"] = np.array(json.dumps([mode, with_mask]))
    np.savez_compressed(os.path.join(HERE, "symmetries.npz"), **data)


# ================================================================================================== update_batch
ENV_A = dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5, max_steps=120)
ENV_B = dict(obs_mode="log2", obs_log2_scale=0.1, reward_mode="sum", base_reward_scale=0.1, empty_tile_reward=0.01,
             bonus_mode="log2", bonus_scale=0.3, endgame_penalty=-0.7, max_steps=100)
MLP_S = dict(hidden_sizes=[32, 16], activation="ReLU", init_distribution="HeNormal", last_init_normal=True)


def _update_cases():
    cases = []
    k = 0
    for baseline in ("off", "each", "batch", "batch_norm"):
        for opt in ("sgd", "adam"):
            for critic in (None, "mse", "huber"):
                ag = dict(gamma=0.99, learning_rate=1e-2, baseline_mode=baseline, optimizer=opt, model_seed=k)
                if critic:
                    ag.update(use_critic=True, critic_loss_type=critic, critic_learning_rate=5e-3, huber_delta=0.5)
                cases.append(dict(name=f"{baseline}-{opt}-{critic or 'reinforce'}", env=ENV_A if k % 2 == 0 else ENV_B,
                                  mlp=MLP_S, agent=ag, n=6, updates=2))
                k += 1
    extra = [
        dict(name="rank3211-batchnorm", env=ENV_B, mlp=MLP_S, agent=dict(
            gamma=0.99, learning_rate=1e-2, baseline_mode="batch_norm", reward_rank_weights=[3.0, 2.0, 1.0, 1.0],
            model_seed=101)),
        dict(name="rank10-critic-adam", env=ENV_A, mlp=MLP_S, agent=dict(
            gamma=0.97, learning_rate=1e-2, baseline_mode="batch", reward_rank_weights=[1.0, 0.0], optimizer="adam",
            use_critic=True, critic_learning_rate=1e-2, model_seed=102)),
        dict(name="aug-batch", env=ENV_A, mlp=MLP_S, agent=dict(
            gamma=0.99, learning_rate=1e-2, baseline_mode="batch", augmentation=True, model_seed=103)),
        dict(name="aug-critic-huber-adam", env=ENV_B, mlp=MLP_S, agent=dict(
            gamma=0.99, learning_rate=1e-2, baseline_mode="batch_norm", augmentation=True, optimizer="adam",
            use_critic=True, critic_loss_type="huber", huber_delta=0.3, model_seed=104)),
        dict(name="onehot-sigmoid-critic", env=dict(ENV_A, obs_mode="onehot"), mlp=dict(
            hidden_sizes=[32, 16], activation="Sigmoid", init_distribution="XavierNormal", last_init_normal=True),
            agent=dict(gamma=0.99, learning_rate=1e-2, baseline_mode="batch", optimizer="adam", use_critic=True,
                       model_seed=105)),
        dict(name="raw-sigmoid-24x40-each", env=dict(ENV_B, obs_mode="raw"), mlp=dict(
            hidden_sizes=[24, 40], activation="Sigmoid", init_distribution="XavierUniform", last_init_normal=True),
            agent=dict(gamma=0.95, learning_rate=1e-2, baseline_mode="each", model_seed=106)),
        dict(name="noclip-off-gamma1", env=ENV_A, mlp=MLP_S, agent=dict(
            gamma=1.0, learning_rate=1e-2, baseline_mode="off", max_grad_norm=1e9, model_seed=107)),
        dict(name="clip005-critic", env=ENV_B, mlp=MLP_S, agent=dict(
            gamma=0.99, learning_rate=1e-2, baseline_mode="batch", max_grad_norm=0.05, use_critic=True,
            model_seed=108)),
        dict(name="runner256-batch-sgd", env=dict(ENV_A, max_steps=1024), mlp=dict(
            hidden_sizes=[256, 256], activation="ReLU", init_distribution="HeNormal", last_init_normal=True),
            agent=dict(gamma=0.99, learning_rate=1e-4, baseline_mode="batch", model_seed=0), n=4, updates=1),
        dict(name="runner256-critic-adam", env=dict(ENV_B, max_steps=1024), mlp=dict(
            hidden_sizes=[256, 256], activation="ReLU", init_distribution="HeNormal", last_init_normal=True),
            agent=dict(gamma=0.99, learning_rate=1e-4, baseline_mode="batch_norm", optimizer="adam", use_critic=True,
                       critic_learning_rate=1e-4, model_seed=1), n=4, updates=1),
        # round 4: one-hot first layers and depth != 2 (the fused-kernel families of g2048_deep.hip); the first is
        # the configuration runner.py documents in its header (runner.py:10-47), max_steps None included
        dict(name="refconf-onehot-256-128-64", env=dict(
            obs_mode="onehot", obs_log2_scale=1.0, reward_mode="log2", base_reward_scale=1.0, bonus_mode="off",
            bonus_scale=1.0, step_reward=0.0, endgame_penalty=0.0, use_action_mask=True, invalid_action_penalty=-1.0,
            max_steps=None, empty_tile_reward=0.05, merge_reward=0.0), mlp=dict(
            hidden_sizes=[256, 128, 64], activation="ReLU", init_distribution="HeNormal", last_init_normal=True),
            agent=dict(gamma=0.99, learning_rate=0.01, baseline_mode="batch", model_seed=0, optimizer="adam",
                       adam_beta1=0.9, adam_beta2=0.999, augmentation=False, use_critic=True,
                       critic_learning_rate=0.0005, critic_loss_type="mse", huber_delta=1.0), n=4, updates=2),
        dict(name="deep3-log2-batch-sgd", env=ENV_A, mlp=dict(
            hidden_sizes=[64, 48, 32], activation="ReLU", init_distribution="HeNormal", last_init_normal=True),
            agent=dict(gamma=0.99, learning_rate=1e-2, baseline_mode="batch", model_seed=109)),
        dict(name="onehot-relu-128x64-huber", env=dict(ENV_B, obs_mode="onehot"), mlp=dict(
            hidden_sizes=[128, 64], activation="ReLU", init_distribution="HeNormal", last_init_normal=True),
            agent=dict(gamma=0.99, learning_rate=1e-2, baseline_mode="batch_norm", optimizer="adam", use_critic=True,
                       critic_loss_type="huber", huber_delta=0.5, critic_learning_rate=5e-3, model_seed=110)),
        dict(name="deep4-onehot-sigmoid-each", env=dict(ENV_A, obs_mode="onehot"), mlp=dict(
            hidden_sizes=[40, 33, 20, 10], activation="Sigmoid", init_distribution="XavierNormal",
            last_init_normal=True), agent=dict(gamma=0.95, learning_rate=1e-2, baseline_mode="each", model_seed=111)),
        dict(name="onehot-relu-aug-critic", env=dict(ENV_A, obs_mode="onehot"), mlp=dict(
            hidden_sizes=[64, 32], activation="ReLU", init_distribution="HeNormal", last_init_normal=True),
            agent=dict(gamma=0.99, learning_rate=1e-2, baseline_mode="batch", augmentation=True, use_critic=True,
                       model_seed=112), n=4),
        # round 5: a one-hot [256, 256] actor-critic -- 64 dense 32x32 weight-gradient tiles, the largest net
        # g2048_deep_grad holds in registers (its 8-wave, 8-tiles-per-wave instantiation)
        dict(name="onehot-relu-256x256-critic-adam", env=dict(ENV_B, obs_mode="onehot", max_steps=300), mlp=dict(
            hidden_sizes=[256, 256], activation="ReLU", init_distribution="HeNormal", last_init_normal=True),
            agent=dict(gamma=0.99, learning_rate=1e-3, baseline_mode="batch", optimizer="adam", use_critic=True,
                       critic_learning_rate=1e-3, model_seed=113), n=4, updates=1),
    ]
    for e in extra:
        e.setdefault("n", 6)
        e.setdefault("updates", 2)
    return cases + extra


def _params_flat(p):
    # copies: the reference's SGD updates parameters in place (src/reinforce_agent.py:568-575)
    return [np.array(a, dtype=np.float32, copy=True) for a in list(p["W"]) + list(p["b"])]


def run_update_case(E, RA, M, case, ci):
    env = E.Game2048Env(E.Game2048EnvConfig(**case["env"]))
    agent = RA.ReinforceAgent(env, M.MLPConfig(**case["mlp"]), RA.ReinforceAgentConfig(**case["agent"]))
    out = {}
    P = f"u{ci}_"
    for j, a in enumerate(_params_flat(agent.params)):
        out[P + f"init_actor_{j}"] = a
    if agent.critic_params is not None:
        for j, a in enumerate(_params_flat(agent.critic_params)):
            out[P + f"init_critic_{j}"] = a
    steplog = []
    orig_sel = agent.select_action

    def sel(obs, rng, action_fn=None, use_greedy=False):
        b = pack(agent.env.game.board)
        a, probs, acts, pres = orig_sel(obs, rng, action_fn, use_greedy)
        steplog.append((b, a, np.asarray(probs, dtype=np.float32).copy()))
        return a, probs, acts, pres

    agent.select_action = sel
    cap: dict = {}
    orig_clip = agent.clip_grads_global_norm

    def clip(gW, gb):
        cap.setdefault("grads", []).append([np.array(g, dtype=np.float32) for g in list(gW) + list(gb)])
        nrm = orig_clip(gW, gb)
        cap.setdefault("norms", []).append(float(nrm))
        return nrm

    agent.clip_grads_global_norm = clip
    orig_adv = agent._compute_advantages

    def adv(values_list, w):
        res = orig_adv(values_list, w)
        cap["adv_in"] = np.concatenate([np.asarray(v, dtype=np.float32) for v in values_list]) \
            if len(values_list) else np.zeros(0, np.float32)
        cap["adv_out"] = np.concatenate([np.asarray(v, dtype=np.float32) for v in res]) \
            if len(res) else np.zeros(0, np.float32)
        cap["adv_w"] = np.asarray(w, dtype=np.float32).copy()
        return res

    agent._compute_advantages = adv
    orig_rw = agent._compute_episode_rank_weights

    def rw(totals):
        res = orig_rw(totals)
        cap["rank_w"] = np.asarray(res, dtype=np.float32).copy()
        return res

    agent._compute_episode_rank_weights = rw
    it_e, it_p = seed_iter(1000 + ci), seed_iter(2000 + ci)
    for u in range(case["updates"]):
        n = case["n"]
        es = [next(it_e) for _ in range(n)]
        ps = [next(it_p) for _ in range(n)]
        trajs = []
        steplog.clear()
        for e_s, p_s in zip(es, ps):
            trajs.append(agent.run_episode(e_s, p_s))
        lens = np.array([len(t["actions"]) for t in trajs], dtype=np.int64)
        assert len(steplog) == lens.sum()
        acts = np.array([s[1] for s in steplog], dtype=np.uint8)
        assert np.array_equal(acts, np.concatenate([np.array(t["actions"], np.uint8) for t in trajs]))
        Q = P + f"up{u}_"
        out[Q + "env_seeds"] = np.array(es, dtype=np.uint64)
        out[Q + "policy_seeds"] = np.array(ps, dtype=np.uint64)
        out[Q + "lengths"] = lens
        out[Q + "boards"] = np.array([s[0] for s in steplog], dtype=np.uint64)
        out[Q + "actions"] = acts
        out[Q + "probs"] = np.array([s[2] for s in steplog], dtype=np.float32)
        out[Q + "rewards"] = np.concatenate([np.array(t["rewards"], dtype=np.float64) for t in trajs])
        out[Q + "total_reward"] = np.array([t["total_reward"] for t in trajs], dtype=np.float64)
        out[Q + "max_tile"] = np.array([t["max_tile"] for t in trajs], dtype=np.int64)
        cap.clear()
        agent.update_batch(trajs)
        out[Q + "rank_w"] = cap["rank_w"]
        out[Q + "adv_in"] = cap["adv_in"]
        out[Q + "adv_out"] = cap["adv_out"]
        out[Q + "adv_w"] = cap["adv_w"]
        out[Q + "actor_norm"] = np.array(cap["norms"][0], dtype=np.float64)
        for j, g in enumerate(cap["grads"][0]):
            out[Q + f"actor_grad_{j}"] = g
        for j, a in enumerate(_params_flat(agent.params)):
            out[Q + f"actor_{j}"] = a
        if agent.critic_params is not None:
            out[Q + "critic_norm"] = np.array(cap["norms"][1], dtype=np.float64)
            for j, g in enumerate(cap["grads"][1]):
                out[Q + f"critic_grad_{j}"] = g
            for j, a in enumerate(_params_flat(agent.critic_params)):
                out[Q + f"critic_{j}"] = a
    return out


def gen_update(E, RA, M, start: int = 0):
    """All update cases, or (start > 0) only cases start.. appended to the existing update.npz, whose first `start`
    cases must be the current list's (their arrays are kept as they are)."""
    cases = _update_cases()
    data = {"cases": np.array(json.dumps(cases))}
    if start:
        with np.load(os.path.join(HERE, "update.npz")) as z:
            old = json.loads(str(z["cases"]))
            assert old[:start] == json.loads(json.dumps(cases[:start])), "existing cases differ from the list"
            for k in z.files:
                if k != "cases" and int(k[1:k.index("_")]) < start:
                    data[k] = z[k]
    for ci, case in enumerate(cases):
        if ci < start:
            continue
        data.update(run_update_case(E, RA, M, case, ci))
        print(f"  update case {ci} {case['name']}: "
              f"{[int(data[f'u{ci}_up{u}_lengths'].sum()) for u in range(case['updates'])]} steps")
    np.savez_compressed(os.path.join(HERE, "update.npz"), **data)


# ================================================================================================== small pieces
def gen_small(E, RA, M):
    env = E.Game2048Env(E.Game2048EnvConfig())
    data = {}
    r = np.random.default_rng(5)
    # compute_returns: fp64 Python rewards (non-dyadic), several gammas
    rewards = [float(x) for x in (r.integers(0, 40, size=700) * 0.1 + r.standard_normal(700) * 1e-3)]
    data["returns_rewards"] = np.array(rewards, dtype=np.float64)
    for gi, g in enumerate((1.0, 0.99, 0.9, 0.5)):
        ag = RA.ReinforceAgent(env, RA.MLPConfig(hidden_sizes=[4]), RA.ReinforceAgentConfig(gamma=g))
        data[f"returns_g{gi}"] = ag.compute_returns(rewards)
        data[f"returns_gamma{gi}"] = np.array(g)
    # rank weights on near-tied totals (distinct fp64 values that round to the same fp32 value) straddling bins
    confs = [[3.0, 2.0, 1.0, 1.0], [1.0, 0.0], [0.5, 1.5, 2.5], [2.0]]
    tot_sets = []
    base = 1234.5678
    t1 = [base + k * 1e-9 for k in range(8)] + [base - 1.0, base + 1.0, 0.1 * 3, 0.3, 0.30000000000000004, 7.0]
    r.shuffle(t1)
    tot_sets.append(t1)
    tot_sets.append([float(x) for x in np.round(r.standard_normal(37) * 10, 1)])           # exact ties
    tot_sets.append([0.1 * k for k in range(20)] + [0.1 * k + 1e-12 for k in range(20)])
    for si, tot in enumerate(tot_sets):
        data[f"rank_totals{si}"] = np.array(tot, dtype=np.float64)
        for cj, conf in enumerate(confs):
            ag = RA.ReinforceAgent(env, RA.MLPConfig(hidden_sizes=[4]),
                                   RA.ReinforceAgentConfig(reward_rank_weights=conf))
            w = ag._compute_episode_rank_weights(tot)
            data[f"rank_w{si}_{cj}"] = np.asarray(w, dtype=np.float32)
    data["rank_confs"] = np.array(json.dumps(confs))
    # weighted stats
    vals = r.standard_normal(500).astype(np.float32) * 3 + 1
    w = np.repeat(r.choice([0.5, 1.0, 2.0], size=50).astype(np.float32), 10)
    ag = RA.ReinforceAgent(env, RA.MLPConfig(hidden_sizes=[4]), RA.ReinforceAgentConfig())
    m, s = ag._compute_weighted_stats(vals, w)
    data.update(ws_values=vals, ws_weights=w, ws_mean=np.array(m, dtype=np.float64), ws_std=np.array(s, dtype=np.float64))
    np.savez_compressed(os.path.join(HERE, "small.npz"), **data)


# ================================================================================================== runner
RUNNER_CONF = {
    "env": dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5, max_steps=200),
    "mlp": dict(hidden_sizes=[32, 16], activation="ReLU", init_distribution="HeNormal", last_init_normal=True),
    "agent": dict(gamma=0.99, learning_rate=1e-2, baseline_mode="batch", model_seed=0, optimizer="adam"),
    "train": dict(batch_size=8, num_batches=3, env_base_seed=3, policy_base_seed=7),
    "eval": dict(num_episodes=12, env_base_seed=12345, policy_base_seed=54321, model_path=None, use_greedy=True),
}


class _Grab(logging.Handler):
    def __init__(self):
        super().__init__(level=logging.INFO)
        self.records = []

    def emit(self, rec):
        self.records.append(rec)


def gen_runner(E, RA, M, ref):
    import runner as R  # noqa: E402  (the reference runner.py, on sys.path via import_reference)

    R.apply_config_overrides_from_dict(json.loads(json.dumps(RUNNER_CONF)))
    env, agent, env_config, mlp_config, agent_config, train_cfg = R.build_training_components()
    data = {"conf": np.array(json.dumps(RUNNER_CONF))}
    with tempfile.TemporaryDirectory() as td:
        R.training_loop(env, agent, env_config, mlp_config, agent_config, train_cfg, Path(td), "golden")
        with open(os.path.join(td, "training_stats.csv"), newline="") as f:
            rows = list(csv.DictReader(f))
        root = logging.getLogger()
        for h in list(root.handlers):
            if isinstance(h, logging.FileHandler):
                root.removeHandler(h)
                h.close()
    data["train_batch"] = np.array([int(x["batch"]) for x in rows], dtype=np.int64)
    for k in ("avg_reward", "max_reward", "min_reward"):
        data["train_" + k] = np.array([float(x[k]) for x in rows], dtype=np.float64)
    data["train_max_tile_counts"] = np.array([json.loads(x["max_tile_counts"]) for x in rows], dtype=np.int64)
    data["train_csv_header"] = np.array(json.dumps(list(rows[0].keys())))
    for j, a in enumerate(_params_flat(agent.params)):
        data[f"train_final_actor_{j}"] = a
    grab = _Grab()
    R.logger.addHandler(grab)
    prev = R.logger.level
    R.logger.setLevel(logging.INFO)
    for gi, greedy in enumerate((True, False)):
        grab.records.clear()
        ecfg = dict(RUNNER_CONF["eval"], use_greedy=greedy)
        R.evaluation_loop(env, agent, env_config, mlp_config, agent_config, ecfg)
        summ = [r for r in grab.records if r.msg.startswith("Evaluation summary")][0]
        tiles = [r for r in grab.records if r.msg.startswith("Max tile counts")][0]
        data[f"eval{gi}_summary"] = np.array([float(x) for x in summ.args[1:]], dtype=np.float64)
        data[f"eval{gi}_episodes"] = np.array(int(summ.args[0]))
        tile_summary = tiles.args if isinstance(tiles.args, dict) else tiles.args[0]   # logging unwraps a lone dict
        data[f"eval{gi}_max_tiles"] = np.array(json.dumps({int(k): v for k, v in tile_summary.items()}))
    R.logger.removeHandler(grab)
    R.logger.setLevel(prev)
    np.savez_compressed(os.path.join(HERE, "runner.npz"), **data)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="")
    ap.add_argument("--update-from", type=int, default=0, help="append update cases from this index on")
    a = ap.parse_args()
    E, RA, M = import_reference(a.ref)
    jobs = dict(env=gen_env, obs=gen_obs, sym=gen_sym, update=lambda E_, RA_, M_: gen_update(E_, RA_, M_, a.update_from),
                small=gen_small)
    for name, fn in jobs.items():
        if a.only and name not in a.only.split(","):
            continue
        fn(E, RA, M)
        print("wrote", name)
    if not a.only or "runner" in a.only.split(","):
        gen_runner(E, RA, M, a.ref)
        print("wrote runner")


if __name__ == "__main__":
    main()
