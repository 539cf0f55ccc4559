"""Loaders for the fixtures tests/golden/make_golden_ref.py generated from the REAL reference (src/env.py,
src/reinforce_agent.py, runner.py).  Test infrastructure only: the oracle rebuilds reference-format observations
(src/env.py:131-171) from the recorded bitboards, so the fixtures store boards, not obs."""
from __future__ import annotations

import json
import os

import numpy as np

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_cache: dict = {}


def load(name: str):
    if name not in _cache:
        with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
            _cache[name] = {k: z[k] for k in z.files}
    return _cache[name]


def env_configs() -> list[dict]:
    return json.loads(str(load("env_steps")["configs"]))


def update_cases() -> list[dict]:
    return json.loads(str(load("update")["cases"]))


def _n_update_cases() -> int:
    with np.load(os.path.join(GOLDEN, "update.npz"), allow_pickle=False) as z:
        return len(json.loads(str(z["cases"])))


N_UPDATE_CASES = _n_update_cases()


def n_layers(case: dict) -> int:
    return len(case["mlp"]["hidden_sizes"]) + 1


def params_of(ci: int, prefix: str, L: int) -> dict:
    """prefix: "init_actor", "init_critic", "up{u}_actor", "up{u}_critic" -> {"W": [...], "b": [...]}."""
    d = load("update")
    flat = [d[f"u{ci}_{prefix}_{j}"] for j in range(2 * L)]
    return {"W": [a.copy() for a in flat[:L]], "b": [a.copy() for a in flat[L:]]}


def has(ci: int, key: str) -> bool:
    return f"u{ci}_{key}" in load("update")


def arr(ci: int, key: str):
    return load("update")[f"u{ci}_{key}"]


def obs_cfg(env: dict) -> dict:
    return dict(obs_mode=env.get("obs_mode", "raw"), obs_log2_scale=env.get("obs_log2_scale", 1.0))


_obs_cache: dict = {}


def obs_for(board: int, env: dict):
    """Reference-format obs of a bitboard under an env config (dict with mask, or the bare board)."""
    key = (int(board), env.get("obs_mode", "raw"), env.get("obs_log2_scale", 1.0), env.get("use_action_mask", True))
    if key not in _obs_cache:
        x, m = O.obs_of_bitboard(int(board), **obs_cfg(env))
        b = x.reshape(4, 4, 17) if x.size == 272 else x.reshape(4, 4)
        _obs_cache[key] = (b, m)
    b, m = _obs_cache[key]
    if env.get("use_action_mask", True):
        return {"board": b.copy(), "action_mask": m.copy()}
    return b.copy()


def trajectories(ci: int, u: int, case: dict) -> list[dict]:
    """The reference trajectory dicts of update u of case ci (src/reinforce_agent.py:240-247), obs rebuilt."""
    P = f"up{u}_"
    lens = arr(ci, P + "lengths")
    boards, acts, rews = arr(ci, P + "boards"), arr(ci, P + "actions"), arr(ci, P + "rewards")
    tot, mt = arr(ci, P + "total_reward"), arr(ci, P + "max_tile")
    out, s = [], 0
    for i, T in enumerate(lens):
        T = int(T)
        out.append({"obs": [obs_for(int(b), case["env"]) for b in boards[s:s + T]],
                    "actions": [int(a) for a in acts[s:s + T]],
                    "rewards": [float(r) for r in rews[s:s + T]],
                    "total_reward": float(tot[i]), "states": [], "max_tile": int(mt[i])})
        s += T
    return out


_exact_cache: dict = {}


def exact_grads(ci: int, u: int, case: dict) -> dict:
    """Pre-clip gradients of update u of case ci evaluated in fp64 (oracle/agent_oracle.py with dtype=float64) at
    the reference's parameters before that update: the exact value of the reference's formula, against which
    the reference's own fp32 sequential accumulation and ours are both measured."""
    key = (ci, u)
    if key not in _exact_cache:
        from oracle import agent_oracle as AO

        L = n_layers(case)
        pre = "init" if u == 0 else f"up{u - 1}"
        crit = has(ci, "init_critic_0")
        ag = {k: v for k, v in case["agent"].items() if k != "model_seed"}
        ora = AO.OracleAgent(params_of(ci, f"{pre}_actor", L), params_of(ci, f"{pre}_critic", L) if crit else None,
                             AO.AgentCfg(**ag, activation=case["mlp"]["activation"]), dtype=np.float64)
        ora.update_batch(trajectories(ci, u, case))
        gW, gb = ora.captured["actor_grads"]
        out = {"actor": gW + gb}
        if crit:
            cW, cb = ora.captured["critic_grads"]
            out["critic"] = cW + cb
        _exact_cache[key] = out
    return _exact_cache[key]


def assert_grad_parity(got, ref, exact_fn, what="") -> None:
    """North-star gradient parity: within 1e-5 normwise-relative of the reference -- or, where the reference's
    own fp32 sequential accumulation over N steps is itself further than that from the exact (fp64) value of its
    formula, at least as close to the exact value as the reference is."""
    e = rel(got, ref)
    if e < 1e-5:
        return
    exact = exact_fn()
    e_got, e_ref = rel(got, exact), rel(ref, exact)
    assert e_got <= max(e_ref, 1e-5), (what, "vs reference", e, "vs exact", e_got, "reference vs exact", e_ref)


def assert_norm_parity(got: float, ref: float, exact_grads_fn, what="") -> None:
    """clip_grads_global_norm's norm: within 1e-5 of the reference's, or at least as close to the norm of the exact
    gradients as the reference's is."""
    if abs(got - ref) <= 1e-5 * ref:
        return
    ex = float(np.sqrt(sum(float(np.sum(np.asarray(g, np.float64) ** 2)) for g in exact_grads_fn())))
    assert abs(got - ex) <= max(abs(ref - ex), 1e-5 * ex), (what, got, ref, ex)


def rel(a, b) -> float:
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)) if b.size else 0.0


def adam_state(agent, critic: bool = False):
    """Copies of the agent's Adam moments ([W..., b...] order, as the gradients) and step counter."""
    if critic:
        mW, vW, mB, vB, t = agent._adam_m_W_c, agent._adam_v_W_c, agent._adam_m_B_c, agent._adam_v_B_c, agent._adam_t_c
    else:
        mW, vW, mB, vB, t = agent._adam_m_W, agent._adam_v_W, agent._adam_m_B, agent._adam_v_B, agent._adam_t
    host = lambda ts: [x.detach().cpu().numpy().astype(np.float64) for x in ts]  # noqa: E731
    return host(mW) + host(mB), host(vW) + host(vB), int(t)


def assert_adam_step_exact(after, before, grads, state, lr, sign, b1, b2, max_norm, what="") -> None:
    """One Adam update (src/reinforce_agent.py:719-770, after clip_grads_global_norm :835-861) checked on the exact
    basis: the parameter step taken equals the fp64 evaluation of the Adam formula -- clip coefficient, moments
    with bias correction, eps outside the sqrt -- applied to OUR pre-clip gradient (held to the exact value of the
    reference's formula by assert_grad_parity) and our previous moments, on every element, within the fp32
    rounding of the step and of the parameter.  (Elements whose gradient is rounding noise take a step of either
    sign of up to ~lr; compared with the reference's own noise they cannot be matched, compared with the formula
    they can.)"""
    m0, v0, t = state
    g = [np.asarray(x, np.float64) for x in grads]
    norm = float(np.sqrt(sum(float(np.sum(x * x)) for x in g)))
    coef = min(1.0, max_norm / max(norm, 1e-8))
    t1 = t + 1
    bc1, bc2 = 1.0 - b1 ** t1, 1.0 - b2 ** t1
    for k, (a, b, gi, m, v) in enumerate(zip(after, before, g, m0, v0)):
        a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
        gc = gi * coef
        mn = b1 * m + (1.0 - b1) * gc
        vn = b2 * v + (1.0 - b2) * gc * gc
        step = sign * lr * (mn / bc1) / (np.sqrt(vn / bc2) + 1e-8)
        tol = 1e-6 * lr + 2.0 ** -23 * np.abs(b) + 1e-5 * np.abs(step)
        bad = np.abs((a - b) - step) > tol
        assert not bad.any(), (what, k, int(bad.sum()), (a - b)[bad][:5], step[bad][:5])
