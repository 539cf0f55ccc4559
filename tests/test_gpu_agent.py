"""GPU parity of the policy / rollout / update hot path against the reference's MLP fixtures and the numpy
restatement of update_batch (oracle/agent_oracle.py).  Tolerances: fp32 forward 1e-5 relative; gradients and
updated parameters within 1e-5 normwise-relative (the north star's "policy gradient within 1e-5 fp32")."""
import os

import numpy as np
import pytest
import torch

from oracle import agent_oracle as AO
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def test_forward_matches_reference_mlp(golden_dir):
    from rl2048_amd.mlp import forward_logits, logits_to_probs

    d = np.load(os.path.join(golden_dir, "mlp.npz"))
    for name in ("he_relu_log2", "xn_onehot", "xu_critic", "normal_linear", "he_onehot_critic"):
        meta = d[f"{name}__meta"]
        L = int(meta[3]) + 1
        p = {"W": [torch.from_numpy(d[f"{name}__W{i}"]).to(DEV) for i in range(L)],
             "b": [torch.from_numpy(d[f"{name}__b{i}"]).to(DEV) for i in range(L)]}
        X = torch.from_numpy(d[f"{name}__X"]).to(DEV)
        for act in ("ReLU", "Sigmoid"):
            lg = forward_logits(p, X, act)[0].cpu().numpy()
            assert _rel(lg, d[f"{name}__logits_{act}"]) < 1e-5, (name, act)
        if f"{name}__mask" in d:
            pr = logits_to_probs(torch.from_numpy(d[f"{name}__logits_ReLU"]).to(DEV),
                                 torch.from_numpy(d[f"{name}__mask"]).to(DEV)).cpu().numpy()
            np.testing.assert_allclose(pr, d[f"{name}__probs"], rtol=1e-5, atol=1e-7)


def _agent(obs_mode="log2", hidden=(32, 16), act="ReLU", use_action_mask=True, **acfg):
    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    env_cfg = Game2048EnvConfig(obs_mode=obs_mode, obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5,
                                max_steps=300, use_action_mask=use_action_mask)
    return ReinforceAgent(env_cfg, MLPConfig(hidden_sizes=list(hidden), activation=act, init_distribution="HeNormal"),
                          ReinforceAgentConfig(**acfg), device=DEV)


def _np_params(p):
    return {k: [t.detach().cpu().numpy().copy() for t in v] for k, v in p.items()}


@pytest.mark.parametrize("path,mask", [("rollout", True), ("policy", True), ("gemm", True), ("rollout", False),
                                       ("gemm", False)])
def test_rollout_transitions_and_sampling_bit_exact(path, mask):
    """rollout_batch == the reference's run_episode: same env stream (transitions replayed in the oracle env) and
    the same policy stream (Generator.choice on the probabilities the device used).  path: "rollout" = the whole
    rollout in one launch (g2048_rollout); "policy" = per-step loop with the fused g2048_policy kernel; "gemm" =
    per-step loop with the GEMM forward + g2048_sample.  mask: use_action_mask (without it the logits are not
    masked, src/reinforce_agent.py:138-145)."""
    agent = _agent(use_action_mask=mask)
    agent.use_fused_policy = path != "gemm"
    agent.use_fused_rollout = path == "rollout"
    assert (agent._fused_policy_spec() is not None) == (path != "gemm")
    n = 48
    env_seeds = [int(s) for s in np.random.default_rng(3).integers(0, 2**62, size=n)]
    pol_seeds = [int(s) for s in np.random.default_rng(4).integers(0, 2**62, size=n)]
    batch = agent.rollout_batch(env_seeds, pol_seeds, record_probs=True)
    acts = batch.actions.cpu().numpy()
    rews = batch.rewards.cpu().numpy()
    lens = batch.lengths.cpu().numpy()
    probs = batch.probs.cpu().numpy()
    boards = batch.boards.cpu().numpy().view(np.uint64)
    for i in range(n):
        env = O.Env(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5, max_steps=300,
                    use_action_mask=mask)
        env.reset(env_seeds[i])
        pr = O.PCG64(pol_seeds[i])
        total = 0.0
        for t in range(lens[i]):
            assert O.pack_exponents(O.values_to_exponents(env.board)) == boards[t, i], (i, t)
            assert pr.choice4(probs[t, i]) == acts[t, i], (i, t)
            r = env.step(int(acts[t, i]))
            assert rews[t, i] == r["reward"]     # fp64 trajectory rewards, bit-exact
            total += r["reward"]
            done = r["terminated"] or r["truncated"]
            assert done == (t == lens[i] - 1)
        assert abs(total - float(batch.total_reward[i])) < 1e-6 * max(1.0, abs(total))
        assert int(batch.max_tile[i]) == env.max_tile_seen


@pytest.mark.parametrize("path", ["rollout", "policy", "gemm"])
def test_rollout_probs_match_numpy_softmax(path):
    agent = _agent()
    agent.use_fused_policy = path != "gemm"
    agent.use_fused_rollout = path == "rollout"
    batch = agent.rollout_batch(list(range(16)), list(range(100, 116)), record_probs=True)
    from rl2048_amd.mlp import forward_logits

    x, mk = agent._obs_from_boards(batch.boards.reshape(-1).contiguous())
    lg = forward_logits({k: [t.cpu() for t in v] for k, v in agent.params.items()}, x.cpu(), "ReLU")[0].numpy()
    p_ref = AO.logits_to_probs(lg, mk.cpu().numpy())
    p_dev = batch.probs.reshape(-1, 4).cpu().numpy()
    valid = (np.arange(batch.T)[:, None] < batch.lengths.cpu().numpy()[None, :]).reshape(-1)
    # the fixture tolerance (tests/test_gpu_ref_fixtures.py: within 2e-6 absolute of the reference's probabilities)
    np.testing.assert_allclose(p_dev[valid], p_ref[valid], rtol=0, atol=2e-6)


CFGS = [
    dict(baseline_mode="off", optimizer="sgd"),
    dict(baseline_mode="each", optimizer="sgd", gamma=0.99),
    dict(baseline_mode="batch", optimizer="adam", gamma=0.99),
    dict(baseline_mode="batch_norm", optimizer="sgd", gamma=0.9, reward_rank_weights=[3.0, 2.0, 1.0, 1.0]),
    dict(baseline_mode="batch", optimizer="sgd", use_critic=True, critic_loss_type="mse", gamma=0.99),
    dict(baseline_mode="batch_norm", optimizer="adam", use_critic=True, critic_loss_type="huber", huber_delta=0.5),
    dict(baseline_mode="each", optimizer="adam", use_critic=True, gamma=0.97),
    dict(baseline_mode="batch", optimizer="sgd", augmentation=True, gamma=0.99),
    dict(baseline_mode="batch_norm", optimizer="sgd", augmentation=True, use_critic=True),
    dict(baseline_mode="off", optimizer="sgd", max_grad_norm=1e9, learning_rate=1e-2),
]


@pytest.mark.parametrize("obs_mode", ["log2", "onehot"])
@pytest.mark.parametrize("acfg", CFGS)
def test_update_matches_oracle(acfg, obs_mode):
    """update_batch (drop-in, reference trajectory dicts) and update_from_batch (device buffer) both equal the
    numpy restatement of src/reinforce_agent.py:357-620: pre-clip gradients, norms, updated parameters."""
    agent = _agent(obs_mode=obs_mode, act="ReLU" if obs_mode == "log2" else "Sigmoid", **acfg)
    p0, c0 = _np_params(agent.params), (_np_params(agent.critic_params) if agent.critic_params else None)
    batch = agent.rollout_batch(list(range(200, 212)), list(range(300, 312)))
    trajs = agent.trajectories_from_batch(batch, with_states=False)
    oc = AO.AgentCfg(**{k: v for k, v in acfg.items()}, activation="ReLU" if obs_mode == "log2" else "Sigmoid")
    ora = AO.OracleAgent(p0, c0, oc)
    ora.update_batch(trajs)
    for path in ("dropin", "device"):
        ag = _agent(obs_mode=obs_mode, act="ReLU" if obs_mode == "log2" else "Sigmoid", **acfg)
        if path == "dropin":
            ag.update_batch(trajs)
        else:
            ag.update_from_batch(batch)
        gW, gb = ora.captured["actor_grads"]
        got = [g.cpu().numpy() for g in ag.last_grads["actor"]]
        for a, b in zip(got, gW + gb):
            assert _rel(a, b) < 1e-5, (path, "actor grad")
        assert abs(ag.last_stats["actor_grad_norm"] - ora.captured["actor_grad_norm"]) <= 1e-5 * ora.captured["actor_grad_norm"] + 1e-12
        for a, b in zip(ag.params["W"] + ag.params["b"], ora.params["W"] + ora.params["b"]):
            np.testing.assert_allclose(a.cpu().numpy(), b, rtol=1e-5, atol=2e-7)
        if acfg.get("use_critic"):
            cW, cb = ora.captured["critic_grads"]
            for a, b in zip([g.cpu().numpy() for g in ag.last_grads["critic"]], cW + cb):
                assert _rel(a, b) < 1e-5, (path, "critic grad")
            for a, b in zip(ag.critic_params["W"] + ag.critic_params["b"], ora.critic_params["W"] + ora.critic_params["b"]):
                np.testing.assert_allclose(a.cpu().numpy(), b, rtol=1e-5, atol=2e-7)


def test_returns_match_reference_formula():
    """compute_returns (src/reinforce_agent.py:255-273): the device fp64 scan stored as fp32 is bit-exact for
    rewards representable in fp32 (the rollout stores rewards as fp32)."""
    agent = _agent(gamma=0.99)
    r = [float(x) for x in np.random.default_rng(0).standard_normal(500).astype(np.float32)]
    ref = AO.OracleAgent({"W": [], "b": []}, None, AO.AgentCfg(gamma=0.99)).compute_returns(r)
    np.testing.assert_array_equal(agent.compute_returns(r), ref)


def test_run_episode_dropin_and_save_load(tmp_path):
    agent = _agent()
    tr = agent.run_episode(123, 456)
    assert set(tr) == {"obs", "actions", "rewards", "total_reward", "states", "max_tile"}
    assert len(tr["obs"]) == len(tr["actions"]) == len(tr["rewards"]) == len(tr["states"])
    assert abs(sum(tr["rewards"]) - tr["total_reward"]) < 1e-6 * max(1, abs(tr["total_reward"]))
    tr2 = agent.run_episode(123, 456)
    assert tr2["actions"] == tr["actions"]
    g = agent.run_episode(123, 456, use_greedy=True)
    assert len(g["actions"]) > 0
    path = str(tmp_path / "m.npz")
    agent.save_model(path)
    a2 = _agent()
    a2.load_model(path)
    for a, b in zip(agent.params["W"], a2.params["W"]):
        assert torch.equal(a, b)
    with np.load(path, allow_pickle=False) as f:
        assert int(f["n_layers"]) == 3 and f["W_0"].shape == (16, 32)


def test_select_action_dropin():
    from rl2048_amd import Game2048Env, Game2048EnvConfig

    env = Game2048Env(Game2048EnvConfig(obs_mode="log2"), device=DEV)
    agent = _agent()
    obs, _ = env.reset(seed=5)
    a, probs, acts, pres = agent.select_action(obs, np.random.default_rng(0))
    assert 0 <= a < 4 and probs.shape == (4,) and abs(probs.sum() - 1) < 1e-5
    assert all(probs[obs["action_mask"] == 0] == 0)
    a2, _, _, _ = agent.select_action(obs, np.random.default_rng(0), action_fn=lambda s, m: int(np.argmax(m)))
    assert a2 == int(np.argmax(obs["action_mask"]))
