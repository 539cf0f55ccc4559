"""CPU: pin the numpy agent oracle's MLP pieces and the product's host-side init against the real src/MLP.py
outputs (tests/golden/mlp.npz), and check the update oracle's internal consistency (manual backprop == autograd
of sum_t w * A_t * log pi(a_t|s_t), the identity the batched GPU update relies on)."""
import os

import numpy as np
import pytest
import torch

from oracle import agent_oracle as AO


@pytest.fixture(scope="module")
def mlp(golden_dir):
    return np.load(os.path.join(golden_dir, "mlp.npz"), allow_pickle=False)


CASES = ["he_relu_log2", "xn_onehot", "xu_critic", "normal_linear", "he_onehot_critic"]


def _params(d, name):
    meta = d[f"{name}__meta"]
    L = int(meta[3]) + 1
    return {"W": [d[f"{name}__W{i}"] for i in range(L)], "b": [d[f"{name}__b{i}"] for i in range(L)]}, meta


@pytest.mark.parametrize("name", CASES)
def test_oracle_forward_vs_reference(mlp, name):
    p, _ = _params(mlp, name)
    X = mlp[f"{name}__X"]
    for act in ("ReLU", "Sigmoid"):
        lg, _, _ = AO.forward_logits(p, X, act)
        np.testing.assert_array_equal(lg, mlp[f"{name}__logits_{act}"])
    if f"{name}__mask" in mlp:
        np.testing.assert_array_equal(AO.logits_to_probs(mlp[f"{name}__logits_ReLU"], mlp[f"{name}__mask"]),
                                      mlp[f"{name}__probs"])


@pytest.mark.parametrize("name", CASES)
def test_product_init_matches_reference(mlp, name):
    """rl2048_amd.mlp.init_model_params draws the same numpy stream as src/MLP.py:45-94 (bit-exact fp32)."""
    from rl2048_amd.mlp import init_model_params

    p_ref, meta = _params(mlp, name)
    din, dout, seed, nh = (int(x) for x in meta[:4])
    hidden = [int(x) for x in meta[4:4 + nh]]
    dist = str(mlp[f"{name}__dist"])
    p = init_model_params(din, hidden, dout, np.random.default_rng(seed), dist, True, device="cpu")
    for a, b in zip(p["W"] + p["b"], p_ref["W"] + p_ref["b"]):
        np.testing.assert_array_equal(a.numpy(), b)


def test_product_init_actor_then_critic_stream(mlp):
    """The critic is drawn from the same Generator right after the actor (src/reinforce_agent.py:62,77,95)."""
    from rl2048_amd.mlp import init_model_params

    rng = np.random.default_rng(0)
    init_model_params(16, [256, 256], 4, rng, "HeNormal", device="cpu")
    pc = init_model_params(16, [256, 256], 1, rng, "HeNormal", device="cpu")
    np.testing.assert_array_equal(pc["W"][0].numpy(), mlp["agent_critic__W0"])
    np.testing.assert_array_equal(pc["W"][1][:8].numpy(), mlp["agent_critic__W1_rows8"])
    np.testing.assert_array_equal(pc["W"][2].numpy(), mlp["agent_critic__W2"])


def test_init_unknown_distribution_raises():
    from rl2048_amd.mlp import init_model_params

    with pytest.raises(ValueError, match="Unsupported init_distribution"):
        init_model_params(16, [8], 4, np.random.default_rng(0), "normal", device="cpu")  # the reference default


def _random_trajs(rng, n, D=16, onehot=False):
    trajs = []
    for _ in range(n):
        T = int(rng.integers(3, 12))
        obs = []
        for _ in range(T):
            if onehot:
                e = rng.integers(0, 17, size=16)
                b = np.eye(17, dtype=np.float32)[e].reshape(4, 4, 17)
            else:
                b = rng.integers(0, 12, size=(4, 4)).astype(np.float32) * 0.25
            m = (rng.random(4) < 0.7).astype(np.int8)
            m[rng.integers(4)] = 1
            obs.append({"board": b, "action_mask": m})
        acts = [int(rng.choice(np.nonzero(o["action_mask"])[0])) for o in obs]
        rews = [float(x) for x in rng.integers(0, 6, size=T) * 0.5]
        trajs.append({"obs": obs, "actions": acts, "rewards": rews, "total_reward": float(sum(rews))})
    return trajs


@pytest.mark.parametrize("baseline", ["off", "each", "batch", "batch_norm"])
def test_manual_backprop_equals_autograd(baseline):
    """The oracle's per-step outer products (src/reinforce_agent.py:536-555) == autograd of
    sum_i sum_t rank_w_i/(T_i n) * A_t * log softmax(masked logits)[a_t] (fp64 to isolate the algebra)."""
    rng = np.random.default_rng(1)
    p = {"W": [rng.standard_normal((16, 8)), rng.standard_normal((8, 4))], "b": [rng.standard_normal(8) * 0.1,
                                                                                   rng.standard_normal(4) * 0.1]}
    p = {k: [a.astype(np.float64) for a in v] for k, v in p.items()}
    cfg = AO.AgentCfg(baseline_mode=baseline, max_grad_norm=1e9, activation="ReLU")
    ag = AO.OracleAgent(p, None, cfg)
    trajs = _random_trajs(rng, 5)
    ag.update_batch(trajs)
    gW, gb = ag.captured["actor_grads"]
    advs = ag.captured["advantages"]
    tp = [torch.tensor(a, requires_grad=True) for a in p["W"] + p["b"]]
    loss = 0.0
    n = len(trajs)
    for tr, A in zip(trajs, advs):
        X = torch.tensor(np.array([o["board"].reshape(-1) for o in tr["obs"]]), dtype=torch.float64)
        M = torch.tensor(np.array([o["action_mask"] for o in tr["obs"]])).bool()
        h = torch.relu(X @ tp[0] + tp[2])
        lg = h @ tp[1] + tp[3]
        lg = torch.where(M, lg, torch.full_like(lg, -1e9))
        lp = torch.log_softmax(lg, dim=-1)[torch.arange(len(tr["actions"])), torch.tensor(tr["actions"])]
        loss = loss + (torch.tensor(A, dtype=torch.float64) * lp).sum() / (len(tr["obs"]) * n)
    loss.backward()
    for a, b in zip(gW + gb, tp[:2] + tp[2:]):
        np.testing.assert_allclose(a, b.grad.numpy(), rtol=1e-4, atol=1e-6)
