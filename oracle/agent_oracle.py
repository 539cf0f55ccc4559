"""CPU ORACLE (test infrastructure only) -- numpy restatement of ReinforceAgent.update_batch.

Literal per-episode / per-timestep restatement of src/reinforce_agent.py:357-620 with its helpers
(compute_returns :255, _compute_advantages :276, _policy_gradient_step :328, _activation_derivative :624,
_backpropagation :639, _compute_episode_rank_weights :681, _adam_update :719, _augment_trajectories :773,
clip_grads_global_norm :835, _compute_weighted_stats :864, _get_grad_logits_critic :884) and of the numpy MLP
(src/MLP.py:130-196).  It captures the pre-clip gradients and the norms so tests can compare the torch/HIP
update against it.

Pinning: src/reinforce_agent.py imports src/env.py, which imports gymnasium (absent here, no stand-in written),
so this restatement cannot be run side by side with the real update_batch.  Its MLP pieces are pinned by the
real src/MLP.py outputs in tests/golden/mlp.npz (tests/test_agent_oracle.py); the update algebra itself is
"parity unpinned" against the reference and is documented as such in DESIGN.md.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass

import numpy as np


# ------------------------------------------------------------------------------------------ MLP (src/MLP.py)
def _act(x, mode):
    if mode == "Sigmoid":
        return 1.0 / (1.0 + np.exp(-x))
    if mode == "ReLU":
        return np.maximum(x, 0.0)
    raise ValueError(mode)


def forward_logits(params, x, mode):
    act = x.astype(np.float32)
    acts, pres = [act], []
    L = len(params["W"])
    for i in range(L):
        z = act @ params["W"][i] + params["b"][i]
        pres.append(z)
        act = _act(z, mode) if i < L - 1 else z
        acts.append(act)
    return act, acts, pres


def logits_to_probs(logits, mask=None):
    if mask is not None:
        logits = np.where(mask.astype(bool), logits, -1e9)
    m = np.max(logits, axis=-1, keepdims=True)
    e = np.exp(logits - m)
    return e / np.sum(e, axis=-1, keepdims=True)


def encode(obs):
    if isinstance(obs, dict):
        return obs["board"].astype(np.float32).flatten(), obs["action_mask"]
    return obs.astype(np.float32).flatten(), None


# ------------------------------------------------------------------------------------------ agent
@dataclass
class AgentCfg:
    gamma: float = 1
    learning_rate: float = 1e-3
    baseline_mode: str = "off"
    reward_rank_weights: list | None = None
    optimizer: str = "sgd"
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    augmentation: bool = False
    use_critic: bool = False
    critic_learning_rate: float = 1e-3
    max_grad_norm: float = 1.0
    critic_loss_type: str = "mse"
    huber_delta: float = 1.0
    activation: str = "ReLU"


class OracleAgent:
    def __init__(self, params, critic_params, cfg: AgentCfg):
        self.params = copy.deepcopy(params)
        self.critic_params = copy.deepcopy(critic_params)
        self.cfg = cfg
        z = lambda p: [np.zeros_like(a, dtype=np.float32) for a in p]  # noqa: E731
        self.mW, self.vW, self.mB, self.vB = z(self.params["W"]), z(self.params["W"]), z(self.params["b"]), z(self.params["b"])
        self.t = 0
        if critic_params is not None:
            cp = self.critic_params
            self.mWc, self.vWc, self.mBc, self.vBc = z(cp["W"]), z(cp["W"]), z(cp["b"]), z(cp["b"])
            self.tc = 0
        self.captured = {}

    # :255
    def compute_returns(self, rewards):
        T = len(rewards)
        out = np.zeros(T, dtype=np.float32)
        G = 0.0
        for t in reversed(range(T)):
            G = rewards[t] + self.cfg.gamma * G
            out[t] = G
        return out

    # :864
    @staticmethod
    def weighted_stats(values, weights):
        sw = np.sum(weights)
        if sw < 1e-8:
            return 0.0, 1.0
        mean = np.sum(values * weights) / sw
        var = np.sum(weights * (values - mean) ** 2) / sw
        return mean, np.sqrt(var)

    # :276
    def advantages(self, returns_list, rank_w):
        mode = self.cfg.baseline_mode
        if mode == "off":
            return [r.astype(np.float32) for r in returns_list]
        if mode == "each":
            return [(r - float(r.mean())).astype(np.float32) for r in returns_list]
        allv = np.concatenate(returns_list)
        allw = np.concatenate([np.full(len(r), rank_w[i]) for i, r in enumerate(returns_list)])
        mean, std = self.weighted_stats(allv, allw)
        if mode == "batch":
            return [(r - mean).astype(np.float32) for r in returns_list]
        if mode == "batch_norm":
            std = max(std, 1e-8)
            return [((r - mean) / std).astype(np.float32) for r in returns_list]
        raise ValueError(f"Unknown baseline mode: {mode}")

    # :681
    def rank_weights(self, totals):
        conf = self.cfg.reward_rank_weights
        n = len(totals)
        if n == 0:
            return np.array([], dtype=np.float32)
        if conf is None or len(conf) == 0:
            return np.ones(n, dtype=np.float32)
        conf = np.asarray(conf, dtype=np.float32)
        order = np.argsort(totals, kind="stable")  # ties: see DESIGN.md (reference uses the default sort)
        w = np.zeros(n, dtype=np.float32)
        for rank, idx in enumerate(order):
            b = int((rank + 0.5) / n * len(conf))
            w[idx] = conf[min(b, len(conf) - 1)]
        mw = np.mean(w)
        return w / mw if mw > 1e-8 else w

    # :624
    def act_deriv(self, z):
        if self.cfg.activation == "Sigmoid":
            s = 1.0 / (1.0 + np.exp(-z))
            return s * (1.0 - s)
        return (z > 0).astype(np.float32)

    # :639
    def backprop(self, params, acts, pres, grad_logits):
        L = len(params["W"])
        gW = [None] * L
        gb = [None] * L
        delta = grad_logits.astype(np.float32)
        for l in reversed(range(L)):
            gW[l] = np.outer(acts[l], delta)
            gb[l] = delta
            if l > 0:
                delta = (delta @ params["W"][l].T) * self.act_deriv(pres[l - 1])
        return gW, gb

    # :884
    def grad_logits_critic(self, v, target):
        diff = v - target
        if self.cfg.critic_loss_type == "mse":
            return diff.astype(np.float32).reshape(-1, 1)
        if self.cfg.critic_loss_type == "huber":
            d = self.cfg.huber_delta
            return np.where(np.abs(diff) <= d, diff, d * np.sign(diff)).astype(np.float32).reshape(-1, 1)
        raise ValueError(self.cfg.critic_loss_type)

    # :835
    def clip(self, gWs, gbs):
        tot = 0.0
        for g in gWs:
            tot += np.linalg.norm(g) ** 2
        for g in gbs:
            tot += np.linalg.norm(g) ** 2
        norm = np.sqrt(tot)
        coef = self.cfg.max_grad_norm / max(norm, 1e-8)
        if coef < 1.0:
            for i in range(len(gWs)):
                gWs[i] *= coef
            for i in range(len(gbs)):
                gbs[i] *= coef
        return norm

    # :719
    def adam(self, gWs, gbs, critic=False):
        c = self.cfg
        if critic:
            P, mW, vW, mB, vB = self.critic_params, self.mWc, self.vWc, self.mBc, self.vBc
            self.tc += 1
            t, lr, sign = self.tc, c.critic_learning_rate, -1.0
        else:
            P, mW, vW, mB, vB = self.params, self.mW, self.vW, self.mB, self.vB
            self.t += 1
            t, lr, sign = self.t, c.learning_rate, 1.0
        b1, b2, eps = c.adam_beta1, c.adam_beta2, 1e-8
        for l in range(len(P["W"])):
            mW[l] = b1 * mW[l] + (1.0 - b1) * gWs[l]
            mB[l] = b1 * mB[l] + (1.0 - b1) * gbs[l]
            vW[l] = b2 * vW[l] + (1.0 - b2) * (gWs[l] * gWs[l])
            vB[l] = b2 * vB[l] + (1.0 - b2) * (gbs[l] * gbs[l])
            P["W"][l] = P["W"][l] + sign * lr * (mW[l] / (1.0 - b1 ** t)) / (np.sqrt(vW[l] / (1.0 - b2 ** t)) + eps)
            P["b"][l] = P["b"][l] + sign * lr * (mB[l] / (1.0 - b1 ** t)) / (np.sqrt(vB[l] / (1.0 - b2 ** t)) + eps)

    # :773 (get_symmetries src/env.py:317-398)
    @staticmethod
    def symmetries(obs, action):
        def rot_a(a):
            return (a - 1) % 4

        def flip_a(a):
            return {1: 3, 3: 1}.get(a, a)

        board, mask = (obs["board"], obs["action_mask"]) if isinstance(obs, dict) else (obs, None)
        out = []
        for b, a, m in ((board.copy(), action, None if mask is None else mask.copy()),
                        (np.fliplr(board.copy()), flip_a(action), None if mask is None else mask[[0, 3, 2, 1]])):
            for _ in range(4):
                out.append(({"board": b, "action_mask": m} if m is not None else b, a))
                b = np.rot90(b, k=1, axes=(0, 1))
                a = rot_a(a)
                m = np.roll(m, shift=-1) if m is not None else None
        return out

    def augment(self, trajs, advs, rank_w):
        out = []
        for tr in trajs:
            aug = [{"obs": [], "actions": [], "rewards": []} for _ in range(8)]
            for t in range(len(tr["obs"])):
                syms = self.symmetries(tr["obs"][t], tr["actions"][t])
                for i in range(8):
                    aug[i]["obs"].append(syms[i][0])
                    aug[i]["actions"].append(syms[i][1])
                    aug[i]["rewards"].append(tr["rewards"][t])
            out.extend(aug)
        return out, [a for a in advs for _ in range(8)], np.repeat(rank_w, 8)

    # :357
    def update_batch(self, trajs):
        c = self.cfg
        returns_list, totals = [], []
        for tr in trajs:
            totals.append(tr["total_reward"])
            if not c.use_critic:
                returns_list.append(self.compute_returns(tr["rewards"]))
        rank_w = self.rank_weights(totals)
        advs = self.advantages(returns_list, rank_w) if not c.use_critic else [None] * len(trajs)
        if c.augmentation:
            trajs, advs, rank_w = self.augment(trajs, advs, rank_w)
        gW = [np.zeros_like(W, dtype=np.float32) for W in self.params["W"]]
        gb = [np.zeros_like(b, dtype=np.float32) for b in self.params["b"]]
        if c.use_critic:
            gWc = [np.zeros_like(W) for W in self.critic_params["W"]]
            gbc = [np.zeros_like(b) for b in self.critic_params["b"]]
        n = len(trajs)
        if n == 0:
            return
        if c.use_critic:
            tds = []
            for tr, rw in zip(trajs, rank_w):
                T = len(tr["obs"])
                if T == 0:
                    tds.append(np.zeros(0, dtype=np.float32))
                    continue
                X = np.array([encode(o)[0] for o in tr["obs"]])
                R = np.array(tr["rewards"], dtype=np.float32)
                Xn = np.concatenate([X[1:], X[-1:]], axis=0)
                v, va, vp = forward_logits(self.critic_params, X, c.activation)
                v = v.flatten()
                vn = forward_logits(self.critic_params, Xn, c.activation)[0].flatten()
                md = np.ones(T, dtype=np.float32)
                md[-1] = 0.0
                tgt = R + c.gamma * vn * md
                td = tgt - v
                tds.append(td.astype(np.float32))
                gl = self.grad_logits_critic(v, tgt)
                for t in range(T):
                    dW, db = self.backprop(self.critic_params, [a[t] for a in va], [p[t] for p in vp], gl[t])
                    w = 1.0 / (T * n) * float(rw)
                    for l in range(len(gWc)):
                        gWc[l] += w * dW[l]
                        gbc[l] += w * db[l]
            advs = self.advantages(tds, rank_w)
            self.captured["td_errors"] = tds
        self.captured["advantages"] = advs
        for tr, adv, rw in zip(trajs, advs, rank_w):
            T = len(tr["obs"])
            if T == 0:
                continue
            enc = [encode(o) for o in tr["obs"]]
            X = np.array([e[0] for e in enc])
            M = np.array([e[1] for e in enc]) if enc[0][1] is not None else None
            lg, acts, pres = forward_logits(self.params, X, c.activation)
            P = logits_to_probs(lg, M)
            w = 1.0 / (T * n) * float(rw)
            for t in range(T):
                oh = np.zeros_like(P[t], dtype=np.float32)
                oh[tr["actions"][t]] = 1.0
                gl = float(adv[t]) * (oh - P[t].astype(np.float32))
                dW, db = self.backprop(self.params, [a[t] for a in acts], [p[t] for p in pres], gl)
                for l in range(len(gW)):
                    gW[l] += w * dW[l]
                    gb[l] += w * db[l]
        self.captured["actor_grads"] = ([g.copy() for g in gW], [g.copy() for g in gb])
        an = self.clip(gW, gb)
        self.captured["actor_grad_norm"] = an
        if c.use_critic:
            self.captured["critic_grads"] = ([g.copy() for g in gWc], [g.copy() for g in gbc])
            self.captured["critic_grad_norm"] = self.clip(gWc, gbc)
        if c.optimizer == "sgd":
            for l in range(len(self.params["W"])):
                self.params["W"][l] += c.learning_rate * gW[l]
                self.params["b"][l] += c.learning_rate * gb[l]
            if c.use_critic:
                for l in range(len(self.critic_params["W"])):
                    self.critic_params["W"][l] -= c.critic_learning_rate * gWc[l]
                    self.critic_params["b"][l] -= c.critic_learning_rate * gbc[l]
        elif c.optimizer == "adam":
            self.adam(gW, gb)
            if c.use_critic:
                self.adam(gWc, gbc, critic=True)
        else:
            raise ValueError(f"Unknown optimizer: {c.optimizer}")
