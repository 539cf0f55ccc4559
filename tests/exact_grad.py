"""Test helper: the exact (fp64) value of update_batch's pre-clip gradients on a device batch, optionally under a
given ReLU activation pattern -- the basis the fp32 gradient paths are held to 1e-5 against.

update_batch (src/reinforce_agent.py:357-555) restated in fp64 torch: returns (compute_returns :255-273) or
critic TD errors (:403-498, _get_grad_logits_critic :884-910), advantages (_compute_advantages :276-325 with
_compute_weighted_stats :864-881), augmentation (_augment_trajectories :773-808: 8 symmetric copies, n_traj = 8 n),
step weights 1 / (T_i n_traj), manual backprop (_backpropagation :639-678).  Independent of the product's gradient
kernels: obs come from g2048_obs and symmetric boards from g2048_symmetries, both pinned bit-exactly to the
reference's own outputs (tests/test_gpu_ref_fixtures.py).

Why a pattern: at millions of samples, fp32 rounding of a pre-activation within ~1e-7 of 0 flips that unit's ReLU
derivative (1 vs 0) for ~1e-6 of the unit-samples, in each fp32 evaluation on different samples (the reference's
own fp32 included).  The flip is not an accumulation error, so "exact value of the formula given the activation
pattern the fp32 evaluation saw" is the basis on which an fp32 gradient can be held to 1e-5:
  * patterns="plain": the patterns of the plain fp32 path (mlp_forward_kept, hipBLASLt) recomputed on the same
    chunks that path uses (agent.chunk_steps), so its GEMMs see identical shapes;
  * a PatternProbe: the patterns the FUSED kernels actually used, read from their own column buffers through
    ReinforceAgent.grad_probe (layer 1: a1 > 0 as the kernel wrote a1; layer 2: d2 != 0 -- where the kernel's
    d2 is 0 because W3 g is 0 the derivative does not matter);
  * None: plain fp64.
V(s') (the critic's TD target) is a forward value -- continuous in the pattern -- and is always plain fp64.
"""
from __future__ import annotations

import torch


def _rel(a, b) -> float:
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double().to(a.device)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _pack_bits(m: torch.Tensor) -> torch.Tensor:
    """bool [H, m] (unit-major, as the column buffers) -> uint8 [m, H / 8]."""
    H, n = m.shape
    w = (1 << torch.arange(8, device=m.device, dtype=torch.int32))
    return (m.t().reshape(n, H // 8, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


def _unpack_bits(p: torch.Tensor) -> torch.Tensor:
    """uint8 [m, H / 8] -> bool [m, H]."""
    w = (1 << torch.arange(8, device=p.device, dtype=torch.int32))
    return ((p.to(torch.int32).unsqueeze(-1) & w) != 0).reshape(p.shape[0], -1)


class PatternProbe:
    """ReinforceAgent.grad_probe that records, per net ("actor" / "critic"), symmetry k and valid step, the ReLU
    pattern the fused gradient kernel used (bit-packed: 2 x 32 B per sample for 256-unit layers)."""

    def __init__(self, K: int, N: int, device):
        self.K, self.N, self.device = K, N, device
        self.store: dict[str, list[torch.Tensor]] = {}
        self.seen: dict[str, torch.Tensor] = {}

    def __call__(self, slot, k, idx, a1t, d2t):
        h1p, h2p = a1t.shape[0], d2t.shape[0]
        if slot not in self.store:
            self.store[slot] = [torch.zeros(self.K, self.N, h1p // 8, dtype=torch.uint8, device=self.device),
                                torch.zeros(self.K, self.N, h2p // 8, dtype=torch.uint8, device=self.device)]
            self.seen[slot] = torch.zeros(self.K, self.N, dtype=torch.int32, device=self.device)
        s1, s2 = self.store[slot]
        s1[k, idx] = _pack_bits(a1t[:h1p] > 0)
        s2[k, idx] = _pack_bits(d2t != 0)
        self.seen[slot][k, idx] += 1

    def masks(self, slot, k, sl: slice, h1: int, h2: int):
        s1, s2 = self.store[slot]
        return _unpack_bits(s1[k, sl])[:, :h1], _unpack_bits(s2[k, sl])[:, :h2]

    def complete(self, slot) -> bool:
        return slot in self.seen and bool((self.seen[slot] == 1).all())


def fwd64(W, b, x, masks=None):
    """fp64 forward of the 2-hidden-layer ReLU net; masks = (layer-1, layer-2) patterns to impose, or None."""
    z1 = x @ W[0] + b[0]
    if masks is not None:
        z1 = torch.where(masks[0], z1.abs().clamp_min(1e-300), -z1.abs())
    a1 = torch.relu(z1)
    z2 = a1 @ W[1] + b[1]
    if masks is not None:
        z2 = torch.where(masks[1], z2.abs().clamp_min(1e-300), -z2.abs())
    a2 = torch.relu(z2)
    return z1, a1, z2, a2, a2 @ W[2] + b[2]


def bwd64(W, x, z1, a1, z2, a2, g, acc):
    """_backpropagation (src/reinforce_agent.py:639-678) summed over rows, fp64, into acc = [dW1..3, db1..3]."""
    acc[2] += a2.t() @ g
    acc[5] += g.sum(0)
    d2 = (g @ W[2].t()) * (z2 > 0)
    acc[1] += a1.t() @ d2
    acc[4] += d2.sum(0)
    d1 = (d2 @ W[1].t()) * (z1 > 0)
    acc[0] += x.t() @ d1
    acc[3] += d1.sum(0)


_U32 = 2.0 ** -24   # fp32 unit roundoff


def _gamma(n: int) -> float:
    """gamma_n = n u / (1 - n u): the classical bound on the relative error of an n-term fp32 dot product
    accumulated by recursive (fmaf-chain) summation, relative to the sum of the terms' magnitudes."""
    return n * _U32 / (1.0 - n * _U32)


def pattern_flip_check(W, b, x, z1, z2, m1, m2, stats: dict, key: str) -> None:
    """Bound the fp32 path's ReLU pattern (m1, m2: bool [m, h], as the kernels used it) against fp64's own
    (z1 > 0, z2 > 0 of the exact forward):
      layer 1:  |fl32(z1) - z1| <= e1 = gamma_{17} (|x| |W1| + |b1|)   (16 obs features + bias; the obs are exact);
      layer 2:  |fl32(z2) - z2| <= e2 = gamma_{h1+1} ((a1 + e1) |W2| + |b2|) + e1 |W2|   (the fp32 a1 differs from
                the exact one by at most e1 per unit -- ReLU is 1-Lipschitz -- and enters an h1-term sum).
    A unit-sample on which the two patterns disagree must therefore have |z| <= e; stats[key] accumulates the
    disagreement counts, the unit-samples compared and the violations of the bound.  A layer-2 row whose kernel
    pattern is all-zero is skipped (the kernel reads its pattern from d2 != 0, and d2 = 0 there because the
    sample's loss gradient g is 0 -- no ReLU is consulted)."""
    st = stats.setdefault(key, dict(n1=0, n2=0, tot1=0, tot2=0, viol1=0, viol2=0, max_ratio=0.0))
    e1 = _gamma(x.shape[1] + 1) * (x.abs() @ W[0].abs() + b[0].abs())
    d1 = (z1 > 0) != m1
    st["n1"] += int(d1.sum())
    st["tot1"] += d1.numel()
    st["viol1"] += int((d1 & (z1.abs() > e1)).sum())
    a1 = torch.relu(z1)
    W2a = W[1].abs()
    e2 = _gamma(W[1].shape[0] + 1) * ((a1 + e1) @ W2a + b[1].abs()) + e1 @ W2a
    live = m2.any(dim=1, keepdim=True)
    d2 = ((z2 > 0) != m2) & live
    st["n2"] += int(d2.sum())
    st["tot2"] += int(live.sum()) * m2.shape[1]
    st["viol2"] += int((d2 & (z2.abs() > e2)).sum())
    for d, z, e in ((d1, z1, e1), (d2, z2, e2)):
        if bool(d.any()):
            st["max_ratio"] = max(st["max_ratio"], float((z.abs()[d] / e[d]).max()))


def _net64(params):
    return [w.double() for w in params["W"]], [b.double() for b in params["b"]]


def _plain_masks(params, x32):
    from rl2048_amd.mlp import mlp_forward_kept

    _, acts = mlp_forward_kept(params, x32, "ReLU")
    return acts[1] > 0, acts[2] > 0


def actions_k(a: torch.Tensor, k: int) -> torch.Tensor:
    """get_symmetries' action map (src/env.py:317-398): fliplr swaps 1 <-> 3, each CCW rotation a -> a - 1."""
    if k >= 4:
        a = torch.where(a == 1, 3, torch.where(a == 3, 1, a))
    return (a - (k & 3)) % 4


def snapshot(agent) -> tuple[dict, dict | None]:
    """Copies of the actor / critic parameters (the update replaces them; the exact value needs the old ones)."""
    cp = lambda P: None if P is None else {k: [t.detach().clone() for t in v] for k, v in P.items()}  # noqa: E731
    return cp(agent.params), cp(agent.critic_params)


def exact_update_grads(agent, batch, patterns=None, chunk: int | None = None, params=None, flip_probe=None,
                       flip_stats: dict | None = None) -> dict:
    """Pre-clip gradients {"actor": [...], "critic": [...]} of update_batch on `batch`, fp64, under `patterns`
    (None, "plain" or a PatternProbe).  params: (actor, critic) parameter dicts (snapshot()) -- default the
    agent's current ones.  Covers the configurations the GPU tests use: ReLU nets, MSE / Huber critic, baselines
    off / batch / batch_norm / each, augmentation; no reward rank weights.  flip_probe (a PatternProbe, with
    patterns=None): also compare the fused kernels' ReLU pattern with fp64's own on every sample
    (pattern_flip_check), counts into flip_stats["actor" / "critic"]."""
    actor_p, critic_p = params if params is not None else (agent.params, agent.critic_params)
    c = agent.agent_config
    assert agent.mlp_config.activation == "ReLU" and not c.reward_rank_weights
    dev = agent.device
    K = 8 if c.augmentation else 1
    if chunk is None:
        chunk = agent.chunk_steps if patterns == "plain" else 1 << 20
    T, n = batch.boards.shape
    lens = batch.lengths.to(torch.int64).to(dev)
    valid = torch.arange(T, device=dev).unsqueeze(1) < lens.unsqueeze(0)
    vidx = valid.reshape(-1).nonzero().squeeze(1)
    N = int(vidx.numel())
    lane, t = vidx % n, vidx // n
    has_next = (t + 1) < lens[lane]
    w_step = 1.0 / (lens[lane].double() * (K * n))
    R64 = batch.rewards.double()
    flat = batch.boards.reshape(-1)
    acts = batch.actions.reshape(-1)[vidx].long()
    use_mask = bool(agent.env_config.use_action_mask)

    def boards(sel_flat, k):
        b = flat[sel_flat].contiguous()
        return agent._symmetry_boards(b, k) if k else b

    def masks_for(slot, params, x32, k, sl):
        if patterns is None:
            return None
        if patterns == "plain":
            return _plain_masks(params, x32)
        h1, h2 = params["W"][0].shape[1], params["W"][1].shape[1]
        return patterns.masks(slot, k, sl, h1, h2)

    out = {}
    n_chunks = [0]

    def tick(what):   # progress on stdout (a long evaluation must keep writing; see gpurun's silence guard)
        n_chunks[0] += 1
        if n_chunks[0] % 32 == 0:
            print(f"[exact_update_grads] {what}: {n_chunks[0]} chunks", flush=True)

    if c.use_critic:
        Wc, bc = _net64(critic_p)
        accc = [torch.zeros_like(p) for p in Wc + bc]
        delta = torch.empty(K, N, dtype=torch.float64, device=dev)
        for k in range(K):
            for s in range(0, N, chunk):
                sl = slice(s, min(s + chunk, N))
                x32 = agent._obs_from_boards(boards(vidx[sl], k))[0]
                hn = has_next[sl]
                xn32 = agent._obs_from_boards(boards(torch.where(hn, vidx[sl] + n, vidx[sl]), k))[0]
                z1, a1, z2, a2, v = fwd64(Wc, bc, x32.double(), masks_for("critic", critic_p, x32, k, sl))
                if flip_probe is not None:
                    pattern_flip_check(Wc, bc, x32.double(), z1, z2,
                                       *flip_probe.masks("critic", k, sl, Wc[0].shape[1], Wc[1].shape[1]),
                                       flip_stats, "critic")
                vn = fwd64(Wc, bc, xn32.double())[4][:, 0]
                r32 = R64.reshape(-1)[vidx[sl]].float().double()      # np.array(rewards, float32) (:420)
                tgt = r32 + c.gamma * vn * hn.double()
                delta[k, sl] = tgt - v[:, 0]
                diff = v[:, 0] - tgt
                if c.critic_loss_type == "huber":
                    diff = torch.where(diff.abs() <= c.huber_delta, diff, c.huber_delta * torch.sign(diff))
                bwd64(Wc, x32.double(), z1, a1, z2, a2, (diff * w_step[sl]).unsqueeze(1), accc)
                tick("critic")
        out["critic"] = accc
        values = delta.float().double()                                # td_errors.astype(float32) (:447)
    else:
        G = torch.zeros(n, dtype=torch.float64, device=dev)
        Gt = torch.empty(T, n, dtype=torch.float64, device=dev)
        for tt in reversed(range(T)):                                  # compute_returns (:255-273)
            G = R64[tt] + c.gamma * G
            Gt[tt] = G
        values = Gt.float().double().reshape(-1)[vidx].unsqueeze(0).expand(K, -1)   # returns stored as float32
    mode = c.baseline_mode
    if mode == "off":
        adv = values
    elif mode in ("batch", "batch_norm"):
        mu = values.mean()
        adv = values - mu
        if mode == "batch_norm":
            adv = adv / ((values - mu).pow(2).mean().sqrt()).clamp_min(1e-8)
    elif mode == "each":
        s_ = torch.zeros(K, n, dtype=torch.float64, device=dev).index_add_(1, lane, values)
        c_ = torch.zeros(n, dtype=torch.float64, device=dev).index_add_(0, lane, torch.ones_like(lane, dtype=torch.float64))
        adv = values - (s_ / c_.clamp_min(1))[:, lane]
    else:
        raise ValueError(mode)
    W, b = _net64(actor_p)
    acc = [torch.zeros_like(p) for p in W + b]
    for k in range(K):
        for s in range(0, N, chunk):
            sl = slice(s, min(s + chunk, N))
            x32, mk = agent._obs_from_boards(boards(vidx[sl], k))
            z1, a1, z2, a2, lg = fwd64(W, b, x32.double(), masks_for("actor", actor_p, x32, k, sl))
            if flip_probe is not None:
                pattern_flip_check(W, b, x32.double(), z1, z2,
                                   *flip_probe.masks("actor", k, sl, W[0].shape[1], W[1].shape[1]), flip_stats, "actor")
            if use_mask:
                lg = torch.where(mk.bool(), lg, torch.full_like(lg, -1e9))
            p = torch.softmax(lg, dim=1)
            oh = torch.nn.functional.one_hot(actions_k(acts[sl], k), 4).double()
            bwd64(W, x32.double(), z1, a1, z2, a2, (oh - p) * (adv[k, sl] * w_step[sl]).unsqueeze(1), acc)
            tick("actor")
    out["actor"] = acc
    return out


def grad_errors(got: dict, ref: dict) -> dict:
    """Normwise-relative error (max abs error / max abs value) per tensor, keyed actor0.. / critic0.."""
    errs = {}
    for which, gs in got.items():
        if gs is None or which not in ref:
            continue
        for j, (g, e) in enumerate(zip(gs, ref[which])):
            errs[f"{which}{j}"] = _rel(g, e)
    return errs


# ----------------------------------------------------------------------------------------------- any depth
def fwd64_deep(W, b, x, act: str, masks=None):
    """fp64 forward of a net of any depth: returns (pre-activations z_l, layer inputs a_0..a_L, output); masks
    (ReLU): the activation pattern of each hidden layer to impose, or None."""
    zs, acts = [], [x]
    a = x
    for l in range(len(W)):
        z = a @ W[l] + b[l]
        if l == len(W) - 1:
            return zs, acts, z
        if act == "ReLU" and masks is not None:
            z = torch.where(masks[l], z.abs().clamp_min(1e-300), -z.abs())
        zs.append(z)
        a = torch.relu(z) if act == "ReLU" else torch.sigmoid(z)
        acts.append(a)
    raise AssertionError("unreachable")


def bwd64_deep(W, zs, acts, g, acc, act: str):
    """_backpropagation (src/reinforce_agent.py:639-678) of any depth, fp64, summed over rows into
    acc = [dW_0..dW_L, db_0..db_L]."""
    L1 = len(W)
    d = g
    for l in range(L1 - 1, -1, -1):
        acc[l] += acts[l].t() @ d
        acc[L1 + l] += d.sum(0)
        if l:
            dh = d @ W[l].t()
            d = dh * ((zs[l - 1] > 0).to(dh.dtype) if act == "ReLU" else acts[l] * (1.0 - acts[l]))


def pattern_flip_check_deep(W, b, x, zs, masks, stats: dict, key: str) -> None:
    """pattern_flip_check for every hidden layer of a net of any depth (x exact -- one-hot or log2 obs): layer l's
    fp32 pre-activation is within e_l = gamma_{n_l + 1} ((a_{l-1} + e_{l-1}) |W_l| + |b_l|) + e_{l-1} |W_l| of the
    exact one (e_0 = 0 on the exact input; n_l = the layer's fan-in).  Rows whose pattern is all-zero in a layer
    are compared too (the kernels' patterns here come from the activations themselves, not from d2)."""
    st = stats.setdefault(key, dict(n=[0] * len(zs), tot=[0] * len(zs), viol=[0] * len(zs), max_ratio=0.0))
    e_prev = torch.zeros_like(x)
    a_prev = x
    for l, z in enumerate(zs):
        Wa = W[l].abs()
        e = _gamma(W[l].shape[0] + 1) * ((a_prev + e_prev) @ Wa + b[l].abs()) + e_prev @ Wa
        d = (z > 0) != masks[l]
        st["n"][l] += int(d.sum())
        st["tot"][l] += d.numel()
        st["viol"][l] += int((d & (z.abs() > e)).sum())
        if bool(d.any()):
            st["max_ratio"] = max(st["max_ratio"], float((z.abs()[d] / e[d]).max()))
        e_prev, a_prev = e, torch.relu(z)


def deep_kernel_masks(agent, P, boards, out_dim: int):
    """The ReLU pattern of every hidden layer as g2048_deep_policy / g2048_deep_grad compute it, read through
    g2048_deep_hidden (bool [m, h_l] per layer)."""
    from rl2048_amd import _lib as L

    dspec = agent._deep_spec(P, out_dim)
    obs_code, hidden, act, harr = dspec
    packed = agent._pack_deep(P, dspec, "probe%d" % out_dim, out_dim)
    m = boards.numel()
    out = []
    for l, h in enumerate(hidden):
        Hp = 32 * ((h + 31) // 32)
        a = torch.empty(m, Hp, dtype=torch.float32, device=boards.device)
        L.check(L.lib().g2048_deep_hidden(L.ptr(packed), len(hidden), harr, act, obs_code,
                                          float(agent.env_config.obs_log2_scale), L.ptr(boards), m, l, L.ptr(a), Hp,
                                          L.stream_handle(boards.device)))
        out.append(a[:, :h] > 0)
    return out


def exact_update_grads_deep(agent, batch, params, patterns: str | None = "plain", flip_stats: dict | None = None):
    """Pre-clip gradients {"actor", "critic"} of update_batch on `batch` in fp64 for a net of ANY depth and obs
    (one-hot included), the obs materialised by g2048_obs.  patterns="plain": the ReLU pattern of the product's own
    fp32 path (ReinforceAgent._forward_kept_steps on the same chunks: the one-hot gather + hipBLASLt GEMMs), imposed
    on the fp64 evaluation; patterns="deep": the pattern of the fused deep kernels (deep_kernel_masks); flip_stats:
    also bound that pattern against fp64's own (pattern_flip_check_deep).
    Covers the configurations the GPU tests use: MSE / Huber critic, baselines off / batch / batch_norm, no
    augmentation, no rank weights."""
    from rl2048_amd.agent import _Steps

    actor_p, critic_p = params
    c = agent.agent_config
    act = agent.mlp_config.activation
    assert not c.augmentation and not c.reward_rank_weights
    dev = agent.device
    steps = _Steps(agent, batch.lengths, batch.actions, batch.rewards, boards=batch.boards)
    n, N = steps.n, steps.N
    lens = steps.lengths
    w_step = 1.0 / (lens[steps.lane].double() * n)
    use_mask = bool(agent.env_config.use_action_mask)

    def net64(P):
        return [w.double() for w in P["W"]], [v.double() for v in P["b"]]

    def x64(sel, nxt=False):
        b = steps.boards_at(sel, 0, nxt)
        x, mk = agent._obs_from_boards(b)
        return x.double(), mk

    def masks_of(P, sel):
        if patterns is None or act != "ReLU":
            return None
        if patterns == "deep":      # the fused kernels' own forward (g2048_deep_hidden: the same code path)
            return deep_kernel_masks(agent, P, steps.boards_at(sel, 0), 1 if P is critic_p else 4)
        with torch.no_grad():
            _, kept, _, _ = agent._forward_kept_steps(P, steps, sel, 0)
        return [a > 0 for a in kept[1:]]

    out = {}
    if c.use_critic:
        Wc, bc = net64(critic_p)
        accc = [torch.zeros_like(p) for p in Wc + bc]
        delta = torch.empty(N, dtype=torch.float64, device=dev)
        for sel in agent._chunks(N):
            x, _ = x64(sel)
            m = masks_of(critic_p, sel)
            zs, acts, v = fwd64_deep(Wc, bc, x, act, m)
            if flip_stats is not None and m is not None:
                pattern_flip_check_deep(Wc, bc, x, fwd64_deep(Wc, bc, x, act)[0], m, flip_stats, "critic")
            xn, _ = x64(sel, nxt=True)
            vn = fwd64_deep(Wc, bc, xn, act)[2][:, 0]
            hn = steps.has_next[sel]
            tgt = steps.rewards[sel].double() + c.gamma * vn * hn.double()
            delta[sel] = tgt - v[:, 0]
            diff = v[:, 0] - tgt
            if c.critic_loss_type == "huber":
                diff = torch.where(diff.abs() <= c.huber_delta, diff, c.huber_delta * torch.sign(diff))
            bwd64_deep(Wc, zs, acts, (diff * w_step[sel]).unsqueeze(1), accc, act)
        out["critic"] = accc
        values = delta.float().double()
    else:
        T = steps.T
        G = torch.zeros(n, dtype=torch.float64, device=dev)
        Gt = torch.empty(T, n, dtype=torch.float64, device=dev)
        R64 = batch.rewards.double()
        for tt in reversed(range(T)):
            G = R64[tt] + c.gamma * G
            Gt[tt] = G
        values = Gt.float().double().reshape(-1)[steps.vidx]
    mode = c.baseline_mode
    if mode in ("batch", "batch_norm"):
        mu = values.mean()
        adv = values - mu
        if mode == "batch_norm":
            adv = adv / ((values - mu).pow(2).mean().sqrt()).clamp_min(1e-8)
    else:
        assert mode == "off", mode
        adv = values
    W, b = net64(actor_p)
    acc = [torch.zeros_like(p) for p in W + b]
    for sel in agent._chunks(N):
        x, mk = x64(sel)
        m = masks_of(actor_p, sel)
        zs, acts, lg = fwd64_deep(W, b, x, act, m)
        if flip_stats is not None and m is not None:
            pattern_flip_check_deep(W, b, x, fwd64_deep(W, b, x, act)[0], m, flip_stats, "actor")
        if use_mask:
            lg = torch.where(mk.bool(), lg, torch.full_like(lg, -1e9))
        p = torch.softmax(lg, dim=1)
        oh = torch.nn.functional.one_hot(steps.actions[sel], 4).double()
        bwd64_deep(W, zs, acts, (oh - p) * (adv[sel] * w_step[sel]).unsqueeze(1), acc, act)
    out["actor"] = acc
    return out
