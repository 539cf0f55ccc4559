"""GPU: the fused actor gradient (g2048_actor_grad + the split-K layer-2 GEMM) against the batched torch backprop
of the same update (mlp_forward_kept / mlp_backward_, itself pinned to the numpy oracle by test_gpu_agent.py) on
the same rollout batch: every pre-clip actor gradient within 1e-5 normwise-relative (fp32 summation order is the
only difference), for padded and full-width nets, ReLU / Sigmoid, log2 / raw obs, masked / unmasked, with
augmentation; plus the drop-in oracle check of update_batch with use_action_mask off."""
import numpy as np
import pytest
import torch

import exact_grad as EG
from oracle import agent_oracle as AO

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def _agent(hidden, act, obs_mode="log2", use_action_mask=True, **acfg):
    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    env_cfg = Game2048EnvConfig(obs_mode=obs_mode, obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5,
                                max_steps=400, use_action_mask=use_action_mask)
    return ReinforceAgent(env_cfg, MLPConfig(hidden_sizes=list(hidden), activation=act, init_distribution="HeNormal"),
                          ReinforceAgentConfig(**acfg), device=DEV)


CASES = [
    dict(hidden=(256, 256), act="ReLU", obs_mode="log2", use_action_mask=True, episodes=96),
    dict(hidden=(32, 16), act="ReLU", obs_mode="log2", use_action_mask=True, episodes=64),
    dict(hidden=(64, 96), act="Sigmoid", obs_mode="raw", use_action_mask=True, episodes=48),
    dict(hidden=(200, 40), act="ReLU", obs_mode="log2", use_action_mask=False, episodes=48),
    dict(hidden=(128, 256), act="Sigmoid", obs_mode="log2", use_action_mask=False, episodes=32, augmentation=True),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['hidden']}-{c['act']}-{c['obs_mode']}-m{int(c['use_action_mask'])}")
def test_fused_actor_grad_matches_batched_backprop(case):
    case = dict(case)
    n = case.pop("episodes")
    acfg = dict(baseline_mode="batch_norm", optimizer="sgd", gamma=0.99, augmentation=case.pop("augmentation", False))
    grads = {}
    batch = None
    for fused in (True, False):
        ag = _agent(**case, **acfg)
        ag.use_fused_grad = fused
        if batch is None:
            batch = ag.rollout_batch(list(range(500, 500 + n)), list(range(900, 900 + n)))
        ag.grad_chunk_steps = 1 << 12   # several chunks, exercising the accumulation across launches
        ag.update_from_batch(batch)
        grads[fused] = [g.cpu().numpy() for g in ag.last_grads["actor"]]
    assert int(batch.lengths.sum()) > 4096
    for i, (a, b) in enumerate(zip(grads[True], grads[False])):
        assert _rel(a, b) < 1e-5, (i, _rel(a, b))


CRITIC_CASES = [
    dict(hidden=(256, 256), act="ReLU", obs_mode="log2", critic_loss_type="mse", episodes=64),
    dict(hidden=(48, 32), act="Sigmoid", obs_mode="raw", critic_loss_type="huber", huber_delta=0.5, episodes=48),
    dict(hidden=(96, 200), act="ReLU", obs_mode="log2", critic_loss_type="huber", huber_delta=2.0, episodes=32,
         augmentation=True),
]


@pytest.mark.parametrize("case", CRITIC_CASES, ids=lambda c: f"{c['hidden']}-{c['act']}-{c['critic_loss_type']}")
def test_fused_critic_grad_matches_batched_backprop(case):
    """The critic branch (V(s'), TD target, TD errors -> actor advantages, MSE / Huber gradient) through
    g2048_critic_grad equals the batched torch backprop: critic and actor pre-clip gradients within 1e-5."""
    case = dict(case)
    n = case.pop("episodes")
    hidden, act, obs_mode = case.pop("hidden"), case.pop("act"), case.pop("obs_mode")
    acfg = dict(baseline_mode="batch", optimizer="sgd", gamma=0.97, use_critic=True, **case)
    grads = {}
    batch = None
    for fused in (True, False):
        ag = _agent(hidden, act, obs_mode=obs_mode, **acfg)
        ag.use_fused_grad = fused
        if batch is None:
            batch = ag.rollout_batch(list(range(700, 700 + n)), list(range(1700, 1700 + n)))
        ag.grad_chunk_steps = 1 << 12
        ag.update_from_batch(batch)
        grads[fused] = ([g.cpu().numpy() for g in ag.last_grads["critic"]],
                        [g.cpu().numpy() for g in ag.last_grads["actor"]])
    for which in (0, 1):
        for i, (a, b) in enumerate(zip(grads[True][which], grads[False][which])):
            assert _rel(a, b) < 1e-5, ("critic" if which == 0 else "actor", i, _rel(a, b))


@pytest.mark.parametrize("critic", [False, True], ids=["actor", "actor_critic"])
def test_fused_grad_one_large_chunk_split_k(critic):
    """One chunk of > 17 x 8192 samples (below the default chunk size, so a single launch): the layer-2 weight
    gradient then runs as a split-K batched GEMM over P = max(1, min(128, m // 8192)) >= 17 column blocks of
    a1^T / d2^T (the small-batch cases above use P = 1), and the kernel's column buffers are wide (ld > 2^17).
    Gradients within 1e-5 of the torch backprop."""
    acfg = dict(baseline_mode="batch", optimizer="sgd", gamma=0.99)
    if critic:
        acfg.update(use_critic=True, critic_loss_type="mse")
    grads = {}
    batch = None
    for fused in (True, False):
        ag = _agent((256, 256), "ReLU", **acfg)
        ag.use_fused_grad = fused
        if batch is None:
            batch = ag.rollout_batch(list(range(4000, 6048)), list(range(9000, 11048)))
        ag.update_from_batch(batch)
        grads[fused] = {k: [g.cpu().numpy() for g in v] for k, v in ag.last_grads.items() if v is not None}
    assert set(grads[True]) == ({"actor", "critic"} if critic else {"actor"})
    m = int(batch.lengths.sum())
    assert m > 17 * 8192 and m <= ag.grad_chunk_steps, m
    for which, gs in grads[True].items():
        for i, (a, b) in enumerate(zip(gs, grads[False][which])):
            assert _rel(a, b) < 1e-5, (which, i, _rel(a, b))


def test_update_matches_oracle_unmasked():
    """update_batch with use_action_mask off (bare-board obs): the device update, with the fused gradient, equals
    the numpy restatement with unmasked probabilities.  (The reference's own update_batch cannot run this case:
    np.array of the per-step None masks broadcasts against the logits and raises)"""
    acfg = dict(baseline_mode="batch", optimizer="adam", gamma=0.99)
    agent = _agent((32, 16), "ReLU", use_action_mask=False, **acfg)
    p0 = {k: [t.detach().cpu().numpy().copy() for t in v] for k, v in agent.params.items()}
    batch = agent.rollout_batch(list(range(200, 212)), list(range(300, 312)))
    trajs = agent.trajectories_from_batch(batch, with_states=False)
    assert not isinstance(trajs[0]["obs"][0], dict)
    ora = AO.OracleAgent(p0, None, AO.AgentCfg(**acfg, activation="ReLU"))
    ora.update_batch(trajs)
    for path in ("dropin", "device"):
        ag = _agent((32, 16), "ReLU", use_action_mask=False, **acfg)
        if path == "dropin":
            ag.update_batch(trajs)
        else:
            ag.update_from_batch(batch)
        gW, gb = ora.captured["actor_grads"]
        for a, b in zip([g.cpu().numpy() for g in ag.last_grads["actor"]], gW + gb):
            assert _rel(a, b) < 1e-5, path
        for a, b in zip(ag.params["W"] + ag.params["b"], ora.params["W"] + ora.params["b"]):
            np.testing.assert_allclose(a.cpu().numpy(), b, rtol=1e-5, atol=2e-7)


def _check_fused_vs_plain(runs, act):
    """runs: {"fused" | "plain": (agent, params before the update, PatternProbe or None)} after update_from_batch on
    the same batch.  Sigmoid: fused within 1e-5 of the torch backprop (no pattern).  ReLU: each path within 1e-5 of
    the exact fp64 value of the formula under the ReLU pattern it computed (tests/exact_grad.py) -- at ~1e5 samples
    the two fp32 forwards round a few pre-activations next to 0 to opposite signs, so they are not compared with
    each other there."""
    (fa, fp0, probe), (pa, pp0, _) = runs["fused"], runs["plain"]
    if act == "Sigmoid":
        for which in ("critic", "actor"):
            for i, (a, b) in enumerate(zip(fa.last_grads[which], pa.last_grads[which])):
                assert _rel(a.cpu().numpy(), b.cpu().numpy()) < 1e-5, (which, i)
        return
    assert probe.complete("actor") and probe.complete("critic")
    errs_f = EG.grad_errors(fa.last_grads, EG.exact_update_grads(fa, runs["batch"], patterns=probe, params=fp0))
    errs_p = EG.grad_errors(pa.last_grads, EG.exact_update_grads(pa, runs["batch"], patterns="plain", params=pp0))
    print("\nfused vs exact under its pattern", errs_f, "\nplain vs exact under its pattern", errs_p)
    assert all(v < 1e-5 for v in errs_f.values()), errs_f
    assert all(v < 1e-5 for v in errs_p.values()), errs_p


@pytest.mark.parametrize("act,records", [("Sigmoid", False), ("ReLU", False), ("ReLU", True)])
@pytest.mark.parametrize("chunk", [4096 + 17, 8192 * 17 + 5])
def test_fused_critic_grad_ragged_chunks(chunk, act, records):
    """Regression for the round-1 hipErrorIllegalAddress seen after the 256x256 critic's V(s') launch
    ("Fault audit"): every chunk of the fused critic + actor gradient is ragged (m not a
    multiple of 32, so the last 32-sample group of each launch is partial), the last chunk is short, and the
    second size makes the split-K layer-2 GEMM run P = 17 column blocks; the device stays healthy (a
    synchronising copy after each update).  records: the actor's d2 as block records (g2048_actor_grad d2_form 2 +
    g2048_dw2_actor; measured slower than the columns, so off by default) instead of columns.  Gradients:
    _check_fused_vs_plain (1e-5)."""
    acfg = dict(baseline_mode="batch", optimizer="sgd", gamma=0.97, use_critic=True, critic_loss_type="mse")
    runs = {}
    batch = None
    for mode in ("fused", "plain"):
        ag = _agent((256, 256), act, **acfg)
        ag.use_fused_grad = mode == "fused"
        ag.actor_d2_records = records
        if batch is None:
            batch = ag.rollout_batch(list(range(3000, 3000 + 1200)), list(range(7000, 7000 + 1200)))
            runs["batch"] = batch
        N = int(batch.lengths.sum())
        ag.grad_chunk_steps = chunk
        probe = EG.PatternProbe(1, N, DEV) if mode == "fused" else None
        ag.grad_probe = probe
        p0 = EG.snapshot(ag)
        ag.update_from_batch(batch)
        torch.cuda.synchronize()
        runs[mode] = (ag, p0, probe)
    assert N % chunk and (N % chunk) % 32 and N > chunk, (N, chunk)
    _check_fused_vs_plain(runs, act)


@pytest.mark.parametrize("aug,tail", [(False, 0), (True, 0), (False, 64), (True, 100000)])
@pytest.mark.parametrize("act,fac", [("Sigmoid", False), ("ReLU", True), ("ReLU", False)])
def test_fused_critic_rows_mode(act, fac, aug, tail):
    """The per-time-row critic pass (ReinforceAgent._critic_grad_rows: rows last-first, each launch's V(s) serving as
    the previous row's V(s'), one column buffer, accumulated partials) forced on a small batch -- hundreds of
    rows, most of them ragged, a column-buffer flush forced by a small chunk -- against the torch backprop: critic
    and actor gradients and the TD errors (through the actor's advantages).  `tail`: rows below that many samples
    run as the one tail launch with its own V(s') forward (0: none; 64: the later rows, handing over to the chain;
    100000: all rows, capped by the column buffer).  `fac`: the ReLU critic's factored d2 records
    (g2048_critic_grad d2_form 1 + g2048_dw2_factored, the default) or d2 columns.  Gradients: _check_fused_vs_plain
    (1e-5 against the exact value under the fused kernels' own ReLU pattern)."""
    acfg = dict(baseline_mode="batch", optimizer="sgd", gamma=0.97, use_critic=True, critic_loss_type="huber",
                huber_delta=0.5, augmentation=aug)
    runs = {}
    batch = None
    for mode in ("fused", "plain"):
        ag = _agent((64, 96), act, obs_mode="log2", **acfg)
        ag.use_fused_grad = mode == "fused"
        ag.critic_rows_min_avg = 0
        ag.critic_tail_row_max = tail
        ag.critic_factored_d2 = fac
        ag.grad_chunk_steps = 4096
        if batch is None:
            batch = ag.rollout_batch(list(range(100, 100 + 160)), list(range(900, 900 + 160)))
            runs["batch"] = batch
        if mode == "fused":
            assert ag._critic_by_rows(_steps_of(ag, batch))
        probe = EG.PatternProbe(8 if aug else 1, int(batch.lengths.sum()), DEV) if mode == "fused" else None
        ag.grad_probe = probe
        p0 = EG.snapshot(ag)
        ag.update_from_batch(batch)
        torch.cuda.synchronize()
        runs[mode] = (ag, p0, probe)
    _check_fused_vs_plain(runs, act)


def _steps_of(agent, batch):
    from rl2048_amd.agent import _Steps

    return _Steps(agent, batch.lengths, batch.actions, batch.rewards, boards=batch.boards)


@pytest.mark.parametrize("h1,h2", [(256, 256), (32, 16), (64, 96), (200, 40), (128, 256)])
@pytest.mark.parametrize("ncols,cpp", [(4096, 2048), (2048 + 16 * 37, 2048), (1 << 16, 4096), (48, 2048)])
def test_dw2_kernel_matches_fp64(h1, h2, ncols, cpp):
    """g2048_dw2 (the layer-2 weight / bias gradient: a1 d2^T and the row sums of d2, three bf16 planes per fp32
    operand on the bf16 MFMA) against fp64 on the same fp32 column buffers (16-column block layout of
    include/g2048.h), with values spanning several orders of magnitude and zero / negative entries: every slab
    within 4e-6 of sum |a d| of the exact value (the bf16 MFMA's accumulation into its fp32 accumulator is measured
    at ~2e-6 of sum |a d| over 2048 columns -- looser than the f32 MFMA's k-ordered fma chain; the gradient-level
    1e-5 checks hold the whole update to the exact value), for full and padded (non-multiple-of-32) hidden sizes,
    a column range starting inside the buffer, and partial last slabs."""
    from rl2048_amd import _lib as L
    from rl2048_amd.agent import _padded_units

    H1p, H2p = _padded_units(h1), _padded_units(h2)
    R = max(H1p, H2p)
    col0 = 32
    ld = col0 + ncols + 32
    g = torch.Generator(device=DEV)
    g.manual_seed(h1 * 1000 + ncols)
    A = torch.zeros(R, ld, device=DEV)
    D = torch.zeros(R, ld, device=DEV)
    A[:h1] = torch.relu(torch.randn(h1, ld, device=DEV, generator=g) *
                        torch.exp(3 * torch.randn(h1, ld, device=DEV, generator=g)))   # activations: >= 0, many zeros
    D[:h2] = torch.randn(h2, ld, device=DEV, generator=g) * torch.exp(2 * torch.randn(h2, ld, device=DEV, generator=g))
    blocked = lambda X: X.reshape(R, ld // 16, 16).permute(1, 0, 2).contiguous()  # noqa: E731 (include/g2048.h)
    a_in, d_in = blocked(A), blocked(D)
    nparts = -(-ncols // cpp)
    part = torch.full((nparts, H1p + 1, H2p), float("nan"), device=DEV)
    lib = L.lib()
    L.check(lib.g2048_dw2(L.ptr(a_in), L.ptr(d_in), h1, h2, ld, col0, ncols, cpp, L.ptr(part), nparts,
                          L.stream_handle(DEV)))
    torch.cuda.synchronize()
    A64, D64 = A[:H1p, col0:col0 + ncols].double(), D[:H2p, col0:col0 + ncols].double()
    for p in range(nparts):
        sl = slice(p * cpp, min((p + 1) * cpp, ncols))
        ref = A64[:, sl] @ D64[:, sl].t()
        bound = A64[:, sl].abs() @ D64[:, sl].abs().t()
        got = part[p, :H1p].double()
        rel = float(((got - ref).abs() / bound.clamp_min(1e-30)).max())
        print(f"slab {p}: max |err| / sum |a d| = {rel:.3g}")
        assert bool(((got - ref).abs() <= 4e-6 * bound + 1e-30).all()), (p, rel)
        db = D64[:, sl].sum(1)
        assert bool(((part[p, H1p].double() - db).abs() <= 4e-6 * D64[:, sl].abs().sum(1) + 1e-30).all()), p
    # bad arguments are rejected, not launched
    with pytest.raises(ValueError):
        L.check(lib.g2048_dw2(L.ptr(a_in), L.ptr(d_in), h1, h2, ld, col0, ncols + 8, cpp, L.ptr(part), nparts,
                              L.stream_handle(DEV)))


@pytest.mark.parametrize("nparts,slab", [(256, 257 * 256), (1, 33 * 32), (13, 1000), (1024, 1377), (1024, 5380),
                                         (37, 63)])
def test_fold_partials_matches_fp64_sum(nparts, slab):
    """g2048_fold_partials (the update's fp64 fold of g2048_dw2 slabs and per-wave partials): acc += the sum over
    slabs, taken in fp64 in a fixed order -- equal to numpy's fp64 sum of the same fp32 values up to fp64 rounding
    of the (different) summation order, adding to what acc held, and bitwise repeatable."""
    from rl2048_amd import _lib as L

    g = torch.Generator(device=DEV)
    g.manual_seed(nparts * 7 + slab)
    part = torch.randn(nparts, slab, device=DEV, generator=g) * torch.exp(4 * torch.randn(nparts, slab, device=DEV,
                                                                                         generator=g))
    acc0 = torch.randn(slab, device=DEV, dtype=torch.float64, generator=g)
    acc = acc0.clone()
    L.check(L.lib().g2048_fold_partials(L.ptr(part), nparts, slab, L.ptr(acc), L.stream_handle(DEV)))
    torch.cuda.synchronize()
    p64 = part.double().cpu().numpy()
    ref = acc0.cpu().numpy() + np.add.reduce(p64, axis=0)
    bound = np.abs(acc0.cpu().numpy()) + np.abs(p64).sum(0)
    assert np.all(np.abs(acc.cpu().numpy() - ref) <= 1e-14 * bound)
    again = acc0.clone()
    L.check(L.lib().g2048_fold_partials(L.ptr(part), nparts, slab, L.ptr(again), L.stream_handle(DEV)))
    torch.cuda.synchronize()
    assert torch.equal(again, acc)
    with pytest.raises(ValueError):
        L.check(L.lib().g2048_fold_partials(None, nparts, slab, L.ptr(acc), L.stream_handle(DEV)))


@pytest.mark.parametrize("h1,h2", [(256, 256), (32, 16), (200, 40)])
@pytest.mark.parametrize("ncols,cpp", [(4096, 2048), (2048 + 16 * 37, 2048), (48, 2048)])
def test_dw2_factored_kernel_matches_fp64(h1, h2, ncols, cpp):
    """g2048_dw2_factored (the ReLU critic's dW2 / db2 from the factored records of g2048_critic_grad d2_form 1:
    a 16-bit mask word per unit and g per column, per 16-column block) against fp64 of W3[j] * sum fl(a1 g) m and
    W3[j] * sum g m on the same inputs: within 4e-6 of the sum of |terms|, full and padded hidden sizes, a column
    range starting inside the buffer and partial last slabs."""
    from rl2048_amd import _lib as L
    from rl2048_amd.agent import _padded_units, _unrecord

    H1p, H2p = _padded_units(h1), _padded_units(h2)
    R = max(H1p, H2p)
    col0 = 32
    ld = col0 + ncols + 32
    g = torch.Generator(device=DEV)
    g.manual_seed(h1 * 7 + ncols)
    A = torch.zeros(R, ld, device=DEV)
    A[:h1] = torch.relu(torch.randn(h1, ld, device=DEV, generator=g) *
                        torch.exp(3 * torch.randn(h1, ld, device=DEV, generator=g)))
    gc = torch.randn(ld, device=DEV, generator=g) * torch.exp(2 * torch.randn(ld, device=DEV, generator=g))
    M = (torch.rand(H2p, ld, device=DEV, generator=g) < 0.5)
    M[h2:] = False
    w3 = torch.zeros(H2p, device=DEV)
    w3[:h2] = torch.randn(h2, device=DEV, generator=g)
    # the records: uint16 mask words at bytes [0, 2 H2p), g at float 128.. of each 1 KiB block
    rec = torch.zeros(ld // 16, 256, device=DEV)
    words = torch.zeros(ld // 16, H2p, dtype=torch.int32, device=DEV)
    for k in range(16):
        words |= M[:, k::16].t().to(torch.int32) << k
    w16 = torch.where(words >= 32768, words - 65536, words).to(torch.int16)
    rec.view(torch.int16)[:, :H2p] = w16
    rec[:, 128:144] = gc.view(-1, 16)
    rec = rec.reshape(-1).contiguous()
    # the record decoder used by the gradient probe gives back fl(g W3[j]) m
    dec = _unrecord(rec, w3, col0, ncols)
    assert torch.equal(dec, ((gc[None, col0:col0 + ncols] * w3[:, None]) * M[:, col0:col0 + ncols].float()))
    blocked = lambda X: X.reshape(R, ld // 16, 16).permute(1, 0, 2).contiguous()  # noqa: E731 (include/g2048.h)
    a_in = blocked(A)
    nparts = -(-ncols // cpp)
    part = torch.full((nparts, H1p + 1, H2p), float("nan"), device=DEV)
    lib = L.lib()
    L.check(lib.g2048_dw2_factored(L.ptr(a_in), L.ptr(rec), L.ptr(w3), h1, h2, ld, col0, ncols, cpp, L.ptr(part),
                                   nparts, L.stream_handle(DEV)))
    torch.cuda.synchronize()
    AG = (A[:H1p, col0:col0 + ncols] * gc[None, col0:col0 + ncols]).double()   # fl(a1 g), then exact
    M64 = M[:, col0:col0 + ncols].double()
    W = w3.double()[None, :]
    G64 = gc[col0:col0 + ncols].double()
    for p in range(nparts):
        sl = slice(p * cpp, min((p + 1) * cpp, ncols))
        ref = (AG[:, sl] @ M64[:, sl].t()) * W
        bound = (AG[:, sl].abs() @ M64[:, sl].t()) * W.abs()
        got = part[p, :H1p].double()
        rel = float(((got - ref).abs() / bound.clamp_min(1e-30)).max())
        print(f"slab {p}: max |err| / sum |terms| = {rel:.3g}")
        assert bool(((got - ref).abs() <= 4e-6 * bound + 1e-30).all()), (p, rel)
        db = (M64[:, sl] @ G64[sl]) * w3.double()
        dbb = (M64[:, sl] @ G64[sl].abs()) * w3.double().abs()
        assert bool(((part[p, H1p].double() - db).abs() <= 4e-6 * dbb + 1e-30).all()), p
