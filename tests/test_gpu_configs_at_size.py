"""GPU: every single-GPU configuration of BASELINE.json run at its real size and checked.

* configs[1] -- 65,536 parallel boards, REINFORCE + the runner-default 16-256-256-4 ReLU MLP: the one-launch
  rollout of 65,536 episodes (runner seed streams), a few hundred sampled episodes replayed in the CPU oracle (every
  board, fp64 reward, termination, and the action as numpy Generator.choice on the recorded probabilities), the
  probabilities against an fp64 forward, then the fused update on all ~8 M steps against an fp64 evaluation of
  update_batch's formula (src/reinforce_agent.py:357-555) over the whole batch.
* configs[2] -- 1,048,576 parallel boards, actor-critic: the same at ~128 M steps (critic MSE on TD errors, TD
  errors -> batch-baseline advantages), critic and actor gradients against fp64.
* configs[4] shard -- 1,048,576 lanes of the fused step with one-hot obs + action mask and the Philox per-lane
  spawn stream, auto-reset: sampled lanes replayed bit-exactly by the oracle's Philox restatement
  (oracle/g2048_oracle.c, pinned by Random123's known answers), spawn-distribution KAT over every lane.
(configs[3], 8-way RCCL, needs the 8-GPU node: tests/test_dp_gloo.py covers its exchange on CPU.)

Gradient tolerance: 1e-5 normwise-relative (max abs error / max abs value per tensor) against the exact fp64 value
of the formula under the ReLU activation pattern each fp32 path computed (tests/exact_grad.py): the fused kernels'
pattern is read from their own column buffers (ReinforceAgent.grad_probe), the plain hipBLASLt path's recomputed
on its own chunks.  At millions of samples fp32 rounding of pre-activations next to 0 flips ReLU derivatives, in
every fp32 evaluation (the reference's included) on different samples; the errors against fp64 with fp64's own
pattern are printed beside.  That basis is itself checked: every unit-sample where the fused pattern differs from
fp64's own must lie within the fp32 accumulation bound of the kink, and such unit-samples must be rare
(tests/exact_grad.py pattern_flip_check).
"""
import numpy as np
import pytest
import torch

import exact_grad as EG
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ENV = dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5, max_steps=1024)


def _rel(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _agent(**acfg):
    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    return ReinforceAgent(Game2048EnvConfig(**ENV), MLPConfig(hidden_sizes=[256, 256], activation="ReLU",
                                                              init_distribution="HeNormal"),
                          ReinforceAgentConfig(**acfg), device=DEV)


def _replay_sampled(batch, env_seeds, pol_seeds, k, seed):
    """Replay k sampled episodes (plus the first / last) in the oracle env + numpy PCG64 policy stream."""
    n = batch.n
    lens = batch.lengths.cpu().numpy()
    idx = sorted(set(np.random.default_rng(seed).choice(n, size=k, replace=False).tolist()) | {0, n - 1})
    it = torch.tensor(idx, device=DEV)
    T = batch.T
    boards = batch.boards[:, it].cpu().numpy().view(np.uint64)
    acts = batch.actions[:, it].cpu().numpy()
    rews = batch.rewards[:, it].cpu().numpy()
    probs = batch.probs[:, it].cpu().numpy()
    tot = batch.total_reward[it].cpu().numpy()
    mt = batch.max_tile[it].cpu().numpy()
    for j, i in enumerate(idx):
        env = O.Env(**ENV)
        env.reset(int(env_seeds[i]))
        pol = O.PCG64(int(pol_seeds[i]))
        total = 0.0
        Ti = int(lens[i])
        assert 0 < Ti <= T
        if j % 50 == 49:
            print(f"  replayed {j + 1} / {len(idx)} episodes", flush=True)
        for t in range(Ti):
            assert boards[t, j] == O.pack_exponents(O.values_to_exponents(env.board)), (i, t)
            assert pol.choice4(probs[t, j]) == acts[t, j], (i, t)
            r = env.step(int(acts[t, j]))
            assert rews[t, j] == r["reward"], (i, t)
            total += r["reward"]
            assert (r["terminated"] or r["truncated"]) == (t == Ti - 1), (i, t)
        assert tot[j] == total and mt[j] == env.max_tile_seen
    return idx


def _check_probs_fp64(agent, batch, idx):
    """The probabilities the rollout drew from vs an fp64 forward + masked softmax of the same boards."""
    it = torch.tensor(idx, device=DEV)
    lens = batch.lengths[it].to(torch.int64)
    b = batch.boards[:, it]
    valid = torch.arange(batch.T, device=DEV).unsqueeze(1) < lens.unsqueeze(0)
    x, mk = agent._obs_from_boards(b[valid].contiguous())
    W, bb = [w.double() for w in agent.params["W"]], [v.double() for v in agent.params["b"]]
    lg = EG.fwd64(W, bb, x.double())[4]
    p = torch.softmax(torch.where(mk.bool(), lg, torch.full_like(lg, -1e9)), dim=1)
    assert float((batch.probs[:, it][valid].double() - p).abs().max()) < 2e-6


def _run_config(episodes, critic, k_sample):
    from rl2048_amd.runner import SeedStream

    agent = _agent(baseline_mode="batch", gamma=0.99, use_critic=critic)
    es, ps = SeedStream(3).take_array(episodes), SeedStream(7).take_array(episodes)
    batch = agent.rollout_batch(es, ps, record_probs=True)
    assert batch.n == episodes
    print(f"\nrollout of {episodes} episodes done; replaying {k_sample} in the oracle", flush=True)
    idx = _replay_sampled(batch, es, ps, k_sample, seed=episodes)
    _check_probs_fp64(agent, batch, idx)
    print("replay and probabilities ok", flush=True)
    batch.probs = None
    N = int(batch.lengths.sum())
    params0 = EG.snapshot(agent)
    # the fused update, recording the ReLU pattern its kernels used (from their own a1^T / d2^T columns)
    probe = EG.PatternProbe(1, N, DEV)
    agent.grad_probe = probe
    stats = agent.update_from_batch(batch)
    agent.grad_probe = None
    nets = ("actor", "critic") if critic else ("actor",)
    assert all(probe.complete(w) for w in nets)
    # the same update through the plain fp32 GEMM path (hipBLASLt, mlp_backward_)
    plain = _agent(baseline_mode="batch", gamma=0.99, use_critic=critic)
    plain.use_fused_grad = False
    plain.update_from_batch(batch)
    exact_f = EG.exact_update_grads(agent, batch, patterns=probe, params=params0)
    errs = EG.grad_errors(agent.last_grads, exact_f)
    del exact_f
    exact_p = EG.exact_update_grads(plain, batch, patterns="plain", params=params0)
    errs_plain = EG.grad_errors(plain.last_grads, exact_p)
    del exact_p
    # plain fp64 (no imposed pattern), and the fused kernels' pattern compared with fp64's own on every unit-sample
    flips: dict = {}
    exact = EG.exact_update_grads(agent, batch, params=params0, flip_probe=probe, flip_stats=flips)
    del probe
    errs_free = EG.grad_errors(agent.last_grads, exact)
    errs_free_plain = EG.grad_errors(plain.last_grads, exact)
    for which in nets:
        en = float(torch.sqrt(sum((e ** 2).sum() for e in exact[which])))
        assert abs(stats[f"{which}_grad_norm"] - en) <= 1e-5 * en, (which, stats[f"{which}_grad_norm"], en)
    fmt = lambda d: ", ".join(f"{k}={v:.2e}" for k, v in d.items())  # noqa: E731
    print(f"\n{episodes} episodes, {N} steps: fused vs fp64 under the fused kernels' ReLU pattern {fmt(errs)} | "
          f"plain fp32 GEMM path vs fp64 under its pattern {fmt(errs_plain)} | vs fp64 with fp64's own pattern: "
          f"fused {fmt(errs_free)}, plain {fmt(errs_free_plain)}")
    # the basis is bounded: every unit-sample where the fused kernels' ReLU pattern differs from fp64's own lies
    # within the fp32 accumulation bound of the kink (|z| <= gamma_n sum |a w|, tests/exact_grad.py
    # pattern_flip_check), and such unit-samples are rare (<= 1e-5 of those compared, per layer and net)
    for which in nets:
        f = flips[which]
        print(f"{which}: ReLU pattern vs fp64's own: layer 1 {f['n1']} of {f['tot1']} unit-samples differ, layer 2 "
              f"{f['n2']} of {f['tot2']}; bound violations {f['viol1']} / {f['viol2']}; max |z| / bound "
              f"{f['max_ratio']:.3f}", flush=True)
        assert f["viol1"] == 0 and f["viol2"] == 0, (which, f)
        assert f["n1"] <= 1e-5 * f["tot1"] and f["n2"] <= 1e-5 * f["tot2"], (which, f)
    # the north star's 1e-5, for both fp32 paths, each against the exact value of the formula under the activation
    # pattern that path computed (module docstring)
    assert all(v < 1e-5 for v in errs.values()), errs
    assert all(v < 1e-5 for v in errs_plain.values()), errs_plain
    return N


def test_configs1_reinforce_65536_boards():
    N = _run_config(1 << 16, critic=False, k_sample=300)
    assert N > 4_000_000


def test_configs2_actor_critic_1m_boards():
    N = _run_config(1 << 20, critic=True, k_sample=200)
    assert N > 64_000_000


def test_configs4_shard_philox_onehot_1m_lanes():
    """configs[4]'s per-GPU shard: 1,048,576 lanes of g2048_step with one-hot obs + mask, Philox spawns and
    auto-reset (max_steps 16 forces resets through the Philox reset path), 48 steps; sampled lanes bit-exact
    against the oracle's Philox env; spawn ratio 2:4 = 0.9:0.1 and uniform cells over all fresh boards."""
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    n = 1 << 20
    cfg = dict(obs_mode="onehot", reward_mode="log2", base_reward_scale=0.5, bonus_mode="log2", max_steps=16)
    # no score output (the throughput configuration): the log2-reward lean step kernel with Philox spawns
    env = VecGame2048Env(n, Game2048EnvConfig(**cfg), device=DEV, rng="philox", auto_reset=True, reset_stride=n,
                         track_score=False)
    env.reset(seed=123_456)
    e = env.boards_exponents().reshape(n, 16)
    nz = e[e > 0]
    assert int(nz.numel()) == 2 * n
    frac2 = float((nz == 1).double().mean())
    assert abs(frac2 - 0.9) < 5 * np.sqrt(0.09 / (2 * n)), frac2
    cells = torch.bincount((e > 0).nonzero()[:, 1], minlength=16).double()
    assert float(cells.min() / cells.mean()) > 0.98
    idx = sorted(set(np.random.default_rng(4).choice(n, size=256, replace=False).tolist()) | {0, 1, 63, 64, n - 1})
    it = torch.tensor(idx, device=DEV)
    ref = {i: O.Env(rng="philox", philox_key=env.philox_key, **cfg) for i in idx}
    seeds = {i: 123_456 + i for i in idx}
    for i in idx:
        ref[i].reset(seeds[i])
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    resets = 0
    for t in range(48):
        acts = torch.randint(0, 4, (n,), dtype=torch.uint8, device=DEV, generator=g)
        env.step_into(acts)
        a, rw, fl = acts[it].cpu().numpy(), env.reward[it].cpu().numpy(), env.flags[it].cpu().numpy()
        bd, ob, mk = env.board[it].cpu().numpy().view(np.uint64), env.obs[it].cpu().numpy(), env.mask[it].cpu().numpy()
        for j, i in enumerate(idx):
            r = ref[i].step(int(a[j]))
            assert rw[j] == np.float32(r["reward"]), (t, i)
            assert bool(fl[j] & 0x02) == r["terminated"] and bool(fl[j] & 0x04) == r["truncated"], (t, i)
            if r["terminated"] or r["truncated"]:
                assert fl[j] & 0x20
                seeds[i] += n
                ref[i].reset(seeds[i])
                resets += 1
            assert bd[j] == O.pack_exponents(O.values_to_exponents(ref[i].board)), (t, i)
            np.testing.assert_array_equal(ob[j], ref[i].obs())
            np.testing.assert_array_equal(mk[j], ref[i].mask())
    assert resets >= 2 * len(idx)
