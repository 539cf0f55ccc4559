"""GPU: the any-depth / one-hot kernels of g2048_deep.hip against fp32 / fp64 references of the same ops.

* g2048_deep_policy (forward only): logits / value of random nets of 1..4 hidden layers (sizes not multiples of
  32 included), ReLU / Sigmoid, on log2 / raw / one-hot obs, against an fp64 forward of the materialised obs
  (src/MLP.py:159-196) -- within fp32 accumulation error;
* g2048_deep_policy (choice): the probabilities against torch's masked softmax of the kernel's own logits, and the
  action against g2048_sample run on those logits with a copy of the same PCG64 streams (the same device
  softmax_select and numpy Generator.choice replay: bit-identical), greedy included, compacted lane lists;
* g2048_onehot_layer1 against act(onehot(obs) @ W1 + b1) in fp64;
* g2048_onehot_dw1 (+ g2048_fold_partials) against X^T D1 / sum D1 in fp64, ragged part sizes.
The end-to-end parity of these paths (rollouts and updates of one-hot / 3- and 4-layer nets, the reference
runner's documented config included) is in tests/test_gpu_ref_fixtures.py against the real reference's outputs.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _lib():
    from rl2048_amd import _lib as L

    L.ensure_device(DEV)
    return L


def _boards(rng, n, hi=11):
    e = rng.integers(0, hi + 1, size=(n, 16))
    e[rng.random((n, 16)) < 0.35] = 0
    b = (e.astype(np.uint64) << (4 * np.arange(16, dtype=np.uint64))).sum(1)
    return torch.from_numpy(b.view(np.int64)).to(DEV), e


def _obs64(e, mode, scale):
    if mode == "onehot":
        x = np.zeros((len(e), 16, 17))
        np.put_along_axis(x, e[:, :, None], 1.0, axis=2)
        return torch.from_numpy(x.reshape(len(e), 272)).to(DEV)
    if mode == "log2":
        return torch.from_numpy((e * np.float32(scale)).astype(np.float32).astype(np.float64)).to(DEV)
    return torch.from_numpy(np.where(e > 0, 2.0 ** e, 0.0)).to(DEV)


def _net(rng, din, hidden, dout):
    sizes = [din] + list(hidden) + [dout]
    W = [torch.from_numpy((rng.standard_normal((a, b)) * np.sqrt(2.0 / a)).astype(np.float32)).to(DEV)
         for a, b in zip(sizes[:-1], sizes[1:])]
    B = [torch.from_numpy((rng.standard_normal(b) * 0.1).astype(np.float32)).to(DEV) for b in sizes[1:]]
    return W, B


def _fwd64(W, B, x, act):
    a = x
    for i, (w, b) in enumerate(zip(W, B)):
        z = a @ w.double() + b.double()
        a = z if i == len(W) - 1 else (torch.relu(z) if act == "ReLU" else torch.sigmoid(z))
    return a


def _fwd64_bound(W, B, x, act):
    """fp64 forward and a rigorous bound on an fp32 evaluation's error: every layer's pre-activation is a sum of
    fan-in + 1 terms, summed in some order with one rounding per operation (the MFMA chain is a k-ordered fmaf chain;
    the partial sums of the output layer add at most 8 more), so |z^ - z| <= gamma_n (|a^| |W| + |b|) + |W| |a^ - a|
    with n = fan-in + 10; ReLU passes the error through (Lipschitz 1), Sigmoid scales it by 1/4 and adds its own
    rounding (expf, one add, one divide: 4 ulp of a)."""
    u = 2.0 ** -24
    a, E = x, torch.zeros_like(x)
    for i, (w, b) in enumerate(zip(W, B)):
        wd, bd = w.double(), b.double()
        n = w.shape[0] + 10
        z = a @ wd + bd
        Ez = (n * u / (1 - n * u)) * ((a.abs() + E) @ wd.abs() + bd.abs()) + E @ wd.abs()
        if i == len(W) - 1:
            return z, Ez
        if act == "ReLU":
            a, E = torch.relu(z), Ez
        else:
            a = torch.sigmoid(z)
            E = 0.25 * Ez + 4 * u * a.abs()
    raise AssertionError("unreachable")


def _pack(L, W, B, obs_code, hidden, dout):
    lib = L.lib()
    harr = (ctypes.c_int32 * len(hidden))(*hidden)
    size = int(lib.g2048_deep_packed_size(obs_code, len(hidden), harr))
    assert size > 0
    packed = torch.empty(size, dtype=torch.float32, device=DEV)
    wp = (ctypes.c_void_p * len(W))(*[w.data_ptr() for w in W])
    bp = (ctypes.c_void_p * len(B))(*[b.data_ptr() for b in B])
    L.check(lib.g2048_deep_pack(wp, bp, obs_code, len(hidden), harr, dout, L.ptr(packed), size, L.stream_handle(DEV)))
    return packed, harr


NETS = [("onehot", [256, 128, 64], "ReLU"), ("onehot", [40, 33, 20, 10], "Sigmoid"), ("onehot", [128, 64], "ReLU"),
        ("log2", [64, 48, 32], "ReLU"), ("raw", [7], "Sigmoid"), ("log2", [256, 256, 256, 256], "ReLU"),
        ("onehot", [1], "ReLU")]


@pytest.mark.parametrize("dout", [4, 1])
@pytest.mark.parametrize("mode,hidden,act", NETS)
def test_deep_forward_matches_fp64(mode, hidden, act, dout):
    L = _lib()
    code = {"raw": L.OBS_RAW, "log2": L.OBS_LOG2, "onehot": L.OBS_ONEHOT}[mode]
    rng = np.random.default_rng(len(hidden) * 7 + hidden[0] + dout)
    din = 272 if mode == "onehot" else 16
    W, B = _net(rng, din, hidden, dout)
    packed, harr = _pack(L, W, B, code, hidden, dout)
    n = 3000 + 17                       # ragged last group; > 2 workgroups per CU of groups on small nets
    b, e = _boards(rng, n)
    out = torch.empty(n, 4, dtype=torch.float32, device=DEV)
    L.check(L.lib().g2048_deep_policy(L.ptr(packed), len(hidden), harr, L.ACT_RELU if act == "ReLU" else L.ACT_SIGMOID,
                                      L.ptr(b), None, None, code, 0.0625, 0, 1, L.RNG_PCG64, None, None, None, 0, None,
                                      None, L.ptr(out), None, n, L.stream_handle(DEV)))
    ref, bound = _fwd64_bound(W, B, _obs64(e, mode, 0.0625), act)
    got = out[:, :dout].double()
    # every output within the fp32 forward-error bound of its fp64 value (raw obs reach 2^15, so a max-normalised
    # tolerance would not be scale-free)
    ratio = float(((got - ref).abs() / bound.clamp_min(1e-300)).max())
    print(f"\n{mode} {hidden} {act}: max |err| / bound = {ratio:.3g}, max rel err {float((got - ref).abs().max() / ref.abs().max()):.3g}")
    assert ratio <= 1.0, ratio
    if dout == 1:
        assert bool((out[:, 1:] == 0).all())


@pytest.mark.parametrize("greedy", [0, 1])
@pytest.mark.parametrize("compact", [False, True])
def test_deep_choice_equals_g2048_sample(greedy, compact):
    """The fused choice == g2048_sample on the kernel's own logits with a copy of the same PCG64 streams."""
    L = _lib()
    lib, st = L.lib(), L.stream_handle(DEV)
    rng = np.random.default_rng(5 + greedy)
    hidden = [256, 128, 64]
    W, B = _net(rng, 272, hidden, 4)
    packed, harr = _pack(L, W, B, L.OBS_ONEHOT, hidden, 4)
    n = 5000 + 3
    b, e = _boards(rng, n)
    seeds = torch.arange(n, dtype=torch.int64, device=DEV) + 777
    rs = torch.empty(2 * n, dtype=torch.int64, device=DEV)
    inc = torch.empty(2 * n, dtype=torch.int64, device=DEV)
    buf = torch.empty(n, dtype=torch.int64, device=DEV)
    L.check(lib.g2048_seed_pcg64(L.ptr(seeds), L.ptr(rs), L.ptr(inc), L.ptr(buf), n, st))
    rs2 = rs.clone()
    idx = torch.from_numpy(np.sort(rng.choice(n, size=n // 3, replace=False)).astype(np.int32)).to(DEV) if compact \
        else None
    m = n // 3 if compact else n
    acts = torch.full((n,), 9, dtype=torch.uint8, device=DEV)
    probs = torch.zeros(n, 4, dtype=torch.float32, device=DEV)
    logits = torch.zeros(n, 4, dtype=torch.float32, device=DEV)
    L.check(lib.g2048_deep_policy(L.ptr(packed), 3, harr, L.ACT_RELU, L.ptr(b), None, L.ptr(idx), L.OBS_ONEHOT, 1.0, 1,
                                  greedy, L.RNG_PCG64, L.ptr(rs), L.ptr(inc), L.ptr(buf), 0, None, L.ptr(probs),
                                  L.ptr(logits), L.ptr(acts), m, st))
    # the same choice from the same logits through g2048_sample (lane state: only the listed lanes active)
    mask = torch.empty(n, 4, dtype=torch.int8, device=DEV)
    L.check(lib.g2048_obs(L.ptr(b), L.OBS_NONE, 1.0, None, L.ptr(mask), n, st))
    ls = torch.zeros(n, dtype=torch.int32, device=DEV)
    sel = idx.long() if compact else torch.arange(n, device=DEV)
    ls[sel] = L.LS_ACTIVE
    acts2 = torch.full((n,), 9, dtype=torch.uint8, device=DEV)
    probs2 = torch.zeros(n, 4, dtype=torch.float32, device=DEV)
    L.check(lib.g2048_sample(L.ptr(logits), L.ptr(mask), L.ptr(ls), greedy, L.RNG_PCG64, L.ptr(rs2), L.ptr(inc),
                             L.ptr(buf), 0, None, L.ptr(probs2), L.ptr(acts2), n, st))
    assert torch.equal(acts, acts2) and torch.equal(probs, probs2)
    if not greedy:
        assert torch.equal(rs, rs2)
    # untouched lanes stay untouched; probabilities are the masked softmax of the logits
    if compact:
        off = torch.ones(n, dtype=torch.bool, device=DEV)
        off[sel] = False
        assert bool((acts[off] == 9).all())
    p_ref = torch.softmax(torch.where(mask[sel].bool(), logits[sel], torch.full_like(logits[sel], -1e9)).double(), 1)
    assert float((probs[sel].double() - p_ref).abs().max()) < 1e-6
    ref = _fwd64(W, B, _obs64(e, "onehot", 1.0), "ReLU")[sel]
    assert float((logits[sel].double() - ref).abs().max() / ref.abs().max()) < 2e-6


@pytest.mark.parametrize("h1,act", [(256, "ReLU"), (100, "Sigmoid"), (33, "ReLU")])
def test_onehot_layer0_bits_equal_plane_emulation(h1, act):
    """A one-hot net's layer 0 (ABI 15: the update's onehot_l0_mfma_kernel, read here through g2048_deep_hidden,
    and deep_forward in the rollout / policy kernels run the same arithmetic) bit for bit equal to its definition
    emulated in torch fp32: W1 split into bf16 planes hi + mid + lo (round to nearest even, exact residuals), per
    board the hi rows of its 16 cells accumulated from 0 in cell order and, separately, ((acc + mid_c) + lo_c) in cell
    order -- one fp32 rounding per add, which is what each v_mfma_f32_32x32x16_bf16 with a one-hot B operand does (one
    exact nonzero product per output) -- then act((hi + lo) + b1)."""
    L = _lib()
    from rl2048_amd.agent import _round32

    rng = np.random.default_rng(h1 + 11)
    W, B = _net(rng, 272, [h1], 4)
    packed, harr = _pack(L, W, B, L.OBS_ONEHOT, [h1], 4)
    n = 4000 + 5
    b, e = _boards(rng, n, hi=15)
    H = _round32(h1)
    out = torch.empty(n, H, dtype=torch.float32, device=DEV)
    code = L.ACT_RELU if act == "ReLU" else L.ACT_SIGMOID
    L.check(L.lib().g2048_deep_hidden(L.ptr(packed), 1, harr, code, L.OBS_ONEHOT, 1.0, L.ptr(b), n, 0, L.ptr(out), H,
                                      L.stream_handle(DEV)))
    w1 = W[0]
    hi = w1.to(torch.bfloat16).float()
    r = w1 - hi
    mid = r.to(torch.bfloat16).float()
    lo = (r - mid).to(torch.bfloat16).float()
    assert torch.equal(hi + mid + lo, w1)                # the split is exact
    rows = torch.from_numpy(17 * np.arange(16) + e).to(DEV)
    acc_h = torch.zeros(n, h1, dtype=torch.float32, device=DEV)
    acc_l = torch.zeros_like(acc_h)
    for c in range(16):
        acc_h = acc_h + hi[rows[:, c]]
        acc_l = (acc_l + mid[rows[:, c]]) + lo[rows[:, c]]
    z = (acc_h + acc_l) + B[0]
    ref = torch.relu(z) if act == "ReLU" else 1.0 / (1.0 + torch.exp(-z))
    got = out[:, :h1]
    if act == "ReLU":
        assert torch.equal(got, ref)
    else:   # the kernel's expf / divide against torch's: the pre-activation bits are what is pinned here
        torch.testing.assert_close(got, ref, rtol=0, atol=2e-7)


@pytest.mark.parametrize("h1,act", [(256, "ReLU"), (100, "Sigmoid"), (64, "ReLU"), (1, "ReLU")])
def test_onehot_layer1_matches_fp64(h1, act):
    L = _lib()
    rng = np.random.default_rng(h1)
    W, B = _net(rng, 272, [h1], 4)
    n = 7001
    b, e = _boards(rng, n, hi=15)
    ld = h1 + 3
    out = torch.full((n, ld), 7.0, dtype=torch.float32, device=DEV)
    L.check(L.lib().g2048_onehot_layer1(L.ptr(W[0]), L.ptr(B[0]), h1, L.ACT_RELU if act == "ReLU" else L.ACT_SIGMOID,
                                        L.ptr(b), n, ld, L.ptr(out), L.stream_handle(DEV)))
    z = _obs64(e, "onehot", 1.0) @ W[0].double() + B[0].double()
    ref = torch.relu(z) if act == "ReLU" else torch.sigmoid(z)
    assert float((out[:, :h1].double() - ref).abs().max() / ref.abs().max()) < 1e-6
    assert bool((out[:, h1:] == 7.0).all())


@pytest.mark.parametrize("h1,m,per", [(256, 20000, 1024), (256, 70001, 4096), (100, 5000, 777), (64, 3, 1024),
                                       (1, 999, 100), (200, 33, 16)])
def test_onehot_dw1_matches_fp64(h1, m, per):
    L = _lib()
    lib, st = L.lib(), L.stream_handle(DEV)
    rng = np.random.default_rng(h1 + m)
    b, e = _boards(rng, m, hi=15)
    d1 = torch.from_numpy(rng.standard_normal((m, h1)).astype(np.float32)).to(DEV)
    nparts = -(-m // per)
    slab = int(lib.g2048_onehot_dw1_slab(h1))
    assert slab == 273 * h1
    part = torch.empty(nparts, slab, dtype=torch.float32, device=DEV)
    L.check(lib.g2048_onehot_dw1(L.ptr(b), L.ptr(d1), h1, m, h1, per, L.ptr(part), nparts, st))
    acc = torch.zeros(slab, dtype=torch.float64, device=DEV)
    L.check(lib.g2048_fold_partials(L.ptr(part), nparts, slab, L.ptr(acc), st))
    X = _obs64(e, "onehot", 1.0)
    ref_w = X.t() @ d1.double()
    ref_b = d1.double().sum(0)
    # dW1: each slab element is an fp32 accumulation (bf16 MFMA, round 5) of the exact products of the one-hot with
    # the three bf16 planes of every delta (d = d0 + d1 + d2 exactly, sum |d_i| <= (1 + 2^-7) |d|): at most 3 per
    # exact terms, 16 per MFMA -- bounded as a sequential fp32 sum of 3 per + 16 terms
    n = 3 * per + 16
    g = n * 2.0 ** -24 / (1 - n * 2.0 ** -24) * (1 + 2.0 ** -7)
    assert bool(((acc[:272 * h1].view(272, h1) - ref_w).abs() <= g * (X.t() @ d1.double().abs()) + 1e-30).all())
    # db1: per lane half a sequential fp32 sum (<= per terms), the halves added once
    g = per * 2.0 ** -24 / (1 - per * 2.0 ** -24)
    assert bool(((acc[272 * h1:] - ref_b).abs() <= g * d1.double().abs().sum(0) + 1e-30).all())
    # and far tighter than that bound in practice: within 1e-6 of the fp64 value normwise
    assert float((acc[:272 * h1].view(272, h1) - ref_w).norm() / ref_w.norm()) < 1e-6
    # rows of a one-hot feature no sample has are exactly zero
    seen = torch.zeros(272, dtype=torch.bool, device=DEV)
    seen[(torch.arange(16, device=DEV) * 17 + torch.from_numpy(e).to(DEV)).reshape(-1)] = True
    assert bool((acc[:272 * h1].view(272, h1)[~seen] == 0).all())


@pytest.mark.parametrize("h1,m,per", [(256, 20000, 1024), (256, 9001, 4096), (100, 5000, 777), (200, 33, 16),
                                       (64, 3, 1024), (6, 1000, 48), (256, 300, 2000)])
def test_onehot_dw1_ring_bits_equal_register_form(h1, m, per):
    """The LDS-DMA ring dW1 kernel (16-byte rows: ld % 4 == 0, round 5) against the register form (taken for any
    other row stride), bit for bit, on the same deltas: same MFMAs, same order.  NaN in the row padding: neither
    may read past unit h1 into a result."""
    L = _lib()
    lib, st = L.lib(), L.stream_handle(DEV)
    rng = np.random.default_rng(7 * h1 + m)
    b, _ = _boards(rng, m, hi=15)
    d = torch.from_numpy(rng.standard_normal((m, h1)).astype(np.float32)).to(DEV)
    slab = int(lib.g2048_onehot_dw1_slab(h1))
    nparts = -(-m // per)
    parts = []
    for ld in (4 * (-(-h1 // 4)) + 4, 4 * (-(-h1 // 4)) + 1):   # ring, register form
        buf = torch.full((m, ld), float("nan"), dtype=torch.float32, device=DEV)
        buf[:, :h1] = d
        part = torch.empty(nparts, slab, dtype=torch.float32, device=DEV)
        L.check(lib.g2048_onehot_dw1(L.ptr(b), L.ptr(buf), h1, m, ld, per, L.ptr(part), nparts, st))
        parts.append(part)
    torch.cuda.synchronize()
    assert not bool(torch.isnan(parts[0]).any())
    assert torch.equal(parts[0].view(torch.int32), parts[1].view(torch.int32))


REFCONF_ENV = dict(obs_mode="onehot", obs_log2_scale=1.0, reward_mode="log2", base_reward_scale=1.0,
                   use_action_mask=True, invalid_action_penalty=-1.0, max_steps=None, empty_tile_reward=0.05)


def _agent(env: dict, hidden, act="ReLU", **acfg):
    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    return ReinforceAgent(Game2048EnvConfig(**env), MLPConfig(hidden_sizes=hidden, activation=act,
                                                              init_distribution="HeNormal"),
                          ReinforceAgentConfig(**acfg), device=DEV)


def test_deep_rollout_refuses_unbounded_growth():
    """max_steps=None: episodes still running when the trajectory buffer would grow past deep_rollout_max_rows raise
    a clear RuntimeError instead of doubling the [T, n] buffers until the device runs out of memory (an episode the
    reference would play forever -- invalid actions allowed -- must not take the process down)."""
    a = _agent(REFCONF_ENV, [64, 32])
    a.deep_rollout_cap0, a.deep_rollout_max_rows = 8, 12
    es = np.arange(7_000, 7_000 + 257, dtype=np.int64)
    with pytest.raises(RuntimeError, match="still running after 8 steps"):
        a.rollout_batch(es, es + 10 ** 9)
    a.deep_rollout_max_rows = 1 << 24                     # and the same agent then rolls out normally
    b = a.rollout_batch(es, es + 10 ** 9)
    assert b.T > 8 and int(b.lengths.min()) > 0


@pytest.mark.parametrize("env,hidden", [(REFCONF_ENV, [256, 128, 64]),
                                        (dict(obs_mode="log2", obs_log2_scale=0.0625, max_steps=None), [256, 256]),
                                        (dict(REFCONF_ENV, max_steps=70), [40, 33, 20, 10])])
def test_deep_rollout_suspend_resume_equals_stepwise(env, hidden):
    """g2048_deep_rollout with a tiny first capacity (every episode is suspended and resumed several times as the
    buffer doubles) == the per-step path (g2048_deep_policy + g2048_step) on the same seeds: every board, action,
    fp64 reward, flag, probability, length, total, max tile and final board; sampled episodes replayed in the oracle
    (env + numpy Generator.choice on the recorded probabilities)."""
    from oracle import oracle as O
    from rl2048_amd import _lib as L

    n = 3001
    es = np.arange(50_000, 50_000 + n, dtype=np.int64)
    ps = es + 10 ** 9
    a = _agent(env, hidden)
    a.deep_rollout_cap0 = 8
    b1 = a.rollout_batch(es, ps, record_probs=True)
    assert a.last_paths()["rollout"].startswith("g2048_deep_rollout")
    a.use_fused_rollout = False
    b2 = a.rollout_batch(es, ps, record_probs=True)
    assert "g2048_deep_policy" in a.last_paths()["rollout"] or "g2048_policy" in a.last_paths()["rollout"]
    assert b1.T == b2.T and b1.T > 8
    assert torch.equal(b1.lengths, b2.lengths)
    valid = torch.arange(b1.T, device=DEV).unsqueeze(1) < b1.lengths.unsqueeze(0)
    for name in ("boards", "actions", "rewards"):
        x, y = getattr(b1, name), getattr(b2, name)
        assert torch.equal(x[valid], y[valid]), name
    assert torch.equal((b1.flags & ~L.F_INACTIVE)[valid], (b2.flags & ~L.F_INACTIVE)[valid])
    if "g2048_deep_policy" in a.last_paths()["rollout"]:   # the same forward code: bit for bit
        assert torch.equal(b1.probs[valid], b2.probs[valid])
    else:   # 2 hidden layers step by g2048_policy, whose output layer sums its partials in another order
        torch.testing.assert_close(b1.probs[valid], b2.probs[valid], rtol=0, atol=2e-6)
    assert torch.equal(b1.total_reward, b2.total_reward) and torch.equal(b1.max_tile, b2.max_tile)
    assert torch.equal(b1.final_boards, b2.final_boards)
    ocfg = {k: v for k, v in env.items()}
    lens = b1.lengths.cpu().numpy()
    for i in [0, 1, n // 2, n - 1] + list(np.random.default_rng(0).choice(n, 20, replace=False)):
        e, pol = O.Env(**ocfg), O.PCG64(int(ps[i]))
        e.reset(int(es[i]))
        total = 0.0
        bb, aa = b1.boards[:, i].cpu().numpy().view(np.uint64), b1.actions[:, i].cpu().numpy()
        rr, pp = b1.rewards[:, i].cpu().numpy(), b1.probs[:, i].cpu().numpy()
        for t in range(int(lens[i])):
            assert bb[t] == O.pack_exponents(O.values_to_exponents(e.board)), (i, t)
            assert pol.choice4(pp[t]) == aa[t], (i, t)
            r = e.step(int(aa[t]))
            assert rr[t] == r["reward"], (i, t)
            total += r["reward"]
            assert (r["terminated"] or r["truncated"]) == (t == lens[i] - 1), (i, t)
        assert float(b1.total_reward[i]) == total


@pytest.mark.parametrize("n", [1, 5, 63, 64, 65, 129])
def test_deep_rollout_ragged_slot_counts(n):
    """The 64-slot one-hot rollout (deep_forward64: one 8-wave workgroup per CU, 64 slots) at episode counts that
    leave slots, workgroups and the last claim ragged -- fewer episodes than one workgroup's slots, one more than a
    full workgroup -- bit for bit the per-step path (g2048_deep_policy + g2048_step) on the same seeds."""
    from rl2048_amd import _lib as L

    es = np.arange(90_000, 90_000 + n, dtype=np.int64)
    ps = es + 10 ** 9
    a = _agent(dict(REFCONF_ENV, max_steps=120), [256, 128, 64])
    b1 = a.rollout_batch(es, ps, record_probs=True)
    assert a.last_paths()["rollout"].startswith("g2048_deep_rollout")
    a.use_fused_rollout = False
    b2 = a.rollout_batch(es, ps, record_probs=True)
    assert b1.T == b2.T and torch.equal(b1.lengths, b2.lengths)
    valid = torch.arange(b1.T, device=DEV).unsqueeze(1) < b1.lengths.unsqueeze(0)
    for name in ("boards", "actions", "rewards", "probs"):
        assert torch.equal(getattr(b1, name)[valid], getattr(b2, name)[valid]), name
    assert torch.equal((b1.flags & ~L.F_INACTIVE)[valid], (b2.flags & ~L.F_INACTIVE)[valid])
    assert torch.equal(b1.total_reward, b2.total_reward) and torch.equal(b1.final_boards, b2.final_boards)


@pytest.mark.parametrize("fused,rows", [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize("env,hidden,act,critic", [(REFCONF_ENV, [256, 128, 64], "ReLU", True),
                                                   (dict(REFCONF_ENV, max_steps=200), [40, 33, 20, 10], "Sigmoid", False),
                                                   (dict(obs_mode="log2", obs_log2_scale=0.0625, max_steps=None),
                                                    [64, 48, 32], "ReLU", True),
                                                   # round 5: 64 dense tiles (the 8-wave, 8-tiles-per-wave kernel)
                                                   (REFCONF_ENV, [256, 256], "ReLU", True),
                                                   # round 5: 128 tiles, two launches (one per range of 64 dW tiles)
                                                   (dict(REFCONF_ENV, max_steps=300), [256, 256, 256], "ReLU", True),
                                                   # 80 log2 tiles, two launches of <= 48 (Sigmoid, a 3-layer net)
                                                   (dict(obs_mode="log2", obs_log2_scale=0.0625, max_steps=300),
                                                    [256, 256, 64], "Sigmoid", False)])
def test_deep_update_at_size_vs_fp64(env, hidden, act, critic, fused, rows):
    """update_from_batch on nets the register-specialised kernels do not cover (the reference runner's documented
    config first: one-hot obs, 256-128-64, actor-critic) over 16,384 episodes of its own rollout: the pre-clip
    gradients within 1e-5 normwise of the exact fp64 value of update_batch's formula under the fp32 path's own
    ReLU pattern (tests/exact_grad.py exact_update_grads_deep), that pattern bounded against fp64's own (every
    disagreement within the fp32 accumulation bound, <= 1e-5 of the unit-samples), and the norms within 1e-5.
    fused: g2048_deep_grad (forward + backward in one kernel; the one-hot first layer by g2048_onehot_dw1's
    scatter); else the gather + hipBLASLt path (g2048_onehot_layer1 / g2048_onehot_dw1 around torch GEMMs).
    rows: the critic by time rows, last first (each launch's V(s) the previous row's V(s'), no V(s') forward),
    forced on this batch size (by default from 16,384 samples per row)."""
    import exact_grad as EG

    if rows and not critic:
        pytest.skip("the row pass is the critic's")
    a = _agent(env, hidden, act, baseline_mode="batch", gamma=0.99, use_critic=critic, optimizer="adam",
               learning_rate=0.01, critic_learning_rate=5e-4)
    a.use_fused_grad = fused
    a.deep_grad_multi_launch = True   # nets past one launch's tile budget: the multi-launch form under test
    if rows:
        a.critic_rows_min_avg = 0
        a.critic_tail_row_max = 256
    n = 16384
    es = np.arange(7, 7 + n, dtype=np.int64)
    batch = a.rollout_batch(es, es + 3 * n)
    params0 = EG.snapshot(a)
    stats = a.update_from_batch(batch)
    paths = a.last_paths()
    if fused:
        assert paths["actor_grad"].startswith("g2048_deep_grad"), paths
        if critic:
            assert paths["critic_grad"].startswith("g2048_deep_grad"), paths
            assert ("time rows" in paths["critic_grad"]) == rows, paths
    elif env["obs_mode"] == "onehot":
        assert "g2048_onehot_layer1" in paths["actor_grad"], paths
    flips: dict = {}
    exact = EG.exact_update_grads_deep(a, batch, params0, "deep" if fused else "plain", flips)
    errs = EG.grad_errors(a.last_grads, exact)
    print(f"\n{env['obs_mode']} {hidden} {act}: {int(batch.lengths.sum())} samples, paths {paths}, errors {errs}, "
          f"flips {flips}", flush=True)
    assert all(v < 1e-5 for v in errs.values()), errs
    for which, f in flips.items():
        assert sum(f["viol"]) == 0, (which, f)
        assert all(k <= 1e-5 * t for k, t in zip(f["n"], f["tot"])), (which, f)
    for which in ("actor", "critic") if critic else ("actor",):
        en = float(torch.sqrt(sum((e ** 2).sum() for e in exact[which])))
        assert abs(stats[f"{which}_grad_norm"] - en) <= 1e-5 * en, (which, stats, en)
