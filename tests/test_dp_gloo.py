"""CPU, world_size 2 (gloo): the data-parallel collectives of the update (rl2048_amd/dp.py) give every rank the
result of the concatenated global batch -- rank weights, weighted baseline statistics and the fused gradient
all-reduce -- which is what makes the N-GPU update equal to the 1-GPU update."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from rl2048_amd import dp

        rng = np.random.default_rng(0)
        totals = rng.integers(0, 50, size=13).astype(np.float64) + rng.random(13)   # distinct totals
        sizes = [6, 7]
        off = sum(sizes[:rank])
        mine = torch.tensor(totals[off:off + sizes[rank]])
        conf = [3.0, 2.0, 1.0, 1.0]
        w_local = dp.rank_weights(mine, conf)
        allg, o = dp.gather_varlen(mine)
        vals = torch.tensor(rng.standard_normal(40), dtype=torch.float32)
        wts = torch.tensor(rng.random(40), dtype=torch.float32)
        vshard, wshard = vals[rank * 20:(rank + 1) * 20], wts[rank * 20:(rank + 1) * 20]
        mean, std = dp.batch_mean_std(vshard, wshard)
        g = [torch.full((3, 2), float(rank + 1)), torch.arange(4, dtype=torch.float32) * (rank + 1)]
        dp.fused_all_reduce_(g)
        # reduce_gradients_: sum over ranks / global episode count (6 + 7), one collective
        h = [torch.full((2, 2), float(rank + 1) * 13.0), torch.ones(3) * (rank + 1) * 26.0]
        dp.reduce_gradients_(h, sizes[rank])
        # the same gathers with the shard sizes known host-side (no size exchange)
        w_local2 = dp.rank_weights(mine, conf, sizes=sizes)
        allg2, o2 = dp.gather_varlen(mine, sizes=sizes)
        # the count path alone, augmented episode counts (8 n) far above 2^24 whose fp32 sum would round
        big = [8 * 8_388_608 + 3, 8 * 1_000_001][rank]
        c = [torch.full((5,), float(rank + 1))]
        dp.reduce_gradients_(c, big)
        q.put((rank, w_local.numpy(), allg.numpy(), o, float(mean), float(std), [t.numpy() for t in g],
               [t.numpy() for t in h], w_local2.numpy(), allg2.numpy(), o2, c[0].numpy()))
    finally:
        dist.destroy_process_group()


def test_dp_collectives_equal_single_process():
    from rl2048_amd import dp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(0)
    totals = rng.integers(0, 50, size=13).astype(np.float64) + rng.random(13)
    vals = rng.standard_normal(40).astype(np.float32)
    wts = rng.random(40).astype(np.float32)
    w_single = dp.rank_weights(torch.tensor(totals), [3.0, 2.0, 1.0, 1.0]).numpy()
    np.testing.assert_array_equal(np.concatenate([res[0][1], res[1][1]]), w_single)
    np.testing.assert_array_equal(res[0][2], totals)
    assert res[0][3] == 0 and res[1][3] == 6
    m1, s1 = (float(x) for x in dp.batch_mean_std(torch.tensor(vals), torch.tensor(wts)))
    from oracle import agent_oracle as AO

    m_ref, s_ref = AO.OracleAgent.weighted_stats(vals, wts)        # src/reinforce_agent.py:864-881 (two-pass)
    assert abs(m1 - float(m_ref)) < 1e-6 and abs(s1 - float(s_ref)) < 1e-6
    for r in (0, 1):
        assert abs(res[r][4] - m1) < 1e-12 and abs(res[r][5] - s1) < 1e-12
        np.testing.assert_array_equal(res[r][6][0], np.full((3, 2), 3.0))
        np.testing.assert_array_equal(res[r][6][1], np.arange(4) * 3.0)
        np.testing.assert_allclose(res[r][7][0], np.full((2, 2), 3.0), rtol=1e-7)     # (13 + 26) / 13
        np.testing.assert_allclose(res[r][7][1], np.full(3, 6.0), rtol=1e-7)          # (26 + 52) / 13
        np.testing.assert_array_equal(res[r][8], res[r][1])
        np.testing.assert_array_equal(res[r][9], totals)
        assert res[r][10] == res[r][3]
        # (1 + 2) * fp32(1 / (67,108,867 + 8,000,008)): the global count is exact
        inv = np.float32(1.0 / (8 * 8_388_608 + 3 + 8 * 1_000_001))
        np.testing.assert_array_equal(res[r][11], np.full(5, np.float32(3.0) * inv, dtype=np.float32))


def test_rank_weights_match_reference_formula():
    """src/reinforce_agent.py:681-716 on distinct totals (single process)."""
    from rl2048_amd import dp
    from oracle import agent_oracle as AO

    rng = np.random.default_rng(5)
    for n in (1, 2, 7, 64):
        totals = rng.permutation(n).astype(np.float64) * 1.5
        for conf in ([1.0, 0.0], [3.0, 2.0, 1.0, 1.0], [1.0], None):
            ref = AO.OracleAgent({"W": [], "b": []}, None, AO.AgentCfg(reward_rank_weights=conf)).rank_weights(
                list(totals))
            got = dp.rank_weights(torch.tensor(totals), conf).numpy()
            np.testing.assert_allclose(got, ref, rtol=1e-6)


@pytest.mark.parametrize("n", [0, 5, 1000])
def test_batch_mean_std_single(n):
    """dp.batch_mean_std (fp64 single-pass) against the reference's two-pass weighted statistics, including the
    empty batch's (0, 1); values with a large mean relative to their spread (the returns' typical shape)."""
    from rl2048_amd import dp
    from oracle import agent_oracle as AO

    rng = np.random.default_rng(n)
    v = (rng.standard_normal(n) * 3 + 250).astype(np.float32)
    w = rng.choice([0.5, 1.0, 3.0], size=n).astype(np.float32)
    got = [float(x) for x in dp.batch_mean_std(torch.tensor(v), torch.tensor(w))]
    ref = AO.OracleAgent.weighted_stats(v.astype(np.float64), w.astype(np.float64))
    assert abs(got[0] - float(ref[0])) < 1e-9 * max(1.0, abs(float(ref[0]))) and abs(got[1] - float(ref[1])) < 1e-9


def test_shard_sizes_partition():
    from rl2048_amd import dp

    for n in (0, 1, 7, 8, 1 << 20, 4_194_304):
        for ws in (1, 2, 3, 8):
            sz = dp.shard_sizes(n, ws)
            assert sum(sz) == n and len(sz) == ws
            assert [dp.shard_bounds(n, r, ws) for r in range(ws)] == [
                (sum(sz[:r]), sum(sz[:r + 1])) for r in range(ws)]


def test_reduce_gradients_single_process_scale():
    """No process group: the gradients are multiplied by fp32(1 / n), the same factor the all-reduce path uses."""
    from rl2048_amd import dp

    n = 8 * 8_388_608 + 3
    t = [torch.full((4,), 3.0)]
    dp.reduce_gradients_(t, n)
    np.testing.assert_array_equal(t[0].numpy(), np.full(4, np.float32(3.0) * np.float32(1.0 / n), dtype=np.float32))


# ---------------------------------------------------------------------------------------------------------------
# world sizes 2, 4 and 8 (gloo, CPU): ragged shards and empty ranks.  Every collective of the update, and the
# sharded actor gradient built from them (per-rank sums of rank_w / T_i-weighted per-step gradients, the
# global batch baseline, ONE reduce_gradients_), equal the single-process values of the whole batch.
# (n, sizes): sizes None = dp.shard_sizes(n, ws) -- shard_bounds' ceil split, whose last ranks are short or empty
_SHARD_CASES = {
    2: [(13, None), (5, [0, 5])],
    4: [(13, None), (9, [3, 0, 4, 2])],
    8: [(13, None), (11, [2, 0, 3, 1, 0, 4, 1, 0]), (3, None)],
}
_CONF = [3.0, 2.0, 1.0, 1.0]


def _episodes(n, seed=7):
    """n small synthetic trajectories (16-float log2-style obs with masks, actions, fp64 rewards) and a 16-8-4 net."""
    rng = np.random.default_rng(seed + n)
    trajs = []
    for i in range(n):
        T = 1 + (7 * i) % 5
        obs = [{"board": rng.integers(0, 12, size=(4, 4)).astype(np.float32) / 4.0,
                "action_mask": (rng.random(4) < 0.8).astype(np.int8) | np.eye(4, dtype=np.int8)[i % 4]}
               for _ in range(T)]
        rewards = list(rng.standard_normal(T) * 2.0 + 0.3)
        trajs.append({"obs": obs, "actions": [int(a) for a in rng.integers(0, 4, size=T)], "rewards": rewards,
                      "total_reward": float(sum(rewards)) + 1e-3 * i})
    params = {"W": [rng.standard_normal((16, 8)) * 0.4, rng.standard_normal((8, 4)) * 0.4],
              "b": [rng.standard_normal(8) * 0.1, rng.standard_normal(4) * 0.1]}
    return trajs, params


def _sharded_actor_grads(trajs, params, sizes, rank):
    """What ReinforceAgent._update does on one rank (REINFORCE, batch baseline, rank weights), in fp64 through the
    pinned oracle's per-step formulas, with the collectives of rl2048_amd/dp.py."""
    from oracle import agent_oracle as AO
    from rl2048_amd import dp

    off = sum(sizes[:rank])
    mine = trajs[off: off + sizes[rank]]
    ag = AO.OracleAgent(params, None, AO.AgentCfg(baseline_mode="batch", reward_rank_weights=_CONF), dtype=np.float64)
    totals = torch.tensor([t["total_reward"] for t in mine], dtype=torch.float64)
    rw = dp.rank_weights(totals, _CONF, sizes=sizes).numpy()
    rets = [ag.compute_returns(t["rewards"]) for t in mine]
    vals = torch.tensor(np.concatenate(rets) if rets else np.zeros(0), dtype=torch.float64)
    wts = torch.tensor(np.concatenate([np.full(len(r), rw[i]) for i, r in enumerate(rets)]) if rets else np.zeros(0),
                       dtype=torch.float64)
    mean, _ = dp.batch_mean_std(vals, wts)
    gW = [np.zeros_like(W) for W in params["W"]]
    gb = [np.zeros_like(b) for b in params["b"]]
    for tr, ret, w_i in zip(mine, rets, rw):
        T = len(tr["obs"])
        X = np.array([AO.encode(o)[0] for o in tr["obs"]], dtype=np.float64)
        M = np.array([AO.encode(o)[1] for o in tr["obs"]])
        lg, acts, pres = AO.forward_logits(ag.params, X, "ReLU", np.float64)
        P = AO.logits_to_probs(lg, M)
        for t in range(T):
            oh = np.zeros(4)
            oh[tr["actions"][t]] = 1.0
            dW, db = ag.backprop(ag.params, [a[t] for a in acts], [p[t] for p in pres],
                                 (ret[t] - float(mean)) * (oh - P[t]))
            for l in range(2):
                gW[l] += float(w_i) / T * dW[l]
                gb[l] += float(w_i) / T * db[l]
    g = [torch.tensor(x) for x in gW + gb]
    dp.reduce_gradients_(g, len(mine))
    return [x.numpy() for x in g]


def _ws_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from rl2048_amd import dp

        out = []
        for n, sizes in _SHARD_CASES[world]:
            sizes = list(dp.shard_sizes(n, world)) if sizes is None else sizes
            off = sum(sizes[:rank])
            rng = np.random.default_rng(100 + n)
            totals = rng.integers(0, 20, size=n).astype(np.float64) + 0.25 * rng.integers(0, 3, size=n)  # with ties
            mine = torch.tensor(totals[off: off + sizes[rank]])
            allg, o = dp.gather_varlen(mine, sizes=sizes)
            allx, ox = dp.gather_varlen(mine)                                   # sizes exchanged
            w = dp.rank_weights(mine, _CONF, sizes=sizes)
            wx = dp.rank_weights(mine, _CONF)
            # per-step values / weights of the shard's episodes (episode i has 1 + i % 3 steps)
            lens = 1 + np.arange(n) % 3
            vals = rng.standard_normal(int(lens.sum())) * 4.0 + 30.0
            wts = np.repeat(rng.choice([0.5, 1.0, 2.0], size=n), lens)
            s0, s1 = int(lens[:off].sum()), int(lens[:off + sizes[rank]].sum())
            mean, std = dp.batch_mean_std(torch.tensor(vals[s0:s1], dtype=torch.float32),
                                          torch.tensor(wts[s0:s1], dtype=torch.float32))
            # gradient sums of this rank's episodes (rank r contributes (r + 1) per episode) / the global count
            h = [torch.full((3, 2), float(rank + 1) * sizes[rank]), torch.ones(4) * float(rank + 1) * sizes[rank]]
            dp.reduce_gradients_(h, sizes[rank])
            trajs, params = _episodes(n)
            grads = _sharded_actor_grads(trajs, params, sizes, rank)
            out.append((sizes, allg.numpy(), o, allx.numpy(), ox, w.numpy(), wx.numpy(), float(mean), float(std),
                        [t.numpy() for t in h], grads))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_world_sizes_ragged_and_empty_shards(world):
    from oracle import agent_oracle as AO
    from rl2048_amd import dp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ws_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out = q.get(timeout=240)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for ci, (n, _) in enumerate(_SHARD_CASES[world]):
        sizes = res[0][ci][0]
        assert sum(sizes) == n and len(sizes) == world
        rng = np.random.default_rng(100 + n)
        totals = rng.integers(0, 20, size=n).astype(np.float64) + 0.25 * rng.integers(0, 3, size=n)
        w_single = dp.rank_weights(torch.tensor(totals), _CONF).numpy()
        lens = 1 + np.arange(n) % 3
        vals = rng.standard_normal(int(lens.sum())) * 4.0 + 30.0
        wts = np.repeat(rng.choice([0.5, 1.0, 2.0], size=n), lens)
        m1, s1 = (float(x) for x in dp.batch_mean_std(torch.tensor(vals, dtype=torch.float32),
                                                     torch.tensor(wts, dtype=torch.float32)))
        trajs, params = _episodes(n)
        ref = AO.OracleAgent(params, None, AO.AgentCfg(baseline_mode="batch", reward_rank_weights=_CONF),
                             dtype=np.float64)
        ref.update_batch(trajs)
        gW, gb = ref.captured["actor_grads"]
        # the same per-step arithmetic in one process (no group): the sharded sums must equal it to rounding; and
        # it is the oracle's update_batch formula (whose baseline sums the weights in fp32, as the reference does)
        single = _sharded_actor_grads(trajs, params, [n], 0)
        for got, want in zip(single, list(gW) + list(gb)):
            assert np.linalg.norm(got - want) <= 1e-6 * max(np.linalg.norm(want), 1e-30)
        w_cat = np.concatenate([res[r][ci][5] for r in range(world)])
        np.testing.assert_array_equal(w_cat, w_single)                        # global ranks, ties by episode order
        np.testing.assert_array_equal(np.concatenate([res[r][ci][6] for r in range(world)]), w_single)
        for r in range(world):
            sz, allg, o, allx, ox, _, _, mean, std, h, grads = res[r][ci]
            assert sz == sizes
            np.testing.assert_array_equal(allg, totals)
            np.testing.assert_array_equal(allx, totals)
            assert o == ox == sum(sizes[:r])
            assert abs(mean - m1) < 1e-9 * abs(m1) and abs(std - s1) < 1e-9 * s1
            # sum over ranks of (r + 1) * sizes[r], over n
            expect = sum((q + 1) * sizes[q] for q in range(world)) / n
            np.testing.assert_allclose(h[0], np.full((3, 2), expect), rtol=1e-6)
            np.testing.assert_allclose(h[1], np.full(4, expect), rtol=1e-6)
            for got, want in zip(grads, single):
                assert np.linalg.norm(got - want) <= 1e-12 * max(np.linalg.norm(want), 1e-30), (world, ci, r)
