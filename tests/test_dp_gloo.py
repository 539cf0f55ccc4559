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
