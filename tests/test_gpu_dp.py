"""GPU, 2 ranks on cuda:0 (gloo transport; the production backend is RCCL): the data-parallel batched training
step (each rank plays its slice of the batch's seeds, then update_from_batch with the fused gradient all-reduce)
yields exactly the parameters of the single-process step on the whole batch (within fp32 reduction-order noise).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ACFG = dict(baseline_mode="batch_norm", optimizer="adam", use_critic=True, gamma=0.99,
            reward_rank_weights=[3.0, 2.0, 1.0, 1.0], learning_rate=1e-3)
N_EP = 24


def _agent():
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    cfg = Game2048EnvConfig(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5,
                            max_steps=200)
    return ReinforceAgent(cfg, MLPConfig(hidden_sizes=[32, 16], activation="ReLU", init_distribution="HeNormal"),
                          ReinforceAgentConfig(**ACFG), device="cuda:0")


def _seeds():
    rng = np.random.default_rng(17)
    return ([int(s) for s in rng.integers(0, 2**62, size=N_EP)], [int(s) for s in rng.integers(0, 2**62, size=N_EP)])


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        agent = _agent()
        es, ps = _seeds()
        per = N_EP // world
        b = agent.rollout_batch(es[rank * per:(rank + 1) * per], ps[rank * per:(rank + 1) * per])
        stats = agent.update_from_batch(b)
        q.put((rank, [t.cpu().numpy() for t in agent.params["W"] + agent.params["b"]],
               [t.cpu().numpy() for t in agent.critic_params["W"] + agent.critic_params["b"]],
               stats["actor_grad_norm"]))
    finally:
        dist.destroy_process_group()


def test_two_rank_update_equals_single_process():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=300)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    agent = _agent()
    es, ps = _seeds()
    stats = agent.update_from_batch(agent.rollout_batch(es, ps))
    ref_a = [t.cpu().numpy() for t in agent.params["W"] + agent.params["b"]]
    ref_c = [t.cpu().numpy() for t in agent.critic_params["W"] + agent.critic_params["b"]]
    for rank in (0, 1):
        for a, b in zip(res[rank][1], ref_a):
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=2e-7)
        for a, b in zip(res[rank][2], ref_c):
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=2e-7)
        assert abs(res[rank][3] - stats["actor_grad_norm"]) <= 1e-5 * stats["actor_grad_norm"]
    for a, b in zip(res[0][1], res[1][1]):   # replicas stay identical
        np.testing.assert_array_equal(a, b)
