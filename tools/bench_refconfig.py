"""Time one training iteration (rollout_batch + update_from_batch) of the reference runner's documented config
(runner.py:10-47: one-hot obs, MLP [256, 128, 64] ReLU, actor-critic MSE, Adam, batch baseline, max_steps None) at
the given episode counts, against the package found under --repo (so a checkout of an earlier round can be timed
by the same script).  One warm-up iteration at every size (rep 0), then the timed one (rep 1) -- the
definition bench.py's train_iteration_reference_runner_config uses; prints one JSON object per iteration.

    python tools/bench_refconfig.py [--repo DIR] [--episodes 65536 1048576]     (G2048_LIB=<path>: an A/B build)
"""
import argparse
import json
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("--repo", default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap.add_argument("--episodes", type=int, nargs="+", default=[65536, 1 << 20])
ap.add_argument("--label", default="")
ap.add_argument("--hidden", type=int, nargs="+", default=[256, 128, 64], help="hidden sizes (other nets, same env)")
ap.add_argument("--no-fused-grad", action="store_true", help="update through the gather + hipBLASLt path (A/B)")
ap.add_argument("--multi-launch", action="store_true",
                help="deep_grad_multi_launch: nets past one launch's tile budget on g2048_deep_grad (A/B)")
args = ap.parse_args()
sys.path.insert(0, os.path.abspath(args.repo))
if os.environ.get("G2048_LIB"):   # an A/B build of the library
    from rl2048_amd import _lib as _L0

    _L0.use_library_for_tools(os.environ["G2048_LIB"])

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rl2048_amd import Game2048EnvConfig  # noqa: E402
from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig  # noqa: E402
from rl2048_amd.mlp import MLPConfig  # noqa: E402

ENV = dict(obs_mode="onehot", obs_log2_scale=1.0, reward_mode="log2", base_reward_scale=1.0, bonus_mode="off",
           bonus_scale=1.0, step_reward=0.0, endgame_penalty=0.0, use_action_mask=True, invalid_action_penalty=-1.0,
           max_steps=None, empty_tile_reward=0.05, merge_reward=0.0)
MLP = dict(hidden_sizes=list(args.hidden), activation="ReLU", init_distribution="HeNormal", last_init_normal=True)
AGENT = dict(gamma=0.99, learning_rate=0.01, baseline_mode="batch", model_seed=0, reward_rank_weights=None,
             optimizer="adam", adam_beta1=0.9, adam_beta2=0.999, augmentation=False, use_critic=True,
             critic_learning_rate=0.0005, critic_loss_type="mse", huber_delta=1.0)
dev = torch.device("cuda", 0)
agent = ReinforceAgent(Game2048EnvConfig(**ENV), MLPConfig(**MLP), ReinforceAgentConfig(**AGENT), device=dev)
if args.no_fused_grad:
    agent.use_fused_grad = False
if args.multi_launch:
    agent.deep_grad_multi_launch = True
for si, E in enumerate(args.episodes):
    for rep in range(2):   # one warm-up iteration at every size, then the timed one (bench.py's definition)
        es = np.arange(3 + (rep + 10 * si) * E, 3 + (rep + 10 * si + 1) * E, dtype=np.int64)
        ps = es + 7 * E
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batch = agent.rollout_batch(es, ps)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        agent.update_from_batch(batch)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rec = {"label": args.label, "hidden": list(args.hidden), "episodes": E, "rep": rep, "env_steps": int(batch.lengths.sum()),
               "longest_episode": batch.T, "rollout_s": round(t1 - t0, 4), "update_s": round(t2 - t1, 4),
               "iteration_s": round(t2 - t0, 4), "env_steps_per_s": int(batch.lengths.sum()) / (t2 - t0),
               "paths": agent.last_paths() if hasattr(agent, "last_paths") else "round-3 code"}
        print(json.dumps(rec), flush=True)
        del batch
