"""TOOL: training-loop throughput on the GPU box -- rollout_batch and update_from_batch timed separately for the
runner-default agent (MLP 16-256-256-4 ReLU, log2 obs, batch baseline), REINFORCE and actor-critic, at several
batch sizes (episodes per update).  One JSON line per configuration.

    python tools/bench_update.py [--episodes 256 4096 65536] [--critic]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if "--repo" in sys.argv:   # time another checkout's package (e.g. the round-3 tree) with this script
    ROOT = os.path.abspath(sys.argv[sys.argv.index("--repo") + 1])
sys.path.insert(0, ROOT)

FLOP_FWD = 2 * (16 * 256 + 256 * 256 + 256 * 4)      # per sample, actor forward
FLOP_BWD = 2 * (256 * 256 + 256 * 256 + 16 * 256 + 2 * 256 * 4)   # dW2, dH1, dW1, dW3 + dH2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, nargs="+", default=[256, 4096, 65536])
    ap.add_argument("--critic", action="store_true")
    ap.add_argument("--max-steps", type=int, default=1024)
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--lib", default=None, help="another build of libg2048 (A/B scripts)")
    ap.add_argument("--repo", default=None, help="import rl2048_amd from this checkout")
    ap.add_argument("--deep-grad", action="store_true",
                    help="the two-layer net through g2048_deep_grad (use_two_layer_grad = False; log2 [256, 256] is "
                         "past its one-launch budget, so this is the multi-launch form)")
    ap.add_argument("--no-actor-records", action="store_true",
                    help="actor d2 as columns + g2048_dw2 instead of d2_form 2 records + g2048_dw2_actor (A/B)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd import _lib as L

    if args.lib:
        L.use_library_for_tools(args.lib)
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for n in args.episodes:
        agent = ReinforceAgent(Game2048EnvConfig(max_steps=args.max_steps),
                               MLPConfig(hidden_sizes=[256, 256], activation="ReLU", init_distribution="HeNormal"),
                               ReinforceAgentConfig(baseline_mode="batch", use_critic=args.critic), device=dev)
        if args.no_actor_records:
            agent.actor_d2_records = False
        if args.deep_grad:
            agent.use_two_layer_grad = False
        for rep in range(args.repeats + 1):
            base = 1000 + rep * n
            es = np.arange(base, base + n, dtype=np.int64)   # seed arrays (SeedStream.take_array form)
            ps = es + 7 * n
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            batch = agent.rollout_batch(es, ps)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            agent.update_from_batch(batch)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if rep == 0:
                continue                       # warm-up (allocator, kernels)
            samples = int(batch.lengths.sum())
            flop = samples * (FLOP_FWD + FLOP_BWD) * (2 if args.critic else 1)
            print(json.dumps({"episodes": n, "critic": args.critic, "T": batch.T, "samples": samples,
                              "rollout_s": round(t1 - t0, 4), "update_s": round(t2 - t1, 4),
                              "rollout_steps_per_s": samples / (t1 - t0), "update_samples_per_s": samples / (t2 - t1),
                              "update_tflops": flop / (t2 - t1) / 1e12, "paths": agent.last_paths()}), flush=True)


if __name__ == "__main__":
    main()
