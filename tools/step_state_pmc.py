"""Step launches from bench.py's synthetic start: S untimed steps, then K more (run under rocprofv3 --pmc to compare
counters of the launches after S = 5 with those after S = 40; tools/step_launch_probe.py has the timings)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import bench

    dev = torch.device("cuda:0")
    args = argparse.Namespace(obs="log2", rng="pcg64", gpus=1, no_auto_reset=False)
    B = 1 << 20
    env = bench.make_env(torch, args, B, 0, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    n = a.skip + a.steps
    actions = torch.randint(0, 4, (n, B), dtype=torch.uint8, device=dev, generator=g)
    for k in range(n):
        env.step_into(actions[k])
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
