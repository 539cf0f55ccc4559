"""TOOL: phase breakdown of the one-launch rollout (diag build): per workgroup, the summed durations of layer 1,
layer 2, logits+choice+env step and claims over the whole rollout, divided by its steps.

    G2048_DIAG_LIB=tools/libg2048_diag.so python tools/diag_rollout.py --episodes 256 8192
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, nargs="+", default=[256, 8192])
    args = ap.parse_args()
    assert os.environ.get("G2048_DIAG_LIB"), "set G2048_DIAG_LIB to the diag build"
    import torch

    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd import _lib as L
    L.use_library_for_tools(os.environ["G2048_DIAG_LIB"])
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    dev = torch.device("cuda", 0)
    lib = L.lib()
    lib.g2048_diag_rollout_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
    agent = ReinforceAgent(Game2048EnvConfig(), MLPConfig(hidden_sizes=[256, 256], activation="ReLU",
                                                          init_distribution="HeNormal"), ReinforceAgentConfig(),
                           device=dev)
    for n in args.episodes:
        for rep in range(2):
            agent.rollout_batch(list(range(rep * n, rep * n + n)), list(range(10 * n, 11 * n)))
        torch.cuda.synchronize()
        buf = np.zeros((4096, 5), dtype=np.uint64)
        got = lib.g2048_diag_rollout_phases(buf.ctypes.data, 4096)
        blocks = min(got, (n + 31) // 32, 256)
        b = buf[:blocks].astype(np.float64)
        steps = b[:, 4]
        per = b[:, :4] / np.maximum(steps[:, None], 1) * 0.01   # us per step (100 MHz)
        print(json.dumps({"episodes": n, "blocks": int(blocks), "steps_mean": float(steps.mean()),
                          "steps_max": float(steps.max()),
                          "us_per_step": {k: round(float(per[:, i].mean()), 2) for i, k in
                                          enumerate(("layer1+barrier", "layer2+barrier", "env+choice", "claims"))}}),
              flush=True)


if __name__ == "__main__":
    main()
