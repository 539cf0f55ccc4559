"""TOOL: phase breakdown of grad_kernel (diag build): per workgroup, wave 0's summed durations of layer 1, layer 2,
softmax / loss + dW3, d2 and d1 + db1 + dW1 over its 32-sample groups of the last launch, divided by its groups.

    G2048_DIAG_LIB=tools/libg2048_diag.so python tools/diag_grad.py [--critic]
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
    ap.add_argument("--episodes", type=int, default=65536)
    ap.add_argument("--critic", action="store_true")
    args = ap.parse_args()
    assert os.environ.get("G2048_DIAG_LIB"), "set G2048_DIAG_LIB to the diag build"
    from rl2048_amd import _lib as _L0

    _L0.use_library_for_tools(os.environ["G2048_DIAG_LIB"])
    import torch

    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd import _lib as L
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    dev = torch.device("cuda", 0)
    lib = L.lib()
    lib.g2048_diag_grad_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
    agent = ReinforceAgent(Game2048EnvConfig(max_steps=1024),
                           MLPConfig(hidden_sizes=[256, 256], activation="ReLU", init_distribution="HeNormal"),
                           ReinforceAgentConfig(baseline_mode="batch", use_critic=args.critic), device=dev)
    n = args.episodes
    batch = agent.rollout_batch(list(range(n)), list(range(7 * n, 8 * n)))
    for _ in range(2):
        agent.update_from_batch(batch)
    torch.cuda.synchronize()
    buf = np.zeros((4096, 6), dtype=np.uint64)
    got = lib.g2048_diag_grad_phases(buf.ctypes.data, 4096)
    b = buf[:min(got, 256)].astype(np.float64)
    b = b[b[:, 5] > 0]
    per = b[:, :5] / b[:, 5:6] * 0.01   # us per group (100 MHz)
    names = ("layer1", "layer2+logits", "softmax+dW3", "d2", "d1+db1+dW1")
    print(json.dumps({"samples": int(batch.lengths.sum()), "blocks": int(len(b)), "groups_per_wave": float(b[:, 5].mean()),
                      "us_per_group": {k: round(float(per[:, i].mean()), 3) for i, k in enumerate(names)},
                      "us_per_group_total": round(float(per.sum(1).mean()), 3),
                      "mfma_floor_us_per_group": {"layer1": 64 * 64 / 2400, "layer2": 1024 * 64 / 2400,
                                                  "dW3": 128 * 32 / 2400, "d1": 1024 * 64 / 2400,
                                                  "dW1": 128 * 32 / 2400}}), flush=True)


if __name__ == "__main__":
    main()
