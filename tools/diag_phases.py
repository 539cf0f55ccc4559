"""TOOL: per-workgroup phase timing of g2048_step (diag build, tools/diag_build.sh) on the bench workload.

    G2048_DIAG_LIB=tools/libg2048_diag.so python tools/diag_phases.py [--rng pcg64 --obs log2 --boards N]

Prints, for a few launches after warm-up, the distribution over workgroups of: entry skew, table fill, main loop,
reset-list build, reset pass, and the span from the first entry to the last exit (s_memrealtime, 100 MHz)."""
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
    ap.add_argument("--rng", default="pcg64")
    ap.add_argument("--obs", default="log2")
    ap.add_argument("--boards", type=int, default=1 << 20)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--launches", type=int, default=5)
    args = ap.parse_args()
    assert os.environ.get("G2048_DIAG_LIB"), "set G2048_DIAG_LIB to the diag build"
    from rl2048_amd import _lib as _L0

    _L0.use_library_for_tools(os.environ["G2048_DIAG_LIB"])
    import torch

    import bench
    from rl2048_amd import _lib as L

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ns = argparse.Namespace(rng=args.rng, obs=args.obs, gpus=1, no_auto_reset=False)
    env = bench.make_env(torch, ns, args.boards, 0, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    acts = torch.randint(0, 4, (args.warmup + args.launches, args.boards), dtype=torch.uint8, device=dev, generator=g)
    for k in range(args.warmup):
        env.step_into(acts[k])
    torch.cuda.synchronize()
    lib = L.lib()
    lib.g2048_diag_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nb = 4096
    buf = np.zeros((nb, 5), dtype=np.uint64)
    for k in range(args.launches):
        buf[:] = 0
        env.step_into(acts[args.warmup + k])
        got = lib.g2048_diag_times(buf.ctypes.data, nb)
        t = buf[:got].astype(np.int64)
        t = t[t[:, 0] > 0]
        t0 = t[:, 0].min()
        rel = (t - t0) * 0.01  # us
        ph = {"entry_skew": rel[:, 0], "fill": rel[:, 1] - rel[:, 0], "loop": rel[:, 2] - rel[:, 1],
              "list": rel[:, 3] - rel[:, 2], "resets": rel[:, 4] - rel[:, 3], "exit": rel[:, 4]}
        out = {"launch": k, "blocks": int(len(t)), "span_us": round(float(rel[:, 4].max()), 2),
               "resets_this_step": int(((env.flags & L.F_RESET) != 0).sum())}
        for name, v in ph.items():
            out[name] = [round(float(np.percentile(v, q)), 2) for q in (0, 50, 100)]
        print(json.dumps(out), flush=True)
        np.save(os.path.join(ROOT, "gpurun_out", f"phases_raw_{k}.npy"), buf[:got])


if __name__ == "__main__":
    main()
