"""TOOL: the one-hot layer-0 kernel (onehot_l0_mfma_kernel) alone, through g2048_deep_hidden(layer 0) on a one-hot
[256, 128, 64] net: K calls over N random boards (default 307,200: about one runner-config gradient chunk).  Run it
under rocprofv3 --kernel-trace --stats for the kernel's own duration; prints the per-call wall time (layer-0 kernel
plus the layer-0 deep_hidden_kernel re-stride).  G2048_LIB=<path> loads an A/B build.

    python tools/bench_l0.py [--boards N] [--calls K]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=307200)
    ap.add_argument("--calls", type=int, default=50)
    a = ap.parse_args()
    if os.environ.get("G2048_LIB"):
        from rl2048_amd import _lib as _L0

        _L0.use_library_for_tools(os.environ["G2048_LIB"])
    import numpy as np
    import torch

    from rl2048_amd import _lib as L

    dev = torch.device("cuda:0")
    lib = L.lib()
    rng = np.random.default_rng(0)
    hidden = [256, 128, 64]
    sizes = [272] + hidden + [4]
    W = [torch.from_numpy((rng.standard_normal((i, o)) * np.sqrt(2.0 / i)).astype(np.float32)).to(dev)
         for i, o in zip(sizes[:-1], sizes[1:])]
    B = [torch.from_numpy((rng.standard_normal(o) * 0.1).astype(np.float32)).to(dev) for o in sizes[1:]]
    harr = (ctypes.c_int32 * 3)(*hidden)
    size = int(lib.g2048_deep_packed_size(L.OBS_ONEHOT, 3, harr))
    packed = torch.empty(size, dtype=torch.float32, device=dev)
    wp = (ctypes.c_void_p * 4)(*[w.data_ptr() for w in W])
    bp = (ctypes.c_void_p * 4)(*[b.data_ptr() for b in B])
    st = L.stream_handle(dev)
    L.check(lib.g2048_deep_pack(wp, bp, L.OBS_ONEHOT, 3, harr, 4, L.ptr(packed), size, st))
    e = rng.integers(0, 16, size=(a.boards, 16))
    e[rng.random((a.boards, 16)) < 0.35] = 0
    b = torch.from_numpy(((e.astype(np.uint64) << (4 * np.arange(16, dtype=np.uint64))).sum(1)).view(np.int64)).to(dev)
    out = torch.empty(a.boards, 256, dtype=torch.float32, device=dev)

    def call():
        L.check(lib.g2048_deep_hidden(L.ptr(packed), 3, harr, L.ACT_RELU, L.OBS_ONEHOT, 1.0, L.ptr(b), a.boards, 0,
                                      L.ptr(out), 256, st))

    for _ in range(5):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.calls):
        call()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.calls
    print(json.dumps({"boards": a.boards, "calls": a.calls, "us_per_call": round(dt * 1e6, 1),
                      "lib": os.path.basename(os.environ.get("G2048_LIB", "shipped"))}), flush=True)


if __name__ == "__main__":
    main()
