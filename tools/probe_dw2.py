"""TOOL: structured-input probe of g2048_dw2 (which columns / rows land where)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rl2048_amd import _lib as L  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
L.ensure_device(dev)
lib = L.lib()


def run(a1t, d2t, h1, h2, ncols, cpp):
    nparts = -(-ncols // cpp)
    part = torch.full((nparts, a1t.shape[0], d2t.shape[0]), float("nan"), device=dev)
    L.check(lib.g2048_dw2(L.ptr(a1t), L.ptr(d2t), h1, h2, a1t.shape[1], 0, ncols, cpp, L.ptr(part), nparts,
                          L.stream_handle(dev)))
    torch.cuda.synchronize()
    return part


for H in (32, 256):
    ld = 64
    for kk in (0, 5, 17, 40):
        a = torch.zeros(H + 1, ld, device=dev)
        a[:H, kk] = torch.arange(H, device=dev, dtype=torch.float32) + 1
        d = torch.zeros(H, ld, device=dev)
        d[:, kk] = (torch.arange(H, device=dev, dtype=torch.float32) + 1) * 1000
        p = run(a, d, H, H, 64, 2048)[0]
        ref = a[:H].double() @ d.double().t()
        err = (p[:H].double() - ref).abs()
        nz = (p[:H] != 0).nonzero()
        print(f"H={H} k={kk}: max err {float(err.max()):.3g}; nonzeros {nz.shape[0]} (want {H*H}); "
              f"p[0,0]={float(p[0,0])} want {float(ref[0,0])}; p[1,2]={float(p[1,2])} want {float(ref[1,2])}; "
              f"db2[0..3]={p[H, :4].tolist()} want {d[:4, kk].tolist()}", flush=True)
    # random
    a = torch.randn(H + 1, 4096, device=dev)
    d = torch.randn(H, 4096, device=dev)
    p = run(a, d, H, H, 4096, 2048)
    ref = a[:H, :2048].double() @ d[:, :2048].double().t()
    print(f"H={H} random: rel err slab0 {float((p[0, :H].double() - ref).abs().max() / ref.abs().max()):.3g}", flush=True)
