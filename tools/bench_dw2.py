"""TOOL: g2048_dw2 alone at the update's chunk size (2^20 columns, 256 x 256 net): time per call by HIP events,
achieved bytes/s on the 2,052 B/column it reads and the fp32-equivalent TFLOP/s; accuracy vs fp64 on one slab.

    python tools/bench_dw2.py [--lib tools/libg2048_x.so ...] [--cols N]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", nargs="*", default=[None])
    ap.add_argument("--cols", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--parts", type=int, nargs="*", default=[256])
    args = ap.parse_args()
    import torch

    from rl2048_amd import _lib as L

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = args.cols
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    a1t = torch.relu(torch.randn(256, n, device=dev, generator=g))   # (random data: the block layout does not matter)
    d2t = torch.randn(256, n, device=dev, generator=g) * 1e-3
    for lib_path in args.lib:
        if lib_path:
            L._lib = None
            L.LIB_PATH = os.path.abspath(lib_path)
        lib = L.lib()
        L._inited_devices.clear()
        L.ensure_device(dev)
        for P in args.parts:
            cpp = max(2048, -(-n // (16 * P)) * 16)
            nparts = -(-n // cpp)
            part = torch.empty(nparts, 257, 256, device=dev)
            s = L.stream_handle(dev)

            def call():
                L.check(lib.g2048_dw2(L.ptr(a1t), L.ptr(d2t), 256, 256, n, 0, n, cpp, L.ptr(part), nparts, s))

            for _ in range(3):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / args.reps * 1e3
            ub = lambda X: X.reshape(n // 16, 256, 16).permute(1, 0, 2).reshape(256, n)  # noqa: E731 (block layout)
            A, D = ub(a1t)[:, :cpp].double(), ub(d2t)[:, :cpp].double()
            ref, bound = A @ D.t(), A.abs() @ D.abs().t()
            err = float(((part[0, :256].double() - ref).abs() / bound.clamp_min(1e-30)).max())
            print(json.dumps({"lib": lib_path or "shipped", "cols": n, "parts": nparts, "us": round(us, 1),
                              "GBps": round(n * 2052 / us / 1e3, 1),
                              "tflops_fp32_equiv": round(2 * 256 * 256 * n / us / 1e6, 1),
                              "max_err_over_sum_abs": err}), flush=True)


if __name__ == "__main__":
    main()
