"""TOOL: the layer-2 weight-gradient GEMM of the fused update (a1t [257, m] x d2t [256, m]^T, m = 2^20 columns) --
hipBLASLt strided-batched split-K over P column blocks in both operand orders, and a single addmm -- timed on one
MI355X (ms per chunk, TFLOP/s).  Picks the variant agent._fused_grad uses."""
import json
import sys
import time

import torch

dev = torch.device("cuda", 0)
m = 1 << 20
H1, H2 = 257, 256
a1t = torch.randn(H1, m, device=dev)
d2t = torch.randn(H2, m, device=dev)
flop = 2.0 * H1 * H2 * m


def bench(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


res = {}
if "--sample-major" in sys.argv:   # a1 / d2 stored [sample][unit] (the kernel's column stores as 16-B runs)
    a1s = torch.randn(m, H1, device=dev)
    d2s = torch.randn(m, H2, device=dev)
    for P in (64, 128, 256):
        q = m // P
        res[f"unit_major_P{P}"] = bench(lambda: torch.bmm(a1t.view(H1, P, q).transpose(0, 1),
                                                          d2t.view(H2, P, q).permute(1, 2, 0)).sum(0))
        res[f"sample_major_P{P}"] = bench(lambda: torch.bmm(a1s.view(P, q, H1).transpose(1, 2),
                                                            d2s.view(P, q, H2)).sum(0))
    for k, v in sorted(res.items(), key=lambda kv: kv[1]):
        print(json.dumps({"variant": k, "ms": round(v, 3), "tflops": round(flop / v / 1e9, 1)}))
    sys.exit(0)
if "--rows" in sys.argv:      # M = 256 (no ones row) against 257, and the db2 row as a separate column sum
    a1s = a1t[:256]
    for P in (64, 128, 256):
        q = m // P
        res[f"bmm_M257_P{P}"] = bench(lambda: torch.bmm(a1t.view(H1, P, q).transpose(0, 1),
                                                        d2t.view(H2, P, q).permute(1, 2, 0)).sum(0))
        res[f"bmm_M256_P{P}"] = bench(lambda: torch.bmm(a1s.reshape(256, P, q).transpose(0, 1),
                                                        d2t.view(H2, P, q).permute(1, 2, 0)).sum(0))
    res["d2_rowsum"] = bench(lambda: d2t.sum(1))
    for k, v in sorted(res.items(), key=lambda kv: kv[1]):
        print(json.dumps({"variant": k, "ms": round(v, 3)}))
    sys.exit(0)
for P in (8, 16, 32, 64, 128, 256):
    q = m // P
    res[f"bmm_a1d2_P{P}"] = bench(lambda: torch.bmm(a1t.view(H1, P, q).transpose(0, 1),
                                                    d2t.view(H2, P, q).permute(1, 2, 0)).sum(0))
    res[f"bmm_d2a1_P{P}"] = bench(lambda: torch.bmm(d2t.view(H2, P, q).transpose(0, 1),
                                                    a1t.view(H1, P, q).permute(1, 2, 0)).sum(0))
res["addmm"] = bench(lambda: a1t @ d2t.t())
for k, v in sorted(res.items(), key=lambda kv: kv[1]):
    print(json.dumps({"variant": k, "ms": round(v, 3), "tflops": round(flop / v / 1e9, 1)}))
