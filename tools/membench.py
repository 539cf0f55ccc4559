"""TOOL: calibrate the achievable bandwidth of g2048_step's access pattern (tools/membench.hip) on the GPU box.

    python tools/membench.py            # prints one JSON line per variant
"""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmembench.so")


class Bufs(ctypes.Structure):
    _fields_ = [(f, ctypes.c_void_p) for f in ("board", "status", "action", "sc", "mt", "score", "rs", "inc", "buf",
                                               "reward", "flags", "mask", "obs")] + [("n", ctypes.c_uint32)]


def main():
    if not os.path.exists(SO):
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO,
                        os.path.join(HERE, "membench.hip")], check=True)
    L = ctypes.CDLL(SO)
    dev = torch.device("cuda", 0)
    n = 1 << 20
    z = lambda dt, *s: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
    t = dict(board=z(torch.int64, n), status=z(torch.uint8, n), action=z(torch.uint8, n), sc=z(torch.int32, n),
             mt=z(torch.uint8, n), score=z(torch.int32, n), rs=z(torch.int64, 2 * n), inc=z(torch.int64, 2 * n),
             buf=z(torch.int64, n), reward=z(torch.float32, n), flags=z(torch.uint8, n), mask=z(torch.int32, n),
             obs=z(torch.float32, n, 16))
    b = Bufs(*[t[k].data_ptr() for k in ("board", "status", "action", "sc", "mt", "score", "rs", "inc", "buf",
                                        "reward", "flags", "mask", "obs")], n)
    stream = torch.cuda.current_stream().cuda_stream
    bytes_alg = 173 * n

    def timeit(fn, reps=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps * 1e3  # us

    out = []
    if "--stream-sweep" in sys.argv:
        # plain streams at the step kernel's traffic per launch (166.8 MB at 1M boards, x8 at 8M), back to back
        # like the bench: a 1:1 copy and a 1:2 read:write stream (the step's byte mix), grid 4096 x 256
        for boards in (1 << 20, 1 << 21, 1 << 22, 1 << 23):
            total = 159 * boards
            nb = (total // 2) & ~15
            src, dst = z(torch.uint8, nb), z(torch.uint8, nb)
            us = timeit(lambda: L.mb_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                          ctypes.c_size_t(nb // 16), 4096, ctypes.c_void_p(stream)))
            out.append(dict(variant=f"float4 copy, {boards} boards' traffic ({2 * nb >> 20} MiB)", us=us,
                            GBs=2 * nb / us / 1e3))
            del src, dst
            nr = (total // 3) & ~15
            src, dst = z(torch.uint8, nr), z(torch.uint8, 2 * nr)
            us = timeit(lambda: L.mb_rw12(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                          ctypes.c_size_t(nr // 16), 4096, ctypes.c_void_p(stream)))
            out.append(dict(variant=f"float4 read 1 : write 2, {boards} boards' traffic ({3 * nr >> 20} MiB)", us=us,
                            GBs=3 * nr / us / 1e3))
            del src, dst
        for o in out:
            print(json.dumps(o), flush=True)
        return
    for work in (0, 16, 32, 64):
        for grid, block, lds in ((256, 1024, 160 * 1024), (256, 1024, 0), (1024, 1024, 0), (4096, 256, 0)):
            us = timeit(lambda: L.mb_twin(ctypes.byref(b), 1, grid, block, work, lds, ctypes.c_void_p(stream)))
            out.append(dict(variant=f"twin work={work} grid={grid}x{block} lds={lds}", us=us, GBs=bytes_alg / us / 1e3))
    for mb in (181,):
        nb = mb * (1 << 20)
        src, dst = z(torch.uint8, nb), z(torch.uint8, nb)
        us = timeit(lambda: L.mb_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                      ctypes.c_size_t(nb // 16), 4096, ctypes.c_void_p(stream)))
        out.append(dict(variant=f"float4 copy {mb} MiB", us=us, GBs=2 * nb / us / 1e3))
        del src, dst
    nb = 1088 * n                                     # the one-hot obs of one 1M-board step
    dst = z(torch.uint8, nb)
    for nt in (0, 1):
        for grid in (1024, 4096, 16384):
            us = timeit(lambda: L.mb_fill(ctypes.c_void_p(dst.data_ptr()), ctypes.c_size_t(nb // 16), grid, nt,
                                          ctypes.c_void_p(stream)))
            out.append(dict(variant=f"float4 fill {nb >> 20} MiB nt={nt} grid={grid}", us=us, GBs=nb / us / 1e3))
    del dst
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    sys.exit(main())
