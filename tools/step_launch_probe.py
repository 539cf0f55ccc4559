"""Where the driver command's per-step time goes above the kernel's own duration (bench.py headline leg).

Interleaved, on one env of the bench's shape (1,048,576 boards, PCG64, log2 obs, packed mask):
  eager    -- bench.py's timed region as it is: ev0, K x step_into from Python, ev1
  queued   -- the same K launches queued behind a GPU sleep so the host is ahead of the GPU when ev0 runs
              (the GPU-side back-to-back time of K launches)
  graph    -- the K step_into calls captured once in a HIP graph (torch.cuda.CUDAGraph), replayed
  freshS   -- (S untimed steps; S = 5 when omitted)  bench.py's exact sequence: a new env of synthetic random-state boards, W = 5 untimed steps, then the
              timed K (the driver's headline: the first steps after the synthetic start, 1-3 % of lanes resetting)
  resetS / sparseS -- as freshS from env.reset's two-tile boards / from synthetic boards with cells 1-3 of
              each row cleared
G2048_LIB=<path> loads an A/B build.    zfreshS / mfreshS -- as freshS with obs_log2_scale 0 (zero obs values) / max_tile_seen starting at 2^12
  reloadS  -- (round 5: buffer age vs board state) the long-running env (hundreds of launches on its buffers) given
              the synthetic random-state boards and lane state again, S untimed steps, then the timed K
  evolvedS -- a new env (freshly initialised buffers) given the long-running env's evolved boards and lane state,
              S untimed steps, then the timed K
  noresetS -- as freshS with auto-reset off (finished lanes go inactive: no reset pass, no reset writes)
  truncN   -- reset rate at will: the long-running env's evolved boards with max_steps = N and lane step counts spread
              uniformly over 0..N-1, so ~1/N of the lanes truncate and auto-reset every step (board state as steady as
              `evolved`); 60 untimed steps, then the timed K
  pollM    -- as trunc1000, then M x 64 MiB of unrelated writes (a scratch fill) just before the timed K: evicts the
              step kernel's working set from the 256 MB Infinity Cache (MALL) without touching the env
  bigS     -- as freshS with the synthetic boards built in one whole-batch pass (~10 temporaries of 128 MiB each, the
              pre-round-5 bench.synthetic_boards) instead of 65,536-board chunks
Also the host cost of one step_into call.  Prints one JSON line per repetition.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--modes", default="eager,queued,graph,fresh")
    a = ap.parse_args()
    if os.environ.get("G2048_LIB"):   # an A/B build (tools/build_variants.py)
        from rl2048_amd import _lib as _L0

        _L0.use_library_for_tools(os.environ["G2048_LIB"])
    import torch

    import bench

    dev = torch.device("cuda:0")
    args = argparse.Namespace(obs="log2", rng="pcg64", gpus=1, no_auto_reset=False)
    B, K = a.boards, a.steps
    env = bench.make_env(torch, args, B, 0, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    actions = torch.randint(0, 4, (K, B), dtype=torch.uint8, device=dev, generator=g)
    for _ in range(400):   # chip warm-up
        env.step_into(actions[0])
    torch.cuda.synchronize()

    # host cost of one call (GPU kept busy by a long sleep so nothing blocks)
    torch.cuda._sleep(400_000_000)
    t0 = time.perf_counter()
    for k in range(K):
        env.step_into(actions[k])
    host_us = (time.perf_counter() - t0) / K * 1e6
    torch.cuda.synchronize()

    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        env.step_into(actions[0])
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(gr):
        for k in range(K):
            env.step_into(actions[k])
    torch.cuda.synchronize()

    def timed(mode):
        if mode.startswith("reload") or mode.startswith("evolved"):
            skip = int(mode.lstrip("reloadevolved") or 5)
            if mode.startswith("reload"):
                fenv = env
                fenv.board.copy_(bench.synthetic_boards(torch, B, 0, dev))
                fenv.set_lane_state(step_count=0, max_tile_exp=2, active=True)
            else:
                fenv = bench.make_env(torch, args, B, 0, dev)
                fenv.board.copy_(env.board)
                fenv.state.copy_(env.state)
            for k in range(skip):
                fenv.step_into(actions[k % K])
            torch.cuda.synchronize()
        elif mode.startswith("trunc") or mode.startswith("poll"):
            N = int(mode[5:]) if mode.startswith("trunc") else 1000
            fenv = bench.make_env(torch, args, B, 0, dev)
            fenv.board.copy_(env.board)
            fenv.state.copy_(env.state)
            fenv._cfg.max_steps = N
            fenv.set_lane_state(step_count=torch.randint(0, N, (B,), device=dev, generator=g), active=True)
            for k in range(60):
                fenv.step_into(actions[k % K])
            if mode.startswith("poll"):
                scratch = torch.empty(int(mode[4:]) << 24, dtype=torch.float32, device=dev)
                scratch.fill_(1.0)
                del scratch
            torch.cuda.synchronize()
        elif mode.startswith("noreset"):
            skip = int(mode.lstrip("noreset") or 5)
            fenv = bench.make_env(torch, argparse.Namespace(obs="log2", rng="pcg64", gpus=1, no_auto_reset=True), B, 0,
                                  dev)
            for k in range(skip):
                fenv.step_into(actions[k % K])
            torch.cuda.synchronize()
        elif mode[0] in "frsmzb":
            skip = int(mode.lstrip("freshsparetmzbig") or 5)
            fenv = bench.make_env(torch, args, B, 0, dev)
            if mode.startswith("big"):
                fenv.board.copy_(bench.synthetic_boards(torch, B, 0, dev, chunk=B))
                fenv.set_lane_state(step_count=0, max_tile_exp=2, active=True)
            if mode.startswith("zfresh"):      # obs values all 0.0 (same stores)
                fenv._cfg.obs_log2_scale = 0.0
            elif mode.startswith("mfresh"):    # max_tile_seen starts at 2^12 instead of 4
                fenv.set_lane_state(max_tile_exp=12)
            if mode.startswith("reset"):     # the boards env.reset dealt (two tiles each)
                fenv.reset(seed=torch.arange(B, dtype=torch.int64, device=dev) + 1_000_003)
            elif mode.startswith("sparse"):  # synthetic boards with 3 of 4 cells cleared
                keep = torch.tensor(0x000F000F000F000F, dtype=torch.int64, device=dev)
                fenv.board.bitwise_and_(keep)
                fenv.set_lane_state(step_count=0, max_tile_exp=2, active=True)
            for k in range(skip):
                fenv.step_into(actions[k % K])
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if mode == "queued":
            torch.cuda._sleep(50_000_000)
        t0 = time.perf_counter()
        e0.record()
        if mode == "graph":
            gr.replay()
        elif mode[0] in "frsmzentpb":
            for k in range(K):
                fenv.step_into(actions[k])
        else:
            for k in range(K):
                env.step_into(actions[k])
        e1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return e0.elapsed_time(e1) / K * 1e3, wall / K * 1e6

    for rep in range(a.reps):
        out = {"rep": rep, "host_us_per_call": round(host_us, 2)}
        for mode in a.modes.split(","):
            ev, wall = timed(mode)
            out[mode] = {"event_us": round(ev, 2), "wall_us": round(wall, 2)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
