#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: env steps/s (whole node) + achieved HBM GB/s on a batch of 1,048,576 4x4 boards
per GPU (configs[2]'s batch; the per-GPU shard of configs[4]).

One "step" = one launch of the fused HIP env step (g2048_step) over the whole per-GPU board batch: slide/merge
(LDS row table) + numpy-PCG64 spawn + reward (fp64) + done/truncation + auto-reset + action mask + log2 obs.
Inputs are synthetic and resident in HBM before timing: random-state boards (each cell empty w.p. 6/16, else an
exponent uniform in 1..12, seed 0x2048), actions uniform over 0..3 (seed 1; invalid no-change moves included),
per-lane seeds seed0 + global lane for auto-reset.  Weak scaling: every GPU owns B boards (lanes
[rank*B, (rank+1)*B)), no collective on the data path.

    python bench.py [--gpus N --steps K --warmup W --boards B --rng pcg64|philox --obs log2|onehot|raw|none]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Extras: `roofline` of the step kernel (SURVEY.md section 8(d)'s algorithmic bytes per
board-step / HIP-event kernel time vs 8 TB/s; the build's layout bytes beside them; `traffic` = HBM bytes per launch
from rocprofv3 FETCH_SIZE/WRITE_SIZE passes when rocprofv3 is present), `cpu_baseline` (the reference's CPU step
loop restated in Python -- oracle/pyref.py, pinned to the reference -- one process per host core, a bounded sample;
the C port beside it), `configs4_onehot_philox` (configs[4]'s per-GPU shard, every rank: the same step leg in Philox
mode writing one-hot obs + int8 mask, 1,122 B / board-step, with its own roofline and PMC traffic),
`train_iteration_dp` (configs[3]'s training iteration per GPU shard, every rank, with the gradient all-reduce inside
the timed region) and, at N=1, `policy_rollout` (env steps/s with the [256,256] ReLU policy MLP + on-device sampling
in the loop; the configs[1] / configs[2] training iterations; the reference runner's documented config).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env steps/sec (whole node) + achieved HBM GB/s, batch=1M 4x4 boards"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
POLICY_FLOP_PER_BOARD = 2 * (16 * 256 + 256 * 256 + 256 * 4)  # 141,312: the runner-default MLP forward
# update per sample: forward + weight / input gradients of layers 2 and 3, weight gradient of layer 1
UPDATE_FLOP_PER_SAMPLE = POLICY_FLOP_PER_BOARD + 2 * (256 * 256 * 2 + 256 * 4 * 2 + 16 * 256)

# ALGORITHMIC bytes per board-step -- SURVEY.md section 8(d)'s table, the roofline's numerator: core (board
# 8/8, action 1, reward 4, flags 1) 22 B + env lane state (step count u16, max tile exp u8, pad) 8 B = 30 B (Philox,
# counter from the step), + the numpy-PCG64-compatible RNG (state 16 r/w, inc 16 r, uinteger 4 + has 1 r/w) = 88 B;
# obs: + 64 B log2 / raw fp32, + 1092 B one-hot fp32 + int8 mask.
SURVEY_RNG_BYTES = {"pcg64": 88, "philox": 30}
SURVEY_OBS_BYTES = {"none": 0, "raw": 64, "log2": 64, "onehot": 1092}
# LAYOUT bytes: what this build's structure-of-arrays lane layout actually moves per board-step (reads / writes):
#   board 8/8, action 1/-, lane state word (step count, max tile, active, PCG64 buffer flag) 4/4, reward -/4,
#   flags -/1, action mask -/1 (packed: g2048_step_out.mask_bits);  PCG64: rng_state 16/16, rng_inc 16/-,
#   rng_uint 4/4;  Philox: lane seed 8/-;  obs: log2/raw -/64, onehot -/1088
CORE_R, CORE_W = 8 + 1 + 4, 8 + 4 + 4 + 1 + 1
RNG_BYTES = {"pcg64": (36, 20), "philox": (8, 0)}
OBS_BYTES = {"none": 0, "raw": 64, "log2": 64, "onehot": 1088}


def survey_bytes_per_step(rng: str, obs: str) -> int:
    return SURVEY_RNG_BYTES[rng] + SURVEY_OBS_BYTES[obs]


def bytes_per_step(rng: str, obs: str) -> tuple[int, int]:
    """Layout bytes (reads, writes) per board-step."""
    r = CORE_R + RNG_BYTES[rng][0]
    w = CORE_W + RNG_BYTES[rng][1] + OBS_BYTES[obs] + (3 if obs == "onehot" else 0)   # one-hot: int8[4] mask
    return r, w


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--boards", type=int, default=1 << 20, help="boards per GPU")
    ap.add_argument("--rng", default="pcg64", choices=["pcg64", "philox"])
    ap.add_argument("--obs", default="log2", choices=["log2", "onehot", "raw", "none"])
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--train-episodes", type=int, default=1 << 19,
                    help="episodes per GPU of the data-parallel training-iteration leg (configs[3]'s shard)")
    ap.add_argument("--no-train", action="store_true", help="skip the data-parallel training-iteration leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default="auto", choices=["auto", "off"])
    ap.add_argument("--no-policy", action="store_true")
    ap.add_argument("--no-configs4", action="store_true",
                    help="skip configs[4]'s Philox + one-hot obs step leg (1,122 B / board-step)")
    ap.add_argument("--no-refconfig", action="store_true",
                    help="skip the reference runner-config training iterations (runner.py:10-47)")
    ap.add_argument("--no-auto-reset", action="store_true", help="diagnostic: finished lanes go inactive")
    ap.add_argument("--chip-warmup-seconds", type=float, default=0.5,
                    help="untimed step launches on a separate env of the same shape before the headline leg")
    ap.add_argument("--trace-steps", type=int, default=0,
                    help="diagnostic: print per-launch kernel us and reset fraction for the first N steps, then exit")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    # tools/ A/B and diag scripts only: measure another build of libg2048 (never the default)
    ap.add_argument("--lib", default=None, help=argparse.SUPPRESS)
    return ap.parse_args()


# ---------------------------------------------------------------------------------------------- inputs
def synthetic_boards(torch, B: int, lane_offset: int, device, seed: int = 0x2048, chunk: int = 1 << 16):
    """Random-state boards: cell empty w.p. 6/16, else exponent uniform over 1..12.
    A counter hash of (global lane, cell) so shards of an N-GPU run are slices of the 1-GPU global batch.
    Built in chunks of 65,536 boards: the whole-batch form made ~10 temporaries of 128 MiB (16 cells x 1M int64)
    whose traffic evicted the step kernel's working set from the 256 MB Infinity Cache (MALL) right before the timed
    launches, which then ran ~2.5 us slower until the working set was back (tools/step_launch_probe.py, round 5)."""
    M = 0x7FFFFFFFFFFFFFFF
    out = torch.empty(B, dtype=torch.int64, device=device)
    shifts = torch.arange(0, 64, 4, dtype=torch.int64, device=device)
    for c0 in range(0, B, chunk):
        n = min(chunk, B - c0)
        idx = (torch.arange(n * 16, dtype=torch.int64, device=device) + (lane_offset + c0) * 16) ^ seed
        h = idx * -0x61C8864680B583EB - 0x61C8864680B583EB  # splitmix64 (0x9E3779B97F4A7C15 as int64), wraps
        h = (h ^ ((h >> 30) & (M >> 29))) * -0x40A7B892E31B1A47
        h = (h ^ ((h >> 27) & (M >> 26))) * -0x6B2FB644ECCEEE15
        h = h ^ ((h >> 31) & (M >> 30))
        u = h & 0xFFFF
        exps = torch.where((u & 15) < 6, torch.zeros_like(u), 1 + ((u >> 4) % 12)).view(n, 16)
        out[c0:c0 + n] = (exps << shifts).sum(dim=1)
    return out


def make_env(torch, args, B, lane_offset, device, rng: str | None = None, obs: str | None = None):
    """The bench env (rng / obs default to the headline's): max_steps 1024, auto-reset, per-lane seeds
    seed0 + global lane, synthetic random-state boards.  The action mask is packed (bit a = action a) except with
    one-hot obs, where it is the obs dict's int8[4] (configs[4]: SURVEY.md section 8(d)'s 1,092 B = obs + mask)."""
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    rng = rng or args.rng
    obs = obs or args.obs
    packed_mask = obs != "onehot"
    cfg = Game2048EnvConfig(obs_mode="log2" if obs == "none" else obs, obs_log2_scale=0.0625,
                            reward_mode="log2", base_reward_scale=0.5, max_steps=1024)
    env = VecGame2048Env(B, cfg, device=device, rng=rng, auto_reset=not args.no_auto_reset,
                         reset_stride=B * max(args.gpus, 1), lane_offset=lane_offset, track_score=False,
                         packed_mask=packed_mask)
    if obs == "none":
        env._out.obs = None
    # per-lane episode seeds (PCG64: default_rng(seed) streams) via g2048_reset, then the random-state boards
    env.reset(seed=torch.arange(B, dtype=torch.int64, device=device) + (1_000_003 + lane_offset))
    env.board.copy_(synthetic_boards(torch, B, lane_offset, device))
    env.set_lane_state(step_count=0, max_tile_exp=2, active=True)
    return env


# ---------------------------------------------------------------------------------------------- PMC traffic
def pmc_traffic(args, rng: str | None = None, obs: str | None = None) -> dict | None:
    """Run this benchmark's step leg twice under rocprofv3 (separate FETCH_SIZE and WRITE_SIZE passes, kernel-trace
    only, per MI355X_MICROARCH.md 'HBM') and return HBM bytes per step-kernel launch (rng / obs: the leg's mode,
    default the headline's).  FETCH_SIZE is doubled: on gfx950 it reports half the bytes of coalesced streaming
    reads."""
    rng = rng or args.rng
    obs = obs or args.obs
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None
    vals = {}
    base = os.path.join(ROOT, "gpurun_out", "pmc") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else None
    if base:
        os.makedirs(base, exist_ok=True)
    # the child is a single-process run on this rank's GPU even under torchrun: no rendezvous variables
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT") and not k.startswith("TORCHELASTIC_")}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        out = tempfile.mkdtemp(prefix=f"pmc_{rng}_{obs}_{counter}_", dir=base)
        cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", out, "-o", "pmc", "--", sys.executable,
               os.path.abspath(__file__), "--pmc-child", "--steps", "10", "--warmup", "3", "--boards",
               str(args.boards), "--rng", rng, "--obs", obs]
        try:
            subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           env=env)
        except Exception:  # noqa: BLE001 -- traffic is optional; report null on any profiler failure
            return None
        rows = []
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            import csv

            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if "step_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                        rows.append(float(row["Counter_Value"]))
        if not rows:
            return None
        vals[counter] = sum(rows[1:] if len(rows) > 1 else rows) / max(len(rows) - 1, 1)
    fetch_b = vals["FETCH_SIZE"] * 1024.0 * 2.0
    write_b = vals["WRITE_SIZE"] * 1024.0
    return {"fetch_bytes": fetch_b, "write_bytes": write_b, "bytes": fetch_b + write_b}


# ---------------------------------------------------------------------------------------------- CPU baseline
def host_cores() -> dict:
    """Cores this process may use: the affinity set, capped by a cgroup CPU quota when there is one (the GPU box
    grants a share of a larger machine; os.cpu_count() reports the whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    return {"cores": max(1, min(aff, int(quota))) if quota else aff, "affinity_cores": aff, "cgroup_cpu_quota": quota}


# oracle/pyref.py's single-core speed relative to the real src/env.py on the same workload, measured in the build
# container where the reference exists (tools/pyref_ratio.py -> profiles/round2/pyref_ratio.txt)
PYREF_OVER_REFERENCE = 1.442


def cpu_baseline(args, seconds: float) -> dict:
    """The reference's CPU step loop on this box's host cores: oracle/pyref.py (the Python + NumPy restatement of
    src/game2048.py + src/env.py, pinned bit for bit to the reference's outputs) as one process per core, each
    stepping its own boards (obs + action mask every step, auto-reset), for a bounded `seconds`.  Beside it the
    C port (oracle/g2048_oracle.c, OpenMP over the same cores)."""
    from oracle import oracle as O
    from oracle import pyref

    hc = host_cores()
    cores = hc["cores"]
    cfg = dict(obs_mode="log2" if args.obs == "none" else args.obs, obs_log2_scale=0.0625, reward_mode="log2",
               base_reward_scale=0.5, max_steps=1024)
    steps, dt = pyref.bench(cores, seconds, cfg)
    out = {"value": steps / dt, "unit": "env steps/s", "cores": cores, "kind": "port",
           "sample": f"oracle/pyref.py (Python + NumPy restatement of src/game2048.py + src/env.py step loop, "
                     f"{args.obs} obs + action mask, numpy PCG64 spawn), {cores} processes x 64 boards, "
                     f"{steps} env steps in {dt:.1f} s",
           "reference_equivalent": steps / dt / PYREF_OVER_REFERENCE,
           "pyref_over_reference_single_core": PYREF_OVER_REFERENCE,
           "affinity_cores": hc["affinity_cores"], "cgroup_cpu_quota": hc["cgroup_cpu_quota"]}
    os.environ["OMP_NUM_THREADS"] = str(cores)
    boards = 64 * cores
    t0 = time.perf_counter()
    csteps, _ = O.bench_env_steps(boards, 32, **cfg)
    cdt = time.perf_counter() - t0
    rounds = max(32, int(32 * min(seconds, 5.0) / max(cdt, 1e-6)))
    t0 = time.perf_counter()
    csteps, _ = O.bench_env_steps(boards, rounds, **cfg)
    cdt = time.perf_counter() - t0
    out["c_port"] = {"value": csteps / cdt, "unit": "env steps/s", "cores": cores,
                     "sample": f"oracle/g2048_oracle.c {boards} boards x {rounds} steps = {csteps} env steps in "
                               f"{cdt:.1f} s, OpenMP"}
    return out


# ---------------------------------------------------------------------------------------------- policy loop
def policy_rollout_rate(torch, B: int, device, steps: int = 20, warmup: int = 5, fused: bool = True) -> dict:
    """Env steps/s with the runner-default policy in the loop: MLP [256,256] ReLU HeNormal fp32 on log2 obs.
    fused: g2048_policy (fp32 MFMA forward + numpy-PCG64 choice straight from the bitboards) -> env step without
    the obs buffer; else hipBLASLt GEMMs (bias + ReLU epilogue) on the env's obs -> g2048_sample -> env step."""
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env
    from rl2048_amd import _lib as L
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    cfg = Game2048EnvConfig(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5)
    agent = ReinforceAgent(cfg, MLPConfig(hidden_sizes=[256, 256], activation="ReLU", init_distribution="HeNormal"),
                           ReinforceAgentConfig(), device=device)
    env = VecGame2048Env(B, cfg, device=device, auto_reset=True, track_score=False)
    env.reset(seed=7)
    lib = L.lib()
    st = torch.empty(2 * B, dtype=torch.int64, device=device)
    inc = torch.empty(2 * B, dtype=torch.int64, device=device)
    buf = torch.empty(B, dtype=torch.int64, device=device)
    seeds = torch.arange(B, dtype=torch.int64, device=device) + 99
    stream = L.stream_handle(device)
    L.check(lib.g2048_seed_pcg64(L.ptr(seeds), L.ptr(st), L.ptr(inc), L.ptr(buf), B, stream))
    acts = torch.empty(B, dtype=torch.uint8, device=device)
    spec = agent._fused_policy_spec()
    packed = agent._packed_policy(spec)

    def one():
        if fused:
            L.check(lib.g2048_policy(L.ptr(packed), spec[0], spec[1], spec[2], L.ptr(env.board), L.ptr(env.state),
                                     None, L.OBS_LOG2, 0.0625, 1, 0, L.RNG_PCG64, L.ptr(st), L.ptr(inc), L.ptr(buf), 0,
                                     None, None, None, L.ptr(acts), B, stream))
            env.step_into(acts, write_obs=False)
        else:
            logits = agent._policy_logits(env.obs)
            L.check(lib.g2048_sample(L.ptr(logits), L.ptr(env.mask), None, 0, 0, L.ptr(st), L.ptr(inc), L.ptr(buf),
                                     0, None, None, L.ptr(acts), B, stream))
            env.step_into(acts)

    with torch.no_grad():
        for _ in range(warmup):
            one()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            one()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    path = ("fused g2048_policy (fp32 MFMA) + step without obs" if fused else
            "hipBLASLt GEMMs + g2048_sample + step with obs")
    return {"value": steps * B / dt, "unit": "env steps/s", "boards": B, "steps": steps,
            "ms_per_step": dt / steps * 1e3, "model": "MLP 16-256-256-4 ReLU fp32 (runner.py defaults)",
            "path": path, "policy_tflops": steps * B * POLICY_FLOP_PER_BOARD / dt / 1e12}


def train_iteration_rate(torch, device, episodes: int = 65536, repeats: int = 2, critic: bool = False) -> dict:
    """One training iteration of configs[1] (65,536 parallel boards, REINFORCE + the runner-default MLP) or, with
    critic=True, of configs[2]'s actor-critic: the batched rollout of one episode per lane (g2048_rollout: fused
    policy + env step) and update_from_batch (fused actor / critic gradient kernels + the layer-2 GEMM, fp32),
    timed separately; the last of `repeats` iterations after one warm-up."""
    import numpy as np

    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    agent = ReinforceAgent(Game2048EnvConfig(), MLPConfig(hidden_sizes=[256, 256], activation="ReLU",
                                                          init_distribution="HeNormal"),
                           ReinforceAgentConfig(baseline_mode="batch", use_critic=critic), device=device)
    out = {}
    for rep in range(repeats + 1):
        base = 1000 + rep * episodes
        # the episode seeds as arrays (the runner's SeedStream.take_array form), made before the timed region
        es = np.arange(base, base + episodes, dtype=np.int64)
        ps = es + 7 * episodes
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batch = agent.rollout_batch(es, ps)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        agent.update_from_batch(batch)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        samples = int(batch.lengths.sum())
        out = {"episodes": episodes, "env_steps": samples, "longest_episode": batch.T, "rollout_s": t1 - t0,
               "update_s": t2 - t1, "iteration_s": t2 - t0, "env_steps_per_s": samples / (t2 - t0),
               "model": ("actor-critic (critic MSE on TD errors)" if critic else "REINFORCE") +
                        ", MLP 16-256-256-4 ReLU fp32, batch baseline (runner.py defaults)"}
        if not critic:
            out["update_tflops"] = samples * UPDATE_FLOP_PER_SAMPLE / (t2 - t1) / 1e12
        del batch
    return out


# The configuration runner.py documents in its header (/root/reference/runner.py:10-47): one-hot obs, a
# 16x17 -> 256 -> 128 -> 64 -> 4 ReLU MLP, actor-critic (MSE), Adam, batch baseline, no max_steps.
REFCONF_ENV = dict(obs_mode="onehot", obs_log2_scale=1.0, reward_mode="log2", base_reward_scale=1.0, bonus_mode="off",
                   bonus_scale=1.0, step_reward=0.0, endgame_penalty=0.0, use_action_mask=True,
                   invalid_action_penalty=-1.0, max_steps=None, empty_tile_reward=0.05, merge_reward=0.0)
REFCONF_MLP = dict(hidden_sizes=[256, 128, 64], activation="ReLU", init_distribution="HeNormal", last_init_normal=True)
REFCONF_AGENT = dict(gamma=0.99, learning_rate=0.01, baseline_mode="batch", model_seed=0, reward_rank_weights=None,
                     optimizer="adam", adam_beta1=0.9, adam_beta2=0.999, augmentation=False, use_critic=True,
                     critic_learning_rate=0.0005, critic_loss_type="mse", huber_delta=1.0)


def train_iteration_refconfig(torch, device, episodes: int, repeats: int = 1) -> dict:
    """One training iteration (rollout_batch of `episodes` episodes + update_from_batch) of the reference runner's
    documented config (REFCONF_*), timed per phase; the last of `repeats` timed iterations after one warm-up."""
    import numpy as np

    from rl2048_amd import Game2048EnvConfig
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    agent = ReinforceAgent(Game2048EnvConfig(**REFCONF_ENV), MLPConfig(**REFCONF_MLP),
                           ReinforceAgentConfig(**REFCONF_AGENT), device=device)
    out = {}
    for rep in range(repeats + 1):
        es = np.arange(3 + rep * episodes, 3 + (rep + 1) * episodes, dtype=np.int64)
        ps = es + 7 * episodes
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batch = agent.rollout_batch(es, ps)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        agent.update_from_batch(batch)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        samples = int(batch.lengths.sum())
        out = {"episodes": episodes, "env_steps": samples, "longest_episode": batch.T, "rollout_s": t1 - t0,
               "update_s": t2 - t1, "iteration_s": t2 - t0, "env_steps_per_s": samples / (t2 - t0),
               "paths": agent.last_paths(),
               "model": "actor-critic (MSE), one-hot obs, MLP 272-256-128-64-4 ReLU fp32, Adam, batch baseline, "
                        "max_steps None (runner.py:10-47)"}
        del batch
    return out


def train_iteration_dp(torch, device, episodes_per_rank: int, rank: int, world: int) -> dict:
    """configs[3]'s training iteration, weak-scaled: every rank plays `episodes_per_rank` episodes of the global
    batch (global episode g = rank * E + i; env seed 1000 + g, policy seed 2**40 + g, so N ranks play a partition
    of one global batch) with the runner-default net (16-256-256-4 ReLU, REINFORCE, batch baseline, SGD), then
    update_from_batch -- whose ONE gradient all-reduce (RCCL over xGMI on a multi-GPU node) is inside the timed
    region.  One warm-up iteration, one timed; time = max over ranks; env steps summed over ranks.  The gradient
    all-reduce alone is timed beside it (20 back-to-back dp.reduce_gradients_ of the same buffer)."""
    import numpy as np
    import torch.distributed as dist

    from rl2048_amd import Game2048EnvConfig, dp
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
    from rl2048_amd.mlp import MLPConfig

    agent = ReinforceAgent(Game2048EnvConfig(), MLPConfig(hidden_sizes=[256, 256], activation="ReLU",
                                                          init_distribution="HeNormal"),
                           ReinforceAgentConfig(baseline_mode="batch", gamma=0.99, learning_rate=1e-4), device=device)
    E = int(episodes_per_rank)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    res = {}
    for it in range(2):
        base = 1000 + it * E * world + rank * E
        es = np.arange(base, base + E, dtype=np.int64)
        ps = es + (1 << 40)
        barrier()
        t0 = time.perf_counter()
        batch = agent.rollout_batch(es, ps)
        batch.shard_sizes = (E,) * world
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        agent.update_from_batch(batch)
        barrier()
        t2 = time.perf_counter()
        res = {"rollout_s": t1 - t0, "update_s": t2 - t1, "iteration_s": t2 - t0,
               "env_steps": int(batch.lengths.sum())}
        del batch
    n_par = sum(p.numel() for p in agent.params["W"] + agent.params["b"])
    buf = [torch.zeros(n_par, dtype=torch.float32, device=device)]
    dp.reduce_gradients_(buf, E)
    barrier()
    t0 = time.perf_counter()
    for _ in range(20):
        dp.reduce_gradients_(buf, E)
    barrier()
    ar_ms = (time.perf_counter() - t0) / 20 * 1e3
    if world > 1:
        t = torch.tensor([res["rollout_s"], res["update_s"], res["iteration_s"], ar_ms], dtype=torch.float64,
                         device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        steps = torch.tensor([res["env_steps"]], dtype=torch.int64, device=device)
        dist.all_reduce(steps)
        res.update(rollout_s=float(t[0]), update_s=float(t[1]), iteration_s=float(t[2]), env_steps=int(steps[0]))
        ar_ms = float(t[3])
    backend = dist.get_backend() if dist.is_initialized() else "none (1 rank)"
    return {"episodes": E * world, "episodes_per_gpu": E, **res,
            "env_steps_per_s": res["env_steps"] / res["iteration_s"],
            "grad_allreduce_ms": ar_ms, "grad_allreduce_bytes": 4 * (n_par + 1), "backend": str(backend),
            "model": "REINFORCE, MLP 16-256-256-4 ReLU fp32, batch baseline (runner.py defaults)",
            "scaling": "weak"}


def time_steps(torch, env, actions, K: int, W: int, world: int):
    """W untimed launches, then EXACTLY K launches bracketed by a barrier + synchronize on both sides; HIP events on
    the launch stream around launches 2..K of the same K (kernel ms per launch = their span / (K - 1)): the GPU is
    idle when the first launch is enqueued, so an event recorded before it would also time the first launch's host
    enqueue latency (~12 us; profiles/round6/r7a/trace_window.json: events 29.3 us against a 28.6 us dispatch span).
    Returns (wall seconds, kernel ms per launch), each the MAX over ranks."""
    import torch.distributed as dist

    for k in range(W):
        env.step_into(actions[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if K == 1:
        ev0.record()
    for k in range(K):
        env.step_into(actions[W + k])
        if k == 0 and K > 1:
            ev0.record()   # fires when launch 1 ends; launches 2..K are queued back to back behind it
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / max(K - 1, 1)
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=env.board.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def onehot_philox_leg(torch, args, B, rank, world, device, actions, K, W, traffic) -> dict:
    """configs[4]'s per-GPU shard (BASELINE.json configs[4]: 8,388,608 boards = 8 x 1,048,576, fused step + one-hot
    obs + Philox per-lane RNG): the same synthetic boards, actions and timing as the headline leg, on
    g2048_step in Philox mode writing the one-hot obs (float32[272], src/env.py:131-150 / src/MLP.py:22-43) and
    the int8[4] action mask every step -- 1,122 algorithmic B per board-step, 92 %
    writes, a 1.1 GB launch: beyond the 256 MB MALL, so its HBM fraction is HBM's."""
    env = make_env(torch, args, B, rank * B, device, rng="philox", obs="onehot")
    elapsed, kern_ms = time_steps(torch, env, actions, K, W, world)
    del env
    torch.cuda.empty_cache()
    sb = survey_bytes_per_step("philox", "onehot")
    rb, wb = bytes_per_step("philox", "onehot")
    alg = sb * B
    achieved = alg / (kern_ms * 1e-3) / 1e9
    out = {"config": f"configs[4] per-GPU shard: {B:,} boards x {world} GPU(s), Philox spawn + one-hot obs + int8 mask",
           "boards_per_gpu": B, "rng": "philox", "obs": "onehot", "steps": K, "warmup": W,
           "value": K * B * world / elapsed, "unit": "env steps/s", "ms_per_step": elapsed / K * 1e3,
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "bytes_per_board_step": sb,
                        "algorithmic_bytes_per_launch": alg, "layout_bytes_per_board_step": rb + wb,
                        "traffic": traffic["bytes"] if traffic else None,
                        "traffic_over_algorithmic": traffic["bytes"] / alg if traffic else None,
                        "kernel_ms": kern_ms, "kernel": "step_kernel (g2048_step, Philox + one-hot obs)"}}
    if traffic:
        out["roofline"]["traffic_detail"] = traffic
    return out


# ---------------------------------------------------------------------------------------------- main
def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        args.gpus = world
    # The profiler passes and the CPU baseline run on rank 0 before this process touches the GPU, at every N: under
    # torchrun the other ranks meanwhile wait in init_process_group (well inside its timeout), so the CPU loop is
    # timed on the same box's host cores in the same run and the roofline carries PMC traffic at N > 1 too.
    traffic = traffic4 = None
    run_c4 = not args.pmc_child and not args.no_configs4
    if rank == 0 and not args.pmc_child and args.traffic == "auto":
        traffic = pmc_traffic(args)
        if run_c4:
            traffic4 = pmc_traffic(args, rng="philox", obs="onehot")
    cpu = None
    if rank == 0 and not args.pmc_child and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, args.cpu_baseline_seconds)

    import torch
    import torch.distributed as dist

    import rl2048_amd  # noqa: F401

    if args.lib:
        from rl2048_amd import _lib as L

        L.use_library_for_tools(args.lib)

    ndev = torch.cuda.device_count()
    device = torch.device("cuda", local_rank % max(ndev, 1))
    torch.cuda.set_device(device)
    if world > 1:
        # rank 0 ran the PMC passes and the CPU baseline before getting here (each bounded by its own timeout, a
        # few minutes at most): the rendezvous timeout is set well above that
        import datetime

        tmo = datetime.timedelta(minutes=30)
        if ndev >= world:
            dist.init_process_group("nccl", device_id=device, timeout=tmo)   # RCCL: one rank per GPU (production)
        else:
            dist.init_process_group("gloo", timeout=tmo)   # rehearsal of the N-rank path with ranks sharing a GPU
    B = args.boards
    # The extra legs (training iterations, policy rollouts) run first, so that the headline env-step leg below is
    # timed on a chip at its working clock: on a cold chip the first ~20 launches of the step kernel run 10-30 %
    # slower (profiles/round3/step_cold_trace.log), which a 20-step run would otherwise fold into the headline.
    train = None
    if not args.pmc_child and not args.no_train and args.train_episodes > 0:
        try:
            train = train_iteration_dp(torch, device, args.train_episodes, rank, world)
        except Exception as e:  # noqa: BLE001 -- an extra, never the headline
            train = {"error": repr(e)}
    policy = None
    if not args.pmc_child and rank == 0 and world == 1 and not args.no_policy:
        try:
            policy = policy_rollout_rate(torch, B, device)
            policy["gemm_path"] = policy_rollout_rate(torch, B, device, fused=False)
            policy["train_iteration_configs1"] = train_iteration_rate(torch, device)
            # configs[2]: 1,048,576 parallel boards, actor-critic (one warm-up, one timed iteration)
            policy["train_iteration_configs2"] = train_iteration_rate(torch, device, episodes=1 << 20, repeats=1,
                                                                      critic=True)
            if not args.no_refconfig:
                # each size: one warm-up iteration, then the timed one (tools/bench_refconfig.py reports the same)
                policy["train_iteration_reference_runner_config"] = {
                    "65536": train_iteration_refconfig(torch, device, 1 << 16),
                    "1048576": train_iteration_refconfig(torch, device, 1 << 20)}
        except Exception as e:  # noqa: BLE001 -- an extra, never the headline
            policy = {"error": repr(e)}
    torch.cuda.empty_cache()
    if world > 1:
        dist.barrier()
    K, W = args.steps, args.warmup
    g = torch.Generator(device=device)
    g.manual_seed(1 + rank)
    actions = torch.randint(0, 4, (K + W, B), dtype=torch.uint8, device=device, generator=g)
    configs4 = None
    if run_c4:   # every rank (weak scaling), before the headline leg: its K launches stay the run's last
        try:
            configs4 = onehot_philox_leg(torch, args, B, rank, world, device, actions, K, W, traffic4)
        except Exception as e:  # noqa: BLE001 -- an extra, never the headline
            configs4 = {"error": repr(e)}
    # Chip warm-up, explicit and independent of the extra legs above: untimed step launches for
    # --chip-warmup-seconds on a separate env of the same shape (on a cold chip the first ~20 launches of the step
    # kernel run 10-30 % slower, profiles/round3/step_cold_trace.log); the headline env below starts from the
    # synthetic random-state boards untouched.
    warm = {"launches": 0, "seconds": 0.0}
    if args.chip_warmup_seconds > 0:
        wenv = make_env(torch, args, B, rank * B, device)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.chip_warmup_seconds:
            for _ in range(32):
                wenv.step_into(actions[warm["launches"] % (K + W)])
                warm["launches"] += 1
            torch.cuda.synchronize()
        warm["seconds"] = time.perf_counter() - t0
        del wenv
    env = make_env(torch, args, B, rank * B, device)
    if args.trace_steps:
        from rl2048_amd import _lib as L

        for k in range(args.trace_steps):
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            env.step_into(actions[k % (K + W)])
            e_.record()
            torch.cuda.synchronize()
            rf = float(((env.flags & L.F_RESET) != 0).float().mean())
            act = float(env.active.float().mean())
            inv = float(((env.flags & L.F_INVALID) != 0).float().mean())
            tiles = float(((((env.board.unsqueeze(1) >> torch.arange(0, 64, 4, device=device)) & 15) != 0)
                           .float().sum(1)).mean())
            print(json.dumps({"step": k, "us": round(s_.elapsed_time(e_) * 1e3, 2), "reset_frac": round(rf, 5),
                              "active_frac": round(act, 4), "invalid_frac": round(inv, 4),
                              "tiles_per_board": round(tiles, 2)}), flush=True)
        return
    # timed region (the reported value): K launches, nothing else on the stream.  HIP events on the launch stream
    # bracket the same K launches: kernel_ms (the roofline's duration) is their average, back to back -- the last K
    # step_kernel dispatches of the run (tools/trace_window.py reads them back from a rocprofv3 kernel trace of this
    # command: profiles/round6/)
    elapsed, kern_ms = time_steps(torch, env, actions, K, W, world)
    if args.pmc_child:
        return
    del actions
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return
    rb, wb = bytes_per_step(args.rng, args.obs)
    sb = survey_bytes_per_step(args.rng, args.obs)
    alg_bytes = sb * B
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    layout_achieved = (rb + wb) * B / (kern_ms * 1e-3) / 1e9
    total_steps = K * B * world
    line = {
        "metric": METRIC, "value": total_steps / elapsed, "unit": "env steps/s", "n_gpus": world, "steps": K,
        "warmup": W, "ms_per_step": elapsed / K * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": f"g2048_step over {B:,} random-state boards per GPU (configs[2] batch): "
                               f"slide/merge + {args.rng} spawn + fp64 reward + done/trunc + auto-reset + action mask (packed) + "
                               f"{args.obs} obs, uniform random actions incl. invalid",
                   "boards_per_gpu": B, "global_boards": B * world, "rng": args.rng, "obs": args.obs,
                   "parallelism": f"dp{world} (board shards, no data-path collective)",
                   "chip_warmup": {"launches": warm["launches"], "seconds": round(warm["seconds"], 3),
                                   "env": "separate env of the same shape (untimed)"}},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic["bytes"] if traffic else None,
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "bytes_per_board_step": sb, "bytes_basis": "SURVEY.md section 8(d) algorithmic bytes",
                     "layout_bytes_per_board_step": rb + wb, "layout_achieved": layout_achieved,
                     "layout_frac": layout_achieved / HBM_PEAK_GBS,
                     "traffic_over_algorithmic": (traffic["bytes"] / alg_bytes) if traffic else None,
                     "kernel_ms": kern_ms, "kernel_ms_basis": "HIP events around launches 2..K of the timed K",
                     "kernel": "step_kernel (g2048_step)"},
        "cpu_baseline": cpu,
    }
    if traffic:
        line["roofline"]["traffic_detail"] = traffic
    if configs4 is not None:
        line["configs4_onehot_philox"] = configs4
    if train is not None:
        line["train_iteration_dp"] = train
    if policy is not None:
        line["policy_rollout"] = policy
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
