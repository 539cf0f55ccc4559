"""runner.py (reference runner.py) on the batched MI355X path.

    python -m rl2048_amd.runner -conf path/to/config.json          # or: python rl2048_amd_runner.py -conf ...
    torchrun --nproc-per-node 8 -m rl2048_amd.runner -conf cfg.json  # data parallel (one process per GPU)

Same JSON schema, DEFAULT_* values, seed streams, batch statistics, CSV schema and checkpoint format as the
reference (runner.py:116-176, :244-261, :495-679, :737-828).  What changes is the execution: each batch of
`batch_size` episodes is played at once, one episode per GPU lane (ReinforceAgent.rollout_batch), and updated
on the device trajectory buffer (update_from_batch) -- the same trajectories and the same update the reference
computes episode by episode.  Under torch.distributed each rank plays a contiguous slice of the batch's
episodes; statistics and checkpoints are global (rank 0 writes files).
"""
from __future__ import annotations

import argparse
import copy
import csv
import dataclasses
import json
import logging
import sys
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, Generator, List

import numpy as np
import torch

from . import dp
from .agent import ReinforceAgent, ReinforceAgentConfig
from .config import Game2048EnvConfig
from .mlp import MLPConfig

logger = logging.getLogger(__name__)

TRAINING_HISTORY_DIR = Path("training_history")
RUN_MODE: str = "Evaluation"

DEFAULT_ENV_KWARGS: Dict[str, Any] = {
    "size": 4, "obs_mode": "log2", "obs_log2_scale": 0.0625, "reward_mode": "log2", "base_reward_scale": 0.5,
    "bonus_mode": "off", "bonus_scale": 1.0, "step_reward": 0.0, "endgame_penalty": 0.0, "use_action_mask": True,
    "invalid_action_penalty": -1.0, "max_steps": 1024, "empty_tile_reward": 0.0, "merge_reward": 0.0,
}
DEFAULT_MLP_KWARGS: Dict[str, Any] = {
    "hidden_sizes": [256, 256], "activation": "ReLU", "init_distribution": "HeNormal", "last_init_normal": True,
}
DEFAULT_AGENT_KWARGS: Dict[str, Any] = {
    "gamma": 0.99, "learning_rate": 1e-4, "baseline_mode": "batch", "model_seed": 0, "reward_rank_weights": None,
    "optimizer": "sgd", "adam_beta1": 0.9, "adam_beta2": 0.999, "augmentation": False, "use_critic": False,
    "critic_learning_rate": 1e-5, "critic_loss_type": "mse", "huber_delta": 1.0,
}
DEFAULT_TRAIN_CONFIG: Dict[str, Any] = {"batch_size": 256, "num_batches": 256, "env_base_seed": 3, "policy_base_seed": 7}
DEFAULT_EVAL_CONFIG: Dict[str, Any] = {"num_episodes": 2048, "env_base_seed": 12345, "policy_base_seed": 54321,
                                       "model_path": None, "use_greedy": True}
DEFAULT_LOG_LEVEL_NAME = "VERBOSE"
TILE_VALUES = [16, 32, 64, 128, 256, 512, 1024, 2048, 4096]

_PRISTINE = copy.deepcopy((DEFAULT_ENV_KWARGS, DEFAULT_MLP_KWARGS, DEFAULT_AGENT_KWARGS, DEFAULT_TRAIN_CONFIG,
                           DEFAULT_EVAL_CONFIG))


# ---------------------------------------------------------------------------------------------- config
def reset_defaults() -> None:
    """Restore the DEFAULT_* dicts (module globals mutate under apply_config_overrides_from_dict)."""
    global RUN_MODE, DEFAULT_LOG_LEVEL_NAME
    for cur, orig in zip((DEFAULT_ENV_KWARGS, DEFAULT_MLP_KWARGS, DEFAULT_AGENT_KWARGS, DEFAULT_TRAIN_CONFIG,
                          DEFAULT_EVAL_CONFIG), _PRISTINE):
        cur.clear()
        cur.update(copy.deepcopy(orig))
    RUN_MODE, DEFAULT_LOG_LEVEL_NAME = "Evaluation", "VERBOSE"


def apply_config_overrides_from_dict(conf: Dict[str, Any]) -> None:
    """runner.py:394-441"""
    global RUN_MODE, DEFAULT_LOG_LEVEL_NAME
    for key, target in (("env", DEFAULT_ENV_KWARGS), ("mlp", DEFAULT_MLP_KWARGS), ("agent", DEFAULT_AGENT_KWARGS),
                        ("train", DEFAULT_TRAIN_CONFIG), ("eval", DEFAULT_EVAL_CONFIG)):
        if isinstance(conf.get(key), dict):
            target.update(conf[key])
    if isinstance(conf.get("run_mode"), str):
        RUN_MODE = conf["run_mode"]
    if isinstance(conf.get("log_level"), str):
        DEFAULT_LOG_LEVEL_NAME = conf["log_level"]


def load_config_from_file(path) -> Dict[str, Any]:
    """runner.py:444-465 (exits with a message on an unreadable / non-object file)."""
    p = Path(path)
    try:
        conf = json.loads(p.read_text(encoding="utf-8"))
    except Exception as e:  # noqa: BLE001
        print(f"[runner] Failed to load config file '{p}': {e}", file=sys.stderr)
        sys.exit(1)
    if not isinstance(conf, dict):
        print(f"[runner] Config file '{p}' must contain a JSON object at root.", file=sys.stderr)
        sys.exit(1)
    apply_config_overrides_from_dict(conf)
    return conf


def log_setup() -> None:
    """runner.py:182-207 (adds the VERBOSE=15 level of src/utils/logging_ext.py)."""
    if not hasattr(logging, "VERBOSE"):
        logging.VERBOSE = 15
        logging.addLevelName(15, "VERBOSE")
    root = logging.getLogger()
    if root.handlers:
        return
    h = logging.StreamHandler(sys.stdout)
    h.setLevel(logging.INFO)
    logging.basicConfig(level=getattr(logging, DEFAULT_LOG_LEVEL_NAME, logging.INFO),
                        format="%(asctime)s [%(name)s] [%(levelname)s] %(message)s", handlers=[h])


def attach_run_file_logger(log_path: Path) -> None:
    """runner.py:210-241"""
    root = logging.getLogger()
    for h in list(root.handlers):
        if isinstance(h, logging.FileHandler):
            root.removeHandler(h)
            h.close()
    log_path.parent.mkdir(parents=True, exist_ok=True)
    fh = logging.FileHandler(log_path, encoding="utf-8")
    fh.setLevel(logging.DEBUG)
    fh.setFormatter(logging.Formatter("%(asctime)s [%(name)s] [%(levelname)s] %(message)s"))
    root.addHandler(fh)


# ---------------------------------------------------------------------------------------------- seeds
def make_fixed_seed_iter(base_seed: int) -> Generator[int, None, None]:
    """runner.py:244-261: default_rng(base).integers(0, int64max, dtype=int64), one per episode."""
    rng = np.random.default_rng(base_seed)
    hi = np.iinfo(np.int64).max
    while True:
        yield int(rng.integers(low=0, high=hi, dtype=np.int64))


class SeedStream:
    """The same stream as make_fixed_seed_iter, drawn a block at a time (numpy's 64-bit bounded draws consume
    the generator identically for size=n and for n scalar calls; tests/test_runner_cpu.py checks it)."""

    def __init__(self, base_seed: int):
        self.rng = np.random.default_rng(base_seed)
        self.hi = np.iinfo(np.int64).max

    def take(self, n: int) -> list[int]:
        return [int(x) for x in self.rng.integers(0, self.hi, size=n, dtype=np.int64)]

    def take_array(self, n: int) -> np.ndarray:
        """take(n) as an int64 array (the batched rollout's fast seed path)."""
        return self.rng.integers(0, self.hi, size=n, dtype=np.int64)

    def skip(self, n: int) -> None:
        """Advance past n seeds (what take(n) consumes), a block at a time."""
        while n > 0:
            k = min(n, 1 << 20)
            self.rng.integers(0, self.hi, size=k, dtype=np.int64)
            n -= k


# ---------------------------------------------------------------------------------------------- helpers
def build_full_config_dict(env_config, mlp_config, agent_config, extra=None) -> Dict[str, Any]:
    """runner.py:264-294"""
    cfg = {"env": dataclasses.asdict(env_config), "mlp": dataclasses.asdict(mlp_config),
           "agent": dataclasses.asdict(agent_config)}
    if extra:
        cfg.update(extra)
    return cfg


def safe_write_json(path: Path, data: Dict[str, Any]) -> None:
    try:
        path.write_text(json.dumps(data, ensure_ascii=False, indent=2), encoding="utf-8")
    except Exception:  # noqa: BLE001 (the reference logs and continues, runner.py:297-307)
        logger.exception("Failed to write JSON config to %s", path)


def safe_append_csv_row(path: Path, fieldnames: List[str], row: Dict[str, Any]) -> None:
    """runner.py:310-332"""
    try:
        exists = path.exists() and path.stat().st_size > 0
        path.parent.mkdir(parents=True, exist_ok=True)
        with path.open("a", newline="", encoding="utf-8") as f:
            w = csv.DictWriter(f, fieldnames=fieldnames)
            if not exists:
                w.writeheader()
            w.writerow(row)
    except Exception:  # noqa: BLE001
        logger.exception("Failed to append row to CSV %s", path)


def create_training_run_dir() -> tuple[Path, str]:
    run_id = datetime.now().strftime("%Y%m%d_%H%M%S")
    run_dir = TRAINING_HISTORY_DIR / run_id
    run_dir.mkdir(parents=True, exist_ok=True)
    return run_dir, run_id


def _shard(n: int) -> tuple[int, int]:
    rank, world = dp.world()
    return dp.shard_bounds(n, rank, world)


def _global_episode_stats(batch) -> tuple[np.ndarray, np.ndarray]:
    tot, _ = dp.gather_varlen(batch.total_reward.to(torch.float64), sizes=batch.shard_sizes)
    mt, _ = dp.gather_varlen(batch.max_tile.to(torch.float64), sizes=batch.shard_sizes)
    return tot.cpu().numpy(), mt.cpu().numpy().astype(np.int64)


# ---------------------------------------------------------------------------------------------- training
def build_training_components(device=None):
    """runner.py:470-492 (the env is a config: the agent owns its vectorised env lanes)."""
    env_config = Game2048EnvConfig(**DEFAULT_ENV_KWARGS)
    mlp_config = MLPConfig(**DEFAULT_MLP_KWARGS)
    agent_config = ReinforceAgentConfig(**DEFAULT_AGENT_KWARGS)
    agent = ReinforceAgent(env_config, mlp_config, agent_config, device=device)
    return agent, env_config, mlp_config, agent_config, dict(DEFAULT_TRAIN_CONFIG)


def training_loop(agent: ReinforceAgent, env_config, mlp_config, agent_config, train_cfg: Dict[str, Any],
                  run_dir: Path, run_id: str) -> List[Dict[str, Any]]:
    """runner.py:495-679 with batched rollouts.  Returns the CSV rows written (rank 0).

    Beyond the reference: train_cfg["checkpoint_every"] = N > 0 writes
    run_dir/checkpoint_latest.npz after every N-th update (actor, critic, Adam state, batch index, best average,
    seed-stream positions); train_cfg["resume_from"] = path continues from such a file, so an interrupted run
    resumed from batch b produces the same later batches as the uninterrupted run."""
    bs = int(train_cfg["batch_size"])
    nb = int(train_cfg["num_batches"])
    ckpt_every = int(train_cfg.get("checkpoint_every") or 0)
    resume_from = train_cfg.get("resume_from")
    rank, _ = dp.world()
    if rank == 0:
        attach_run_file_logger(run_dir / f"train_{run_id}.log")
        full = build_full_config_dict(env_config, mlp_config, agent_config,
                                      extra={"run_mode": "Training", "train": train_cfg})
        safe_write_json(run_dir / "config.json", full)
    csv_path = run_dir / "training_stats.csv"
    fields = ["batch", "avg_reward", "max_reward", "min_reward", "max_tile_counts"]
    env_stream = SeedStream(int(train_cfg["env_base_seed"]))
    pol_stream = SeedStream(int(train_cfg["policy_base_seed"]))
    tile_index = {t: i for i, t in enumerate(TILE_VALUES)}
    best = float("-inf")
    rows: List[Dict[str, Any]] = []
    step = 0
    if resume_from:
        extra = agent.load_checkpoint(str(resume_from))
        if int(extra["batch_size"]) != bs or int(extra["env_base_seed"]) != int(train_cfg["env_base_seed"]) or \
                int(extra["policy_base_seed"]) != int(train_cfg["policy_base_seed"]):
            raise ValueError("resume_from: batch_size / base seeds differ from the checkpoint's run")
        step = int(extra["batch"])
        best = float(extra["best_avg_reward"])
        env_stream.skip(int(extra["env_seeds_drawn"]))
        pol_stream.skip(int(extra["policy_seeds_drawn"]))
        logger.info("Resumed from %s at batch %d", resume_from, step)
    lo, hi = _shard(bs)
    while nb <= 0 or step < nb:
        env_seeds, pol_seeds = env_stream.take_array(bs), pol_stream.take_array(bs)
        batch = agent.rollout_batch(env_seeds[lo:hi], pol_seeds[lo:hi])
        batch.shard_sizes = dp.shard_sizes(bs, dp.world()[1])
        step += 1
        totals, max_tiles = _global_episode_stats(batch)
        r32 = totals.astype(np.float32)
        avg_r, max_r, min_r = float(r32.mean()), float(r32.max()), float(r32.min())
        counts = [0] * len(TILE_VALUES)
        for mt in max_tiles:
            if int(mt) in tile_index:
                counts[tile_index[int(mt)]] += 1
        info = f"{step}/{nb}" if nb > 0 else f"{step} (infinite)"
        logger.info(f"Batch {info}: avg_reward={avg_r:.2f}, max_reward={max_r:.2f}, min_reward={min_r:.2f}, "
                    f"max_tile_counts={dict(zip(TILE_VALUES, counts))}")
        is_record = avg_r > best
        if is_record:
            best = avg_r
        if step > 30 and is_record and rank == 0:    # runner.py:642-660 (checkpoint before the update)
            path = run_dir / f"model_{datetime.now().strftime('%H%M%S')}_step{step}.npz"
            try:
                agent.save_model(str(path))
                logger.info("Saved model checkpoint: step=%d, avg_reward=%.4f, file=%s", step, avg_r, path)
            except Exception:  # noqa: BLE001
                logger.exception("Failed to save model checkpoint to %s", path)
        agent.update_from_batch(batch)
        row = {"batch": step, "avg_reward": avg_r, "max_reward": max_r, "min_reward": min_r,
               "max_tile_counts": json.dumps(counts, ensure_ascii=False)}
        if rank == 0:
            safe_append_csv_row(csv_path, fields, row)
        rows.append(row)
        if ckpt_every > 0 and step % ckpt_every == 0 and rank == 0:
            agent.save_checkpoint(str(run_dir / "checkpoint_latest.npz"), extra={
                "batch": step, "best_avg_reward": best, "batch_size": bs, "env_seeds_drawn": step * bs,
                "policy_seeds_drawn": step * bs, "env_base_seed": int(train_cfg["env_base_seed"]),
                "policy_base_seed": int(train_cfg["policy_base_seed"])})
    logger.info("Training finished.")
    return rows


def training(device=None) -> List[Dict[str, Any]]:
    agent, env_config, mlp_config, agent_config, train_cfg = build_training_components(device)
    run_dir, run_id = create_training_run_dir()
    return training_loop(agent, env_config, mlp_config, agent_config, train_cfg, run_dir, run_id)


# ---------------------------------------------------------------------------------------------- evaluation
def evaluation_loop(agent: ReinforceAgent, eval_cfg: Dict[str, Any], chunk: int = 65536) -> Dict[str, Any]:
    """runner.py:737-828: num_episodes episodes with fixed seed streams (greedy by default), batched."""
    n = int(eval_cfg["num_episodes"])
    greedy = bool(eval_cfg.get("use_greedy", True))
    env_seeds = SeedStream(int(eval_cfg["env_base_seed"])).take_array(n)
    pol_seeds = SeedStream(int(eval_cfg["policy_base_seed"])).take_array(n)
    totals, tiles = [], []
    for s in range(0, n, chunk):
        e, p = env_seeds[s:s + chunk], pol_seeds[s:s + chunk]
        lo, hi = _shard(len(e))
        b = agent.rollout_batch(e[lo:hi], p[lo:hi], use_greedy=greedy)
        b.shard_sizes = dp.shard_sizes(len(e), dp.world()[1])
        t, m = _global_episode_stats(b)
        totals.append(t)
        tiles.append(m)
    tot = np.concatenate(totals).astype(np.float32)
    mts = np.concatenate(tiles)
    hist = {int(t): int((mts == t).sum()) for t in sorted(set(mts.tolist()))}
    summary = {"episodes": int(n), "avg_reward": float(tot.mean()), "max_reward": float(tot.max()),
               "min_reward": float(tot.min()),
               "max_tile_counts": {t: {"count": c, "pct": round(c / n * 100.0, 2)} for t, c in hist.items()}}
    logger.info("Evaluation summary: episodes=%d, avg_reward=%.2f, max_reward=%.2f, min_reward=%.2f", n,
                summary["avg_reward"], summary["max_reward"], summary["min_reward"])
    logger.info("Max tile counts: %s", summary["max_tile_counts"])
    return summary


def evaluation(device=None) -> Dict[str, Any]:
    env_config = Game2048EnvConfig(**DEFAULT_ENV_KWARGS)
    agent = ReinforceAgent(env_config, MLPConfig(**DEFAULT_MLP_KWARGS), ReinforceAgentConfig(**DEFAULT_AGENT_KWARGS),
                           device=device)
    mp = DEFAULT_EVAL_CONFIG.get("model_path")
    if mp:
        try:
            agent.load_model(str(mp))
        except Exception:  # noqa: BLE001 (runner.py:723-732: fall back to the random init)
            logger.exception("Failed to load model from '%s', continue with randomly initialized weights.", mp)
    return evaluation_loop(agent, dict(DEFAULT_EVAL_CONFIG))


# ---------------------------------------------------------------------------------------------- CLI
def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description="2048 REINFORCE runner (configuration via JSON file), MI355X path.")
    ap.add_argument("-conf", "--conf", dest="conf", type=str, help="Path to configuration JSON file.")
    return ap.parse_args(argv)


def main(argv=None) -> None:
    import os

    import torch.distributed as dist

    args = parse_args(argv)
    if args.conf:
        load_config_from_file(args.conf)
    log_setup()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", torch.cuda.current_device())
    logger.info("Runner started with mode=%s", RUN_MODE)
    if RUN_MODE.lower() == "training":
        training(device)
    else:
        evaluation(device)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
