"""GPU: the runner harness on the batched path reproduces the reference's per-episode loop (runner.py:581-677,
737-828): batch statistics of the first batch equal those of run_episode called episode by episode with the same
seed streams, CSV / config / checkpoint files follow the reference's layout, and the CLI runs end to end."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONF = {"env": {"obs_mode": "log2", "max_steps": 200}, "mlp": {"hidden_sizes": [32, 16]},
        "agent": {"baseline_mode": "batch", "learning_rate": 1e-3, "use_critic": True, "optimizer": "adam"},
        "train": {"batch_size": 12, "num_batches": 3, "env_base_seed": 3, "policy_base_seed": 7},
        "eval": {"num_episodes": 10, "env_base_seed": 11, "policy_base_seed": 13, "use_greedy": True}}


@pytest.fixture()
def R():
    from rl2048_amd import runner

    runner.reset_defaults()
    runner.apply_config_overrides_from_dict(CONF)
    yield runner
    runner.reset_defaults()


def test_training_loop_matches_episode_loop(R, tmp_path):
    agent, ec, mc, ac, tc = R.build_training_components(DEV)
    ref_agent, *_ = R.build_training_components(DEV)
    es, ps = R.make_fixed_seed_iter(3), R.make_fixed_seed_iter(7)
    ref = [ref_agent.run_episode(next(es), next(ps)) for _ in range(12)]
    rows = R.training_loop(agent, ec, mc, ac, tc, tmp_path, "t")
    assert len(rows) == 3
    tot = np.array([t["total_reward"] for t in ref], dtype=np.float32)
    assert rows[0]["avg_reward"] == pytest.approx(float(tot.mean()), rel=1e-6)
    assert rows[0]["max_reward"] == pytest.approx(float(tot.max()), rel=1e-6)
    assert rows[0]["min_reward"] == pytest.approx(float(tot.min()), rel=1e-6)
    counts = [sum(1 for t in ref if t["max_tile"] == v) for v in R.TILE_VALUES]
    assert json.loads(rows[0]["max_tile_counts"]) == counts
    lines = (tmp_path / "training_stats.csv").read_text().strip().splitlines()
    assert lines[0] == "batch,avg_reward,max_reward,min_reward,max_tile_counts" and len(lines) == 4
    cfg = json.loads((tmp_path / "config.json").read_text())
    assert cfg["run_mode"] == "Training" and cfg["mlp"]["hidden_sizes"] == [32, 16]


def test_evaluation_loop_matches_episode_loop(R):
    agent, *_ = R.build_training_components(DEV)
    s = R.evaluation_loop(agent, dict(R.DEFAULT_EVAL_CONFIG))
    es, ps = R.make_fixed_seed_iter(11), R.make_fixed_seed_iter(13)
    ref = [agent.run_episode(next(es), next(ps), use_greedy=True) for _ in range(10)]
    tot = np.array([t["total_reward"] for t in ref], dtype=np.float32)
    assert s["avg_reward"] == pytest.approx(float(tot.mean()), rel=1e-6)
    assert sum(v["count"] for v in s["max_tile_counts"].values()) == 10


def test_cli_training_run(tmp_path):
    conf = dict(CONF, run_mode="Training", log_level="INFO")
    conf["train"] = dict(CONF["train"], num_batches=2)
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(conf))
    r = subprocess.run([sys.executable, "-m", "rl2048_amd.runner", "-conf", str(p)], cwd=tmp_path, timeout=240,
                       capture_output=True, text=True, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    runs = list((tmp_path / "training_history").iterdir())
    assert len(runs) == 1 and (runs[0] / "training_stats.csv").exists()


def test_resume_reproduces_uninterrupted_run(R, tmp_path):
    """checkpoint_every / resume_from: batches 3-4 of a run resumed from its batch-2 checkpoint equal those of the
    uninterrupted 4-batch run, and so do the final actor / critic parameters and Adam state."""
    tc = dict(R.DEFAULT_TRAIN_CONFIG, num_batches=4)
    agent, ec, mc, ac, _ = R.build_training_components(DEV)
    (tmp_path / "full_run").mkdir()
    full = R.training_loop(agent, ec, mc, ac, tc, tmp_path / "full_run", "f")
    a1, *_ = R.build_training_components(DEV)
    (tmp_path / "part1").mkdir()
    R.training_loop(a1, ec, mc, ac, dict(tc, num_batches=2, checkpoint_every=2), tmp_path / "part1", "p1")
    ck = tmp_path / "part1" / "checkpoint_latest.npz"
    assert ck.exists()
    a2, *_ = R.build_training_components(DEV)
    (tmp_path / "part2").mkdir()
    rest = R.training_loop(a2, ec, mc, ac, dict(tc, resume_from=str(ck)), tmp_path / "part2", "p2")
    assert [r["batch"] for r in rest] == [3, 4]
    for got, ref in zip(rest, full[2:]):
        assert got["max_tile_counts"] == ref["max_tile_counts"]
        for k in ("avg_reward", "max_reward", "min_reward"):
            assert got[k] == pytest.approx(ref[k], rel=1e-5, abs=1e-5)
    sa, sb = agent.checkpoint_state(), a2.checkpoint_state()
    assert sorted(sa) == sorted(sb)
    for k in sa:
        np.testing.assert_allclose(sb[k], sa[k], rtol=1e-5, atol=1e-6, err_msg=k)
    # the checkpoint's actor loads as a reference model file (src/MLP.py:97-107 keys)
    from rl2048_amd.mlp import load_model_params

    p = load_model_params(str(ck))
    assert len(p["W"]) == len(agent.params["W"])
