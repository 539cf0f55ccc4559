"""CPU: runner harness host logic (seed streams, config overrides, CSV schema) -- no GPU work."""
import json

import numpy as np
import pytest


@pytest.fixture()
def R():
    from rl2048_amd import runner

    runner.reset_defaults()
    yield runner
    runner.reset_defaults()


def test_seed_stream_blocks_equal_iterator(R, golden_dir):
    """SeedStream.take(n) reproduces make_fixed_seed_iter (runner.py:244-261) across block boundaries."""
    import os

    for base in (3, 7, 12345, 54321):
        it = R.make_fixed_seed_iter(base)
        ref = [next(it) for _ in range(700)]
        s = R.SeedStream(base)
        got = s.take(1) + s.take(255) + s.take(256) + s.take(188)
        assert got == ref
        s2 = R.SeedStream(base)
        assert [int(x) for x in s2.take_array(300)] + s2.take(400) == ref
    d = np.load(os.path.join(golden_dir, "pcg64.npz"))
    assert R.SeedStream(3).take(64) == [int(x) for x in d["fixed_seed_iter3"]]
    assert R.SeedStream(7).take(64) == [int(x) for x in d["fixed_seed_iter7"]]


def test_config_overrides_and_file(R, tmp_path):
    conf = {"env": {"obs_mode": "onehot", "max_steps": None}, "mlp": {"hidden_sizes": [64]},
            "agent": {"use_critic": True}, "train": {"batch_size": 8}, "eval": {"num_episodes": 3},
            "run_mode": "Training", "log_level": "INFO"}
    p = tmp_path / "c.json"
    p.write_text(json.dumps(conf))
    R.load_config_from_file(p)
    assert R.DEFAULT_ENV_KWARGS["obs_mode"] == "onehot" and R.DEFAULT_ENV_KWARGS["max_steps"] is None
    assert R.DEFAULT_ENV_KWARGS["reward_mode"] == "log2"           # untouched defaults survive
    assert R.DEFAULT_MLP_KWARGS["hidden_sizes"] == [64]
    assert R.DEFAULT_AGENT_KWARGS["use_critic"] is True
    assert R.DEFAULT_TRAIN_CONFIG["batch_size"] == 8 and R.DEFAULT_EVAL_CONFIG["num_episodes"] == 3
    assert R.RUN_MODE == "Training" and R.DEFAULT_LOG_LEVEL_NAME == "INFO"
    bad = tmp_path / "bad.json"
    bad.write_text("[1, 2]")
    with pytest.raises(SystemExit):
        R.load_config_from_file(bad)


def test_defaults_match_reference(R):
    """runner.py:116-176 defaults."""
    assert R.DEFAULT_ENV_KWARGS == {"size": 4, "obs_mode": "log2", "obs_log2_scale": 0.0625, "reward_mode": "log2",
                                    "base_reward_scale": 0.5, "bonus_mode": "off", "bonus_scale": 1.0,
                                    "step_reward": 0.0, "endgame_penalty": 0.0, "use_action_mask": True,
                                    "invalid_action_penalty": -1.0, "max_steps": 1024, "empty_tile_reward": 0.0,
                                    "merge_reward": 0.0}
    assert R.DEFAULT_TRAIN_CONFIG == {"batch_size": 256, "num_batches": 256, "env_base_seed": 3, "policy_base_seed": 7}
    assert R.DEFAULT_EVAL_CONFIG["env_base_seed"] == 12345 and R.DEFAULT_EVAL_CONFIG["use_greedy"] is True


def test_csv_schema(R, tmp_path):
    p = tmp_path / "training_stats.csv"
    fields = ["batch", "avg_reward", "max_reward", "min_reward", "max_tile_counts"]
    R.safe_append_csv_row(p, fields, {"batch": 1, "avg_reward": 1.5, "max_reward": 2.0, "min_reward": 1.0,
                                      "max_tile_counts": json.dumps([0] * 9)})
    R.safe_append_csv_row(p, fields, {"batch": 2, "avg_reward": 2.5, "max_reward": 3.0, "min_reward": 2.0,
                                      "max_tile_counts": json.dumps([1] + [0] * 8)})
    lines = p.read_text().strip().splitlines()
    assert lines[0] == ",".join(fields) and len(lines) == 3


def test_seed_stream_skip(R):
    """SeedStream.skip(n) consumes exactly what take(n) does (resume support)."""
    for base, n in ((3, 0), (7, 1), (12345, 700), (54321, (1 << 20) + 17)):
        ref = R.SeedStream(base)
        ref.take(n)
        s = R.SeedStream(base)
        s.skip(n)
        assert s.take(40) == ref.take(40)
