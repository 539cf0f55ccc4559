"""TOOL (build container only -- /root/reference does not exist on the GPU box): speed of oracle/pyref.py, the
Python restatement bench.py times as its CPU baseline, against the REAL reference on the same single-core workload
(Game2048Env.step with uniform random actions incl. invalid, obs + action mask every step, reset on episode end).

    python tools/pyref_ratio.py [--seconds 10]     # -> profiles/round2/pyref_ratio.txt
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CFG = dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5, max_steps=1024)


def run(make, step, seconds):
    rng = np.random.default_rng(0)
    env, seed, steps = make(), 1000, 0
    env.reset(seed=seed) if hasattr(env, "metadata") else env.reset(seed)
    t_end = time.perf_counter() + seconds
    t0 = time.perf_counter()
    while time.perf_counter() < t_end:
        if step(env, int(rng.integers(4))):
            seed += 1
            env.reset(seed=seed) if hasattr(env, "metadata") else env.reset(seed)
        steps += 1
    return steps / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden_ref import import_reference

    E, _, _ = import_reference("/root/reference")
    from oracle import pyref

    def ref_step(env, act):
        obs, r, te, tr, info = env.step(act)      # obs dict carries the board encoding and the action mask
        return te or tr

    def py_step(env, act):
        r, te, tr, _ = env.step(act)
        env.obs()
        env.game.action_mask()
        return te or tr

    ref = run(lambda: E.Game2048Env(E.Game2048EnvConfig(**CFG)), ref_step, a.seconds)
    py = run(lambda: pyref.PyEnv(**CFG), py_step, a.seconds)
    lines = [f"workload: Game2048Env.step + log2 obs + action mask, uniform random actions, {a.seconds:.0f} s each, "
             f"one core",
             f"reference src/env.py : {ref:10.0f} env steps/s",
             f"oracle/pyref.py      : {py:10.0f} env steps/s",
             f"ratio pyref / reference = {py / ref:.3f}"]
    out = "\n".join(lines)
    print(out)
    with open(os.path.join(ROOT, "profiles", "round2", "pyref_ratio.txt"), "w") as f:
        f.write(out + "\n")


if __name__ == "__main__":
    main()
