"""GPU parity of g2048_step at the batch sizes the bench runs (the LDS-table path: >= 16,384 lanes) and at its
edges, against the CPU oracle on sampled lanes (every lane would be minutes of oracle time):

* the LDS path with frequent auto-resets (block-compacted reset list) on a ragged batch;
* a mass truncation in which every lane resets in the same launch, so every workgroup's LDS reset list overflows
  and the per-lane fallback runs -- all 4M boards are also checked against g2048_reset of the next seeds;
* the launch split above 2^27 lanes (32-bit byte offsets per launch), sampled around the split.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CFG = dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5)


def _sample(n, k, seed, extra=()):
    g = np.random.default_rng(seed)
    idx = set(int(i) for i in g.choice(n, size=min(k, n), replace=False))
    for i in (0, 1, 63, 64, 1023, 1024, 1025, n - 2, n - 1) + tuple(extra):
        if 0 <= i < n:
            idx.add(int(i))
    return np.array(sorted(idx), dtype=np.int64)


def _run(n, steps, max_steps, k, seed, stride=None, extra=(), lean=False):
    """lean: the throughput configuration of bench.py (no score output, packed action mask): the log2-reward lean
    step kernel (RK 1)."""
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    cfg = dict(CFG, max_steps=max_steps)
    stride = stride or n
    env = VecGame2048Env(n, Game2048EnvConfig(**cfg), device=DEV, auto_reset=True, reset_stride=stride,
                         track_score=not lean, packed_mask=lean)
    env.reset(seed=seed)                               # lane i: seed + i
    idx = _sample(n, k, seed, extra)
    it = torch.from_numpy(idx).to(DEV)
    ref = {int(i): O.Env(**cfg) for i in idx}
    seeds = {int(i): seed + int(i) for i in idx}
    for i, e in ref.items():
        e.reset(seeds[i])
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    resets = 0
    for t in range(steps):
        acts = torch.randint(0, 4, (n,), dtype=torch.uint8, device=DEV, generator=g)
        env.step_into(acts)
        a = acts[it].cpu().numpy()
        rw = env.reward[it].cpu().numpy()
        fl = env.flags[it].cpu().numpy()
        bd = env.board[it].cpu().numpy().view(np.uint64)
        ob = env.obs[it].cpu().numpy()
        mk = env.action_mask[it].cpu().numpy()
        for j, i in enumerate(idx):
            i = int(i)
            r = ref[i].step(int(a[j]))
            assert rw[j] == np.float32(r["reward"]), (t, i)
            assert bool(fl[j] & 0x02) == r["terminated"] and bool(fl[j] & 0x04) == r["truncated"], (t, i)
            if r["terminated"] or r["truncated"]:
                assert fl[j] & 0x20, (t, i)            # auto-reset: the lane now holds the next episode
                seeds[i] += stride
                ref[i].reset(seeds[i])
                resets += 1
            assert bd[j] == O.pack_exponents(O.values_to_exponents(ref[i].board)), (t, i)
            np.testing.assert_array_equal(ob[j], ref[i].obs())
            np.testing.assert_array_equal(mk[j], ref[i].mask())
    return env, resets


@pytest.mark.parametrize("lean", [False, True])
def test_lds_path_autoreset_sampled_vs_oracle(lean):
    env, resets = _run(20000 + 37, steps=100, max_steps=40, k=256, seed=4242, lean=lean)
    assert resets > 256                                # every sampled lane went through >= 2 resets


def test_bench_workload_lean_path_sampled_vs_oracle():
    """bench.py's headline workload exactly -- 1,048,576 random-state boards (tiles up to 2^12, so large merges
    and max_tile_seen updates from 4), PCG64 lane streams from env.reset, log2 obs + log2 reward, packed mask, no
    score output: the lean step kernel -- with sampled lanes replayed bit-exactly by the oracle from the same
    boards and streams (rewards, flags, boards, obs, masks, max_tile_seen; auto-resets included)."""
    import bench
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    n = 1 << 20
    cfg = dict(obs_mode="log2", obs_log2_scale=0.0625, reward_mode="log2", base_reward_scale=0.5, max_steps=1024)
    env = VecGame2048Env(n, Game2048EnvConfig(**cfg), device=DEV, auto_reset=True, reset_stride=n,
                         track_score=False, packed_mask=True)
    env.reset(seed=torch.arange(n, dtype=torch.int64, device=DEV) + 1_000_003)
    env.board.copy_(bench.synthetic_boards(torch, n, 0, DEV))
    env.set_lane_state(step_count=0, max_tile_exp=2, active=True)
    idx = _sample(n, 300, 99)
    it = torch.from_numpy(idx).to(DEV)
    start = env.boards_values()[it].cpu().numpy().reshape(-1, 16)
    ref, seeds = {}, {}
    for j, i in enumerate(idx):
        i = int(i)
        seeds[i] = 1_000_003 + i
        e = O.Env(**cfg)
        e.reset(seeds[i])                              # the lane's PCG64 stream after its reset's two spawns
        for c in range(16):
            e.e.game.board[c] = int(start[j, c])       # then the synthetic board, as bench.make_env does
        e.e.step_count, e.e.max_tile_seen = 0, 4
        ref[i] = e
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    bonus_updates = 0
    for t in range(40):
        acts = torch.randint(0, 4, (n,), dtype=torch.uint8, device=DEV, generator=g)
        env.step_into(acts)
        a, rw, fl = acts[it].cpu().numpy(), env.reward[it].cpu().numpy(), env.flags[it].cpu().numpy()
        bd, ob = env.board[it].cpu().numpy().view(np.uint64), env.obs[it].cpu().numpy()
        mk, mt = env.action_mask[it].cpu().numpy(), env.max_tile_seen[it].cpu().numpy()
        for j, i in enumerate(idx):
            i = int(i)
            before = ref[i].max_tile_seen
            r = ref[i].step(int(a[j]))
            bonus_updates += ref[i].max_tile_seen != before
            assert rw[j] == np.float32(r["reward"]), (t, i)
            assert bool(fl[j] & 0x02) == r["terminated"] and bool(fl[j] & 0x04) == r["truncated"], (t, i)
            assert bool(fl[j] & 0x08) == r["invalid"], (t, i)
            if r["terminated"] or r["truncated"]:
                assert fl[j] & 0x20, (t, i)
                seeds[i] += n
                ref[i].reset(seeds[i])
            assert bd[j] == O.pack_exponents(O.values_to_exponents(ref[i].board)), (t, i)
            np.testing.assert_array_equal(ob[j], ref[i].obs())
            np.testing.assert_array_equal(mk[j], ref[i].mask())
            assert mt[j] == ref[i].max_tile_seen, (t, i)
    assert bonus_updates > len(idx)                    # max_tile_seen rose from 4 on most sampled lanes


def test_mass_truncation_overflows_reset_list():
    """max_steps=3 from a common start: every lane truncates at step 3 and 6, i.e. ~16 resets per lane-slot of a
    persistent workgroup -- more than its LDS reset list holds, so the per-lane fallback runs."""
    n = (1 << 22) + 5
    env, resets = _run(n, steps=7, max_steps=3, k=128, seed=77)
    assert resets >= 2 * 128
    # every lane truncated at steps 3 and 6 (a fresh game cannot end within 3 moves) and has stepped once since
    assert bool((env.step_count == 1).all())


def test_mass_reset_boards_equal_g2048_reset():
    """All lanes of a mass truncation hold exactly Game2048.reset(seed + stride) afterwards."""
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    n = (1 << 22) + 5
    cfg = Game2048EnvConfig(**dict(CFG, max_steps=1))
    env = VecGame2048Env(n, cfg, device=DEV, auto_reset=True, reset_stride=n)
    env.reset(seed=1000)
    env.step_into(torch.zeros(n, dtype=torch.uint8, device=DEV))    # every lane truncates (max_steps=1)
    fresh = VecGame2048Env(n, cfg, device=DEV)
    fresh.reset(seed=1000 + n)
    assert bool(((env.flags & 0x20) != 0).all())
    assert torch.equal(env.board, fresh.board)
    assert torch.equal(env.obs, fresh.obs) and torch.equal(env.mask, fresh.mask)
    assert bool((env.step_count == 0).all()) and bool((env.score == 0).all())


def test_split_launch_above_2_27_lanes():
    n = (1 << 27) + 3001
    s = 1 << 27
    _run(n, steps=4, max_steps=1024, k=64, seed=5,
         extra=(s - 65, s - 64, s - 2, s - 1, s, s + 1, s + 63, s + 64, s + 1023, s + 1024))
