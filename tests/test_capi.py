"""CPU checks of the drop-in boundary: libg2048.so loads, exports every function include/g2048.h declares, the
ctypes struct images match the C layouts, and argument validation rejects bad calls before any launch.
No compute call is made (there is no GPU here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "g2048.h")


@pytest.fixture(scope="module")
def L():
    from rl2048_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib


def _declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(g2048_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_expected_api():
    assert _declared_functions() == sorted([
        "g2048_abi_version", "g2048_last_error", "g2048_init", "g2048_seed_pcg64", "g2048_reset", "g2048_step",
        "g2048_obs", "g2048_move", "g2048_sample", "g2048_returns", "g2048_symmetries", "g2048_policy_packed_size",
        "g2048_policy_pack", "g2048_policy", "g2048_rollout", "g2048_grad_packed_size", "g2048_grad_partial_size",
        "g2048_grad_pack", "g2048_actor_grad_waves", "g2048_actor_grad", "g2048_critic_grad", "g2048_dw2",
        "g2048_fold_partials", "g2048_dw2_factored", "g2048_dw2_actor", "g2048_deep_packed_size", "g2048_deep_pack", "g2048_deep_policy",
        "g2048_deep_rollout", "g2048_deep_hidden", "g2048_deep_grad_pack_size", "g2048_deep_grad_slab", "g2048_deep_grad_parts",
        "g2048_deep_grad_passes",
        "g2048_deep_grad_pack", "g2048_deep_grad", "g2048_onehot_layer1", "g2048_onehot_dw1_slab", "g2048_onehot_dw1"])


def test_library_exports_every_declared_symbol(L):
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (g2048_\w+)", out))
    missing = set(_declared_functions()) - exported
    assert not missing, missing
    lib = L.lib()
    assert lib.g2048_abi_version() == L.ABI_VERSION
    assert set(L.EXPORTED_SYMBOLS) == set(_declared_functions())


def test_gfx950_code_object_present(L):
    """The fat binary embeds an amdgcn gfx950 code object (the offload bundle id names the target)."""
    data = open(L.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_struct_layouts_match_header(L, tmp_path):
    import ctypes

    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "g2048.h"\nint main(void){printf("%zu %zu %zu %zu %zu\\n",'
                   ' sizeof(g2048_env_cfg), sizeof(g2048_lanes), sizeof(g2048_step_out),'
                   ' offsetof(g2048_env_cfg, base_reward_scale), offsetof(g2048_env_cfg, max_steps)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I" + os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [ctypes.sizeof(L.EnvCfg), ctypes.sizeof(L.Lanes), ctypes.sizeof(L.StepOut),
                   L.EnvCfg.base_reward_scale.offset, L.EnvCfg.max_steps.offset]


def test_argument_validation_without_gpu(L):
    """Bad arguments are rejected with G2048_EINVAL before anything touches a device."""
    import ctypes

    lib = L.lib()
    assert lib.g2048_obs(None, 1, 1.0, None, None, 4, None) == L.G2048_EINVAL
    assert lib.g2048_obs(ctypes.c_void_p(8), 7, 1.0, None, None, 4, None) == L.G2048_EINVAL
    assert b"obs_mode" in lib.g2048_last_error()
    assert lib.g2048_returns(None, None, 0.9, None, 4, 4, None) == L.G2048_EINVAL
    assert lib.g2048_symmetries(None, None, None, None, -1, None) == L.G2048_EINVAL
    cfg = L.EnvCfg()
    cfg.reward_mode = 5
    lanes = L.Lanes()
    out = L.StepOut()
    rc = lib.g2048_step(ctypes.byref(lanes), None, ctypes.byref(cfg), ctypes.byref(out), 0, 0, 0, 0, 1, None)
    assert rc == L.G2048_EINVAL and b"reward mode" in lib.g2048_last_error()
    cfg.reward_mode, cfg.max_steps = 0, L.MAX_STEPS_LIMIT + 1      # the 20-bit lane step count
    rc = lib.g2048_step(ctypes.byref(lanes), None, ctypes.byref(cfg), ctypes.byref(out), 0, 0, 0, 0, 1, None)
    assert rc == L.G2048_EINVAL and b"max_steps" in lib.g2048_last_error()
    cfg.max_steps = -1                                                  # Philox draws need a finite max_steps
    q = ctypes.c_void_p(8)
    plan = L.Lanes(q, q, q, None, None, None)
    pout = L.StepOut(q, q, None, None, None, None, None, None, None)
    rc = lib.g2048_step(ctypes.byref(plan), q, ctypes.byref(cfg), ctypes.byref(pout), L.RNG_PHILOX, 0, 0, 0, 1, None)
    assert rc == L.G2048_EINVAL and b"Philox" in lib.g2048_last_error()
    from rl2048_amd.config import Game2048EnvConfig, env_cfg_struct

    with pytest.raises(ValueError, match="max_steps"):
        env_cfg_struct(Game2048EnvConfig(max_steps=1 << 20))
    assert env_cfg_struct(Game2048EnvConfig(max_steps=L.MAX_STEPS_LIMIT)).max_steps == L.MAX_STEPS_LIMIT
    with pytest.raises(ValueError):
        L.check(L.G2048_EINVAL)
    # fused policy: shape / mode validation (no launch)
    assert lib.g2048_policy_packed_size(256, 256) == 8 * 8 * 64 + 8 * 32 + 8 * 8 * 16 * 64 + 8 * 32 + 8 * 128 + 4
    assert lib.g2048_policy_packed_size(0, 16) == -1 and lib.g2048_policy_packed_size(16, 300) == -1
    p = ctypes.c_void_p(8)
    assert lib.g2048_policy_pack(p, p, p, p, p, p, 272, 32, 32, p, 1 << 20, None) == L.G2048_EINVAL
    assert b"obs width" in lib.g2048_last_error()
    assert lib.g2048_policy_pack(p, p, p, p, p, p, 16, 32, 32, p, 10, None) == L.G2048_EINVAL
    args = [p, 32, 32, L.ACT_RELU, p, None, None, L.OBS_ONEHOT, 1.0, 1, 0, L.RNG_PHILOX, None, None, None, 0, None,
            None, None, p, 4, None]
    assert lib.g2048_policy(*args) == L.G2048_EINVAL and b"obs_mode" in lib.g2048_last_error()
    args[7], args[3] = L.OBS_LOG2, 7
    assert lib.g2048_policy(*args) == L.G2048_EINVAL and b"activation" in lib.g2048_last_error()
    args[3], args[11] = L.ACT_RELU, L.RNG_PCG64
    assert lib.g2048_policy(*args) == L.G2048_EINVAL and b"PCG64" in lib.g2048_last_error()
    # fused actor gradient: sizes and argument checks (no launch)
    assert lib.g2048_grad_packed_size(256, 256) == 8 * 8 * 1024 and lib.g2048_grad_packed_size(0, 5) == -1
    assert lib.g2048_grad_partial_size(256, 256) == 17 * 256 + 4 * 256 + 4
    assert lib.g2048_grad_partial_size(20, 40) == 17 * 32 + 4 * 64 + 4
    assert lib.g2048_grad_pack(p, 32, 32, p, 10, None) == L.G2048_EINVAL and b"too small" in lib.g2048_last_error()
    gargs = [p, p, 32, 32, L.ACT_RELU, L.OBS_LOG2, 1.0, 1, p, p, p, 40, 48, p, p, p, 1024, 0, None]
    assert lib.g2048_actor_grad(*gargs) == L.G2048_EINVAL and b"ld" in lib.g2048_last_error()   # ld % 32 != 0
    gargs[12] = 32
    assert lib.g2048_actor_grad(*gargs) == L.G2048_EINVAL   # ld < n
    gargs[12], gargs[5] = 64, L.OBS_ONEHOT
    assert lib.g2048_actor_grad(*gargs) == L.G2048_EINVAL and b"obs_mode" in lib.g2048_last_error()
    cargs = [p, p, 32, 32, L.ACT_RELU, L.OBS_LOG2, 1.0, 2, 1.0, p, p, p, None, None, 40, 128, 0, 64, p, p, p, 0, 1024,
             0, None, None]
    assert lib.g2048_critic_grad(*cargs) == L.G2048_EINVAL and b"critic loss" in lib.g2048_last_error()
    cargs[7] = 0
    for col_off, ncols in ((16, 64), (0, 32), (96, 64), (-32, 64)):   # unaligned, < n, past ld, negative
        cargs[16], cargs[17] = col_off, ncols
        assert lib.g2048_critic_grad(*cargs) == L.G2048_EINVAL and b"column window" in lib.g2048_last_error()
    cargs[16], cargs[17] = 0, 64
    cargs[4], cargs[23] = L.ACT_SIGMOID, 1      # the factored d2 form needs ReLU's 0/1 derivative
    assert lib.g2048_critic_grad(*cargs) == L.G2048_EINVAL and b"factored" in lib.g2048_last_error()
    cargs[4], cargs[23] = L.ACT_RELU, 2
    assert lib.g2048_critic_grad(*cargs) == L.G2048_EINVAL and b"factored" in lib.g2048_last_error()
    # in-kernel TD targets (g2048_td_rows, ABI 14): every buffer required; the deep kernel takes them for the critic only
    td = L.TdRows(8, 8, 8, None, 8, 0.99, 0)
    cargs[4], cargs[23], cargs[10], cargs[24] = L.ACT_RELU, 0, None, ctypes.byref(td)
    assert lib.g2048_critic_grad(*cargs) == L.G2048_EINVAL and b"TD-row" in lib.g2048_last_error()
    td.v_next = 8
    hs2 = (ctypes.c_int32 * 2)(64, 32)
    gd = [p, p, 2, hs2, L.ACT_RELU, L.OBS_LOG2, 1.0, 0, p, p, p, 0, 0, 1.0, None, None, None, None, 10, p, 4,
          ctypes.byref(td), None]
    assert lib.g2048_deep_grad(*gd) == L.G2048_EINVAL and b"TD rows are for the critic" in lib.g2048_last_error()
    dargs = [p, p, None, 32, 32, 64, 0, 64, 64, p, 1, None]   # factored dW2 without W3
    assert lib.g2048_dw2_factored(*dargs) == L.G2048_EINVAL and b"NULL" in lib.g2048_last_error()


def test_deep_sizes_and_validation_without_gpu(L):
    """The any-depth / one-hot entry points (g2048_deep.hip): packed sizes and slab layouts agree with the host's
    own layout (agent._deep_slab_layout), the coverage limits (<= 4 hidden layers of <= 256 units; the fused
    gradient: <= 64 dense 32x32 weight-gradient tiles on one-hot obs, <= 48 on log2 / raw) and the argument checks, all before any launch."""
    import ctypes

    from rl2048_amd.agent import ReinforceAgent, _round32

    lib = L.lib()
    arr = lambda hs: (ctypes.c_int32 * len(hs))(*hs)   # noqa: E731

    def packed(obs, hs):
        t = [_round32(h) // 32 for h in hs]
        n = (272 * 32 * t[0] if obs == L.OBS_ONEHOT else t[0] * 512) + 32 * t[0]
        for l in range(1, len(hs)):
            n += 1024 * t[l] * t[l - 1] + 32 * t[l]
        n += 32 * t[-1] * 4 + 4
        # one-hot: + W1's bf16-plane A fragments, [nt0][16 cells][3 planes][64 lanes][4 dwords] (round 5)
        return n + (t[0] * 16 * 3 * 64 * 4 if obs == L.OBS_ONEHOT else 0)

    for obs, hs in ((L.OBS_ONEHOT, [256, 128, 64]), (L.OBS_LOG2, [40, 33, 20, 10]), (L.OBS_RAW, [1]),
                    (L.OBS_ONEHOT, [128, 64])):
        assert lib.g2048_deep_packed_size(obs, len(hs), arr(hs)) == packed(obs, hs), (obs, hs)
    for obs, hs in ((L.OBS_LOG2, [16] * 5), (L.OBS_LOG2, [257]), (L.OBS_LOG2, [0, 8]), (7, [32])):
        assert lib.g2048_deep_packed_size(obs, len(hs), arr(hs)) == -1, (obs, hs)
    # the fused gradient's partial slab == the layout the host folds it with; nets past its tile budget -> -1
    for obs, hs in ((L.OBS_ONEHOT, [256, 128, 64]), (L.OBS_LOG2, [64, 48, 32]), (L.OBS_RAW, [40, 33, 20, 10]),
                    (L.OBS_LOG2, [128, 128, 128]), (L.OBS_ONEHOT, [256, 256]), (L.OBS_ONEHOT, [200, 250])):
        pw, pb = ReinforceAgent._deep_slab_layout(hs, obs == L.OBS_ONEHOT)
        assert lib.g2048_deep_grad_slab(obs, len(hs), arr(hs)) == pb[-1] + 4, (obs, hs)
        t = [_round32(h) // 32 for h in hs]
        nb = sum(t[l] * t[l - 1] * 1024 for l in range(1, len(hs)))
        assert lib.g2048_deep_grad_pack_size(obs, len(hs), arr(hs)) == max(nb, 1)
    # past one launch's accumulator budget (64 tiles one-hot, 48 log2 / raw): covered by one launch per tile range
    # (round 5), the same slab
    for obs, hs in ((L.OBS_ONEHOT, [256, 256, 256]), (L.OBS_ONEHOT, [256, 256, 32]), (L.OBS_LOG2, [256, 256]),
                    (L.OBS_ONEHOT, [256] * 4)):
        pw, pb = ReinforceAgent._deep_slab_layout(hs, obs == L.OBS_ONEHOT)
        assert lib.g2048_deep_grad_slab(obs, len(hs), arr(hs)) == pb[-1] + 4, (obs, hs)
        assert lib.g2048_deep_grad_parts(obs, len(hs), arr(hs)) > 0, (obs, hs)
        assert lib.g2048_deep_grad_passes(obs, len(hs), arr(hs)) > 1, (obs, hs)
    # within one launch's budget: one pass (what ReinforceAgent._deep_grad_spec gates on)
    for obs, hs in ((L.OBS_ONEHOT, [256, 128, 64]), (L.OBS_ONEHOT, [256, 256]), (L.OBS_LOG2, [64, 48, 32])):
        assert lib.g2048_deep_grad_passes(obs, len(hs), arr(hs)) == 1, (obs, hs)
    # not a net of the any-depth kernels at all (5 hidden layers)
    for obs, hs in ((L.OBS_LOG2, [32] * 5),):
        assert lib.g2048_deep_grad_slab(obs, len(hs), arr(hs)) == -1, (obs, hs)
        assert lib.g2048_deep_grad_parts(obs, len(hs), arr(hs)) == -1, (obs, hs)
        assert lib.g2048_deep_grad_passes(obs, len(hs), arr(hs)) == -1, (obs, hs)
    # workgroups that fill the chip: one per CU (64-sample groups for one-hot nets of <= 40 tiles, round 6)
    cus = lib.g2048_deep_grad_parts(L.OBS_LOG2, 3, arr([64, 48, 32]))
    assert cus > 0
    assert lib.g2048_deep_grad_parts(L.OBS_ONEHOT, 3, arr([256, 128, 64])) == cus
    assert lib.g2048_deep_grad_parts(L.OBS_ONEHOT, 2, arr([256, 256])) == cus
    assert lib.g2048_onehot_dw1_slab(256) == 273 * 256 and lib.g2048_onehot_dw1_slab(0) == -1
    assert lib.g2048_onehot_dw1_slab(257) == -1
    p = ctypes.c_void_p(8)
    hs = arr([32, 32])
    assert lib.g2048_deep_pack(p, p, L.OBS_LOG2, 5, arr([32] * 5), 4, p, 1 << 20, None) == L.G2048_EINVAL
    assert b"hidden layers" in lib.g2048_last_error()
    assert lib.g2048_deep_pack(p, p, L.OBS_LOG2, 2, hs, 3, p, 1 << 20, None) == L.G2048_EINVAL
    assert b"output width" in lib.g2048_last_error()
    assert lib.g2048_deep_pack(p, p, L.OBS_LOG2, 2, hs, 4, p, 10, None) == L.G2048_EINVAL
    assert b"too small" in lib.g2048_last_error()
    assert lib.g2048_deep_grad_pack(p, L.OBS_LOG2, 2, hs, p, 10, None) == L.G2048_EINVAL
    assert lib.g2048_onehot_layer1(p, p, 32, 7, p, 4, 32, p, None) == L.G2048_EINVAL
    assert b"activation" in lib.g2048_last_error()
    assert lib.g2048_onehot_layer1(p, p, 32, L.ACT_RELU, p, 4, 16, p, None) == L.G2048_EINVAL   # ld < h1
    assert lib.g2048_onehot_dw1(p, p, 64, 100, 64, 30, p, 3, None) == L.G2048_EINVAL           # 3 != ceil(100/30)
    assert b"nparts" in lib.g2048_last_error()
    assert lib.g2048_onehot_dw1(p, p, 300, 100, 300, 30, p, 4, None) == L.G2048_EINVAL
    assert lib.g2048_onehot_layer1(p, p, 32, L.ACT_RELU, None, 0, 32, None, None) == L.G2048_OK   # m == 0: no-op


def test_config_validation_messages():
    from rl2048_amd.config import Game2048EnvConfig, env_cfg_struct

    for kw, msg in ((dict(obs_mode="x"), "Unsupported obs_mode"), (dict(reward_mode="x"), "Unsupported reward mode"),
                    (dict(bonus_mode="x"), "Unsupported bonus mode")):
        with pytest.raises(ValueError, match=msg):
            env_cfg_struct(Game2048EnvConfig(**kw))
    assert env_cfg_struct(Game2048EnvConfig(max_steps=None)).max_steps == -1
    assert env_cfg_struct(Game2048EnvConfig(max_steps=0)).max_steps == 0


def test_philox_needs_finite_max_steps():
    """Philox's draw counter is the 20-bit lane step count, so a Philox env without max_steps is refused at
    construction (before any device is touched); PCG64 without max_steps is fine."""
    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    with pytest.raises(ValueError, match="finite max_steps"):
        VecGame2048Env(4, Game2048EnvConfig(max_steps=None), device="cpu", rng="philox")


def test_no_cpu_fallback():
    """The product path refuses to run without a HIP device instead of falling back to CPU."""
    import torch

    from rl2048_amd import Game2048EnvConfig, VecGame2048Env

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no CPU fallback|no HIP device"):
        VecGame2048Env(4, Game2048EnvConfig(), device="cpu")
