"""TOOL: where deep_grad_kernel's time goes, phase by phase, on the reference runner config (runner.py:10-47:
one-hot obs, [256, 128, 64] ReLU, actor-critic MSE, Adam).  Needs the stamp build:

    python tools/build_variants.py --tu g2048_deep.hip deepdiag=G2048_DEEP_DIAG=1
    python tools/diag_deep.py [--episodes 262144] [--lib tools/libg2048_deepdiag.so]

Each wave adds the s_memtime cycles of every phase of every 32-sample group it runs (a phase ends at the barrier
that closes it, so it includes the wait for the slowest wave); printed: cycles per group per phase (mean over waves)
for one update (actor + critic launches), and the same as a share of the group.  The MFMA floor per group for this
net (the busiest wave's MFMA cycles, its SIMD shared with the other workgroup's wave) is printed beside it."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--episodes", type=int, default=262144)
ap.add_argument("--lib", default="tools/libg2048_deepdiag.so")
ap.add_argument("--label", default="")
ap.add_argument("--nb", type=int, default=64, help="samples per gradient group of the net's instantiation")
ap.add_argument("--rollout", action="store_true", help="stamp the rollout (deep_rollout_kernel) instead of the update")
ap.add_argument("--rollout-waves", type=int, default=8, help="waves per rollout workgroup (8: 64 slots, 4: 32 slots)")
args = ap.parse_args()
from rl2048_amd import _lib as L  # noqa: E402

L.use_library_for_tools(args.lib)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rl2048_amd import Game2048EnvConfig  # noqa: E402
from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig  # noqa: E402
from rl2048_amd.mlp import MLPConfig  # noqa: E402

ENV = dict(obs_mode="onehot", obs_log2_scale=1.0, reward_mode="log2", base_reward_scale=1.0, bonus_mode="off",
           bonus_scale=1.0, step_reward=0.0, endgame_penalty=0.0, use_action_mask=True, invalid_action_penalty=-1.0,
           max_steps=None, empty_tile_reward=0.05, merge_reward=0.0)
MLP = dict(hidden_sizes=[256, 128, 64], activation="ReLU", init_distribution="HeNormal", last_init_normal=True)
AGENT = dict(gamma=0.99, learning_rate=0.01, baseline_mode="batch", model_seed=0, reward_rank_weights=None,
             optimizer="adam", adam_beta1=0.9, adam_beta2=0.999, augmentation=False, use_critic=True,
             critic_learning_rate=0.0005, critic_loss_type="mse", huber_delta=1.0)
NS = 15   # kDiagSlots (g2048_deep.hip): the last slot counts groups / steps
# gradient kernel slots: the top dense layer's dW / delta / db and the lower layers' apart, the first dense layer's
# forward and the deeper ones' apart
PHASES = ["boards", "layer0", "dense_fwd_l1", "out_partials", "logits_g", "out_bwd", "dW_top", "db_top",
          "first_layer_out", "dense_fwd_l2+", "dW_lower", "delta_top", "delta_lower", "db_lower"]
dev = torch.device("cuda", 0)
agent = ReinforceAgent(Game2048EnvConfig(**ENV), MLPConfig(**MLP), ReinforceAgentConfig(**AGENT), device=dev)
lib = L.lib()
lib.g2048_diag_deep_stamps.argtypes = [ctypes.c_void_p]
slots = 4096 * NS
buf = torch.zeros(slots, dtype=torch.int64, device=dev)
E = args.episodes
RPHASES = ["top+boards", "layer0", "dense", "out_partials", "owners_rest", "claim", "owner_logits_choice",
           "owner_env_step", "owner_row_stores"]
for rep in range(2 if args.rollout else 0):
    # deep_rollout_kernel: per step of a workgroup, wave 0 (whose lanes own the episode slots: logits, choice, env
    # step, trajectory row) and the other waves (which wait for it at the next step's first barrier)
    es = np.arange(3 + rep * E, 3 + (rep + 1) * E, dtype=np.int64)
    torch.cuda.synchronize()
    buf.zero_()
    lib.g2048_diag_deep_stamps(ctypes.c_void_p(buf.data_ptr()))
    batch = agent.rollout_batch(es, es + 7 * E)
    torch.cuda.synchronize()
    lib.g2048_diag_deep_stamps(None)
    W = args.rollout_waves
    d = buf.view(-1, W, NS).cpu().numpy().astype(np.float64)
    d = d[d[:, 0, NS - 1] > 0]
    out = {"label": args.label, "rep": rep, "episodes": E, "steps": int(batch.lengths.sum()), "workgroups": int(d.shape[0]),
           "steps_per_workgroup": float(d[:, 0, NS - 1].mean())}
    for name, ws in (("wave0", [0]), ("waves1_%d" % (W - 1), list(range(1, W)))):
        per = (d[:, ws, :9] / d[:, ws, NS - 1:NS]).reshape(-1, 9).mean(axis=0)
        out[name] = {"cycles_per_step": round(per.sum()), "phases_cycles": {p: round(v) for p, v in zip(RPHASES, per)}}
    print(json.dumps(out), flush=True)
for rep in range(0 if args.rollout else 2):
    es = np.arange(3 + rep * E, 3 + (rep + 1) * E, dtype=np.int64)
    batch = agent.rollout_batch(es, es + 7 * E)
    torch.cuda.synchronize()
    buf.zero_()
    lib.g2048_diag_deep_stamps(ctypes.c_void_p(buf.data_ptr()))
    agent.update_from_batch(batch)
    torch.cuda.synchronize()
    lib.g2048_diag_deep_stamps(None)
    d = buf.view(-1, NS).cpu().numpy().astype(np.float64)
    d = d[d[:, NS - 1] > 0]
    per = d[:, :NS - 1] / d[:, NS - 1:NS]                      # cycles per group, per wave
    mean = per.mean(axis=0)
    tot = mean.sum()
    print(json.dumps({"label": args.label, "rep": rep, "episodes": E, "samples": int(batch.lengths.sum()),
                      "waves": int(d.shape[0]), "groups_per_wave": float(d[:, NS - 1].mean()),
                      "cycles_per_group": round(tot),
                      # the busiest SIMD's MFMA cycles per group of --nb samples (dense fp32 chains and dW tiles,
                      # 1920 v_mfma_f32_32x32x2f32 of 64 cycles per 32 samples over 4 SIMDs, plus the layer-0 bf16
                      # MFMAs: 65.5 k cycles per 64 samples)
                      "mfma_floor_cycles_per_group": 65536 * args.nb // 64,
                      "phases_cycles": {p: round(v) for p, v in zip(PHASES, mean)},
                      "phases_share": {p: round(v / tot, 3) for p, v in zip(PHASES, mean)}}), flush=True)
