"""MI355X-native hot path of pqpeqr/RL-2048-with-Reinforce-and-Actor-Critic.

Import as ``rl2048_amd`` (the repo-root shim ``rl2048_amd.py`` maps that name onto this directory, whose own
name is not a Python identifier).

    from rl2048_amd import VecGame2048Env, Game2048Env, Game2048EnvConfig, Game2048
    from rl2048_amd.mlp import MLPConfig, init_model_params, forward_logits, logits_to_probs
    from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig

The GPU work happens in libg2048.so (csrc/g2048.hip, C ABI in include/g2048.h); there is no CPU fallback.
"""
from ._lib import build as build_library  # noqa: F401
from .config import Game2048EnvConfig  # noqa: F401
from .env import Game2048, Game2048Env  # noqa: F401
from .vec_env import VecGame2048Env, decode_merged  # noqa: F401

__all__ = ["Game2048EnvConfig", "Game2048", "Game2048Env", "VecGame2048Env", "decode_merged", "build_library"]
