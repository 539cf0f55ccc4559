import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
from rl2048_amd import Game2048EnvConfig
from rl2048_amd.agent import ReinforceAgent, ReinforceAgentConfig
from rl2048_amd.mlp import MLPConfig
from rl2048_amd.vec_env import _as_u64_seeds
dev = torch.device("cuda", 0)
agent = ReinforceAgent(Game2048EnvConfig(), MLPConfig(hidden_sizes=[256, 256], activation="ReLU", init_distribution="HeNormal"), ReinforceAgentConfig(), device=dev)
n = 65536
for rep in range(3):
    es = list(range(rep * n, rep * n + n)); ps = list(range(10 * n, 11 * n))
    torch.cuda.synchronize(); t0 = time.perf_counter()
    a = _as_u64_seeds(es, n, 0, dev); torch.cuda.synchronize(); t1 = time.perf_counter()
    cap = 1024
    x = torch.empty(cap, n, dtype=torch.int64, device=dev); y = torch.zeros(cap, n, dtype=torch.float32, device=dev)
    torch.cuda.synchronize(); t2 = time.perf_counter()
    b = agent.rollout_batch(es, ps); torch.cuda.synchronize(); t3 = time.perf_counter()
    agent.update_from_batch(b); torch.cuda.synchronize(); t4 = time.perf_counter()
    print(f"seeds->tensor {1e3*(t1-t0):.2f} ms  alloc {1e3*(t2-t1):.2f} ms  rollout_batch {1e3*(t3-t2):.2f} ms  update {1e3*(t4-t3):.2f}", flush=True)
    del x, y
