import faulthandler, sys, os, time, traceback
faulthandler.dump_traceback_later(240, exit=True)
sys.path.insert(0, os.getcwd())
t0=time.time()
import torch
print("torch", torch.__version__, torch.cuda.is_available(), time.time()-t0, flush=True)
import rl2048_amd
from rl2048_amd import _lib as L
lib = L.lib()
print("abi", lib.g2048_abi_version(), flush=True)
try:
    L.ensure_device(torch.device("cuda", 0))
    print("init ok", flush=True)
except Exception:
    traceback.print_exc(); sys.stdout.flush()
    rc = lib.g2048_init(0); print("rc", rc, lib.g2048_last_error(), flush=True)
import numpy as np
from rl2048_amd import VecGame2048Env, Game2048EnvConfig
env = VecGame2048Env(8, Game2048EnvConfig(max_steps=None), device="cuda:0", record_merged=True)
print("env ok", flush=True)
env.reset(seed=[1,2,3,4,5,6,7,8]); torch.cuda.synchronize()
print("reset ok", env.board.cpu().numpy().view(np.uint64), flush=True)
from oracle import oracle as O
for s in range(1,9):
    g = O.Game(); g.reset(s); print(s, hex(O.pack_exponents(O.values_to_exponents(g.board))), flush=True)
env.step(torch.tensor([0,1,2,3,0,1,2,3], device="cuda:0")); torch.cuda.synchronize()
print("step ok", env.board.cpu().numpy().view(np.uint64), env.flags.cpu().numpy(), env.reward.cpu().numpy(), flush=True)
big = VecGame2048Env(100000, Game2048EnvConfig(max_steps=None), device="cuda:0")
big.reset(seed=1); torch.cuda.synchronize(); print("big reset ok", flush=True)
for i in range(5):
    big.step(torch.randint(0,4,(100000,), device="cuda:0")); torch.cuda.synchronize()
print("big step ok", big.flags[:10].cpu().numpy(), flush=True)
