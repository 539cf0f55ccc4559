import torch, time
dev = torch.device("cuda", 0)
torch.manual_seed(0)
for m in (1000, 262144):
    a = torch.randn(m, 256, device=dev); w = torch.randn(256, 256, device=dev) * 0.06; b = torch.randn(256, device=dev)
    ref = torch.addmm(b.double(), a.double(), w.double())
    for name, fn in (("addmm", lambda: torch.addmm(b, a, w)), ("addmm_act", lambda: torch._addmm_activation(b, a, w))):
        y = fn(); torch.cuda.synchronize()
        r = ref if name == "addmm" else torch.relu(ref)
        err = ((y.double() - r).abs().max() / r.abs().max()).item()
        t0 = time.perf_counter()
        for _ in range(20): fn()
        torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 20
        print(f"m={m} {name}: max rel err {err:.2e}  {dt*1e6:.1f} us  {2*m*256*256/dt/1e12:.1f} TF", flush=True)
print("allow_tf32", torch.backends.cuda.matmul.allow_tf32, "precision", torch.get_float32_matmul_precision())
