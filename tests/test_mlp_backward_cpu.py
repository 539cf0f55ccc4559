"""CPU: the batched manual backprop used by the update (mlp.mlp_backward_, restating
src/reinforce_agent.py:_backpropagation :639-678) equals torch autograd of the same MLP, including the split-K
weight-gradient path (row blocks + remainder) and both activations."""
import pytest
import torch


@pytest.mark.parametrize("act", ["ReLU", "Sigmoid"])
@pytest.mark.parametrize("m", [7, 4096, 9000])
def test_manual_backprop_equals_autograd(act, m):
    from rl2048_amd.mlp import mlp_backward_, mlp_forward_kept

    g = torch.Generator().manual_seed(m + len(act))
    sizes = [16, 64, 32, 4]
    W = [torch.randn(sizes[i], sizes[i + 1], generator=g, dtype=torch.float64) * 0.3 for i in range(3)]
    b = [torch.randn(sizes[i + 1], generator=g, dtype=torch.float64) * 0.1 for i in range(3)]
    x = torch.randn(m, 16, generator=g, dtype=torch.float64)
    gout = torch.randn(m, 4, generator=g, dtype=torch.float64)
    gW = [torch.zeros_like(w, dtype=torch.float32) for w in W]
    gb = [torch.zeros_like(v, dtype=torch.float32) for v in b]
    pf = {"W": [w.float() for w in W], "b": [v.float() for v in b]}
    out, kept = mlp_forward_kept(pf, x.float(), act)
    mlp_backward_(pf, kept, act, gout.float(), gW, gb)
    # autograd reference in float64
    Wr = [w.clone().requires_grad_(True) for w in W]
    br = [v.clone().requires_grad_(True) for v in b]
    a = x
    for i in range(3):
        z = a @ Wr[i] + br[i]
        a = (torch.relu(z) if act == "ReLU" else torch.sigmoid(z)) if i < 2 else z
    grads = torch.autograd.grad(a, Wr + br, grad_outputs=gout)
    for got, ref in zip(gW + gb, grads):
        err = float((got.double() - ref).abs().max() / (ref.abs().max() + 1e-30))
        assert err < 2e-5, err
