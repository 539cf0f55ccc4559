"""The policy / critic MLP of src/MLP.py on PyTorch-ROCm (fp32; the dense layers run on hipBLASLt).

Same names, parameter layout and numbers as the reference: params = {"W": [W_0..W_L], "b": [b_0..b_L]} with
W_l of shape [in, out] (``x @ W + b``), fp32, initialised by the SAME numpy Generator draws in the same order
(src/MLP.py:45-94), so a given model_seed yields bit-identical weights.  Tensors live on the agent's device.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Literal

import numpy as np
import torch

ActivationMode = Literal["Sigmoid", "ReLU"]


@dataclass
class MLPConfig:
    hidden_sizes: list[int] = field(default_factory=list)
    activation: ActivationMode = "Sigmoid"
    init_distribution: str = "XavierNormal"
    last_init_normal: bool = True   # accepted for config compatibility; dead code in the reference (src/MLP.py:69)

    @property
    def num_layers(self) -> int:
        return len(self.hidden_sizes)


def encode_observation(obs):
    """src/MLP.py:22-43.  obs: dict {"board", "action_mask"} or a bare board; numpy or torch, single or batched
    (a leading batch dim is kept when the board has 3 (raw/log2) or 4 (onehot) dims)."""
    if isinstance(obs, dict):
        board, mask = obs["board"], obs["action_mask"]
    else:
        board, mask = obs, None
    if isinstance(board, torch.Tensor):
        batched = board.dim() in (3, 4) and not (board.dim() == 3 and board.shape[-1] == 17)
        x = board.to(torch.float32).reshape(board.shape[0], -1) if batched else board.to(torch.float32).reshape(-1)
    else:
        x = np.asarray(board).astype(np.float32).flatten()
    return x, mask


def _draw_layer(rng: np.random.Generator, dist: str, din: int, dout: int) -> np.ndarray:
    if dist == "XavierNormal":
        return rng.normal(0.0, np.sqrt(2.0 / (din + dout)), size=(din, dout)).astype(np.float32)
    if dist == "HeNormal":
        return rng.normal(0.0, np.sqrt(2.0 / din), size=(din, dout)).astype(np.float32)
    if dist == "XavierUniform":
        lim = np.sqrt(6.0 / (din + dout))
        return rng.uniform(-lim, lim, size=(din, dout)).astype(np.float32)
    if dist == "Normal":
        return rng.standard_normal((din, dout), dtype=np.float32) * 0.01
    raise ValueError(f"Unsupported init_distribution: {dist}")


def init_model_params(input_dim: int, hidden_sizes: list[int], output_dim: int, rng: np.random.Generator,
                      init_distribution: str = "normal", last_init_normal: bool = True, device=None) -> dict[str, Any]:
    """src/MLP.py:45-94: one draw per layer, in order, from `rng` (host numpy -- the reference's init stream),
    biases zero, then the fp32 tensors are placed on `device`."""
    sizes = [input_dim] + list(hidden_sizes) + [output_dim]
    Ws, bs = [], []
    for din, dout in zip(sizes[:-1], sizes[1:]):
        Ws.append(torch.from_numpy(_draw_layer(rng, init_distribution, din, dout)).to(device))
        bs.append(torch.zeros(dout, dtype=torch.float32, device=device))
    return {"W": Ws, "b": bs}


def load_model_params(file_path: str = "params.npz", device=None) -> dict[str, Any]:
    """src/MLP.py:97-107 (npz keys n_layers, W_i, b_i; loaded without pickle)."""
    with np.load(file_path, allow_pickle=False) as data:
        n = int(data["n_layers"])
        return {"W": [torch.from_numpy(np.array(data[f"W_{i}"], dtype=np.float32)).to(device) for i in range(n)],
                "b": [torch.from_numpy(np.array(data[f"b_{i}"], dtype=np.float32)).to(device) for i in range(n)]}


def save_model_params(params: dict[str, Any], file_path: str = "params.npz") -> None:
    """src/MLP.py:110-126 -- the same npz layout, so checkpoints interoperate with the reference."""
    Ws, bs = list(params["W"]), list(params["b"])
    assert len(Ws) == len(bs), "W/b layer count mismatch"
    data = {"n_layers": np.array(len(Ws), dtype=np.int64)}
    for i, (W, b) in enumerate(zip(Ws, bs)):
        data[f"W_{i}"] = W.detach().cpu().numpy() if isinstance(W, torch.Tensor) else np.asarray(W)
        data[f"b_{i}"] = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    np.savez(file_path, **data)


def apply_activation(x: torch.Tensor, mode: str) -> torch.Tensor:
    """src/MLP.py:130-136"""
    if mode == "Sigmoid":
        return torch.sigmoid(x)
    if mode == "ReLU":
        return torch.relu(x)
    raise ValueError(f"Unsupported activation: {mode}")


def forward_logits(params: dict[str, list[torch.Tensor]], x: torch.Tensor, activation_mode: str,
                   keep_cache: bool = True):
    """src/MLP.py:159-196: z_i = a_i @ W_i + b_i, activation on hidden layers, identity on the last.
    Returns (logits, activations [a_0..a_L], pre_activations [z_0..z_{L-1}]) like the reference."""
    Ws, bs = params["W"], params["b"]
    assert len(Ws) == len(bs), "W/b layer count mismatch"
    act = x.to(torch.float32)
    acts, pres = ([act], []) if keep_cache else (None, None)
    for i, (W, b) in enumerate(zip(Ws, bs)):
        if not keep_cache and activation_mode == "ReLU" and act.dim() == 2 and i < len(Ws) - 1 and \
                not (torch.is_grad_enabled() and (act.requires_grad or W.requires_grad or b.requires_grad)):
            # rollout / inference: bias + ReLU in the hipBLASLt epilogue (no separate pass over the [n, 256]
            # activations; same fp32 values as relu(addmm)); it has no autograd formula, so not under grad
            act = torch._addmm_activation(b, act, W, use_gelu=False)
            continue
        z = torch.addmm(b, act, W) if act.dim() == 2 else act @ W + b
        if keep_cache:
            pres.append(z)
        act = apply_activation(z, activation_mode) if i < len(Ws) - 1 else z
        if keep_cache:
            acts.append(act)
    return act, acts, pres


def _wgrad_(out: torch.Tensor, a: torch.Tensor, d: torch.Tensor) -> None:
    """out += a^T d for a [m, p], d [m, q] with m >> p, q (the weight gradient of a batch): split-K as a batched
    GEMM over row blocks plus one reduction, so the few output tiles are spread over the whole chip instead of
    each walking all m rows (a plain addmm of these shapes gets a handful of workgroups)."""
    m = a.shape[0]
    P = min(128, m // 2048)
    if P >= 2:
        q = m // P
        mm = P * q
        part = torch.bmm(a[:mm].view(P, q, -1).transpose(1, 2), d[:mm].view(P, q, -1))
        out.add_(part.sum(0))
        if mm < m:
            out.addmm_(a[mm:].t(), d[mm:])
    else:
        out.addmm_(a.t(), d)


def mlp_forward_kept(params: dict[str, list[torch.Tensor]], x: torch.Tensor | None, activation_mode: str,
                     a1: torch.Tensor | None = None):
    """forward_logits (src/MLP.py:159-196) keeping the layer inputs a_0..a_{L-1} for mlp_backward_.  a1: the first
    hidden layer's activations computed elsewhere (the one-hot gather, g2048_onehot_layer1); then x is not needed
    and a_0 is kept as None."""
    Ws, bs = params["W"], params["b"]
    if a1 is not None:
        acts, a, first = [None, a1], a1, 1
    else:
        acts = [x.to(torch.float32)]
        a, first = acts[0], 0
    for i in range(first, len(Ws)):
        if i < len(Ws) - 1 and activation_mode == "ReLU" and a.dim() == 2:
            a = torch._addmm_activation(bs[i], a, Ws[i], use_gelu=False)   # bias + ReLU in the GEMM epilogue
            acts.append(a)
            continue
        z = torch.addmm(bs[i], a, Ws[i])
        if i < len(Ws) - 1:
            a = apply_activation(z, activation_mode)
            acts.append(a)
        else:
            a = z
    return a, acts


def mlp_backward_(params: dict[str, list[torch.Tensor]], acts: list[torch.Tensor], activation_mode: str,
                  grad_out: torch.Tensor, grad_W: list[torch.Tensor], grad_b: list[torch.Tensor],
                  first_layer_grad=None) -> None:
    """The manual backprop of src/reinforce_agent.py:_backpropagation (:639-678) and _activation_derivative
    (:624-636) for a whole batch at once: given the kept layer inputs (mlp_forward_kept) and dL/d(output) =
    grad_out [m, out], ACCUMULATE dL/dW_i = a_i^T d_i and dL/db_i = sum_rows d_i into grad_W / grad_b (tensors
    shaped like the params), with d_{i-1} = (d_i W_i^T) * act'(a_i); act' = 1[a > 0] (ReLU) or a (1 - a)
    (Sigmoid), computed from the kept activation.  first_layer_grad(d1): accumulates layer 0's weight and bias
    gradient from its delta instead (the one-hot scatter, g2048_onehot_dw1; acts[0] is then None)."""
    Ws = params["W"]
    d = grad_out
    for i in range(len(Ws) - 1, -1, -1):
        if i == 0 and first_layer_grad is not None:
            first_layer_grad(d)
            break
        _wgrad_(grad_W[i], acts[i], d)
        grad_b[i].add_(d.sum(0))
        if i > 0:
            h = acts[i]
            dh = d @ Ws[i].t()
            if activation_mode == "ReLU":
                d = torch.ops.aten.threshold_backward(dh, h, 0.0)   # dh * 1[h > 0] in one pass
            elif activation_mode == "Sigmoid":
                d = dh.mul_(h * (1.0 - h))
            else:
                raise ValueError(f"Unsupported activation: {activation_mode}")


def masked_logits(logits: torch.Tensor, action_mask: torch.Tensor | None) -> torch.Tensor:
    if action_mask is None:
        return logits
    return torch.where(action_mask.to(torch.bool), logits, torch.full_like(logits, -1e9))


def logits_to_probs(logits: torch.Tensor, action_mask: torch.Tensor | None = None) -> torch.Tensor:
    """src/MLP.py:139-156: where(mask, logits, -1e9), max-shifted softmax over the last axis."""
    z = masked_logits(logits, action_mask)
    e = torch.exp(z - z.max(dim=-1, keepdim=True).values)
    return e / e.sum(dim=-1, keepdim=True)
