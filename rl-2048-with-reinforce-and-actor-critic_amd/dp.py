"""Data-parallel collectives of the update (one process per GPU, torch.distributed; "nccl" = RCCL on ROCm).

The env step needs no communication (boards are independent; each rank owns a contiguous global lane range).
Per update_batch the only exchanges are tiny except one:
  * episode totals  -> all-gather (global reward ranks, src/reinforce_agent.py:681-716)
  * baseline sums   -> all-reduce of 2 + 1 fp64 scalars ('batch' / 'batch_norm', :864-881)
  * gradients       -> ONE fused fp32 all-reduce of actor + critic gradients, before clipping (:558-561)
The fused buffer is 0.3-1.1 MB for the reference configs: latency-bound on xGMI, so a single bucket is the
right size (no bucketing / overlap needed at this size).  These helpers are device-agnostic (gloo on CPU in
the tests, RCCL on the GPUs).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def active(group=None) -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


def world(group=None) -> tuple[int, int]:
    if not active(group):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def all_reduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    if active(group):
        dist.all_reduce(t, group=group)
    return t


def gather_varlen(x: torch.Tensor, group=None) -> tuple[torch.Tensor, int]:
    """Concatenate a 1-D tensor of per-rank length across ranks (rank order).  Returns (all, my offset)."""
    if not active(group):
        return x, 0
    rank, ws = world(group)
    n = torch.tensor([x.numel()], dtype=torch.int64, device=x.device)
    sizes = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    padded = torch.zeros(max(sizes), dtype=x.dtype, device=x.device)
    padded[: x.numel()] = x
    parts = [torch.zeros_like(padded) for _ in range(ws)]
    dist.all_gather(parts, padded, group=group)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)]), sum(sizes[:rank])


def fused_all_reduce_(tensors: list[torch.Tensor], group=None) -> None:
    """Sum every tensor across ranks with one collective on a flat buffer (in place)."""
    if not active(group) or not tensors:
        return
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, group=group)
    off = 0
    for t in tensors:
        t.copy_(flat[off: off + t.numel()].view_as(t))
        off += t.numel()


def rank_weights(totals: torch.Tensor, conf, group=None) -> torch.Tensor:
    """_compute_episode_rank_weights (src/reinforce_agent.py:681-716) over the GLOBAL batch; returns this rank's
    slice.  Episode ranks come from a stable sort of the fp64 totals (the Python floats the reference sorts,
    :701); exact ties keep episode order, where the reference's default numpy sort leaves their order
    machine-dependent.  Weights are fp32 as in the reference: conf[bin] / mean, the mean an fp32 division of the
    (exact) weight sum by n.  No host synchronisation."""
    n_local = totals.numel()
    if conf is None or len(conf) == 0:
        return torch.ones(n_local, dtype=torch.float32, device=totals.device)
    all_tot, offset = gather_varlen(totals.to(torch.float64), group)
    n = all_tot.numel()
    confs = torch.tensor(list(conf), dtype=torch.float32, device=totals.device)
    order = torch.argsort(all_tot, stable=True)
    ranks = torch.arange(n, device=totals.device, dtype=torch.float64)
    bins = torch.clamp(((ranks + 0.5) / n * len(conf)).to(torch.int64), max=len(conf) - 1)
    w = torch.empty(n, dtype=torch.float32, device=totals.device)
    w[order] = confs[bins]
    # np.mean of the fp32 weights: the sum of a few distinct conf values is exact in fp64, then one fp32 division
    mw = (w.double().sum().to(torch.float32) / torch.tensor(float(n), dtype=torch.float32, device=w.device))
    w = torch.where(mw > 1e-8, w / mw, w)
    return w[offset: offset + n_local].contiguous()


def weighted_stats(values: torch.Tensor, weights: torch.Tensor, group=None) -> tuple[float, float]:
    """_compute_weighted_stats (src/reinforce_agent.py:864-881) across ranks: two-pass, fp64 accumulation."""
    w = weights.double()
    v = values.double()
    sums = torch.stack([w.sum(), (w * v).sum()])
    all_reduce_sum_(sums, group)
    if float(sums[0]) < 1e-8:
        return 0.0, 1.0
    mean = sums[1] / sums[0]
    var_num = (w * (v - mean) ** 2).sum().reshape(1)
    all_reduce_sum_(var_num, group)
    return float(mean), float(torch.sqrt(var_num[0] / sums[0]))


def global_count(n_local: int, device, group=None) -> int:
    t = torch.tensor([n_local], dtype=torch.int64, device=device)
    all_reduce_sum_(t, group)
    return int(t.item())
