"""Data-parallel collectives of the update (one process per GPU, torch.distributed; "nccl" = RCCL on ROCm).

The env step needs no communication (boards are independent; each rank owns a contiguous global lane range).
Per update_batch there is ONE gradient all-reduce, plus two tiny exchanges only where the configuration needs
global statistics before the gradient pass:
  * gradients       -> ONE fused fp32 all-reduce of actor + critic gradients and the episode count, before
                       clipping (src/reinforce_agent.py:558-561); the 1 / n_traj weight is applied after it
  * baseline sums   -> 'batch' / 'batch_norm' only: one all-reduce of 3 fp64 scalars (:864-881)
  * episode totals  -> reward_rank_weights only: an all-gather (global reward ranks, :681-716)
None of them synchronises the host when the caller passes the shard sizes of the global batch (``sizes``: the
episode count of every rank's shard, known to whoever sharded the batch -- shard_sizes()); without them
gather_varlen first exchanges the sizes, which costs one host synchronisation.  The fused buffer is 0.3-1.1 MB for
the reference configs: latency-bound on xGMI, so a single bucket is the right size (no bucketing / overlap needed
at this size).  These helpers are device-agnostic (gloo on CPU in the tests, RCCL on the GPUs).  Whenever a
process group is initialised -- world size 1 included -- the collectives run through it, so a one-rank RCCL group
exercises the device-backend path on one GPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def active(group=None) -> bool:
    """A process group is initialised (any world size): the collectives go through it."""
    return dist.is_available() and dist.is_initialized()


def world(group=None) -> tuple[int, int]:
    if not active(group):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def shard_bounds(n: int, rank: int, ws: int) -> tuple[int, int]:
    """Episodes [lo, hi) of rank `rank` when a global batch of n episodes is split into ws contiguous shards of
    ceil(n / ws) (the last ones shorter or empty)."""
    per = (n + ws - 1) // ws
    lo = min(rank * per, n)
    return lo, min(lo + per, n)


def shard_sizes(n: int, ws: int) -> tuple[int, ...]:
    """The episode count of every rank's shard (shard_bounds) -- host-known, so the collectives need no size
    exchange."""
    return tuple(hi - lo for lo, hi in (shard_bounds(n, r, ws) for r in range(ws)))


def all_reduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    if active(group):
        dist.all_reduce(t, group=group)
    return t


def gather_varlen(x: torch.Tensor, group=None, sizes=None) -> tuple[torch.Tensor, int]:
    """Concatenate a 1-D tensor of per-rank length across ranks (rank order).  Returns (all, my offset).
    sizes: every rank's length (host-known, e.g. shard_sizes) -- then no host synchronisation; None exchanges
    the lengths first (one all-gather read back on the host)."""
    if not active(group):
        return x, 0
    rank, ws = world(group)
    if sizes is None:
        n = torch.tensor([x.numel()], dtype=torch.int64, device=x.device)
        parts_n = [torch.zeros_like(n) for _ in range(ws)]
        dist.all_gather(parts_n, n, group=group)
        sizes = [int(s) for s in torch.cat(parts_n).tolist()]      # the one host synchronisation
    sizes = [int(s) for s in sizes]
    if len(sizes) != ws or sizes[rank] != x.numel():
        raise ValueError(f"gather_varlen: sizes {sizes} do not match world size {ws} / this rank's {x.numel()}")
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


def rank_weights(totals: torch.Tensor, conf, group=None, sizes=None) -> torch.Tensor:
    """_compute_episode_rank_weights (src/reinforce_agent.py:681-716) over the GLOBAL batch; returns this rank's
    slice.  Episode ranks come from a stable sort of the fp64 totals (the Python floats the reference sorts,
    :701); exact ties keep episode order, where the reference's default numpy sort leaves their order
    machine-dependent.  Weights are fp32 as in the reference: conf[bin] / mean, the mean an fp32 division of the
    (exact) weight sum by n.  No host synchronisation when `sizes` (every rank's episode count) is given."""
    n_local = totals.numel()
    if conf is None or len(conf) == 0:
        return torch.ones(n_local, dtype=torch.float32, device=totals.device)
    all_tot, offset = gather_varlen(totals.to(torch.float64), group, sizes)
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


def batch_mean_std(values: torch.Tensor, weights: torch.Tensor, group=None) -> tuple[torch.Tensor, torch.Tensor]:
    """_compute_weighted_stats (src/reinforce_agent.py:864-881) over the global batch: the fp64 sums
    [sum w, sum w v, sum w v^2] of every rank in ONE all-reduce, then mean and the (single-pass, fp64) weighted
    standard deviation as device scalars -- no host synchronisation.  sum w < 1e-8 gives (0, 1) like the
    reference.  (In fp64 the single-pass variance loses ~1e-16 (mu / sigma)^2 relative: far below the fp32 the
    reference computes these statistics in.)"""
    w = weights.double()
    v = values.double()
    sums = torch.stack([w.sum(), (w * v).sum(), (w * v * v).sum()])
    all_reduce_sum_(sums, group)
    ok = sums[0] >= 1e-8
    sw = torch.where(ok, sums[0], torch.ones_like(sums[0]))
    mean = sums[1] / sw
    var = torch.clamp(sums[2] / sw - mean * mean, min=0.0)
    return torch.where(ok, mean, torch.zeros_like(mean)), torch.where(ok, torch.sqrt(var), torch.ones_like(var))


# the episode count travels in the fp32 gradient buffer as base-2^16 digits: each digit sum is exact in fp32 for
# up to 256 ranks (256 * 65535 < 2^24), and counts up to 2^48 are representable
_COUNT_DIGITS = 3


def _count_digits(n: int) -> list[float]:
    n = int(n)
    if n < 0 or n >= 1 << (16 * _COUNT_DIGITS):
        raise ValueError(f"episode count {n} out of range")
    return [float((n >> (16 * d)) & 0xFFFF) for d in range(_COUNT_DIGITS)]


def reduce_gradients_(tensors: list[torch.Tensor], n_local: int, group=None) -> None:
    """Finish the gradients of update_batch across ranks with ONE collective: every rank accumulated its
    episodes' sum of rank_w / T_i-weighted per-step gradients; the flat fp32 buffer of all of them (actor +
    critic) plus this rank's episode count (as exact base-2^16 digits) is all-reduced, the global count is rebuilt
    exactly in fp64 on the device, and every gradient is multiplied by fp32(1 / count) -- the 1 / n_traj of
    src/reinforce_agent.py:467, :533 (n_traj = 8 n with augmentation).  No host synchronisation.  Without a process
    group: the same multiply by 1 / n_local, the Python scalar rounded to each tensor's own dtype (no host-to-device
    copy, no host sync)."""
    if not tensors:
        return
    if not active(group):
        inv = 1.0 / max(int(n_local), 1)
        for t in tensors:
            t.mul_(inv)
        return
    dev, dt = tensors[0].device, tensors[0].dtype
    flat = torch.cat([t.reshape(-1) for t in tensors] +
                     [torch.tensor(_count_digits(n_local), dtype=dt, device=dev)])
    dist.all_reduce(flat, group=group)
    digits = flat[-_COUNT_DIGITS:].double()
    scale = torch.tensor([float(1 << (16 * d)) for d in range(_COUNT_DIGITS)], dtype=torch.float64, device=dev)
    count = (digits * scale).sum().clamp(min=1.0)
    grads = flat[:-_COUNT_DIGITS]
    grads.mul_((1.0 / count).to(dt))
    off = 0
    for t in tensors:
        t.copy_(grads[off: off + t.numel()].view_as(t))
        off += t.numel()
