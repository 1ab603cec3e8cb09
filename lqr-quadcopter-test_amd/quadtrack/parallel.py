"""Episode sharding across GPUs and the one metric exchange.

Episodes are independent, so a multi-GPU run is one process per GPU
(torch.distributed, backend "nccl" = RCCL over xGMI) that owns a contiguous
range of global episode indices; seeds and per-episode parameters are
functions of the global index, so results do not depend on the world size.
The only communication is at the end: the EvaluationSummary
(utils/metrics.py:341-390) reductions — sums for the means, a second centred
pass for the population std (np.std), and an all-gather of each rank's
best/worst episode for the first-occurrence argmax/argmin.
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from . import core

F64 = torch.float64


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) share of rank `rank` (earlier ranks take the remainder)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _dist_on(group) -> bool:
    return dist.is_available() and dist.is_initialized()


def _all_reduce(t: torch.Tensor, group, op=None):
    """all_reduce that works for nccl (device tensors) and gloo (host copies)."""
    op = op or dist.ReduceOp.SUM
    if dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t


def _all_gather(t: torch.Tensor, group) -> list[torch.Tensor]:
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        h = t.cpu()
        out = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(out, h, group=group)
        return out
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return out


def summary_from_partials(met: torch.Tensor, criteria, group=None, distributed=True, global_offset: int = 0):
    """EvaluationSummary from per-episode metric rows [MET_ROWS, n] on this
    rank (and, when distributed, every other rank's)."""
    from .utils.metrics import EvaluationSummary, SuccessCriteria

    crit = criteria if criteria is not None else SuccessCriteria()
    min_ratio = crit.min_on_target_ratio
    use_dist = distributed and _dist_on(group)
    p1 = core.summary_partials(met)
    sums = p1[0:5].clone()
    if use_dist:
        _all_reduce(sums, group)
    s = sums.cpu().tolist()
    count = int(round(s[4]))
    if count == 0:
        return EvaluationSummary()
    mu_r, mu_e = s[0] / count, s[1] / count
    p2 = core.summary_partials(met, mu_r, mu_e)
    m2 = p2[5:7].clone()
    if use_dist:
        _all_reduce(m2, group)
    m2 = m2.cpu().tolist()
    ext = p1[7:11].clone()  # max, argmax, min, argmin (local indices)
    if met.shape[1] == 0:
        ext = torch.tensor([float("-inf"), -1.0, float("inf"), -1.0], dtype=F64, device=met.device)
    else:
        ext[1] += global_offset
        ext[3] += global_offset
    parts = [ext.cpu().tolist()]
    if use_dist:
        parts = [g.cpu().tolist() for g in _all_gather(ext, group)]
    best = max((p for p in parts if p[1] >= 0), key=lambda p: (p[0], -p[1]))
    worst = min((p for p in parts if p[3] >= 0), key=lambda p: (p[2], p[3]))
    succ = int(round(s[3]))
    return EvaluationSummary(
        total_episodes=count, successful_episodes=succ, success_rate=succ / count,
        mean_on_target_ratio=mu_r, std_on_target_ratio=(m2[0] / count) ** 0.5, mean_tracking_error=mu_e,
        std_tracking_error=(m2[1] / count) ** 0.5, mean_control_effort=s[2] / count,
        best_episode_idx=int(best[1]), worst_episode_idx=int(worst[3]), meets_criteria=mu_r >= min_ratio)


def reduce_summary(met: torch.Tensor, criteria, group=None, global_offset: int = 0):
    from .utils.metrics import SuccessCriteria

    c = SuccessCriteria(criteria.min_on_target_ratio, criteria.min_episode_duration, criteria.target_radius)
    return summary_from_partials(met, c, group=group, distributed=True, global_offset=global_offset)
