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

F64 = torch.float64


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) share of rank `rank` (earlier ranks take the remainder)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def dist_on() -> bool:
    return dist.is_available() and dist.is_initialized()


def all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM all-reduce; nccl (RCCL) on device tensors, gloo via host copies."""
    if not dist_on():
        return t
    if dist.get_backend(group) == "gloo" and t.device.type != "cpu":
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)
    return t


def all_gather_rows(t: torch.Tensor, group=None) -> list[list[float]]:
    if not dist_on():
        return [t.cpu().tolist()]
    world = dist.get_world_size(group)
    src = t.cpu() if dist.get_backend(group) == "gloo" else t
    out = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(out, src, group=group)
    return [o.cpu().tolist() for o in out]


def pick_extremes(parts: list[list[float]]) -> tuple[int, int]:
    """First-occurrence argmax / argmin over ranks from [max, argmax, min, argmin]
    rows with GLOBAL indices (-1 = rank had no episodes)."""
    have_max = [p for p in parts if p[1] >= 0]
    have_min = [p for p in parts if p[3] >= 0]
    best = max(have_max, key=lambda p: (p[0], -p[1]))
    worst = min(have_min, key=lambda p: (p[2], p[3]))
    return int(best[1]), int(worst[3])


def summary_from_stats(sums: list[float], m2: list[float], best: int, worst: int, min_ratio: float):
    """EvaluationSummary from reduced statistics: sums = [sum ratio, sum err,
    sum effort, sum success, count], m2 = centred squares [ratio, err]."""
    from .utils.metrics import EvaluationSummary

    count = int(round(sums[4]))
    if count == 0:
        return EvaluationSummary()
    mu_r, mu_e = sums[0] / count, sums[1] / count
    succ = int(round(sums[3]))
    return EvaluationSummary(
        total_episodes=count, successful_episodes=succ, success_rate=succ / count, mean_on_target_ratio=mu_r,
        std_on_target_ratio=(m2[0] / count) ** 0.5, mean_tracking_error=mu_e,
        std_tracking_error=(m2[1] / count) ** 0.5, mean_control_effort=sums[2] / count, best_episode_idx=best,
        worst_episode_idx=worst, meets_criteria=mu_r >= min_ratio)


def summary_from_partials(met: torch.Tensor, criteria, group=None, distributed=True, global_offset: int = 0):
    """EvaluationSummary of per-episode metric rows [MET_ROWS, n] on this rank
    (and, when torch.distributed is initialised, on every other rank): two
    passes of the qt_summary kernel and three tiny collectives."""
    from . import core
    from .utils.metrics import EvaluationSummary, SuccessCriteria

    crit = criteria if criteria is not None else SuccessCriteria()
    use_dist = distributed and dist_on()
    p1 = core.summary_partials(met)
    sums = p1[0:5].clone()
    if use_dist:
        all_reduce_sum(sums, group)
    s = sums.cpu().tolist()
    count = int(round(s[4]))
    if count == 0:
        return EvaluationSummary()
    p2 = core.summary_partials(met, s[0] / count, s[1] / count)
    m2 = p2[5:7].clone()
    if use_dist:
        all_reduce_sum(m2, group)
    ext = p1[7:11].clone()
    if met.shape[1] == 0:
        ext = torch.tensor([float("-inf"), -1.0, float("inf"), -1.0], dtype=F64, device=met.device)
    else:
        ext[1] += global_offset
        ext[3] += global_offset
    parts = all_gather_rows(ext, group) if use_dist else [ext.cpu().tolist()]
    best, worst = pick_extremes(parts)
    return summary_from_stats(s, m2.cpu().tolist(), best, worst, crit.min_on_target_ratio)


def reduce_summary(met: torch.Tensor, criteria, group=None, global_offset: int = 0):
    from .utils.metrics import SuccessCriteria

    c = SuccessCriteria(criteria.min_on_target_ratio, criteria.min_episode_duration, criteria.target_radius)
    return summary_from_partials(met, c, group=group, distributed=True, global_offset=global_offset)
