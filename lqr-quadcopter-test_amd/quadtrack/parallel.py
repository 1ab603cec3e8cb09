"""Episode sharding across GPUs and the one metric exchange.

Episodes are independent, so a multi-GPU run is one process per GPU
(torch.distributed, backend "nccl" = RCCL over xGMI) that owns a contiguous
range of global episode indices; seeds and per-episode parameters are
functions of the global index, so results do not depend on the world size.
The only communication is at the end: the EvaluationSummary
(utils/metrics.py:341-390) reductions — the means and population stds in
numpy's own summation order (per-block pairwise sums, qt_summary_numpy,
gathered and folded in global block order), counts, and an all-gather of
each rank's best/worst episode for the first-occurrence argmax/argmin.
"""

from __future__ import annotations

import math

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
        std_on_target_ratio=math.sqrt(m2[0] / count), mean_tracking_error=mu_e,
        std_tracking_error=math.sqrt(m2[1] / count), mean_control_effort=sums[2] / count, best_episode_idx=best,
        worst_episode_idx=worst, meets_criteria=mu_r >= min_ratio)


def _gather_padded(t: torch.Tensor, group=None) -> list[torch.Tensor]:
    """all_gather of [r, c_rank] tensors whose column counts differ by rank
    (padded to the largest); returns each rank's tensor at its own width, on
    t's device."""
    c = torch.tensor([float(t.shape[1])], dtype=F64, device=t.device)
    widths = [int(v[0]) for v in all_gather_rows(c, group)]
    cmax = max(widths)
    pad = torch.zeros(t.shape[0], cmax, dtype=F64, device=t.device)
    pad[:, :t.shape[1]] = t
    src = pad.cpu() if dist.get_backend(group) == "gloo" else pad
    out = [torch.empty_like(src) for _ in widths]
    dist.all_gather(out, src, group=group)
    return [o[:, :w].to(t.device) for o, w in zip(out, widths)]


def _np_sums(met: torch.Tensor, pass_: int, mu_r: float, mu_e: float, group, use_dist: bool) -> list[float]:
    """np.add.reduce of this pass's rows over every rank's episodes, in global
    episode order (the shards tile the global range at multiples of the numpy
    block, checked by the caller): each rank's block sums, gathered in rank
    order, folded from 0.0."""
    from . import core

    blocks = core.summary_numpy_blocks(met, pass_, mu_r, mu_e)
    if use_dist:
        blocks = torch.cat(_gather_padded(blocks, group), dim=1)
    return [core.np_fold(row) for row in blocks.cpu().tolist()]


def _shard_layout(n: int, global_offset: int, device, group) -> list[tuple[int, int]]:
    """(global offset, episodes) of every rank, in rank order."""
    rows = all_gather_rows(torch.tensor([float(global_offset), float(n)], dtype=F64, device=device), group)
    return [(int(o), int(c)) for o, c in rows]


def summary_from_partials(met: torch.Tensor, criteria, group=None, distributed=True, global_offset: int = 0,
                          exact: bool = True):
    """EvaluationSummary of per-episode metric rows [MET_ROWS, n] on this rank
    (and, when torch.distributed is initialised, on every other rank).

    exact (default): means and stds in numpy's summation order
    (qt_summary_numpy), equal to the reference's np.mean / np.std
    (utils/metrics.py:380-384) bit for bit on the same per-episode metrics.
    When the ranks' shards do not start at multiples of numpy's 8,192-element
    block (in rank order), the metric rows are all-gathered first (one
    [MET_ROWS, N] copy per rank).  exact=False: the fixed-order tree sums of
    qt_summary_parts (~1e-15 relative from numpy's), three tiny collectives."""
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
    ext = p1[7:11].clone()
    if met.shape[1] == 0:
        ext = torch.tensor([float("-inf"), -1.0, float("inf"), -1.0], dtype=F64, device=met.device)
    else:
        ext[1] += global_offset
        ext[3] += global_offset
    parts = all_gather_rows(ext, group) if use_dist else [ext.cpu().tolist()]
    best, worst = pick_extremes(parts)
    if exact:
        src, np_dist = met, use_dist
        if use_dist:
            layout = _shard_layout(met.shape[1], global_offset, met.device, group)
            pos, tiled = 0, True
            for o, c in layout:
                tiled = tiled and o == pos and (c == 0 or pos % core.NP_BLOCK == 0)
                pos += c
            if not tiled:  # numpy's blocks straddle shards: reduce the whole array on every rank
                ordered = sorted(zip(layout, _gather_padded(met, group)), key=lambda z: z[0][0])
                src = torch.cat([m for _, m in ordered], dim=1).contiguous()
                np_dist = False
        s[0:3] = _np_sums(src, 0, 0.0, 0.0, group, np_dist)
        m2 = _np_sums(src, 1, s[0] / count, s[1] / count, group, np_dist)
    else:
        p2 = core.summary_partials(met, s[0] / count, s[1] / count)
        m2t = p2[5:7].clone()
        if use_dist:
            all_reduce_sum(m2t, group)
        m2 = m2t.cpu().tolist()
    return summary_from_stats(s, m2, best, worst, crit.min_on_target_ratio)


def reduce_summary(met: torch.Tensor, criteria, group=None, global_offset: int = 0):
    from .utils.metrics import SuccessCriteria

    c = SuccessCriteria(criteria.min_on_target_ratio, criteria.min_episode_duration, criteria.target_radius)
    return summary_from_partials(met, c, group=group, distributed=True, global_offset=global_offset)
