"""Evaluation metrics — drop-in for the reference's
`quadcopter_tracking.utils.metrics` (utils/metrics.py:1-433).

Dataclasses and report text keep the reference's fields and layout.  The
reductions run in the HIP metrics kernel (`qt_metrics_from_arrays`): every
list-based helper lays its arrays out as [steps][xyz][episodes] and lets one
lane stream one episode, exactly the accumulation the fused rollout kernel
does in-register (quadtrack.rollout).
"""

from __future__ import annotations

import logging
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import _abi, core
from .._abi import MET, TERM_REASONS

logger = logging.getLogger(__name__)
F64 = torch.float64


@dataclass
class SuccessCriteria:
    min_on_target_ratio: float = 0.8
    min_episode_duration: float = 30.0
    target_radius: float = 0.5


@dataclass
class EpisodeMetrics:
    episode_duration: float = 0.0
    on_target_ratio: float = 0.0
    mean_tracking_error: float = 0.0
    max_tracking_error: float = 0.0
    rms_tracking_error: float = 0.0
    total_control_effort: float = 0.0
    mean_control_effort: float = 0.0
    overshoot_count: int = 0
    max_overshoot: float = 0.0
    success: bool = False
    termination_reason: str = ""
    action_violations: int = 0

    def to_dict(self) -> dict:
        return {k: getattr(self, k) for k in self.__dataclass_fields__}


@dataclass
class EvaluationSummary:
    total_episodes: int = 0
    successful_episodes: int = 0
    success_rate: float = 0.0
    mean_on_target_ratio: float = 0.0
    std_on_target_ratio: float = 0.0
    mean_tracking_error: float = 0.0
    std_tracking_error: float = 0.0
    mean_control_effort: float = 0.0
    best_episode_idx: int = 0
    worst_episode_idx: int = 0
    meets_criteria: bool = False
    episode_metrics: list[EpisodeMetrics] = field(default_factory=list)

    def to_dict(self) -> dict:
        d = {k: getattr(self, k) for k in self.__dataclass_fields__ if k != "episode_metrics"}
        d["episode_metrics"] = [m.to_dict() for m in self.episode_metrics]
        return d


def _crit(criteria: SuccessCriteria | None, window: int = 10):
    c = criteria or SuccessCriteria()
    return core.criteria(c.min_on_target_ratio, c.min_episode_duration, c.target_radius, window)


def _kernel_metrics(qpos, tpos, actions, last_time, crit) -> np.ndarray:
    """One episode per column: qpos/tpos [S, 3, n], actions [S, 4, n] (numpy)
    -> met [MET_ROWS, n] numpy, via qt_metrics_from_arrays."""
    dev = _abi.require_gpu()
    S, _, n = qpos.shape
    q = core.to_device(qpos, dev)
    t = core.to_device(tpos, dev)
    a = core.to_device(actions, dev)
    steps = torch.full((n,), S, dtype=torch.int32, device=dev)
    lt = core.to_device(np.broadcast_to(np.asarray(last_time, float), (n,)), dev)
    return core.metrics_from_arrays(crit, q, t, a, steps, lt).cpu().numpy()


def compute_tracking_error(quad_positions, target_positions) -> np.ndarray:
    """Per-step distance (metrics.py:144-162): each row is a one-step episode
    whose mean error is that row's distance."""
    qp, tp = np.asarray(quad_positions, dtype=np.float64), np.asarray(target_positions, dtype=np.float64)
    if qp.shape != tp.shape:
        raise ValueError(f"Shape mismatch: quad {qp.shape} vs target {tp.shape}")
    if qp.shape[0] == 0:
        return np.zeros(0)
    N = qp.shape[0]
    met = _kernel_metrics(qp.T[None], tp.T[None], np.zeros((1, 4, N)), 0.0, _crit(None))
    return met[MET["mean_tracking_error"]]


def _errors_as_episode(tracking_errors):
    e = np.asarray(tracking_errors, dtype=np.float64).reshape(-1)
    S = e.size
    qp = np.zeros((S, 3, 1))
    qp[:, 0, 0] = e  # distance of (e, 0, 0) from the origin is |e|
    return qp, np.zeros((S, 3, 1))


def compute_on_target_ratio(tracking_errors, target_radius: float) -> float:
    """Fraction of steps with error <= radius (metrics.py:165-179)."""
    if len(tracking_errors) == 0:
        return 0.0
    qp, tp = _errors_as_episode(tracking_errors)
    met = _kernel_metrics(qp, tp, np.zeros((qp.shape[0], 4, 1)), 0.0,
                          _crit(SuccessCriteria(target_radius=target_radius)))
    return float(met[MET["on_target_ratio"], 0])


def compute_control_effort(actions) -> tuple[float, float]:
    """(sum, mean) of per-step action norms (metrics.py:182-202)."""
    a = np.asarray(actions, dtype=np.float64)
    if len(a) == 0:
        return 0.0, 0.0
    S = a.shape[0]
    met = _kernel_metrics(np.zeros((S, 3, 1)), np.zeros((S, 3, 1)), a.reshape(S, 4, 1), 0.0, _crit(None))
    return float(met[MET["total_control_effort"], 0]), float(met[MET["mean_control_effort"], 0])


def detect_overshoots(tracking_errors, target_radius: float, window_size: int = 10) -> tuple[int, float]:
    """Overshoot state machine (metrics.py:205-261)."""
    if len(tracking_errors) < window_size:
        return 0, 0.0
    qp, tp = _errors_as_episode(tracking_errors)
    met = _kernel_metrics(qp, tp, np.zeros((qp.shape[0], 4, 1)), 0.0,
                          _crit(SuccessCriteria(target_radius=target_radius), window_size))
    return int(met[MET["overshoot_count"], 0]), float(met[MET["max_overshoot"], 0])


def compute_episode_metrics(episode_data: list[dict], criteria: SuccessCriteria | None = None,
                            episode_info: dict | None = None) -> EpisodeMetrics:
    """All metrics of one episode from its step records (metrics.py:264-338)."""
    if criteria is None:
        criteria = SuccessCriteria()
    if not episode_data:
        return EpisodeMetrics(success=False, termination_reason="no_data")
    qp = np.array([d["quadcopter_position"] for d in episode_data], dtype=np.float64)
    tp = np.array([d["target_position"] for d in episode_data], dtype=np.float64)
    ac = np.array([d["action"] for d in episode_data], dtype=np.float64)
    last_time = float(episode_data[-1]["time"])
    met = _kernel_metrics(qp[:, :, None], tp[:, :, None], ac[:, :, None], last_time, _crit(criteria))[:, 0]
    reason, viol = "", 0
    if episode_info:
        reason = episode_info.get("termination_reason", "")
        viol = episode_info.get("action_violations", 0)
    return EpisodeMetrics(
        episode_duration=float(met[MET["episode_duration"]]), on_target_ratio=float(met[MET["on_target_ratio"]]),
        mean_tracking_error=float(met[MET["mean_tracking_error"]]),
        max_tracking_error=float(met[MET["max_tracking_error"]]),
        rms_tracking_error=float(met[MET["rms_tracking_error"]]),
        total_control_effort=float(met[MET["total_control_effort"]]),
        mean_control_effort=float(met[MET["mean_control_effort"]]),
        overshoot_count=int(met[MET["overshoot_count"]]), max_overshoot=float(met[MET["max_overshoot"]]),
        success=bool(met[MET["success"]]), termination_reason=reason, action_violations=viol)


def metrics_matrix(episode_metrics_list: list[EpisodeMetrics]) -> torch.Tensor:
    """EpisodeMetrics list -> [MET_ROWS, n] device tensor (the rollout layout)."""
    dev = _abi.require_gpu()
    rows = np.zeros((_abi.MET_ROWS, len(episode_metrics_list)))
    for j, m in enumerate(episode_metrics_list):
        rows[MET["on_target_ratio"], j] = m.on_target_ratio
        rows[MET["mean_tracking_error"], j] = m.mean_tracking_error
        rows[MET["mean_control_effort"], j] = m.mean_control_effort
        rows[MET["success"], j] = float(bool(m.success))
    return core.to_device(rows, dev)


def compute_evaluation_summary(episode_metrics_list: list[EpisodeMetrics],
                               criteria: SuccessCriteria | None = None) -> EvaluationSummary:
    """Summary statistics over episodes (metrics.py:341-390) via qt_summary."""
    from ..parallel import summary_from_partials

    if criteria is None:
        criteria = SuccessCriteria()
    if not episode_metrics_list:
        return EvaluationSummary()
    met = metrics_matrix(episode_metrics_list)
    s = summary_from_partials(met, criteria, group=None, distributed=False)
    s.episode_metrics = list(episode_metrics_list)
    return s


def format_metrics_report(summary: EvaluationSummary) -> str:
    """Human-readable report, same layout as metrics.py:393-433."""
    em = summary.episode_metrics

    def ep_line(label, idx):
        if not em:
            return f"{label} Episode: N/A"
        return f"{label} Episode: #{idx + 1} ({em[idx].on_target_ratio:.1%} on-target)"

    lines = [
        "=" * 60, "EVALUATION SUMMARY", "=" * 60, "",
        f"Total Episodes: {summary.total_episodes}",
        f"Successful Episodes: {summary.successful_episodes}",
        f"Success Rate: {summary.success_rate:.1%}", "",
        "Tracking Performance:",
        f"  Mean On-Target Ratio: {summary.mean_on_target_ratio:.1%} (± {summary.std_on_target_ratio:.1%})",
        f"  Mean Tracking Error: {summary.mean_tracking_error:.3f}m (± {summary.std_tracking_error:.3f}m)",
        f"  Mean Control Effort: {summary.mean_control_effort:.3f}", "",
        ep_line("Best", summary.best_episode_idx), ep_line("Worst", summary.worst_episode_idx), "",
        f"SUCCESS CRITERIA MET: {'YES' if summary.meets_criteria else 'NO'}", "=" * 60,
    ]
    return "\n".join(lines)


__all__ = ["SuccessCriteria", "EpisodeMetrics", "EvaluationSummary", "compute_tracking_error",
           "compute_on_target_ratio", "compute_control_effort", "detect_overshoots", "compute_episode_metrics",
           "compute_evaluation_summary", "format_metrics_report", "TERM_REASONS"]
