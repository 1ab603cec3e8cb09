"""Metric reductions (reference utils/metrics.py)."""

from .metrics import (
    EpisodeMetrics,
    EvaluationSummary,
    SuccessCriteria,
    compute_control_effort,
    compute_episode_metrics,
    compute_evaluation_summary,
    compute_on_target_ratio,
    compute_tracking_error,
    detect_overshoots,
    format_metrics_report,
)

__all__ = ["EpisodeMetrics", "EvaluationSummary", "SuccessCriteria", "compute_control_effort",
           "compute_episode_metrics", "compute_evaluation_summary", "compute_on_target_ratio",
           "compute_tracking_error", "detect_overshoots", "format_metrics_report"]
