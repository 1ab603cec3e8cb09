"""quadtrack — MI355X-native batched quadcopter-tracking hot path.

Drop-in for the closed-loop `RiccatiLQRController.compute_action` ->
`QuadcopterEnv.step` path of AgentFoundryExamples/lqr-quadcopter-test: the
same env / controller / metrics API (package `quadcopter_tracking` there),
backed by hand-written HIP kernels for gfx950 (libquadtrack.so, C ABI in
include/quadtrack.h), plus batched tensors APIs that run tens of thousands of
episodes per launch.  There is no CPU fallback: without the built library or
a visible GPU the numeric calls raise.
"""

from . import _abi
from .controllers import (
    BaseController,
    BatchedLQR,
    BatchedPID,
    BatchedRiccatiLQR,
    LQRController,
    PIDController,
    RiccatiLQRController,
    batched_controller,
    solve_dare,
)
from .env import BatchedQuadcopterEnv, EnvConfig, QuadcopterEnv, TargetMotion
from .eval import BatchedEvaluator, Evaluator, evaluate_batched, load_controller, run_hyperparameter_sweep
from .rollout import RolloutResult, run_closed_loop
from .utils import EpisodeMetrics, EvaluationSummary, SuccessCriteria, compute_episode_metrics

__version__ = "0.1.0"

__all__ = ["BaseController", "BatchedLQR", "BatchedPID", "BatchedRiccatiLQR", "LQRController", "PIDController",
           "RiccatiLQRController", "batched_controller", "solve_dare",
           "BatchedQuadcopterEnv", "EnvConfig", "QuadcopterEnv", "TargetMotion", "Evaluator", "BatchedEvaluator", "evaluate_batched",
           "load_controller", "run_hyperparameter_sweep", "RolloutResult", "run_closed_loop", "EpisodeMetrics", "EvaluationSummary",
           "SuccessCriteria", "compute_episode_metrics", "_abi"]
