"""Controllers on the north-star path (reference controllers/__init__.py exports
the Riccati controller, its heuristic-LQR fallback and the plugin base)."""

from .base import ACTION_KEYS, DEFAULT_ACTION_LIMITS, ActionLimits, BaseController, validate_action
from .lqr import BatchedLQR, LQRController, heuristic_gains
from .pid import BatchedPID, PIDController
from .riccati_lqr import (
    BatchedRiccatiLQR,
    RiccatiLQRController,
    build_augmented_lqi_system,
    build_linearized_system,
    solve_dare,
)

VALID_CONTROLLER_TYPES = ("lqr", "pid", "riccati_lqr", "lqi")


def batched_controller(controller_type: str = "riccati_lqr", config: dict | None = None, device=None, **per_episode):
    """Batched gains for the fused closed loop by controller type (the
    batched counterpart of eval.load_controller, eval.py:472-513):
    "riccati_lqr" / "lqi" -> BatchedRiccatiLQR, "lqr" -> BatchedLQR (heuristic
    gains), "pid" -> BatchedPID.  Per-episode arrays go to the constructor."""
    config = dict(config or {})
    if controller_type == "lqi":
        config["use_lqi"] = True
        config.setdefault("q_int", [0.01, 0.01, 0.1])
        controller_type = "riccati_lqr"
    cls = {"riccati_lqr": BatchedRiccatiLQR, "lqr": BatchedLQR, "pid": BatchedPID}.get(controller_type)
    if cls is None:
        raise ValueError(f"Unknown controller type: {controller_type}")
    return cls(config, device=device, **per_episode)

__all__ = [
    "ACTION_KEYS", "DEFAULT_ACTION_LIMITS", "ActionLimits", "BaseController", "validate_action", "LQRController",
    "BatchedLQR", "PIDController", "BatchedPID", "batched_controller", "heuristic_gains", "BatchedRiccatiLQR",
    "RiccatiLQRController", "build_augmented_lqi_system", "build_linearized_system", "solve_dare",
    "VALID_CONTROLLER_TYPES",
]
