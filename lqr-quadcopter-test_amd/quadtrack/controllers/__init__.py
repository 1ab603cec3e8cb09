"""Controllers on the north-star path (reference controllers/__init__.py exports
the Riccati controller, its heuristic-LQR fallback and the plugin base)."""

from .base import ACTION_KEYS, DEFAULT_ACTION_LIMITS, ActionLimits, BaseController, validate_action
from .lqr import LQRController, heuristic_gains
from .riccati_lqr import (
    BatchedRiccatiLQR,
    RiccatiLQRController,
    build_augmented_lqi_system,
    build_linearized_system,
    solve_dare,
)

VALID_CONTROLLER_TYPES = ("lqr", "riccati_lqr", "lqi")

__all__ = [
    "ACTION_KEYS", "DEFAULT_ACTION_LIMITS", "ActionLimits", "BaseController", "validate_action", "LQRController",
    "heuristic_gains", "BatchedRiccatiLQR", "RiccatiLQRController", "build_augmented_lqi_system",
    "build_linearized_system", "solve_dare", "VALID_CONTROLLER_TYPES",
]
