"""Controller plugin interface — drop-in for the reference's
`quadcopter_tracking.controllers.base` (controllers/base.py:1-135).

Action schema: {"thrust", "roll_rate", "pitch_rate", "yaw_rate"}; ENU sign
conventions (+pitch_rate -> +x, +roll_rate -> -y, +thrust -> +z).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

ACTION_KEYS = ("thrust", "roll_rate", "pitch_rate", "yaw_rate")


@dataclass
class ActionLimits:
    """Default output limits shared by the controllers (base.py:31-56)."""

    min_thrust: float = 0.0
    max_thrust: float = 20.0
    max_rate: float = 3.0

    def clip_action(self, action: dict) -> dict:
        lo = {"thrust": self.min_thrust}
        hi = {"thrust": self.max_thrust}
        return {k: np.clip(action[k], lo.get(k, -self.max_rate), hi.get(k, self.max_rate)) for k in ACTION_KEYS}


DEFAULT_ACTION_LIMITS = ActionLimits()


def validate_action(action: dict) -> None:
    """Raise KeyError / TypeError for a malformed action dict (base.py:63-80)."""
    for key in ACTION_KEYS:
        if key not in action:
            raise KeyError(f"Action missing required key: '{key}'")
        if not isinstance(action[key], (int, float)):
            raise TypeError(f"Action['{key}'] must be numeric, got {type(action[key]).__name__}")


class BaseController:
    """Controller base class (base.py:83-135): subclasses implement compute_action."""

    def __init__(self, name: str = "base", config: dict | None = None, mass: float = 1.0, gravity: float = 9.81):
        self.name = name
        self.config = config or {}
        self.mass = mass
        self.gravity = gravity

    def compute_action(self, observation: dict) -> dict:
        raise NotImplementedError("Subclasses must implement compute_action")

    def reset(self) -> None:
        pass
