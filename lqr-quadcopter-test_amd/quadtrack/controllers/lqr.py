"""Heuristic LQR controller — the DARE-failure fallback of the Riccati
controller (controllers/__init__.py:398-700 of the reference,
riccati_lqr.py:747-777).  Closed-form per-axis double-integrator gains
(`_compute_gains`, __init__.py:522-574); the control law runs in the same HIP
controller kernel as the Riccati controller (6-column K, no integral).
"""

from __future__ import annotations

import numpy as np

from .base import BaseController
from .riccati_lqr import _OneEpisodeKernel, _ensure_array, _obs15, _validate_observation, ctrl_params


def heuristic_gains(q_pos, q_vel, r_thrust: float, r_rate: float) -> np.ndarray:
    """K (4 x 6): z -> thrust, y -> -roll, x -> +pitch, no yaw row."""
    q_pos, q_vel = np.asarray(q_pos, float), np.asarray(q_vel, float)
    K = np.zeros((4, 6))
    with np.errstate(invalid="ignore"):
        K[0, 2] = np.sqrt(q_pos[2] / r_thrust)
        K[0, 5] = np.sqrt(2 * np.sqrt(q_pos[2] / r_thrust) + q_vel[2] / r_thrust)
        K[1, 1] = -np.sqrt(q_pos[1] / r_rate)
        K[1, 4] = -np.sqrt(2 * np.sqrt(q_pos[1] / r_rate) + q_vel[1] / r_rate)
        K[2, 0] = np.sqrt(q_pos[0] / r_rate)
        K[2, 3] = np.sqrt(2 * np.sqrt(q_pos[0] / r_rate) + q_vel[0] / r_rate)
    return K


class LQRController(BaseController):
    def __init__(self, config: dict | None = None, device=None):
        config = config or {}
        super().__init__(name="lqr", config=config, mass=config.get("mass", 1.0), gravity=config.get("gravity", 9.81))
        self.max_thrust = config.get("max_thrust", 20.0)
        self.min_thrust = config.get("min_thrust", 0.0)
        self.max_rate = config.get("max_rate", 3.0)
        self.hover_thrust = self.mass * self.gravity
        self.feedforward_enabled = config.get("feedforward_enabled", False)
        self.ff_velocity_gain = _ensure_array(config.get("ff_velocity_gain", [0.0, 0.0, 0.0]))
        self.ff_acceleration_gain = _ensure_array(config.get("ff_acceleration_gain", [0.0, 0.0, 0.0]))
        self.ff_max_velocity = config.get("ff_max_velocity", 10.0)
        self.ff_max_acceleration = config.get("ff_max_acceleration", 5.0)
        self.last_control_components: dict | None = None
        if config.get("K") is not None:
            self.K = np.array(config["K"])
            if self.K.shape != (4, 6):
                raise ValueError(f"K matrix must have shape (4, 6), got {self.K.shape}")
        else:
            self.K = heuristic_gains(config.get("q_pos", [0.0001, 0.0001, 16.0]),
                                     config.get("q_vel", [0.0036, 0.0036, 4.0]),
                                     config.get("r_thrust", 1.0), config.get("r_rate", 1.0))
        self._kernel = _OneEpisodeKernel(self.K, 6, device)
        self._ctrl = ctrl_params(0.01, self.hover_thrust, self.min_thrust, self.max_thrust, self.max_rate, False,
                                 self.feedforward_enabled, 0.0, 0.0, self.ff_velocity_gain, self.ff_acceleration_gain,
                                 self.ff_max_velocity, self.ff_max_acceleration)

    def compute_action(self, observation: dict) -> dict:
        _validate_observation(observation)
        out = self._kernel(self._ctrl, _obs15(observation))
        d = out[7:23]
        self.last_control_components = {"feedback_u": d[6:10].copy(), "ff_velocity_term": d[10:13].copy(),
                                        "ff_acceleration_term": d[13:16].copy()}
        return {"thrust": float(out[0]), "roll_rate": float(out[1]), "pitch_rate": float(out[2]),
                "yaw_rate": float(out[3])}

    def get_control_components(self) -> dict | None:
        return self.last_control_components

    def reset(self) -> None:
        self.last_control_components = None
