"""Heuristic LQR controller — the DARE-failure fallback of the Riccati
controller (controllers/__init__.py:398-700 of the reference,
riccati_lqr.py:747-777).  Closed-form per-axis double-integrator gains
(`_compute_gains`, __init__.py:522-574); the control law runs in the same HIP
controller kernel as the Riccati controller (6-column K, no integral).
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _abi, core
from ..step import BatchedControlMixin
from .base import BaseController
from .riccati_lqr import _OneEpisodeKernel, _ensure_array, _obs15, _validate_observation, ctrl_params


def heuristic_gains(q_pos, q_vel, r_thrust, r_rate) -> np.ndarray:
    """K (4 x 6): z -> thrust, y -> -roll, x -> +pitch, no yaw row
    (`_compute_gains`, __init__.py:522-574).  Broadcasts: q_pos / q_vel [..., 3]
    and r_thrust / r_rate [...] give K [..., 4, 6]."""
    q_pos, q_vel = np.asarray(q_pos, float), np.asarray(q_vel, float)
    r_thrust, r_rate = np.asarray(r_thrust, float), np.asarray(r_rate, float)
    shape = np.broadcast_shapes(q_pos.shape[:-1], q_vel.shape[:-1], r_thrust.shape, r_rate.shape)
    K = np.zeros(shape + (4, 6))
    with np.errstate(invalid="ignore", divide="ignore"):
        K[..., 0, 2] = np.sqrt(q_pos[..., 2] / r_thrust)
        K[..., 0, 5] = np.sqrt(2 * np.sqrt(q_pos[..., 2] / r_thrust) + q_vel[..., 2] / r_thrust)
        K[..., 1, 1] = -np.sqrt(q_pos[..., 1] / r_rate)
        K[..., 1, 4] = -np.sqrt(2 * np.sqrt(q_pos[..., 1] / r_rate) + q_vel[..., 1] / r_rate)
        K[..., 2, 0] = np.sqrt(q_pos[..., 0] / r_rate)
        K[..., 2, 3] = np.sqrt(2 * np.sqrt(q_pos[..., 0] / r_rate) + q_vel[..., 0] / r_rate)
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

    def to_batched(self, device=None) -> "BatchedLQR":
        """Shared-gain batched view for the fused closed loop."""
        return BatchedLQR({**self.config, "K": self.K}, device=device or self._kernel.dev)


class BatchedLQR(BatchedControlMixin):
    """Heuristic-LQR gains (LQRController, __init__.py:398-700) for a batch of
    episodes, for the fused closed loop (6-column K, no integral).  Shared, or
    per episode when any of q_pos / q_vel [n, 3], r_thrust / r_rate [n],
    K [n, 4, 6] or mass [n] is given."""

    kind = "lqr"
    k_cols = 6
    use_lqi = False

    def __init__(self, config: dict | None = None, device=None, *, q_pos=None, q_vel=None, r_thrust=None,
                 r_rate=None, K=None, mass=None, ff_velocity_gain=None, ff_acceleration_gain=None):
        config = dict(config or {})
        self.config = config
        self.device = _abi.require_gpu(device)
        self.gravity = config.get("gravity", 9.81)
        base_mass = float(config.get("mass", 1.0))
        if isinstance(mass, torch.Tensor):
            mass = mass.detach().to("cpu", torch.float64).numpy()
        given = {k: v for k, v in (("q_pos", q_pos), ("q_vel", q_vel), ("r_thrust", r_thrust), ("r_rate", r_rate),
                                   ("K", K), ("mass", mass), ("ff_velocity_gain", ff_velocity_gain),
                                   ("ff_acceleration_gain", ff_acceleration_gain)) if v is not None}
        lens = {len(v) for v in given.values()}
        if len(lens) > 1:
            raise ValueError(f"per-episode arrays disagree on the episode count: {sorted(lens)}")
        m = lens.pop() if lens else 1
        self.per_episode = bool(given)
        self.num_problems = m
        if K is None and config.get("K") is not None:
            K = np.broadcast_to(np.asarray(config["K"], float), (m, 4, 6))
        if K is not None:
            Km = np.asarray(K, float)
            if Km.shape[-2:] != (4, 6):
                raise ValueError(f"K matrix must have shape (4, 6), got {Km.shape[-2:]}")
            Km = np.broadcast_to(Km, (m, 4, 6))
        else:
            pick = lambda v, key, default: np.broadcast_to(  # noqa: E731
                np.asarray(v if v is not None else config.get(key, default), float),
                (m, 3) if key in ("q_pos", "q_vel") else (m,))
            Km = heuristic_gains(pick(q_pos, "q_pos", [0.0001, 0.0001, 16.0]),
                                 pick(q_vel, "q_vel", [0.0036, 0.0036, 4.0]), pick(r_thrust, "r_thrust", 1.0),
                                 pick(r_rate, "r_rate", 1.0))
        self.K = torch.as_tensor(np.array(Km.reshape(m, 24).T, order="C"), dtype=torch.float64, device=self.device)
        self.k_structured = core.gains_structured(self.K, 6)
        self.mass = torch.as_tensor(np.broadcast_to(np.asarray(mass if mass is not None else base_mass, float),
                                                    (m,)).copy(), device=self.device)
        self.hover = (self.mass * self.gravity).contiguous() if mass is not None else None
        self.hover_thrust = base_mass * self.gravity
        self.ctrl = ctrl_params(0.01, self.hover_thrust, config.get("min_thrust", 0.0), config.get("max_thrust", 20.0),
                                config.get("max_rate", 3.0), False, config.get("feedforward_enabled", False), 0.0, 0.0,
                                config.get("ff_velocity_gain", [0.0, 0.0, 0.0]),
                                config.get("ff_acceleration_gain", [0.0, 0.0, 0.0]),
                                config.get("ff_max_velocity", 10.0), config.get("ff_max_acceleration", 5.0))
        self.status = torch.zeros(m, dtype=torch.int8, device=self.device)
        # per-episode feed-forward gains (qt_batch.ff): the tuner's ff ranges
        self.ff = None
        if ff_velocity_gain is not None or ff_acceleration_gain is not None:
            self.ff = core.ff_rows(
                m, self.device, True,
                ff_velocity_gain if ff_velocity_gain is not None else config.get("ff_velocity_gain", 0.0),
                ff_acceleration_gain if ff_acceleration_gain is not None else config.get("ff_acceleration_gain", 0.0),
                config.get("ff_max_velocity", 10.0))

    def gains(self) -> torch.Tensor:
        return self.K.T.reshape(-1, 4, 6)

    def repeat_episodes(self, k: int) -> "BatchedLQR":
        import copy

        out = copy.copy(self)
        if k == 1 and self.per_episode:
            return out
        rep = lambda t: None if t is None else t.repeat_interleave(k, dim=-1).contiguous()  # noqa: E731
        out.K, out.mass, out.hover, out.status = rep(self.K), rep(self.mass), rep(self.hover), rep(self.status)
        out.ff = rep(self.ff)
        out.num_problems = self.num_problems * k
        out.per_episode = True
        out.integral_state = None
        return out
