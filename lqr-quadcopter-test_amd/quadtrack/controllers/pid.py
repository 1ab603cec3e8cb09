"""PID controller on MI355X — drop-in for the reference's `PIDController`
(controllers/__init__.py:116-396) and its batched form.

The control law runs in the HIP controller kernels: `qt_compute_action` with
k_cols = 3 (gains kp | ki | kd) for the one-episode drop-in, and the fused
closed-loop rollout for batches (`quadtrack.rollout.run_closed_loop`), where
the integral error and the last observation time live in the rollout state
(`integ[4][n]`).  The integral advances by pos_error * (t - t_last) only when
that step is positive and is clipped to +-integral_limit (default 0, i.e. no
integral action, 263-271); yaw rate is always 0.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _abi, core
from ..step import BatchedControlMixin
from .base import BaseController
from .riccati_lqr import _OneEpisodeKernel, _ensure_array, _obs15, _validate_observation, ctrl_params

F64 = torch.float64

_DEFAULT_KP = [0.01, 0.01, 4.0]
_DEFAULT_KI = [0.0, 0.0, 0.0]
_DEFAULT_KD = [0.06, 0.06, 2.0]


def _pid_ctrl(config: dict, hover_thrust: float):
    return ctrl_params(0.0, hover_thrust, config.get("min_thrust", 0.0), config.get("max_thrust", 20.0),
                       config.get("max_rate", 3.0), False, config.get("feedforward_enabled", False),
                       config.get("integral_limit", 0.0), 0.0, config.get("ff_velocity_gain", [0.0, 0.0, 0.0]),
                       config.get("ff_acceleration_gain", [0.0, 0.0, 0.0]), config.get("ff_max_velocity", 10.0),
                       config.get("ff_max_acceleration", 5.0))


class PIDController(BaseController):
    """PID position controller (controllers/__init__.py:116-396), GPU-backed.

    Same config keys (kp_pos/kp, ki_pos/ki, kd_pos/kd as scalars or 3-vectors,
    integral_limit, feedforward_*, ff_max_*, output limits, mass, gravity),
    attributes and `get_control_components()` terms."""

    def __init__(self, config: dict | None = None, device=None):
        config = config or {}
        super().__init__(name="pid", config=config, mass=config.get("mass", 1.0), gravity=config.get("gravity", 9.81))
        self.kp_pos = _ensure_array(config.get("kp_pos", config.get("kp", _DEFAULT_KP)))
        self.ki_pos = _ensure_array(config.get("ki_pos", config.get("ki", _DEFAULT_KI)))
        self.kd_pos = _ensure_array(config.get("kd_pos", config.get("kd", _DEFAULT_KD)))
        self.feedforward_enabled = config.get("feedforward_enabled", False)
        self.ff_velocity_gain = _ensure_array(config.get("ff_velocity_gain", [0.0, 0.0, 0.0]))
        self.ff_acceleration_gain = _ensure_array(config.get("ff_acceleration_gain", [0.0, 0.0, 0.0]))
        self.ff_max_velocity = config.get("ff_max_velocity", 10.0)
        self.ff_max_acceleration = config.get("ff_max_acceleration", 5.0)
        self.integral_limit = config.get("integral_limit", 0.0)
        self.max_thrust = config.get("max_thrust", 20.0)
        self.min_thrust = config.get("min_thrust", 0.0)
        self.max_rate = config.get("max_rate", 3.0)
        self.hover_thrust = self.mass * self.gravity
        self.integral_error = np.zeros(3)
        self._last_time: float | None = None
        self.last_control_components: dict | None = None
        gains = np.stack([self.kp_pos, self.ki_pos, self.kd_pos]).astype(float)
        self._kernel = _OneEpisodeKernel(gains, 3, device)
        self._ctrl = _pid_ctrl(config, self.hover_thrust)

    def compute_action(self, observation: dict) -> dict:
        _validate_observation(observation)
        now = float(observation.get("time", 0.0))
        integ = np.append(np.asarray(self.integral_error, float),
                          np.nan if self._last_time is None else float(self._last_time))
        out = self._kernel(self._ctrl, np.append(_obs15(observation), now), integ)
        self.integral_error = out[4:7].copy()
        self._last_time = now
        d = out[8:26]
        self.last_control_components = {
            "p_term": d[0:3].copy(), "i_term": d[3:6].copy(), "d_term": d[6:9].copy(),
            "ff_velocity_term": d[9:12].copy(), "ff_acceleration_term": d[12:15].copy(),
            "total_correction": d[15:18].copy(),
        }
        return {"thrust": float(out[0]), "roll_rate": float(out[1]), "pitch_rate": float(out[2]),
                "yaw_rate": float(out[3])}

    def get_control_components(self) -> dict | None:
        return self.last_control_components

    def reset(self) -> None:
        self.integral_error = np.zeros(3)
        self._last_time = None
        self.last_control_components = None

    def to_batched(self, device=None) -> "BatchedPID":
        return BatchedPID(self.config, device=device or self._kernel.dev)


class BatchedPID(BatchedControlMixin):
    """PID gains for a batch of episodes (shared, or per episode when any of
    kp_pos / ki_pos / kd_pos [n, 3] or mass [n] is given), for the fused
    closed loop.  Each episode starts from a fresh controller (integral 0,
    no previous observation time), as `reset()` leaves it (__init__.py:389-393)."""

    kind = "pid"
    k_cols = 3
    use_lqi = False
    k_structured = True

    def __init__(self, config: dict | None = None, device=None, *, kp_pos=None, ki_pos=None, kd_pos=None,
                 mass=None, ff_velocity_gain=None, ff_acceleration_gain=None):
        config = dict(config or {})
        self.config = config
        self.device = _abi.require_gpu(device)
        self.gravity = config.get("gravity", 9.81)
        base_mass = float(config.get("mass", 1.0))
        if isinstance(mass, torch.Tensor):
            mass = mass.detach().to("cpu", F64).numpy()
        given = {k: v for k, v in (("kp_pos", kp_pos), ("ki_pos", ki_pos), ("kd_pos", kd_pos), ("mass", mass),
                                   ("ff_velocity_gain", ff_velocity_gain),
                                   ("ff_acceleration_gain", ff_acceleration_gain)) if v is not None}
        lens = {len(v) for v in given.values()}
        if len(lens) > 1:
            raise ValueError(f"per-episode arrays disagree on the episode count: {sorted(lens)}")
        m = lens.pop() if lens else 1
        self.per_episode = bool(given)
        self.num_problems = m

        def gain(arr, key, alt, default):
            v = arr if arr is not None else _ensure_array(config.get(key, config.get(alt, default)))
            return np.broadcast_to(np.asarray(v, float), (m, 3))

        G = np.concatenate([gain(kp_pos, "kp_pos", "kp", _DEFAULT_KP), gain(ki_pos, "ki_pos", "ki", _DEFAULT_KI),
                            gain(kd_pos, "kd_pos", "kd", _DEFAULT_KD)], axis=1)  # [m, 9]
        self.K = torch.as_tensor(np.array(G.T, order="C"), dtype=F64, device=self.device)
        self.mass = torch.as_tensor(np.broadcast_to(np.asarray(mass if mass is not None else base_mass, float),
                                                    (m,)).copy(), device=self.device)
        self.hover = (self.mass * self.gravity).contiguous() if mass is not None else None
        self.hover_thrust = base_mass * self.gravity
        self.ctrl = _pid_ctrl(config, self.hover_thrust)
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
        """[m, 3, 3]: rows kp, ki, kd."""
        return self.K.T.reshape(-1, 3, 3)

    def repeat_episodes(self, k: int) -> "BatchedPID":
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
