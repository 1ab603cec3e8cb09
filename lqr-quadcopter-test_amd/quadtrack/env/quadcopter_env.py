"""Single-episode QuadcopterEnv on the GPU — drop-in for the reference's
`quadcopter_tracking.env.QuadcopterEnv` (env/quadcopter_env.py:45-667).

Same constructor, reset/step signatures, observation dict (fresh numpy
copies), info keys, exceptions, history and violation records.  The physics
(action validation, RK4/Euler, constraints, target, error, termination) runs
in the HIP reset / step kernels (qt_reset, qt_env_step) on a one-episode
state kept in mapped page-locked host memory (core.MappedBlock): a step is
one launch and one stream sync, with no copies; the host side keeps only the
reference's bookkeeping (counters, violation strings, history).
Seeding follows the reference exactly: the env and target streams are
`numpy.random.default_rng` generators re-created on a seeded reset and
continued on an unseeded one (quadcopter_env.py:108-139).
"""

from __future__ import annotations

import ctypes as C
import logging

import numpy as np

from .. import _abi, core
from .._abi import ACC_ON_POST, ACC_ROWS, ACC_STEPS, TERM_REASONS, Batch, State
from .config import EnvConfig, as_env_config
from .target_motion import TargetMotion

logger = logging.getLogger(__name__)


class QuadcopterEnv:
    POS_X, POS_Y, POS_Z = 0, 1, 2
    VEL_X, VEL_Y, VEL_Z = 3, 4, 5
    ROLL, PITCH, YAW = 6, 7, 8
    ROLL_RATE, PITCH_RATE, YAW_RATE = 9, 10, 11
    STATE_DIM = 12
    ACTION_DIM = 4

    def __init__(self, config: dict | EnvConfig | None = None, device=None):
        self.config = as_env_config(config)
        self.params = self.config.to_params()
        self.device = _abi.require_gpu(device)
        self.target = TargetMotion(params=self.config.target, seed=self.config.seed)
        # the one episode's arrays (qt_state / qt_batch with n = 1), mapped for the kernels
        blk = self._blk = core.MappedBlock(4096)
        self._x, x_d = blk.take(12)
        self._integ, integ_d = blk.take(core.INTEG_ROWS)
        self._t, t_d = blk.take(1)
        self._acc, acc_d = blk.take(ACC_ROWS)
        self._tg, tg_d = blk.take(9)
        self._pat, pat_d = blk.take(4)
        self._off, self._off_d = blk.take(3)
        self._act, self._act_d = blk.take(4)
        self._err, self._err_d = blk.take(1)
        self._flags, flags_d = blk.take(4, np.int8)  # on_target, done, term, violation
        self._flag_d = [C.c_void_p(flags_d.value + i) for i in range(4)]
        self._cstate = State(x_d, integ_d, t_d, acc_d, tg_d)
        self._cbatch = Batch()
        self._cbatch.n, self._cbatch.pattern, self._cbatch.k_cols = 1, pat_d, 6
        self._state_vector = np.zeros(self.STATE_DIM)
        self._target_obs = np.zeros(9)
        self._time = 0.0
        self._step_count = 0
        self._initialized = False
        self._history: list[dict] = []
        self._action_violations: list[dict] = []
        self._on_target_count = 0
        self._total_steps = 0
        self._rng = np.random.default_rng(self.config.seed)

    def _stream(self):
        return _abi.stream_of(self.device)

    # ----------------------------------------------------------------- reset
    def reset(self, seed: int | None = None) -> dict:
        if seed is not None:
            self._rng = np.random.default_rng(seed)
            self.target = TargetMotion(params=self.config.target, seed=seed)
        self.target.reset(seed=seed)
        self._off[:] = self._rng.uniform(-0.5, 0.5, 3)
        self._pat[:] = np.asarray(self.target.raw_draws, dtype=np.float64).reshape(4)
        lib, s = _abi.load(), self._stream()
        _abi.check(lib.qt_reset(C.byref(self.params), C.byref(self._cbatch), self._off_d, self._cstate, s), "qt_reset")
        core.sync(s)
        self._pull()
        self._time = 0.0
        self._step_count = 0
        self._on_target_count = 0
        self._total_steps = 0
        self._history = []
        self._action_violations = []
        self._initialized = True
        return self._get_observation()

    def _pull(self):
        self._state_vector = self._x.copy()
        self._target_obs = self._tg.copy()

    # ------------------------------------------------------------------ step
    def _parse_action(self, action) -> tuple[np.ndarray, list[str]]:
        """Parsing and the violation messages of _parse_and_validate_action
        (quadcopter_env.py:234-293); the clipping itself happens in the kernel."""
        if isinstance(action, dict):
            vec = np.array([action.get("thrust", 0.0), action.get("roll_rate", 0.0), action.get("pitch_rate", 0.0),
                            action.get("yaw_rate", 0.0)], dtype=np.float64)
        else:
            vec = np.asarray(action, dtype=np.float64)
            if vec.shape != (4,):
                raise ValueError(f"Action array must have shape (4,), got {vec.shape}")
        msgs = []
        v = vec
        if not np.all(np.isfinite(v)):
            msgs.append("Action contains NaN or Inf values")
            logger.warning("Action contains NaN or Inf, replacing with zeros")
            v = np.nan_to_num(v, nan=0.0, posinf=0.0, neginf=0.0)
        q = self.config.quadcopter
        if v[0] < q.min_thrust:
            msgs.append(f"Thrust {v[0]:.2f} below min {q.min_thrust:.2f}")
        elif v[0] > q.max_thrust:
            msgs.append(f"Thrust {v[0]:.2f} above max {q.max_thrust:.2f}")
        for i, name in enumerate(("roll_rate", "pitch_rate", "yaw_rate"), start=1):
            if abs(v[i]) > q.max_angular_rate:
                msgs.append(f"{name} {v[i]:.2f} exceeds limit {q.max_angular_rate:.2f}")
        return vec, msgs

    def step(self, action) -> tuple[dict, float, bool, dict]:
        if not self._initialized:
            raise RuntimeError("Environment not initialized. Call reset() first.")
        vec, violations = self._parse_action(action)
        if violations:
            self._action_violations.append({"step": self._step_count, "time": self._time, "violations": violations})
        self._act[:] = vec
        lib, s, f = _abi.load(), self._stream(), self._flag_d
        _abi.check(lib.qt_env_step(C.byref(self.params), C.byref(self._cbatch), self._act_d, self._cstate,
                                   self._err_d, f[0], f[1], f[2], f[3], s), "qt_env_step")
        core.sync(s)
        self._pull()
        self._time = float(self._t[0])
        err = float(self._err[0])
        term = int(self._flags[2])
        applied = self._applied_action(vec)
        self._step_count += 1
        self._total_steps += 1
        obs = self._get_observation()
        on = err <= self.config.success_criteria.target_radius
        if on:
            self._on_target_count += 1
        done = term != 0
        info = {
            "time": self._time,
            "step": self._step_count,
            "tracking_error": err,
            "on_target": on,
            "on_target_ratio": self._on_target_count / self._total_steps if self._total_steps > 0 else 0.0,
            "action_violations": len(self._action_violations),
        }
        if done:
            info["termination_reason"] = TERM_REASONS[term]
            info["episode_length"] = self._time
            info["success"] = self._evaluate_success()
        if self.config.logging.enabled:
            self._record_step(obs, applied, -err, info)
        return obs, -err, done, info

    def _applied_action(self, vec: np.ndarray) -> np.ndarray:
        q = self.config.quadcopter
        v = np.nan_to_num(vec, nan=0.0, posinf=0.0, neginf=0.0)
        v[0] = min(max(v[0], q.min_thrust), q.max_thrust)
        v[1:] = np.clip(v[1:], -q.max_angular_rate, q.max_angular_rate)
        return v

    def _evaluate_success(self) -> bool:
        """quadcopter_env.py:537-553"""
        if self._time < self.config.success_criteria.min_episode_duration:
            return False
        ratio = self._on_target_count / self._total_steps if self._total_steps > 0 else 0.0
        return ratio >= self.config.success_criteria.min_on_target_ratio

    def _record_step(self, observation, action, reward, info) -> None:
        if self._step_count % self.config.logging.log_interval == 0:
            self._history.append({
                "time": self._time, "step": self._step_count,
                "quadcopter_position": observation["quadcopter"]["position"].tolist(),
                "quadcopter_velocity": observation["quadcopter"]["velocity"].tolist(),
                "quadcopter_attitude": observation["quadcopter"]["attitude"].tolist(),
                "target_position": observation["target"]["position"].tolist(),
                "target_velocity": observation["target"]["velocity"].tolist(),
                "action": action.tolist(), "reward": reward, "tracking_error": info["tracking_error"],
                "on_target": info["on_target"],
            })

    # ----------------------------------------------------------- observation
    def _get_observation(self) -> dict:
        s, tg = self._state_vector, self._target_obs
        return {
            "quadcopter": {"position": s[0:3].copy(), "velocity": s[3:6].copy(), "attitude": s[6:9].copy(),
                           "angular_velocity": s[9:12].copy()},
            "target": {"position": tg[0:3].copy(), "velocity": tg[3:6].copy(), "acceleration": tg[6:9].copy()},
            "time": self._time,
        }

    def get_history(self) -> list[dict]:
        return self._history.copy()

    def get_action_violations(self) -> list[dict]:
        return self._action_violations.copy()

    def render(self, mode: str = "dict") -> dict | None:
        return self._get_observation() if mode == "dict" else None

    @property
    def state(self) -> dict:
        return self._get_observation()

    @property
    def time(self) -> float:
        return self._time

    @property
    def dt(self) -> float:
        return self.config.simulation.dt

    @property
    def is_initialized(self) -> bool:
        return self._initialized

    def get_state_vector(self) -> np.ndarray:
        return self._state_vector.copy()

    def set_state_vector(self, state: np.ndarray) -> None:
        if state.shape != (self.STATE_DIM,):
            raise ValueError(f"State must have shape ({self.STATE_DIM},), got {state.shape}")
        self._state_vector = state.copy()
        self._x[:] = state  # the kernels read the mapped state directly

    @staticmethod
    def hover_action(mass: float = 1.0, gravity: float = 9.81) -> dict:
        return {"thrust": mass * gravity, "roll_rate": 0.0, "pitch_rate": 0.0, "yaw_rate": 0.0}


__all__ = ["QuadcopterEnv", "ACC_ON_POST", "ACC_STEPS"]
