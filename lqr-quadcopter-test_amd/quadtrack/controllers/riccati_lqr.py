"""Riccati-LQR / LQI controller on MI355X — drop-in for the reference's
`quadcopter_tracking.controllers.riccati_lqr` (controllers/riccati_lqr.py).

* `RiccatiLQRController` keeps the reference's constructor keys, getters,
  exceptions and dict I/O (riccati_lqr.py:345-1086).  Its DARE runs in the
  batched SDA kernel (qt_dare_batched) and every `compute_action` runs the
  HIP controller kernel (qt_compute_action) on a one-episode batch.
* `BatchedRiccatiLQR` solves one DARE per episode (or one shared) on the GPU
  and drives the fused closed-loop kernel (quadtrack.rollout) or batched
  `compute_action` calls on tensors.
* `solve_dare`, `build_linearized_system`, `build_augmented_lqi_system`
  mirror riccati_lqr.py:119-316.
"""

from __future__ import annotations

import ctypes as C
import logging

import numpy as np
import torch

from .. import _abi, core
from .._abi import DARE_NO_CONVERGE, DARE_OK, DARE_Q_NOT_PSD, DARE_R_NOT_PD, CtrlParams
from ..step import BatchedControlMixin
from .base import BaseController

logger = logging.getLogger(__name__)

F64 = torch.float64
_DARE_MSG = {DARE_NO_CONVERGE: "no convergence of the doubling iteration",
             _abi.DARE_SINGULAR: "singular matrix in the doubling iteration"}


def _raise_for_status(st: int):
    """Map a qt_dare_status to the reference's exceptions (riccati_lqr.py:166-178)."""
    if st == DARE_Q_NOT_PSD:
        raise ValueError("Q matrix must be positive semi-definite")
    if st == DARE_R_NOT_PD:
        raise ValueError("R matrix must be positive definite")
    if st != DARE_OK:
        raise RuntimeError(f"DARE solver failed: {_DARE_MSG.get(st, st)}")


# --------------------------------------------------------------- model


def build_linearized_system(dt: float, mass: float = 1.0, gravity: float = 9.81) -> tuple[np.ndarray, np.ndarray]:
    """Discrete hover model x = [p, v], u = [thrust_delta, roll, pitch, yaw]
    (riccati_lqr.py:187-263): A = I + A_c dt, B = B_c dt."""
    A = np.eye(6)
    for i in range(3):
        A[i, 3 + i] = 1.0 * dt
    B = np.zeros((6, 4))
    B[5, 0] = (1.0 / mass) * dt
    B[4, 1] = -gravity * dt
    B[3, 2] = gravity * dt
    return A, B


def build_augmented_lqi_system(A: np.ndarray, B: np.ndarray, dt: float) -> tuple[np.ndarray, np.ndarray]:
    """Integral-augmented model (riccati_lqr.py:266-316): int_{k+1} = int_k + dt p_k."""
    n, m = A.shape[0], B.shape[1]
    A_aug = np.zeros((n + 3, n + 3))
    A_aug[:n, :n] = A
    A_aug[n:, :3] = np.eye(3) * dt
    A_aug[n:, n:] = np.eye(3)
    B_aug = np.zeros((n + 3, m))
    B_aug[:n, :] = B
    return A_aug, B_aug


def _diag_rows(v, k: int, m: int, device) -> torch.Tensor:
    """Diagonal weights -> [k, m] float64 on device: a shared k-vector is
    broadcast on the device, per-episode [m, k] values are copied once."""
    if isinstance(v, torch.Tensor):  # device draws (workloads.tuner_candidate_tensors) stay on the device
        t = v.detach().to(device=device, dtype=torch.float64)
        return t.reshape(k, 1).expand(k, m) if t.numel() == k else t.reshape(m, k).T
    a = np.asarray(v, dtype=np.float64)
    if a.size == k:
        return torch.as_tensor(a.reshape(k, 1).copy(), device=device).expand(k, m)
    return torch.as_tensor(np.array(np.broadcast_to(a, (m, k)).T, order="C"), device=device)


def _soa(mats: np.ndarray, device) -> torch.Tensor:
    """[m, r, c] -> [r*c, m] float64 on device."""
    mats = np.asarray(mats, dtype=np.float64)
    return torch.as_tensor(np.ascontiguousarray(mats.reshape(mats.shape[0], -1).T), device=device)


def solve_dare(A: np.ndarray, B: np.ndarray, Q: np.ndarray, R: np.ndarray, device=None):
    """Solve the DARE and return (P, K) (riccati_lqr.py:119-184), on the GPU.

    Raises ValueError for shape / definiteness problems and RuntimeError when
    the solver fails, like the reference."""
    A, B, Q, R = (np.asarray(x, dtype=np.float64) for x in (A, B, Q, R))
    n = A.shape[0]
    m = B.shape[1] if B.ndim == 2 else -1
    if A.shape != (n, n):
        raise ValueError(f"A must be square, got shape {A.shape}")
    if B.shape != (n, m):
        raise ValueError(f"B must have shape ({n}, m), got {B.shape}")
    if Q.shape != (n, n):
        raise ValueError(f"Q must have shape ({n}, {n}), got {Q.shape}")
    if R.shape != (m, m):
        raise ValueError(f"R must have shape ({m}, {m}), got {R.shape}")
    if n > 16 or m > 8:
        raise ValueError(f"device DARE supports n <= 16 states and m <= 8 inputs, got n={n}, m={m}")
    dev = _abi.require_gpu(device)
    K, P, status, _ = core.dare_dense(_soa(A[None], dev), _soa(B[None], dev), _soa(Q[None], dev),
                                      _soa(R[None], dev), ab_per_problem=False)
    _raise_for_status(int(status.item()))
    return P[:, 0].cpu().numpy().reshape(n, n), K[:, 0].cpu().numpy().reshape(m, n)


# ---------------------------------------------------------- config parsing


def _ensure_array(value, size: int = 3) -> np.ndarray:
    return np.array([value] * size) if np.isscalar(value) else np.array(value)


def _validate_q_int(q_int) -> np.ndarray:
    """riccati_lqr.py:553-600 (same messages)."""
    if np.isscalar(q_int):
        logger.info("Scalar q_int=%.4f coerced to [%.4f, %.4f, %.4f] for all axes", q_int, q_int, q_int, q_int)
        arr = np.array([q_int, q_int, q_int])
    else:
        arr = np.array(q_int)
    if len(arr) != 3:
        raise ValueError(
            f"q_int must have exactly 3 elements (one per position axis x, y, z), got {len(arr)} elements. "
            f"Provide a 3-element list like [0.01, 0.01, 0.1] or a scalar.")
    if np.any(arr < 0):
        bad = [f"{'xyz'[i]}={arr[i]:.4f}" for i in np.where(arr < 0)[0]]
        raise ValueError(f"q_int weights must be non-negative, but got negative values for: {', '.join(bad)}. "
                         f"Use positive weights or zero to disable integral action on an axis.")
    return arr


def _build_Q(config: dict, use_lqi: bool, q_int: np.ndarray) -> np.ndarray:
    """riccati_lqr.py:602-672."""
    if config.get("Q") is not None:
        Q = np.array(config["Q"])
        if use_lqi:
            if Q.shape == (9, 9):
                return Q
            if Q.shape == (6, 6):
                Qa = np.zeros((9, 9))
                Qa[:6, :6] = Q
                Qa[6:, 6:] = np.diag(q_int)
                return Qa
            raise ValueError(f"Q matrix for LQI must have shape (9, 9) or (6, 6), got {Q.shape}")
        if Q.shape != (6, 6):
            raise ValueError(f"Q matrix must have shape (6, 6), got {Q.shape}")
        return Q
    q_pos = np.array(config.get("q_pos", [0.0001, 0.0001, 16.0]))
    q_vel = np.array(config.get("q_vel", [0.0036, 0.0036, 4.0]))
    if len(q_pos) != 3:
        raise ValueError(f"q_pos must have 3 elements, got {len(q_pos)}")
    if len(q_vel) != 3:
        raise ValueError(f"q_vel must have 3 elements, got {len(q_vel)}")
    return np.diag(np.concatenate([q_pos, q_vel, q_int] if use_lqi else [q_pos, q_vel]))


def _build_R(config: dict) -> np.ndarray:
    """riccati_lqr.py:674-700."""
    if config.get("R") is not None:
        R = np.array(config["R"])
        if R.shape != (4, 4):
            raise ValueError(f"R matrix must have shape (4, 4), got {R.shape}")
        return R
    r = np.array(config.get("r_controls", [1.0, 1.0, 1.0, 1.0]))
    if len(r) != 4:
        raise ValueError(f"r_controls must have 4 elements, got {len(r)}")
    return np.diag(r)


def _is_diag(M: np.ndarray) -> bool:
    return bool(np.all(M == np.diag(np.diag(M))))


def ctrl_params(dt, hover_thrust, min_thrust, max_thrust, max_rate, use_lqi, feedforward_enabled, integral_limit,
                integral_zero_threshold, ff_velocity_gain, ff_acceleration_gain, ff_max_velocity,
                ff_max_acceleration) -> CtrlParams:
    c = CtrlParams()
    c.dt, c.hover_thrust = float(dt), float(hover_thrust)
    c.min_thrust, c.max_thrust, c.max_rate = float(min_thrust), float(max_thrust), float(max_rate)
    c.use_lqi, c.feedforward_enabled = int(bool(use_lqi)), int(bool(feedforward_enabled))
    c.integral_limit, c.integral_zero_threshold = float(integral_limit), float(integral_zero_threshold)
    fv, fa = _ensure_array(ff_velocity_gain), _ensure_array(ff_acceleration_gain)
    for i in range(3):
        c.ff_velocity_gain[i] = float(fv[i])
        c.ff_acceleration_gain[i] = float(fa[i])
    c.ff_max_velocity, c.ff_max_acceleration = float(ff_max_velocity), float(ff_max_acceleration)
    return c


def _validate_observation(observation: dict) -> None:
    """riccati_lqr.py:319-342."""
    for key in ("quadcopter", "target"):
        if key not in observation:
            raise KeyError(f"Observation missing required key: '{key}'")
    for key in ("position", "velocity", "attitude", "angular_velocity"):
        if key not in observation["quadcopter"]:
            raise KeyError(f"Observation['quadcopter'] missing required key: '{key}'")
    for key in ("position", "velocity"):
        if key not in observation["target"]:
            raise KeyError(f"Observation['target'] missing required key: '{key}'")


class _OneEpisodeKernel:
    """qt_compute_action on one observation, its inputs and outputs in mapped
    page-locked host memory (core.MappedBlock): a call is one launch and one
    stream sync, no copies; the gains stay in device memory.
    Output row: action (4) | integral (3 LQR/LQI; 4 PID: integral error + last
    observation time) | diagnostics (16; 18 PID: p, i, d, ff terms, total
    correction) | saturation flag."""

    def __init__(self, K: np.ndarray, k_cols: int, device):
        self.dev = _abi.require_gpu(device)
        self.k_cols = k_cols
        self.ni, self.nd = (4, 18) if k_cols == 3 else (3, 16)
        self.K = torch.as_tensor(np.ascontiguousarray(K[:, :k_cols].reshape(-1, 1)), dtype=F64, device=self.dev)
        blk = self._blk = core.MappedBlock(1024)
        self.buf, buf_d = blk.take(4 + self.ni + self.nd + 1)
        self.obs, self.obs_d = blk.take(16)
        self.sat, self.sat_d = blk.take(1, np.int8)
        self.act_d = buf_d
        self.integ_d = C.c_void_p(buf_d.value + 4 * 8)
        self.diag_d = C.c_void_p(buf_d.value + (4 + self.ni) * 8)
        self.batch = _abi.Batch()
        self.batch.n, self.batch.K, self.batch.k_cols = 1, _abi.ptr(self.K), k_cols

    def zero_integral(self):
        self.buf[4:7] = 0.0

    def __call__(self, ctrl: CtrlParams, obs: np.ndarray, integ: np.ndarray | None = None):
        no = obs.size
        self.obs[:no] = obs
        if integ is not None:
            self.buf[4:4 + self.ni] = integ
        s = _abi.stream_of(self.dev)
        _abi.check(_abi.load().qt_compute_action(C.byref(ctrl), C.byref(self.batch), self.obs_d, self.integ_d,
                                                 self.act_d, self.sat_d, self.diag_d, s), "qt_compute_action")
        core.sync(s)
        self.buf[-1] = float(self.sat[0])
        return self.buf.copy()


def _obs15(observation: dict) -> np.ndarray:
    q, t = observation["quadcopter"], observation["target"]
    acc = t.get("acceleration", None)
    return np.concatenate([np.asarray(q["position"], float), np.asarray(q["velocity"], float),
                           np.asarray(t["position"], float), np.asarray(t["velocity"], float),
                           np.zeros(3) if acc is None else np.asarray(acc, float)])


# -------------------------------------------------------- drop-in controller


class RiccatiLQRController(BaseController):
    """Riccati-LQR / LQI controller (riccati_lqr.py:345-1086), GPU-backed."""

    def __init__(self, config: dict | None = None, device=None):
        config = config or {}
        mass = config.get("mass", 1.0)
        gravity = config.get("gravity", 9.81)
        self.dt = config.get("dt", 0.01)
        super().__init__(name="riccati_lqr", config=config, mass=mass, gravity=gravity)
        self.device = device
        self.max_thrust = config.get("max_thrust", 20.0)
        self.min_thrust = config.get("min_thrust", 0.0)
        self.max_rate = config.get("max_rate", 3.0)
        self.hover_thrust = self.mass * self.gravity
        self.use_lqi = config.get("use_lqi", False)
        self.q_int = _validate_q_int(config.get("q_int", [0.0, 0.0, 0.0]))
        self.integral_limit = config.get("integral_limit", 10.0)
        self.integral_zero_threshold = config.get("integral_zero_threshold", 0.01)
        self.integral_state: np.ndarray | None = np.zeros(3) if self.use_lqi else None
        self.K_pd: np.ndarray | None = None
        self.K_i: np.ndarray | None = None
        self.feedforward_enabled = config.get("feedforward_enabled", False)
        self.ff_velocity_gain = _ensure_array(config.get("ff_velocity_gain", [0.0, 0.0, 0.0]))
        self.ff_acceleration_gain = _ensure_array(config.get("ff_acceleration_gain", [0.0, 0.0, 0.0]))
        self.ff_max_velocity = config.get("ff_max_velocity", 10.0)
        self.ff_max_acceleration = config.get("ff_max_acceleration", 5.0)
        self._saturation_count = 0
        self.A, self.B = build_linearized_system(dt=self.dt, mass=self.mass, gravity=self.gravity)
        self.A_aug: np.ndarray | None = None
        self.B_aug: np.ndarray | None = None
        if self.use_lqi:
            self.A_aug, self.B_aug = build_augmented_lqi_system(self.A, self.B, self.dt)
        self.Q = _build_Q(config, self.use_lqi, self.q_int)
        self.R = _build_R(config)
        self.fallback_on_failure = config.get("fallback_on_failure", True)
        self.fallback_controller = None
        self._using_fallback = False
        self.P = None
        self.K = None
        self.dare_iterations = 0
        self._solve_riccati()
        self.last_control_components: dict | None = None
        self._kernel = None
        self._ctrl = None
        if not self._using_fallback:
            k_cols = 9 if self.use_lqi else 6
            self._kernel = _OneEpisodeKernel(self.K, k_cols, device)
            self._ctrl = ctrl_params(self.dt, self.hover_thrust, self.min_thrust, self.max_thrust, self.max_rate,
                                     self.use_lqi, self.feedforward_enabled, self.integral_limit,
                                     self.integral_zero_threshold, self.ff_velocity_gain, self.ff_acceleration_gain,
                                     self.ff_max_velocity, self.ff_max_acceleration)

    # -- gain solve (riccati_lqr.py:702-777)
    def _solve_riccati(self) -> None:
        n = 9 if self.use_lqi else 6
        try:
            if self.Q.shape != (n, n):
                raise ValueError(f"Q must have shape ({n}, {n}), got {self.Q.shape}")
            dev = _abi.require_gpu(self.device)
            structured = _is_diag(self.Q) and _is_diag(self.R)
            K, P, status, iters = core.dare_batched(n, self.dt, self.gravity,
                                                    torch.tensor([float(self.mass)], dtype=F64, device=dev),
                                                    _soa(self.Q[None], dev), _soa(self.R[None], dev), structured)
            _raise_for_status(int(status.item()))
            self.K = K[:, 0].cpu().numpy().reshape(4, n)
            self.P = P[:, 0].cpu().numpy().reshape(n, n)
            self.dare_iterations = int(iters.item())
            if self.use_lqi:
                self.K_pd, self.K_i = self.K[:, :6], self.K[:, 6:]
            else:
                self.K_pd, self.K_i = self.K, np.zeros((4, 3))
            self._using_fallback = False
        except (ValueError, RuntimeError) as e:
            if isinstance(e, _abi.QuadtrackError):
                raise
            logger.warning("DARE solver failed: %s", e)
            if not self.fallback_on_failure:
                raise
            logger.warning("Falling back to heuristic LQR controller")
            self._create_fallback_controller()
            self._using_fallback = True

    def _create_fallback_controller(self) -> None:
        from .lqr import LQRController

        r_rate = (self.R[1, 1] + self.R[2, 2] + self.R[3, 3]) / 3
        self.fallback_controller = LQRController(config={
            "mass": self.mass, "gravity": self.gravity,
            "q_pos": [self.Q[0, 0], self.Q[1, 1], self.Q[2, 2]],
            "q_vel": [self.Q[3, 3], self.Q[4, 4], self.Q[5, 5]],
            "r_thrust": self.R[0, 0], "r_rate": r_rate,
            "max_thrust": self.max_thrust, "min_thrust": self.min_thrust, "max_rate": self.max_rate,
        }, device=self.device)

    # -- control law (riccati_lqr.py:779-967)
    def compute_action(self, observation: dict) -> dict:
        if self._using_fallback and self.fallback_controller is not None:
            return self.fallback_controller.compute_action(observation)
        _validate_observation(observation)
        out = self._kernel(self._ctrl, _obs15(observation))
        if self.use_lqi:
            self.integral_state = out[4:7].copy()
        sat = bool(out[23] != 0.0)
        if sat:
            self._saturation_count += 1
        d = out[7:23]
        self.last_control_components = {
            "state_error": d[0:6].copy(), "feedback_u": d[6:10].copy(), "ff_velocity_term": d[10:13].copy(),
            "ff_acceleration_term": d[13:16].copy(), "K_matrix": self.K.copy(), "is_saturated": sat,
        }
        if self.use_lqi:
            self.last_control_components["integral_state"] = self.integral_state.copy()
            self.last_control_components["K_pd"] = self.K_pd.copy()
            self.last_control_components["K_i"] = self.K_i.copy()
        return {"thrust": float(out[0]), "roll_rate": float(out[1]), "pitch_rate": float(out[2]),
                "yaw_rate": float(out[3])}

    # -- getters (riccati_lqr.py:969-1071)
    def get_control_components(self) -> dict | None:
        return self.last_control_components

    def get_saturation_count(self) -> int:
        return self._saturation_count

    def is_using_fallback(self) -> bool:
        return self._using_fallback

    def get_gain_matrix(self) -> np.ndarray | None:
        return self.K if not self._using_fallback else None

    def get_riccati_solution(self) -> np.ndarray | None:
        return self.P if not self._using_fallback else None

    def get_integral_gains(self) -> np.ndarray | None:
        return self.K_i if self.use_lqi and not self._using_fallback else None

    def get_pd_gains(self) -> np.ndarray | None:
        return self.K_pd if self.use_lqi and not self._using_fallback else None

    def get_integral_state(self) -> np.ndarray | None:
        if self.use_lqi and self.integral_state is not None:
            return self.integral_state.copy()
        return None

    def reset_integral_state(self) -> None:
        if self.use_lqi and self.integral_state is not None:
            self.integral_state = np.zeros(3)
            if self._kernel is not None:
                self._kernel.zero_integral()

    def is_lqi_mode(self) -> bool:
        return self.use_lqi

    def reset(self) -> None:
        self.last_control_components = None
        self._saturation_count = 0
        if self.use_lqi and self.integral_state is not None:
            self.integral_state = np.zeros(3)
            if self._kernel is not None:
                self._kernel.zero_integral()
        if self.fallback_controller is not None:
            self.fallback_controller.reset()

    # -- batched view of this controller (shared gains)
    def to_batched(self, device=None) -> "BatchedRiccatiLQR":
        return BatchedRiccatiLQR(self.config, device=device or self.device)


# ----------------------------------------------------------- batched gains


class BatchedRiccatiLQR(BatchedControlMixin):
    """Per-episode (or shared) Riccati-LQR / LQI gains on the GPU.

    `config` holds the shared options (the RiccatiLQRController keys).  Any of
    q_pos [n,3], q_vel [n,3], r_controls [n,4], q_int [n,3], mass [n], Q
    [n,k,k], R [n,4,4] given as per-episode arrays gives each episode its own
    DARE (batched SDA kernel) — the ControllerTuner candidate sweep
    (controllers/tuning.py:832-928) and per-episode masses (SURVEY §8d
    configs 4-5).  Failed problems fall back to the heuristic gains per
    episode (riccati_lqr.py:737-777) unless fallback_on_failure is False.
    """

    kind = "riccati_lqr"

    def __init__(self, config: dict | None = None, device=None, *, q_pos=None, q_vel=None, r_controls=None,
                 q_int=None, mass=None, Q=None, R=None, ff_velocity_gain=None, ff_acceleration_gain=None):
        config = dict(config or {})
        self.config = config
        self.device = _abi.require_gpu(device)
        dev = self.device
        self.dt = config.get("dt", 0.01)
        self.gravity = config.get("gravity", 9.81)
        self.use_lqi = bool(config.get("use_lqi", False))
        self.n_state = 9 if self.use_lqi else 6
        self.k_cols = self.n_state
        base_mass = float(config.get("mass", 1.0))
        per_arrays = (q_pos, q_vel, r_controls, q_int, mass, Q, R, ff_velocity_gain, ff_acceleration_gain)
        per = [a is not None for a in per_arrays]
        lens = [len(a) for a in per_arrays if a is not None]
        if lens and len(set(lens)) != 1:
            raise ValueError(f"per-episode arrays disagree on the episode count: {lens}")
        m = lens[0] if lens else 1
        self.per_episode = any(per)
        self.num_problems = m
        qi = _validate_q_int(config.get("q_int", [0.0, 0.0, 0.0]))
        n = self.n_state
        # shared full Q / R from the config (RiccatiLQRController's "Q" / "R" keys,
        # riccati_lqr.py:568-577, 637-641), unless per-episode arrays are given
        if Q is None and config.get("Q") is not None:
            Qs = _build_Q(config, self.use_lqi, qi).astype(float)
            Q = np.broadcast_to(Qs, (m,) + Qs.shape).copy()
        if R is None and config.get("R") is not None:
            R = np.broadcast_to(_build_R(config).astype(float), (m, 4, 4)).copy()
        if Q is None:
            # diagonal weights (every BASELINE config and the tuner's candidates):
            # the diagonals go to the device as [n, m] and the SoA matrices are
            # filled there, no [m, n, n] host arrays
            blocks = [(q_pos, config.get("q_pos", [1e-4, 1e-4, 16.0])),
                      (q_vel, config.get("q_vel", [0.0036, 0.0036, 4.0]))]
            if self.use_lqi:
                blocks.append((q_int, qi))
            Q_soa = torch.zeros(n * n, m, dtype=torch.float64, device=dev)
            q_diag = True
            for b, (per_ep, shared_v) in enumerate(blocks):
                d = _diag_rows(per_ep if per_ep is not None else shared_v, 3, m, dev)
                q_diag = q_diag and not bool(torch.isnan(d).any())  # as Q == Q * I judges a NaN: the dense solver
                Q_soa[torch.arange(3 * b, 3 * b + 3, device=dev) * (n + 1)] = d
        else:
            Qm = np.asarray(Q, float)
            if self.use_lqi and Qm.shape[1:] == (6, 6):
                Qa = np.zeros((m, 9, 9))
                Qa[:, :6, :6] = Qm
                Qa[:, 6:, 6:] = np.diag(qi)
                Qm = Qa
            if Qm.shape != (m, n, n):
                raise ValueError(f"per-episode Q / R must be [{m},{n},{n}] / [{m},4,4]")
            q_diag = bool(np.all(Qm == Qm * np.eye(n)))
            Q_soa = _soa(Qm, dev)
        if R is None:
            d = _diag_rows(r_controls if r_controls is not None else config.get("r_controls", [1.0] * 4), 4, m, dev)
            R_soa = torch.zeros(16, m, dtype=torch.float64, device=dev)
            R_soa[torch.arange(4, device=dev) * 5] = d
            r_diag = not bool(torch.isnan(d).any())
        else:
            Rm = np.asarray(R, float)
            if Rm.shape != (m, 4, 4):
                raise ValueError(f"per-episode Q / R must be [{m},{n},{n}] / [{m},4,4]")
            r_diag = bool(np.all(Rm == Rm * np.eye(4)))
            R_soa = _soa(Rm, dev)
        structured = q_diag and r_diag
        self.structured = structured
        if isinstance(mass, torch.Tensor):  # per-episode masses already on the device stay there
            self.mass = mass.detach().to(device=dev, dtype=torch.float64).reshape(m).contiguous()
        else:
            self.mass = torch.as_tensor(
                np.broadcast_to(np.asarray(mass if mass is not None else base_mass, float), (m,)).copy(), device=dev)
        self.K, self.P, self.status, self.iters = core.dare_batched(
            self.n_state, self.dt, self.gravity, self.mass, Q_soa, R_soa, structured)
        self.k_structured = core.gains_structured(self.K, self.k_cols)
        self.fallback_on_failure = config.get("fallback_on_failure", True)
        bad = self.status != DARE_OK
        if bool(bad.any()):
            first = int(torch.nonzero(bad)[0, 0])
            if not self.fallback_on_failure:
                _raise_for_status(int(self.status[first]))
            logger.warning("DARE failed for %d of %d problems; heuristic gains used there", int(bad.sum()), m)
        self.hover = (self.mass * self.gravity).contiguous() if mass is not None else None
        self.hover_thrust = base_mass * self.gravity
        self.ctrl = ctrl_params(self.dt, self.hover_thrust, config.get("min_thrust", 0.0),
                                config.get("max_thrust", 20.0), config.get("max_rate", 3.0), self.use_lqi,
                                config.get("feedforward_enabled", False), config.get("integral_limit", 10.0),
                                config.get("integral_zero_threshold", 0.01),
                                config.get("ff_velocity_gain", [0.0, 0.0, 0.0]),
                                config.get("ff_acceleration_gain", [0.0, 0.0, 0.0]),
                                config.get("ff_max_velocity", 10.0), config.get("ff_max_acceleration", 5.0))
        # Per-episode feed-forward (qt_batch.ff): per-candidate gains (the tuner's
        # ff ranges, controllers/tuning.py:689-735), and the heuristic fallback of a
        # failed DARE, which runs without feed-forward (riccati_lqr.py:764-776).
        ff_on = bool(config.get("feedforward_enabled", False)) or ff_velocity_gain is not None or \
            ff_acceleration_gain is not None
        self.ff = None
        if ff_on and (ff_velocity_gain is not None or ff_acceleration_gain is not None or bool(bad.any())):
            self.ff = core.ff_rows(
                m, dev, True,
                ff_velocity_gain if ff_velocity_gain is not None else config.get("ff_velocity_gain", [0.0] * 3),
                ff_acceleration_gain if ff_acceleration_gain is not None else
                config.get("ff_acceleration_gain", [0.0] * 3),
                config.get("ff_max_velocity", 10.0), off=bad.cpu().numpy())
        self.integral_state: torch.Tensor | None = None

    @property
    def using_fallback(self) -> torch.Tensor:
        return self.status != DARE_OK

    def gains(self) -> torch.Tensor:
        """K as [m, 4, k_cols]."""
        return self.K.T.reshape(-1, 4, self.k_cols)

    def riccati_solution(self) -> torch.Tensor:
        return self.P.T.reshape(-1, self.n_state, self.n_state)

    def repeat_episodes(self, k: int) -> "BatchedRiccatiLQR":
        """A view with every gain set used by k consecutive episodes (problem j
        -> episodes j*k .. j*k+k-1): the tuner's candidates x evaluation
        episodes (tuning.py:874-906) without re-solving any DARE."""
        import copy

        out = copy.copy(self)
        if k == 1 and self.per_episode:
            return out
        rep = lambda t: None if t is None else t.repeat_interleave(k, dim=-1).contiguous()  # noqa: E731
        out.K, out.P = rep(self.K), rep(self.P)
        out.status, out.iters, out.mass, out.hover = rep(self.status), rep(self.iters), rep(self.mass), rep(self.hover)
        out.ff = rep(self.ff)
        out.num_problems = self.num_problems * k
        out.per_episode = True
        out.integral_state = None
        return out

