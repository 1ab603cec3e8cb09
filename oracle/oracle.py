"""ctypes front end of the CPU restatement (oracle/qt_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.  It carries its
own copy of the parameter schema (env/config.py:11-95 and
controllers/riccati_lqr.py:418-535 of the reference) so that it does not lean
on the code it checks.

Seeding: the reference draws its random episode parameters with
`numpy.random.default_rng(seed)` (env/quadcopter_env.py:122-137,
env/target_motion.py:285-353).  numpy is a dependency of the reference, not
the reference itself, and it is installed here and on the GPU box, so the
oracle uses numpy's own generator for the draws; tests/golden/rng_draws.npz
pins these draws against the reference's reset().
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libqt_oracle.so")

MOTIONS = ("stationary", "linear", "circular", "sinusoidal", "figure8")
MET_FIELDS = ("episode_duration", "on_target_ratio", "mean_tracking_error", "max_tracking_error",
              "rms_tracking_error", "total_control_effort", "mean_control_effort", "overshoot_count",
              "max_overshoot", "success", "termination_code", "action_violations",
              "env_on_target_ratio", "steps")
N_MET = len(MET_FIELDS)
DARE_STATUS = {1: "Q not PSD", 2: "R not PD", 3: "no convergence", 4: "singular"}


class EnvParams(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("mass", "gravity", "drag_linear", "drag_angular", "min_thrust",
                                           "max_thrust", "max_angular_rate", "dt", "max_episode_time",
                                           "max_velocity", "max_angular_velocity", "max_position")] + [
        ("integrator", C.c_int32), ("motion", C.c_int32)] + [
        (k, C.c_double) for k in ("speed", "amplitude", "frequency", "radius")] + [
        ("center", C.c_double * 3), ("max_acceleration", C.c_double)] + [
        (k, C.c_double) for k in ("target_radius", "min_on_target_ratio", "min_episode_duration")]


class CtrlParams(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("dt", "hover_thrust", "min_thrust", "max_thrust", "max_rate")] + [
        ("use_lqi", C.c_int32), ("feedforward_enabled", C.c_int32),
        ("integral_limit", C.c_double), ("integral_zero_threshold", C.c_double),
        ("ff_velocity_gain", C.c_double * 3), ("ff_acceleration_gain", C.c_double * 3),
        ("ff_max_velocity", C.c_double), ("ff_max_acceleration", C.c_double)]


class Criteria(C.Structure):
    _fields_ = [("min_on_target_ratio", C.c_double), ("min_episode_duration", C.c_double),
                ("target_radius", C.c_double), ("overshoot_window", C.c_int32), ("pad_", C.c_int32)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        dp = P(C.c_double)
        L.oq_target_state.argtypes = [P(EnvParams), C.c_int, dp, C.c_double, dp]
        L.oq_env_step.argtypes = [P(EnvParams), C.c_int, dp, C.c_double, dp, dp, dp, dp, dp, P(C.c_int)]
        L.oq_env_step.restype = C.c_int
        L.oq_compute_action.argtypes = [P(CtrlParams), dp, C.c_int, C.c_double, dp, dp, dp]
        L.oq_compute_action.restype = C.c_int
        L.oq_compute_action_pid.argtypes = [P(CtrlParams), dp, C.c_double, dp, dp, dp, dp]
        L.oq_episode.argtypes = [P(EnvParams), P(CtrlParams), P(Criteria), C.c_int, dp, C.c_double, C.c_double,
                                 dp, C.c_int, dp, C.c_int, dp, dp, dp, dp]
        L.oq_rollout.argtypes = [P(EnvParams), P(CtrlParams), P(Criteria), C.c_long, P(C.c_int8), dp, dp, dp,
                                 dp, C.c_int, C.c_long, dp, C.c_int, dp, dp, dp]
        L.oq_rollout.restype = C.c_int
        L.oq_build_system.argtypes = [C.c_int, C.c_double, C.c_double, C.c_double, dp, dp]
        L.oq_dare.argtypes = [C.c_int, dp, dp, dp, dp, dp, dp, C.c_int, C.c_double]
        L.oq_dare.restype = C.c_int
        L.oq_heuristic_gains.argtypes = [dp, dp, C.c_double, C.c_double, dp]
        L.oq_set_threads.argtypes = [C.c_int]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# ------------------------------------------------------------------ schema


def env_params(cfg: dict | None = None) -> EnvParams:
    """EnvConfig.from_dict defaults (reference env/config.py:97-173)."""
    cfg = cfg or {}
    q = cfg.get("quadcopter", {})
    s = dict(cfg.get("simulation", {}))
    t = cfg.get("target", {})
    sc = dict(cfg.get("success_criteria", {}))
    if "dt" in cfg and "dt" not in s:
        s["dt"] = cfg["dt"]
    if "episode_length" in cfg:
        s["max_episode_time"] = cfg["episode_length"]
    if "radius_requirement" in t:
        sc.setdefault("target_radius", t["radius_requirement"])
    e = EnvParams()
    e.mass = q.get("mass", 1.0)
    e.gravity = q.get("gravity", 9.81)
    e.drag_linear = q.get("drag_coeff_linear", 0.1)
    e.drag_angular = q.get("drag_coeff_angular", 0.01)
    e.min_thrust = q.get("min_thrust", 0.0)
    e.max_thrust = q.get("max_thrust", 20.0)
    e.max_angular_rate = q.get("max_angular_rate", 3.0)
    e.dt = s.get("dt", 0.01)
    e.max_episode_time = s.get("max_episode_time", 30.0)
    e.max_velocity = s.get("max_velocity", 50.0)
    e.max_angular_velocity = s.get("max_angular_velocity", 10.0)
    e.max_position = s.get("max_position", 1000.0)
    e.integrator = 1 if s.get("integrator", "rk4") == "euler" else 0
    e.motion = MOTIONS.index(t.get("motion_type", "stationary").lower())
    e.speed = t.get("speed", 1.0)
    e.amplitude = t.get("amplitude", 2.0)
    e.frequency = t.get("frequency", 0.5)
    e.radius = t.get("radius", 2.0)
    c = t.get("center", (0.0, 0.0, 1.0))
    for i in range(3):
        e.center[i] = c[i]
    e.max_acceleration = t.get("max_acceleration", 5.0)
    e.target_radius = sc.get("target_radius", 0.5)
    e.min_on_target_ratio = sc.get("min_on_target_ratio", 0.8)
    e.min_episode_duration = sc.get("min_episode_duration", 30.0)
    return e


def criteria(min_on_target_ratio=0.8, min_episode_duration=30.0, target_radius=0.5, window=10) -> Criteria:
    """utils/metrics.py:26-39 defaults, detect_overshoots window 10 (metrics.py:208)."""
    return Criteria(min_on_target_ratio, min_episode_duration, target_radius, window, 0)


def _vec3(v):
    return [float(v)] * 3 if np.isscalar(v) else [float(x) for x in v]


def _base_params(cfg: dict, integral_limit_default: float) -> CtrlParams:
    """Output clamps and feed-forward options shared by the three controllers."""
    c = CtrlParams()
    c.dt = cfg.get("dt", 0.01)
    c.hover_thrust = cfg.get("mass", 1.0) * cfg.get("gravity", 9.81)
    c.min_thrust = cfg.get("min_thrust", 0.0)
    c.max_thrust = cfg.get("max_thrust", 20.0)
    c.max_rate = cfg.get("max_rate", 3.0)
    c.use_lqi = 0
    c.feedforward_enabled = int(bool(cfg.get("feedforward_enabled", False)))
    c.integral_limit = cfg.get("integral_limit", integral_limit_default)
    c.integral_zero_threshold = cfg.get("integral_zero_threshold", 0.01)
    fv, fa = _vec3(cfg.get("ff_velocity_gain", 0.0)), _vec3(cfg.get("ff_acceleration_gain", 0.0))
    for i in range(3):
        c.ff_velocity_gain[i] = fv[i]
        c.ff_acceleration_gain[i] = fa[i]
    c.ff_max_velocity = cfg.get("ff_max_velocity", 10.0)
    c.ff_max_acceleration = cfg.get("ff_max_acceleration", 5.0)
    return c


def pid_controller(cfg: dict | None = None):
    """PIDController.__init__ (controllers/__init__.py:158-241): (CtrlParams,
    gains [kp, ki, kd] 3 x 3, kcols = 3)."""
    cfg = dict(cfg or {})
    c = _base_params(cfg, 0.0)
    kp = _vec3(cfg.get("kp_pos", cfg.get("kp", [0.01, 0.01, 4.0])))
    ki = _vec3(cfg.get("ki_pos", cfg.get("ki", [0.0, 0.0, 0.0])))
    kd = _vec3(cfg.get("kd_pos", cfg.get("kd", [0.06, 0.06, 2.0])))
    return c, np.array([kp, ki, kd], dtype=float), 3


def lqr_controller(cfg: dict | None = None):
    """LQRController.__init__ (controllers/__init__.py:449-574): heuristic or
    given K, no integral: (CtrlParams, K 4 x 6, kcols = 6)."""
    cfg = dict(cfg or {})
    c = _base_params(cfg, 0.0)
    if cfg.get("K") is not None:
        K = np.array(cfg["K"], dtype=float)
    else:
        K = heuristic_gains(cfg.get("q_pos", [1e-4, 1e-4, 16.0]), cfg.get("q_vel", [0.0036, 0.0036, 4.0]),
                            cfg.get("r_thrust", 1.0), cfg.get("r_rate", 1.0))
    return c, K, 6


def compute_action_pid(c: CtrlParams, gains, obs16, state):
    """state: integral[3] + last time (NaN = None); returns (u, state, diag[18])."""
    state = _f64(state).copy()
    u = np.zeros(4)
    diag = np.zeros(18)
    lib().oq_compute_action_pid(C.byref(c), _dp(_f64(gains)), c.hover_thrust, _dp(_f64(obs16)), _dp(state),
                                _dp(u), _dp(diag))
    return u, state, diag


def controller(cfg: dict | None = None):
    """RiccatiLQRController.__init__ (riccati_lqr.py:418-535): returns
    (CtrlParams, K 4 x kcols, kcols, fallback_flag, P).  cfg["controller"]
    "pid" / "lqr" selects PIDController / LQRController (K = their gains,
    kcols 3 / 6, no fallback, P None)."""
    cfg = dict(cfg or {})
    kind = cfg.pop("controller", "riccati_lqr")
    if kind == "pid":
        c, K, kc = pid_controller(cfg)
        return c, K, kc, False, None
    if kind == "lqr":
        c, K, kc = lqr_controller(cfg)
        return c, K, kc, False, None
    mass = cfg.get("mass", 1.0)
    g = cfg.get("gravity", 9.81)
    dt = cfg.get("dt", 0.01)
    lqi = bool(cfg.get("use_lqi", False))
    c = CtrlParams()
    c.dt = dt
    c.hover_thrust = mass * g
    c.min_thrust = cfg.get("min_thrust", 0.0)
    c.max_thrust = cfg.get("max_thrust", 20.0)
    c.max_rate = cfg.get("max_rate", 3.0)
    c.use_lqi = int(lqi)
    c.feedforward_enabled = int(bool(cfg.get("feedforward_enabled", False)))
    c.integral_limit = cfg.get("integral_limit", 10.0)
    c.integral_zero_threshold = cfg.get("integral_zero_threshold", 0.01)
    fv, fa = _vec3(cfg.get("ff_velocity_gain", 0.0)), _vec3(cfg.get("ff_acceleration_gain", 0.0))
    for i in range(3):
        c.ff_velocity_gain[i] = fv[i]
        c.ff_acceleration_gain[i] = fa[i]
    c.ff_max_velocity = cfg.get("ff_max_velocity", 10.0)
    c.ff_max_acceleration = cfg.get("ff_max_acceleration", 5.0)
    q_int = _vec3(cfg.get("q_int", [0.0, 0.0, 0.0]))
    n = 9 if lqi else 6
    if cfg.get("Q") is not None:
        Q = np.array(cfg["Q"], dtype=float)
        if lqi and Q.shape == (6, 6):
            Qa = np.zeros((9, 9))
            Qa[:6, :6] = Q
            Qa[6:, 6:] = np.diag(q_int)
            Q = Qa
    else:
        Q = np.diag(list(cfg.get("q_pos", [1e-4, 1e-4, 16.0])) + list(cfg.get("q_vel", [0.0036, 0.0036, 4.0]))
                    + (q_int if lqi else []))
    R = np.array(cfg["R"], dtype=float) if cfg.get("R") is not None else np.diag(cfg.get("r_controls", [1.0] * 4))
    ok = _psd(Q) and _pd(R)
    P = None
    if ok:
        try:
            P, K = dare(n, *system(n, dt, mass, g), Q, R)
        except RuntimeError:
            ok = False
    if not ok:  # _create_fallback_controller (riccati_lqr.py:747-777): no LQI, no feed-forward
        c.use_lqi = 0
        c.feedforward_enabled = 0
        r_rate = (R[1, 1] + R[2, 2] + R[3, 3]) / 3
        K = heuristic_gains(np.diag(Q)[:3], np.diag(Q)[3:6], R[0, 0], r_rate)
        return c, K, 6, True, None
    return c, K, n, False, P


def _psd(M):  # riccati_lqr.py:57-84
    return np.allclose(M, M.T, atol=1e-8) and not np.any(np.linalg.eigvalsh(M) < -1e-10)


def _pd(M):  # riccati_lqr.py:87-116
    return np.allclose(M, M.T, atol=1e-8) and not np.any(np.linalg.eigvalsh(M) <= 1e-10)


# ------------------------------------------------------------------- DARE


def system(n, dt, mass=1.0, gravity=9.81):
    A = np.zeros((n, n))
    B = np.zeros((n, 4))
    lib().oq_build_system(n, dt, mass, gravity, _dp(A), _dp(B))
    return A, B


def dare(n, A, B, Q, R, max_iter=64, tol=1e-14):
    A, B, Q, R = (_f64(x) for x in (A, B, Q, R))
    P = np.zeros((n, n))
    K = np.zeros((4, n))
    it = lib().oq_dare(n, _dp(A), _dp(B), _dp(Q), _dp(R), _dp(P), _dp(K), max_iter, tol)
    if it < 0:
        raise RuntimeError(f"DARE solver failed: {DARE_STATUS.get(-it, it)}")
    return P, K


def heuristic_gains(qpos, qvel, r_thrust, r_rate):
    K = np.zeros((4, 6))
    with np.errstate(invalid="ignore"):
        lib().oq_heuristic_gains(_dp(_f64(qpos)), _dp(_f64(qvel)), float(r_thrust), float(r_rate), _dp(K))
    return K


# ------------------------------------------------------------------ reset


def draws(motion: str | int, seeds) -> tuple[np.ndarray, np.ndarray]:
    """Per-seed reset() draws: pattern[N,4] raw, offset[N,3]
    (quadcopter_env.py:122-137; target_motion.py:318-366)."""
    m = MOTIONS[motion] if isinstance(motion, (int, np.integer)) else motion
    seeds = list(seeds)
    pat = np.zeros((len(seeds), 4))
    off = np.zeros((len(seeds), 3))
    for i, s in enumerate(seeds):
        s = int(s)
        r = np.random.default_rng(s)
        if m == "linear":
            pat[i, :3] = r.standard_normal(3)
        elif m == "circular":
            pat[i, 0] = r.uniform(0, 2 * np.pi)
        elif m == "sinusoidal":
            pat[i, :3] = r.uniform(0, 2 * np.pi, 3)
        off[i] = np.random.default_rng(s).uniform(-0.5, 0.5, 3)
    return pat, off


def target_state(e: EnvParams, motion: int, pat, t: float) -> np.ndarray:
    out = np.zeros(9)
    p = _f64(np.resize(np.asarray(pat, float), 4))
    lib().oq_target_state(C.byref(e), int(motion), _dp(p), float(t), _dp(out))
    return out


def initial_state(e: EnvParams, motion: int, pat, off) -> np.ndarray:
    x = np.zeros(12)
    x[:3] = target_state(e, motion, pat, 0.0)[:3] + off
    return x


def env_step(e: EnvParams, motion: int, pat, mass: float, x, t: float, action):
    x = _f64(x).copy()
    tt = C.c_double(t)
    tgt = np.zeros(9)
    err = C.c_double()
    viol = C.c_int()
    p = _f64(np.resize(np.asarray(pat, float), 4))
    term = lib().oq_env_step(C.byref(e), int(motion), _dp(p), float(mass), _dp(x), C.byref(tt),
                             _dp(_f64(action)), _dp(tgt), C.byref(err), C.byref(viol))
    return x, tt.value, tgt, err.value, viol.value, term


def compute_action(c: CtrlParams, K, kcols, obs15, integ):
    integ = _f64(integ).copy()
    u = np.zeros(4)
    sat = lib().oq_compute_action(C.byref(c), _dp(_f64(K)), kcols, c.hover_thrust, _dp(_f64(obs15)),
                                  _dp(integ), _dp(u))
    return u, integ, sat


def episode(e, c, cr, motion, pat, mass, hover, K, kcols, x0, max_steps=-1, record=False):
    met = np.zeros(N_MET)
    xf = np.zeros(12)
    integ = np.zeros(3)
    rec = np.zeros((int(round(e.max_episode_time / e.dt)) + 8 if max_steps < 0 else max_steps, 16)) if record else None
    lib().oq_episode(C.byref(e), C.byref(c), C.byref(cr), int(motion), _dp(_f64(np.resize(pat, 4))), float(mass),
                     float(hover), _dp(_f64(K)), kcols, _dp(_f64(x0)), int(max_steps), _dp(met), _dp(xf),
                     _dp(integ), _dp(rec) if record else None)
    return met, xf, integ, rec


def rollout(e, c, cr, motion, pat, mass, hover, K, kcols, k_per_episode, x0, max_steps=-1, threads=None):
    """Many independent episodes (AoS numpy inputs).  Returns (met[N,14], xf[N,12],
    integ[N,3], threads_used)."""
    if threads is not None:
        lib().oq_set_threads(int(threads))
    n = len(x0)
    met = np.zeros((n, N_MET))
    xf = np.zeros((n, 12))
    integ = np.zeros((n, 3))
    mo = None if motion is None else np.ascontiguousarray(motion, dtype=np.int8)
    used = lib().oq_rollout(
        C.byref(e), C.byref(c), C.byref(cr), n, mo.ctypes.data_as(C.POINTER(C.c_int8)) if mo is not None else None,
        _dp(_f64(pat)), _dp(_f64(mass)) if mass is not None else None,
        _dp(_f64(hover)) if hover is not None else None, _dp(_f64(K)), kcols,
        (9 if kcols == 3 else 4 * kcols) if k_per_episode else 0, _dp(_f64(x0)), int(max_steps), _dp(met), _dp(xf), _dp(integ))
    return met, xf, integ, used


# --------------------------------------------- numpy's summation order
# compute_evaluation_summary (utils/metrics.py:380-384) takes np.mean / np.std
# of per-episode lists.  numpy (the reference's dependency; 2.2 here) reduces a
# contiguous float64 vector in buffer blocks of NP_BLOCK elements, adding each
# block's pairwise sum (numpy/_core/src/umath/loops_utils.h.src,
# pairwise_sum) to a running total in order.  Pure-Python restatement, the
# checker of qt_summary_numpy; pinned against numpy itself in tests/test_oracle.py.
NP_BLOCK = 8192


def np_pairwise(a, lo: int, n: int) -> float:
    if n < 8:
        r = 0.0
        for i in range(n):
            r += a[lo + i]
        return r
    if n <= 128:
        r = [a[lo + j] for j in range(8)]
        i = 8
        while i < n - n % 8:
            for j in range(8):
                r[j] += a[lo + i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[lo + i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return np_pairwise(a, lo, n2) + np_pairwise(a, lo + n2, n - n2)


def np_blocks(a) -> list[float]:
    """Per-block pairwise sums of a float sequence (qt_summary_numpy's output)."""
    a = [float(v) for v in a]
    return [np_pairwise(a, lo, min(NP_BLOCK, len(a) - lo)) for lo in range(0, len(a), NP_BLOCK)]


def np_sum(a) -> float:
    """np.add.reduce of a 1-D float64 sequence, restated."""
    s = 0.0
    for v in np_blocks(a):
        s += v
    return s


def np_mean_std(a) -> tuple[float, float]:
    """(np.mean(a), np.std(a)) restated: mean = sum / n; std = sqrt(sum((x - mean) * (x - mean)) / n)."""
    a = [float(v) for v in a]
    n = len(a)
    mu = np_sum(a) / n
    return mu, float(np.sqrt(np_sum([(x - mu) * (x - mu) for x in a]) / n))
