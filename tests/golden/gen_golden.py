"""Generate the committed golden fixtures under tests/golden/ from the reference.

Test infrastructure only.  This script runs in the build container, where the
reference checkout is mounted read-only at /root/reference; it imports the
reference's pure-Python package (with a no-op stand-in for the absent
`python-dotenv` module, which the reference only uses to read a .env file,
`utils/__init__.py:33,256`) and records its outputs as plain arrays.  Nothing
of the reference travels: the outputs are data (inputs + expected outputs).

Usage:  python tests/golden/gen_golden.py  [--out tests/golden]

Fixture files (all float64 unless noted):
  dare_cases.npz      K/P of `RiccatiLQRController` / `solve_dare`
                      (riccati_lqr.py:119-184, 418-535, 702-777)
  rng_draws.npz       reset() draws per seed and motion type
                      (quadcopter_env.py:111-150, target_motion.py:306-369)
  target_states.npz   TargetMotion.get_state(t) (target_motion.py:29-411)
  actions.npz         RiccatiLQRController.compute_action on observation
                      sequences (riccati_lqr.py:779-967)
  controller_actions.npz  PIDController / LQRController.compute_action with
                      observation times (controllers/__init__.py:116-700)
  open_loop.npz      QuadcopterEnv.step under fixed action sequences
                      (quadcopter_env.py:152-465)
  closed_loop.npz     closed-loop episodes: selected-step states/actions and
                      per-episode metrics (eval.py:95-167, utils/metrics.py:264-338)
  scenarios.json      the env/controller configs each closed-loop scenario used
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import types

import numpy as np

REF_SRC = "/root/reference/src"

MOTIONS = ["stationary", "linear", "circular", "sinusoidal", "figure8"]
TERM_CODES = {"": 0, "time_limit": 1, "position_bounds": 2, "numerical_instability": 3}


def import_reference():
    if "dotenv" not in sys.modules:
        stub = types.ModuleType("dotenv")
        stub.load_dotenv = lambda *a, **k: False
        sys.modules["dotenv"] = stub
    sys.path.insert(0, REF_SRC)
    import logging

    logging.disable(logging.WARNING)
    from quadcopter_tracking.controllers.riccati_lqr import (  # noqa: F401
        RiccatiLQRController,
        solve_dare,
    )
    from quadcopter_tracking.env import QuadcopterEnv, TargetMotion  # noqa: F401
    from quadcopter_tracking.env.config import TargetParams  # noqa: F401
    from quadcopter_tracking.utils import metrics  # noqa: F401

    import quadcopter_tracking as qt

    return qt


# --------------------------------------------------------------------------- DARE


def gen_dare(qt):
    from quadcopter_tracking.controllers.riccati_lqr import RiccatiLQRController

    cases = []  # (cfg dict)
    cases.append({"dt": 0.01})
    cases.append({"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2]})
    cases.append({"dt": 0.01, "use_lqi": True, "q_int": [0.01, 0.01, 0.1]})
    cases.append({"dt": 0.01, "use_lqi": True, "q_int": [0.0, 0.0, 0.0]})
    cases.append({"dt": 0.02, "mass": 1.5, "gravity": 9.8})
    cases.append({"dt": 0.005, "mass": 0.5, "use_lqi": True, "q_int": 0.05})
    rng = np.random.default_rng(2024)
    for i in range(48):
        lqi = i % 3 == 0
        c = {
            "dt": 0.01,
            "mass": float(rng.uniform(0.8, 1.2)),
            "q_pos": list(rng.uniform([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0])),
            "q_vel": list(rng.uniform([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0])),
            "r_controls": list(rng.uniform(0.5, 2.0, 4)),
        }
        if lqi:
            c["use_lqi"] = True
            c["q_int"] = [0.0, 0.0, 0.0] if i % 2 == 0 else list(rng.uniform(1e-4, 0.1, 3))
        cases.append(c)
    # full (non-diagonal) SPD Q / R
    for i in range(8):
        lqi = i % 2 == 1
        n = 6
        M = rng.normal(size=(n, n)) * 0.3
        Q = M @ M.T + np.diag([1e-4, 1e-4, 16.0, 3.6e-3, 3.6e-3, 4.0])
        Mr = rng.normal(size=(4, 4)) * 0.2
        R = Mr @ Mr.T + np.eye(4)
        c = {"dt": 0.01, "Q": Q.tolist(), "R": R.tolist()}
        if lqi:
            c["use_lqi"] = True
            c["q_int"] = [1e-3, 2e-3, 1e-2]
        cases.append(c)
    # config-4 candidates: tuner random-search order from default_rng(42)
    # (controllers/tuning.py:683-728, scripts/controller_autotune.py:375-383)
    r42 = np.random.default_rng(42)
    for i in range(64):
        c = {
            "dt": 0.01,
            "q_pos": [float(r42.uniform(lo, hi)) for lo, hi in zip([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0])],
            "q_vel": [float(r42.uniform(lo, hi)) for lo, hi in zip([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0])],
            "r_controls": [float(r42.uniform(0.5, 2.0)) for _ in range(4)],
        }
        cases.append(c)
    # invalid weights -> heuristic fallback (riccati_lqr.py:737-777, __init__.py:522-574)
    cases.append({"dt": 0.01, "q_pos": [-1.0, 1e-4, 16.0]})
    cases.append({"dt": 0.01, "r_controls": [1.0, 0.0, 1.0, 1.0]})
    cases.append({"dt": 0.01, "r_controls": [2.0, 0.5, 1.0, 3.0], "q_vel": [0.01, -0.5, 4.0]})

    C = len(cases)
    out = {
        "n": np.zeros(C, np.int32),
        "dt": np.zeros(C),
        "mass": np.zeros(C),
        "gravity": np.zeros(C),
        "Q": np.zeros((C, 9, 9)),
        "R": np.zeros((C, 4, 4)),
        "K": np.zeros((C, 4, 9)),
        "P": np.zeros((C, 9, 9)),
        "fallback": np.zeros(C, np.int32),
    }
    for i, c in enumerate(cases):
        ctl = RiccatiLQRController(config=dict(c))
        n = 9 if ctl.use_lqi else 6
        out["n"][i] = n
        out["dt"][i] = ctl.dt
        out["mass"][i] = ctl.mass
        out["gravity"][i] = ctl.gravity
        out["Q"][i, :n, :n] = ctl.Q
        out["R"][i] = ctl.R
        if ctl.is_using_fallback():
            out["fallback"][i] = 1
            out["K"][i, :, :6] = ctl.fallback_controller.K
        else:
            out["K"][i, :, :n] = ctl.K
            out["P"][i, :n, :n] = ctl.P
    out["configs_json"] = np.array(json.dumps(cases))
    return out


# --------------------------------------------------------------------------- RNG


def gen_rng(qt):
    from quadcopter_tracking.env import QuadcopterEnv

    seeds = list(range(0, 256)) + [1000, 4095, 12345, 65535, 99991, 2**31 - 1, 10**9, 2**40 + 7]
    S = len(seeds)
    out = {"seeds": np.array(seeds, np.int64)}
    for m in MOTIONS:
        env = QuadcopterEnv({"target": {"motion_type": m}, "logging": {"enabled": False}})
        x0 = np.zeros((S, 3))
        p0 = np.zeros((S, 3))
        extra = np.zeros((S, 3))
        for j, s in enumerate(seeds):
            obs = env.reset(seed=s)
            x0[j] = obs["quadcopter"]["position"]
            p0[j] = obs["target"]["position"]
            pat = env.target._pattern
            if m == "linear":
                extra[j] = pat.direction
            elif m == "circular":
                extra[j, 0] = pat.initial_angle
            elif m == "sinusoidal":
                extra[j] = pat.phase
        out[f"{m}_x0"] = x0
        out[f"{m}_p0"] = p0
        out[f"{m}_param"] = extra
    return out


# --------------------------------------------------------------------------- targets


TARGET_VARIANTS = [
    {},
    {"speed": 2.5, "amplitude": 3.0, "frequency": 0.8, "radius": 1.5, "center": [1.0, -2.0, 3.0]},
    {"speed": 4.0, "amplitude": 0.7, "frequency": 1.7, "radius": 0.5, "max_acceleration": 2.0},
]


def gen_targets(qt):
    from quadcopter_tracking.env import TargetMotion
    from quadcopter_tracking.env.config import TargetParams

    times = np.concatenate([np.arange(0, 3001, 7) * 0.01, [0.123456, 17.5, 29.999, 30.0]])
    out = {"times": times}
    seeds = [0, 7, 42]
    for vi, var in enumerate(TARGET_VARIANTS):
        for m in MOTIONS:
            kw = dict(var)
            if "center" in kw:
                kw["center"] = tuple(kw["center"])
            tp = TargetParams(motion_type=m, **kw)
            P = np.zeros((len(seeds), len(times), 9))
            for si, s in enumerate(seeds):
                tm = TargetMotion(params=tp, seed=s)
                tm.reset(seed=s)
                for ti, t in enumerate(times):
                    st = tm.get_state(float(t))
                    P[si, ti, 0:3] = st["position"]
                    P[si, ti, 3:6] = st["velocity"]
                    P[si, ti, 6:9] = st["acceleration"]
            out[f"v{vi}_{m}"] = P
    out["seeds"] = np.array(seeds)
    out["variants_json"] = np.array(json.dumps(TARGET_VARIANTS))
    return out


# --------------------------------------------------------------------------- controller


ACTION_CASES = [
    {"dt": 0.01},
    {"dt": 0.01, "use_lqi": True, "q_int": [0.01, 0.01, 0.1]},
    {"dt": 0.01, "use_lqi": True, "q_int": [0.01, 0.01, 0.1], "integral_limit": 0.05},
    {"dt": 0.01, "use_lqi": True, "q_int": [0.01, 0.01, 0.1], "integral_zero_threshold": 0.3},
    {"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2], "integral_limit": 0.0},
    {"dt": 0.01, "feedforward_enabled": True, "ff_velocity_gain": [0.5, 0.3, 0.1],
     "ff_acceleration_gain": [0.2, 0.2, 0.4], "ff_max_velocity": 1.5, "ff_max_acceleration": 2.0},
    {"dt": 0.01, "use_lqi": True, "q_int": [0.01, 0.01, 0.1], "feedforward_enabled": True,
     "ff_velocity_gain": 0.25, "ff_acceleration_gain": 0.5},
    {"dt": 0.01, "max_thrust": 12.0, "min_thrust": 5.0, "max_rate": 0.5, "mass": 0.9},
    {"dt": 0.01, "q_pos": [-1.0, 1e-4, 16.0], "feedforward_enabled": True,
     "ff_velocity_gain": 0.3, "ff_acceleration_gain": 0.3},  # fallback controller path
]


def gen_actions(qt):
    from quadcopter_tracking.controllers.riccati_lqr import RiccatiLQRController

    rng = np.random.default_rng(77)
    T = 120
    out = {}
    obs_arr = np.zeros((T, 15))  # qpos, qvel, tpos, tvel, tacc
    # a slowly drifting observation sequence with occasional large jumps
    base = rng.normal(size=15)
    for k in range(T):
        base = base + 0.05 * rng.normal(size=15)
        if k % 37 == 5:
            base[6:9] += rng.normal(size=3) * 8.0
        obs_arr[k] = base
        obs_arr[k, 2] += 1.0
    obs_arr[10:14, 6:9] = obs_arr[10:14, 0:3] + 0.001  # below zero threshold
    out["obs"] = obs_arr
    for ci, c in enumerate(ACTION_CASES):
        ctl = RiccatiLQRController(config=dict(c))
        A = np.zeros((T, 4))
        I = np.zeros((T, 3))
        for k in range(T):
            o = obs_arr[k]
            obs = {
                "quadcopter": {"position": o[0:3].copy(), "velocity": o[3:6].copy(),
                               "attitude": np.zeros(3), "angular_velocity": np.zeros(3)},
                "target": {"position": o[6:9].copy(), "velocity": o[9:12].copy(),
                           "acceleration": o[12:15].copy()},
            }
            a = ctl.compute_action(obs)
            A[k] = [a["thrust"], a["roll_rate"], a["pitch_rate"], a["yaw_rate"]]
            st = ctl.get_integral_state()
            if st is not None:
                I[k] = st
        out[f"case{ci}_action"] = A
        out[f"case{ci}_integral"] = I
    out["cases_json"] = np.array(json.dumps(ACTION_CASES))
    return out


CONTROLLER_CASES = [
    {"controller": "pid"},
    {"controller": "pid", "kp_pos": 0.5, "ki_pos": [0.1, 0.2, 0.3], "kd_pos": [0.1, 0.1, 1.0],
     "integral_limit": 0.05},
    {"controller": "pid", "ki_pos": [0.05, 0.05, 0.5], "integral_limit": 2.0, "feedforward_enabled": True,
     "ff_velocity_gain": [0.5, 0.5, 0.2], "ff_acceleration_gain": 0.4, "ff_max_velocity": 1.0,
     "ff_max_acceleration": 0.7, "mass": 1.4, "max_rate": 0.5},
    {"controller": "lqr"},
    {"controller": "lqr", "q_pos": [1e-3, 2e-3, 9.0], "r_thrust": 2.0, "r_rate": 0.25,
     "feedforward_enabled": True, "ff_velocity_gain": 0.3, "ff_acceleration_gain": [0.2, 0.3, 0.4]},
    {"controller": "lqr", "K": [[0.0, 0.1, 3.0, 0.0, 0.2, 2.0], [0.05, -0.3, 0.0, 0.1, -0.6, 0.0],
                                [0.3, 0.02, 0.0, 0.7, 0.0, 0.01], [0.01, 0.01, 0.0, 0.0, 0.0, 0.02]]},
]


def gen_controller_actions(qt):
    """PIDController / LQRController.compute_action (controllers/__init__.py:243-396, 576-700)
    on an observation sequence with a `time` entry (the PID integrates over
    time differences; a repeated and a decreasing time are included)."""
    rng = np.random.default_rng(78)
    T = 150
    obs_arr = np.zeros((T, 15))
    times = np.zeros(T)
    base = rng.normal(size=15)
    t = 0.0
    for k in range(T):
        base = base + 0.05 * rng.normal(size=15)
        if k % 41 == 7:
            base[6:9] += rng.normal(size=3) * 6.0
        obs_arr[k] = base
        obs_arr[k, 2] += 1.0
        if k == 60:
            pass  # repeated time: dt = 0
        elif k == 100:
            t = 0.37  # time going backwards: dt < 0
        elif k > 0:
            t += 0.01
        times[k] = t
    out = {"obs": obs_arr, "time": times}
    for ci, c in enumerate(CONTROLLER_CASES):
        ctl = make_controller(c)
        A = np.zeros((T, 4))
        I = np.zeros((T, 3))
        for k in range(T):
            o = obs_arr[k]
            obs = {
                "quadcopter": {"position": o[0:3].copy(), "velocity": o[3:6].copy(),
                               "attitude": np.zeros(3), "angular_velocity": np.zeros(3)},
                "target": {"position": o[6:9].copy(), "velocity": o[9:12].copy(),
                           "acceleration": o[12:15].copy()},
                "time": float(times[k]),
            }
            a = ctl.compute_action(obs)
            A[k] = [a["thrust"], a["roll_rate"], a["pitch_rate"], a["yaw_rate"]]
            if hasattr(ctl, "integral_error"):
                I[k] = ctl.integral_error
        out[f"case{ci}_action"] = A
        out[f"case{ci}_integral"] = I
        if c["controller"] == "lqr":
            out[f"case{ci}_K"] = np.array(ctl.K)
    out["cases_json"] = np.array(json.dumps(CONTROLLER_CASES))
    return out


# --------------------------------------------------------------------------- open loop


OPEN_LOOP = [
    {"motion": "stationary", "seed": 0, "env": {}},
    {"motion": "circular", "seed": 3, "env": {}},
    {"motion": "figure8", "seed": 5, "env": {"simulation": {"integrator": "euler"}}},
    {"motion": "sinusoidal", "seed": 9, "env": {"quadcopter": {"mass": 1.3, "drag_coeff_linear": 0.3,
                                                               "drag_coeff_angular": 0.05, "max_thrust": 25.0,
                                                               "min_thrust": 2.0, "max_angular_rate": 2.0},
                                                "simulation": {"max_velocity": 4.0, "max_angular_velocity": 1.5}}},
    {"motion": "linear", "seed": 11, "env": {"simulation": {"max_position": 3.0}}},
]


def gen_open_loop(qt):
    from quadcopter_tracking.env import QuadcopterEnv

    rng = np.random.default_rng(5)
    T = 400
    actions = np.zeros((T, 4))
    actions[:, 0] = rng.uniform(-5, 30, T)
    actions[:, 1:] = rng.uniform(-6, 6, (T, 3))
    actions[17, 2] = np.nan
    actions[18, 0] = np.inf
    actions[19, 3] = -np.inf
    actions[50:120, 0] = 9.81 + rng.normal(0, 0.5, 70)
    actions[50:120, 1:] = rng.normal(0, 0.3, (70, 3))
    out = {"actions": actions}
    for ci, case in enumerate(OPEN_LOOP):
        cfg = json.loads(json.dumps(case["env"]))
        cfg.setdefault("target", {})["motion_type"] = case["motion"]
        cfg["logging"] = {"enabled": False}
        env = QuadcopterEnv(cfg)
        env.reset(seed=case["seed"])
        X = np.full((T + 1, 12), np.nan)
        info_arr = np.full((T, 6), np.nan)  # err, on_target_ratio, violations, done, reason, time
        X[0] = env.get_state_vector()
        for k in range(T):
            obs, r, done, info = env.step(actions[k].copy())
            X[k + 1] = env.get_state_vector()
            info_arr[k] = [info["tracking_error"], info["on_target_ratio"], info["action_violations"],
                           float(done), TERM_CODES[info.get("termination_reason", "")], info["time"]]
            if done:
                break
        out[f"case{ci}_states"] = X
        out[f"case{ci}_info"] = info_arr
    out["cases_json"] = np.array(json.dumps(OPEN_LOOP))
    return out


# --------------------------------------------------------------------------- closed loop


REC_STEPS = np.unique(np.concatenate([np.arange(0, 50), np.arange(0, 3000, 100), np.arange(2950, 3000)]))


def make_controller(ctl_cfg):
    """controller kind from the scenario's "controller" key (default riccati_lqr)."""
    from quadcopter_tracking.controllers import LQRController, PIDController
    from quadcopter_tracking.controllers.riccati_lqr import RiccatiLQRController

    cfg = dict(ctl_cfg)
    kind = cfg.pop("controller", "riccati_lqr")
    return {"riccati_lqr": RiccatiLQRController, "pid": PIDController, "lqr": LQRController}[kind](config=cfg)


def run_episode(qt, env_cfg, ctl_cfg, seed):
    """Evaluator.run_episode semantics (eval.py:95-167) with a fresh controller
    per episode.  Returns the recorded per-step arrays and metrics."""
    from quadcopter_tracking.env import QuadcopterEnv
    from quadcopter_tracking.utils.metrics import compute_episode_metrics

    env = QuadcopterEnv(env_cfg)
    ctl = make_controller(ctl_cfg)
    obs = env.reset(seed=seed)
    x0 = env.get_state_vector()
    data, states, acts, ints = [], [], [], []
    done = False
    info = {}
    while not done:
        a = ctl.compute_action(obs)
        nobs, r, done, info = env.step(a)
        data.append({
            "time": info["time"],
            "quadcopter_position": obs["quadcopter"]["position"].tolist(),
            "target_position": obs["target"]["position"].tolist(),
            "action": [a["thrust"], a["roll_rate"], a["pitch_rate"], a["yaw_rate"]],
        })
        states.append(env.get_state_vector())
        acts.append(data[-1]["action"])
        if hasattr(ctl, "get_integral_state"):
            st = ctl.get_integral_state()
        else:  # PID integral error (controllers/__init__.py:229)
            st = getattr(ctl, "integral_error", None)
        ints.append(np.array(st) if st is not None else np.zeros(3))
        obs = nobs
    m = compute_episode_metrics(data, None, info)
    met = np.array([
        m.episode_duration, m.on_target_ratio, m.mean_tracking_error, m.max_tracking_error,
        m.rms_tracking_error, m.total_control_effort, m.mean_control_effort, m.overshoot_count,
        m.max_overshoot, float(m.success), TERM_CODES[m.termination_reason], m.action_violations,
        info["on_target_ratio"], len(data),
    ])
    return x0, np.array(states), np.array(acts), np.array(ints), met


METRIC_FIELDS = ["episode_duration", "on_target_ratio", "mean_tracking_error", "max_tracking_error",
                 "rms_tracking_error", "total_control_effort", "mean_control_effort", "overshoot_count",
                 "max_overshoot", "success", "termination_code", "action_violations",
                 "env_on_target_ratio", "steps"]


def closed_loop_scenarios():
    sc = []
    lqr = {"dt": 0.01}
    lqi = {"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2]}
    for m in MOTIONS:
        for name, c in (("lqr", lqr), ("lqi", lqi)):
            sc.append({"name": f"{m}_{name}", "env": {"target": {"motion_type": m}},
                       "ctl": c, "seeds": [0, 1, 42, 12345], "record": True})
    # config 4 style: circular, per-episode Q/R (tuner order from default_rng(42))
    r42 = np.random.default_rng(42)
    per = []
    for i in range(12):
        per.append({
            "dt": 0.01,
            "q_pos": [float(r42.uniform(lo, hi)) for lo, hi in zip([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0])],
            "q_vel": [float(r42.uniform(lo, hi)) for lo, hi in zip([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0])],
            "r_controls": [float(r42.uniform(0.5, 2.0)) for _ in range(4)],
        })
    sc.append({"name": "cfg4_circular_perQR", "env": {"target": {"motion_type": "circular"}},
               "ctl_per_episode": per, "seeds": list(range(12)), "record": False})
    # config 5 style: motion = i mod 5, per-episode mass from default_rng(1e9 + i)
    envs, ctls = [], []
    for i in range(15):
        mass = float(np.random.default_rng(10**9 + i).uniform(0.8, 1.2))
        envs.append({"target": {"motion_type": MOTIONS[i % 5]}, "quadcopter": {"mass": mass}})
        ctls.append({"dt": 0.01, "mass": mass})
    sc.append({"name": "cfg5_mixed_mass", "env_per_episode": envs, "ctl_per_episode": ctls,
               "seeds": list(range(15)), "record": False})
    ff = {"dt": 0.01, "feedforward_enabled": True, "ff_velocity_gain": [0.4, 0.4, 0.2],
          "ff_acceleration_gain": [0.3, 0.3, 0.5], "ff_max_velocity": 10.0, "ff_max_acceleration": 5.0}
    for m in ("circular", "figure8", "sinusoidal", "linear"):
        sc.append({"name": f"ff_{m}", "env": {"target": {"motion_type": m, "max_acceleration": 1.0}},
                   "ctl": ff, "seeds": [0, 3], "record": m == "figure8"})
    sc.append({"name": "euler_circular", "env": {"target": {"motion_type": "circular"},
                                                 "simulation": {"integrator": "euler"}},
               "ctl": lqr, "seeds": [0, 2], "record": True})
    sc.append({"name": "bounds_sinusoidal_lqi", "env": {"target": {"motion_type": "sinusoidal"},
                                                        "simulation": {"max_position": 40.0}},
               "ctl": lqi, "seeds": [0, 1, 2], "record": False})
    sc.append({"name": "short_episode", "env": {"target": {"motion_type": "linear", "speed": 2.0},
                                                "simulation": {"max_episode_time": 2.5}},
               "ctl": {"dt": 0.01, "use_lqi": True, "q_int": [0.01, 0.01, 0.1]}, "seeds": [4, 5], "record": True})
    sc.append({"name": "custom_plant", "env": {"target": {"motion_type": "sinusoidal", "amplitude": 1.0,
                                                          "frequency": 0.2, "center": [2.0, 1.0, 5.0]},
                                               "quadcopter": {"mass": 1.2, "drag_coeff_linear": 0.2,
                                                              "max_thrust": 30.0},
                                               "success_criteria": {"target_radius": 0.8,
                                                                    "min_episode_duration": 10.0}},
               "ctl": {"dt": 0.01, "mass": 1.2, "max_thrust": 30.0, "q_pos": [1e-3, 1e-3, 20.0]},
               "seeds": [6, 7], "record": False})
    # PID and heuristic-LQR controllers in the same loop
    pid = {"controller": "pid"}
    for m in MOTIONS:
        sc.append({"name": f"pid_{m}", "env": {"target": {"motion_type": m}}, "ctl": pid,
                   "seeds": [0, 1, 42], "record": m in ("linear", "circular")})
    sc.append({"name": "pid_integral_sinusoidal", "env": {"target": {"motion_type": "sinusoidal"}},
               "ctl": {"controller": "pid", "kp_pos": [0.02, 0.02, 5.0], "ki_pos": [0.005, 0.005, 0.8],
                       "kd_pos": [0.08, 0.08, 2.5], "integral_limit": 1.5},
               "seeds": [0, 5], "record": True})
    sc.append({"name": "pid_ff_circular", "env": {"target": {"motion_type": "circular", "speed": 3.0}},
               "ctl": {"controller": "pid", "feedforward_enabled": True, "ff_velocity_gain": [0.3, 0.3, 0.1],
                       "ff_acceleration_gain": [0.2, 0.2, 0.4], "ff_max_velocity": 2.5,
                       "ff_max_acceleration": 1.0, "ki_pos": 0.01, "integral_limit": 0.5},
               "seeds": [1, 2], "record": True})
    sc.append({"name": "pid_saturating_linear", "env": {"target": {"motion_type": "linear", "speed": 4.0}},
               "ctl": {"controller": "pid", "kp_pos": [2.0, 2.0, 30.0], "kd_pos": [1.0, 1.0, 10.0],
                       "max_thrust": 18.0, "max_rate": 2.0},
               "seeds": [3], "record": True})
    for m in ("stationary", "linear", "circular"):
        sc.append({"name": f"lqr_heuristic_{m}", "env": {"target": {"motion_type": m}},
                   "ctl": {"controller": "lqr"}, "seeds": [0, 7], "record": m == "circular"})
    sc.append({"name": "lqr_heuristic_custom_ff", "env": {"target": {"motion_type": "sinusoidal"}},
               "ctl": {"controller": "lqr", "q_pos": [2e-4, 3e-4, 20.0], "q_vel": [5e-3, 4e-3, 5.0],
                       "r_thrust": 0.8, "r_rate": 1.5, "feedforward_enabled": True,
                       "ff_velocity_gain": 0.2, "ff_acceleration_gain": [0.1, 0.1, 0.3]},
               "seeds": [2, 9], "record": False})
    return sc


def gen_closed_loop(qt):
    out = {"rec_steps": REC_STEPS}
    scen = closed_loop_scenarios()
    for s in scen:
        E = len(s["seeds"])
        X0 = np.zeros((E, 12))
        MET = np.zeros((E, len(METRIC_FIELDS)))
        FIN = np.zeros((E, 15))
        RS = np.full((E, len(REC_STEPS), 12), np.nan)
        RA = np.full((E, len(REC_STEPS), 4), np.nan)
        RI = np.full((E, len(REC_STEPS), 3), np.nan)
        for e, seed in enumerate(s["seeds"]):
            env_cfg = json.loads(json.dumps(s["env_per_episode"][e] if "env_per_episode" in s else s["env"]))
            env_cfg["logging"] = {"enabled": False}
            ctl_cfg = s["ctl_per_episode"][e] if "ctl_per_episode" in s else s["ctl"]
            x0, st, ac, it, met = run_episode(qt, env_cfg, ctl_cfg, seed)
            X0[e] = x0
            MET[e] = met
            FIN[e, :12] = st[-1]
            FIN[e, 12:] = it[-1]
            if s["record"]:
                n = len(st)
                ok = REC_STEPS < n
                RS[e, ok] = st[REC_STEPS[ok]]
                RA[e, ok] = ac[REC_STEPS[ok]]
                RI[e, ok] = it[REC_STEPS[ok]]
        out[f"{s['name']}_x0"] = X0
        out[f"{s['name']}_metrics"] = MET
        out[f"{s['name']}_final"] = FIN
        if s["record"]:
            out[f"{s['name']}_rec_state"] = RS
            out[f"{s['name']}_rec_action"] = RA
            out[f"{s['name']}_rec_integral"] = RI
        print(f"  {s['name']}: mean err {MET[:, 2].mean():.6f}", flush=True)
    return out, scen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    args = ap.parse_args()
    qt = import_reference()
    np.savez_compressed(os.path.join(args.out, "dare_cases.npz"), **gen_dare(qt))
    print("dare done", flush=True)
    np.savez_compressed(os.path.join(args.out, "rng_draws.npz"), **gen_rng(qt))
    print("rng done", flush=True)
    np.savez_compressed(os.path.join(args.out, "target_states.npz"), **gen_targets(qt))
    print("targets done", flush=True)
    np.savez_compressed(os.path.join(args.out, "actions.npz"), **gen_actions(qt))
    np.savez_compressed(os.path.join(args.out, "controller_actions.npz"), **gen_controller_actions(qt))
    print("actions done", flush=True)
    np.savez_compressed(os.path.join(args.out, "open_loop.npz"), **gen_open_loop(qt))
    print("open loop done", flush=True)
    cl, scen = gen_closed_loop(qt)
    np.savez_compressed(os.path.join(args.out, "closed_loop.npz"), **cl)
    with open(os.path.join(args.out, "scenarios.json"), "w") as f:
        json.dump({"metric_fields": METRIC_FIELDS, "term_codes": TERM_CODES, "motions": MOTIONS,
                   "scenarios": scen}, f, indent=1)
    print("closed loop done", flush=True)


if __name__ == "__main__":
    main()
