"""The yaw-at-rest loop's safe horizon under randomised limits: fast flavour
(horizon, no per-step vote) against the exact step (recording forces it) on
the same episodes, for 12 seeded configurations that push each stop
condition into the horizons — low speed clamps, close position bounds, odd
episode lengths, other time steps and rate limits, light and heavy plants,
LQR / LQI / PID, the last three with the Euler integrator.  Decisions (steps, termination codes, counts) must be
identical, values within 1e-9 (the two paths contract FMAs differently).
Both are also checked against the oracle (oracle/qt_oracle.c, the reference's
step restated) run on the same limits, masses, seeds and controller: step
counts and termination codes exact, every other metric and the final state
within 1e-5 absolute / 1e-8 relative (north star; reference
quadcopter_env.py:428-465 termination, 513-535 constraints).  GPU only."""

import numpy as np
import pytest

import oracle as O
from test_gpu_parity import FIELDS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qt():
    import quadtrack

    quadtrack._abi.require_gpu()
    return quadtrack


def _config(i):
    r = np.random.default_rng(1000 + i)
    motion = ["stationary", "linear", "circular", "sinusoidal", "figure8"][i % 5]
    dt = float(r.choice([0.005, 0.01, 0.02]))
    env = {"target": {"motion_type": motion, "speed": float(r.uniform(0.5, 4.0))},
           "simulation": {"dt": dt, "max_velocity": float(r.uniform(2.0, 8.0)),
                          "max_position": float(r.uniform(3.0, 30.0)),
                          "max_episode_time": float(np.round(r.uniform(4.0, 12.0), 3))},
           "quadcopter": {"max_angular_rate": 3.0}}
    if i >= 12:  # the Euler closed form (make_rate_lin) under the same randomised limits
        env["simulation"]["integrator"] = "euler"
    kind = ["riccati_lqr", "lqi", "pid"][i % 3]
    ctl = {"dt": dt, "max_rate": float(r.uniform(1.0, 3.0))}
    if kind == "riccati_lqr":
        ctl.update(q_pos=[float(r.uniform(1e-4, 5.0))] * 2 + [16.0])
    mass = r.uniform(0.4, 2.0, 256)
    return env, kind, ctl, mass


@pytest.mark.parametrize("i", range(15))
def test_horizon_randomised_limits(qt, i):
    from quadtrack.controllers import batched_controller
    from quadtrack.rollout import run_closed_loop

    env, kind, ctl_cfg, mass = _config(i)
    ctl = batched_controller(kind, ctl_cfg)
    n = 256
    fast = run_closed_loop(ctl, env, n=n, seeds=np.arange(n), plant_mass=mass)
    exact = run_closed_loop(ctl, env, n=n, seeds=np.arange(n), plant_mass=mass, record=True)
    mf, me = fast.metrics.cpu().numpy(), exact.metrics.cpu().numpy()
    for k, f in enumerate(FIELDS):
        if f in ("overshoot_count", "success", "termination_code", "action_violations", "steps"):
            np.testing.assert_array_equal(mf[k], me[k], err_msg=f)
        else:
            np.testing.assert_allclose(mf[k], me[k], rtol=1e-9, atol=1e-9, err_msg=f)
    np.testing.assert_allclose(fast.state.x.cpu().numpy(), exact.state.x.cpu().numpy(), rtol=1e-9, atol=1e-9)
    # the oracle on the same limit set
    om, oxf = _oracle(env, kind, ctl_cfg, mass, n)
    for k, f in enumerate(FIELDS):
        if f in ("termination_code", "steps"):
            np.testing.assert_array_equal(mf[k], om[:, k], err_msg=f)
        else:
            np.testing.assert_allclose(mf[k], om[:, k], rtol=1e-8, atol=1e-5, err_msg=f)
    np.testing.assert_allclose(fast.state.x.cpu().numpy().T, oxf, rtol=1e-8, atol=1e-5)


def _oracle(env_cfg, kind, ctl_cfg, mass, n):
    """The oracle's rollout of _config's episodes: per-episode plant mass, the
    controller's own hover thrust (its mass stays 1 kg), seeds 0..n-1."""
    cfg = dict(ctl_cfg)
    if kind == "lqi":  # batched_controller("lqi"): use_lqi with its default q_int
        cfg.update(use_lqi=True, q_int=[0.01, 0.01, 0.1])
    elif kind == "pid":
        cfg["controller"] = "pid"
    c, K, kc, fb, _ = O.controller(cfg)
    assert not fb
    e = O.env_params(env_cfg)
    pat, off = O.draws(int(e.motion), range(n))
    x0 = np.array([O.initial_state(e, int(e.motion), pat[i], off[i]) for i in range(n)])
    met, xf, _, _ = O.rollout(e, c, O.criteria(), None, pat, mass, None, K, kc, False, x0)
    return met, xf
