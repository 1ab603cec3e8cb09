"""The yaw-at-rest loop's safe horizon (csrc/qt_kernels.hpp yaw0_horizon,
csrc/qt_device.hpp make_horizon): its per-step bounds checked against the
steps the oracle actually takes.  CPU only.

The fast loop runs up to H steps without its stop vote when every lane is
farther than H per-step bounds from each stop condition (speed clamp,
position bound, tilt clamp, time limit).  The bounds come from the closed-form
step (integrate_yaw0): a speed grows by at most the thrust + gravity reach of
one RK4 step, a position moves by at most |pv| vmax plus that reach, roll and
pitch move by at most (|ay| + |au|) max_rate.  Here they are restated from the
same RK4 recurrences and every step of saturating closed-loop episodes
(thrust and tilt at their clips, heavy and light plants, LQI runs that
diverge, PID) must stay inside them; the largest observed fraction of each
bound shows that they are not vacuous.
"""

import numpy as np
import pytest

import oracle as O


def rk4_linear(lam, h, y, f):
    """qt_device.hpp rk4_linear: stage values of y' = f_i - lam y."""
    k1 = f[0] - lam * y
    y2 = y + 0.5 * h * k1
    k2 = f[1] - lam * y2
    y3 = y + 0.5 * h * k2
    k3 = f[2] - lam * y3
    y4 = y + h * k3
    k4 = f[3] - lam * y4
    return (y2, y3, y4, y + h / 6.0 * (k1 + 2.0 * k2 + 2.0 * k3 + k4), h / 6.0 * (y + 2.0 * y2 + 2.0 * y3 + y4))


def step_bounds(e, c, mass):
    """make_horizon + yaw0_horizon's per-lane bounds (dv, dp, dang, tstep)."""
    h, inv_m = e.dt, 1.0 / mass
    lam = 10.0 + e.drag_angular
    ay = rk4_linear(lam, h, 1.0, [0.0] * 4)[4]
    au = rk4_linear(lam, h, 0.0, [10.0] * 4)[4]
    delta = e.drag_linear * inv_m
    o = rk4_linear(delta, h, 1.0, [0.0] * 4)
    cv, pv = o[3], o[4]
    wv, pa = [], []
    for i in range(4):
        f = [0.0] * 4
        f[i] = 1.0
        oi = rk4_linear(delta, h, 0.0, f)
        wv.append(oi[3])
        if i < 3:
            pa.append(oi[4])
    g = -mass * e.gravity * inv_m
    gv, gp = g * sum(wv), g * sum(pa)
    tmax = max(abs(c.min_thrust), abs(c.max_thrust))
    vmax = e.max_velocity * (1.0 - 1e-12)
    dv = (tmax * inv_m * sum(abs(w) for w in wv) + abs(gv)) * (1 + 1e-9) + e.max_velocity * 1e-14
    dp = (abs(pv) * vmax + tmax * inv_m * sum(abs(p) for p in pa) + abs(gp)) * (1 + 1e-9) + e.max_position * 1e-15
    dang = (abs(ay) + abs(au)) * c.max_rate * (1 + 1e-9) + 2e-15
    tstep = (e.dt + (abs(e.max_episode_time) + e.dt) * 4.5e-16) * (1 + 1e-9)
    assert 0.0 <= cv <= 1.0
    return dv, dp, dang, tstep


CASES = [
    # (name, env cfg, controller cfg, initial offset scale)
    ("lqr_far", {"target": {"motion_type": "linear"}}, {}, 40.0),
    ("lqr_heavy_far", {"target": {"motion_type": "circular"}, "quadcopter": {"mass": 1.8}}, {"mass": 1.8}, 30.0),
    ("lqr_light_aggressive", {"target": {"motion_type": "sinusoidal"}, "quadcopter": {"mass": 0.4}},
     {"mass": 0.4, "q_pos": [10.0, 10.0, 40.0], "q_vel": [1.0, 1.0, 4.0]}, 20.0),
    ("lqi_sinusoidal", {"target": {"motion_type": "sinusoidal"}}, {"use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2]}, 0.5),
    ("lqi_far", {"target": {"motion_type": "figure8"}}, {"use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2]}, 25.0),
    ("pid_far", {"target": {"motion_type": "linear"}}, {"controller": "pid", "kp": [2.0, 2.0, 6.0]}, 15.0),
    ("no_drag_fast", {"target": {"motion_type": "linear", "speed": 8.0},
                      "quadcopter": {"drag_coeff_linear": 0.0, "drag_coeff_angular": 0.0}}, {}, 60.0),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_horizon_step_bounds_hold(case):
    name, env_cfg, ctl_cfg, scale = case
    e = O.env_params(env_cfg)
    c, K, kc, _, _ = O.controller(dict(ctl_cfg))
    mass = env_cfg.get("quadcopter", {}).get("mass", 1.0)
    dv, dp, dang, tstep = step_bounds(e, c, mass)
    cr = O.criteria()
    rng = np.random.default_rng(len(name))
    worst = np.zeros(4)
    for ep in range(6):
        pat, _ = O.draws(e.motion, [ep])
        x0 = O.initial_state(e, e.motion, pat[0], rng.uniform(-scale, scale, 3))
        x0[3:6] = rng.uniform(-3.0, 3.0, 3)
        x0[6:8] = rng.uniform(-0.8, 0.8, 2)
        x0[9:11] = rng.uniform(-c.max_rate, c.max_rate, 2)
        _, _, _, rec = O.episode(e, c, cr, e.motion, pat[0], mass, c.hover_thrust, K, kc, x0, record=True)
        xs = np.vstack([x0[None, :], rec[:, :12]])
        xs = xs[: int(np.count_nonzero(np.any(rec != 0.0, axis=1))) + 1]
        assert len(xs) > 100
        sp = np.linalg.norm(xs[:, 3:6], axis=1)
        dsp = sp[1:] - sp[:-1]
        dpos = np.max(np.abs(xs[1:, :3] - xs[:-1, :3]), axis=1)
        dtilt = np.max(np.abs(xs[1:, 6:8] - xs[:-1, 6:8]), axis=1)
        assert np.all(dsp <= dv), (name, dsp.max(), dv)
        assert np.all(dpos <= dp), (name, dpos.max(), dp)
        assert np.all(dtilt <= dang), (name, dtilt.max(), dang)
        worst = np.maximum(worst, [dsp.max() / dv, dpos.max() / dp, dtilt.max() / dang, 0.0])
    # the time bound: t advances by fl(t + dt) - t
    t, dts = 0.0, []
    while t < e.max_episode_time:
        t1 = t + e.dt
        dts.append(t1 - t)
        t = t1
    assert max(dts) <= tstep
    # not vacuous: the saturating cases reach a good part of each bound
    if name in ("lqr_far", "no_drag_fast"):
        assert worst[0] > 0.3 and worst[2] > 0.3, worst


def tie_binade(dt):
    """make_horizon's tie binade (qt_device.hpp): dt = m 2^q with m odd; the
    exponent E of the t binade [2^E, 2^(E+1)) whose ulp is 2^(q+1)."""
    m, q = np.frexp(dt)
    m, q = int(m * 2.0**53), int(q) - 53
    while m % 2 == 0:
        m //= 2
        q += 1
    return q + 53


@pytest.mark.parametrize("dt", [0.01, 0.005, 0.02, 1.0 / 64, 0.1, 0.001])
def test_time_step_constant_per_binade(dt):
    """The folded target rotor (qt_kernels.hpp rotor_fold) rests on this: in
    every binade of t but the tie binade, fl(t + dt) - t is one value (t is a
    multiple of the binade's ulp), and the horizon never crosses a binade
    edge.  Checked over the steps of episodes started at an even and at an
    odd multiple of each binade's ulp; in the tie binade round-half-even
    gives two values, by the parity of t's last bit."""
    e_tie = tie_binade(dt)
    seen_tie = False
    for e in range(-8, 8):
        lo, hi = 2.0**e, 2.0**(e + 1)
        if hi <= dt:
            continue
        steps = set()
        for t in (lo, np.nextafter(lo, hi)):
            k = 0
            while t + dt < hi and k < 4000:
                t1 = t + dt
                steps.add(t1 - t)
                t = t1
                k += 1
        if not steps:
            continue
        if e == e_tie:
            assert len(steps) == 2, (dt, e)
            seen_tie = True
        else:
            assert len(steps) == 1, (dt, e, sorted(steps)[:3])
    assert seen_tie or not (-8 <= e_tie < 8)
