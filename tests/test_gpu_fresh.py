"""qt_rollout_fresh (ABI 8): reset -> rollout -> episode metrics in one launch
set (the reset state formed in the rollout kernel's prologue, the metrics
rows written in its epilogue) against the three separate calls, bit for bit,
for every step flavour: the yaw-at-rest fast loop (LQR, LQI, PID, dense
gains, feed-forward), the staged fast step, the exact step (Euler), waves the
fast kernel leaves to the exact pass, a motion-grouped batch (the grouped
kernel, which takes qt_reset / metrics_kernel around its launch), the empty
batch and nsteps = 0.  GPU only."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qt():
    import quadtrack

    quadtrack._abi.require_gpu()
    return quadtrack


def _both(ctl, env_cfg, n, nsteps, motion=None, plant_mass=None, poison=None, dirty=False):
    from quadtrack import core
    from quadtrack.env.config import EnvConfig
    from quadtrack.rollout import build_batch

    cfg = EnvConfig.from_dict(env_cfg)
    env = cfg.to_params()
    crit = core.criteria()
    batch = build_batch(ctl, cfg, n, seeds=np.arange(n), motion=motion, plant_mass=plant_mass)
    if batch.groups is not None:
        batch, _ = batch.physical_groups()
    if poison is not None:  # a non-finite start: its wave fails the fast flavour's test
        batch.offset[0, poison] = float("nan")
    out = []
    for fresh in (True, False):
        st = core.RolloutState.empty(n, batch.device)
        if dirty:  # a reused state buffer: every row holds an old value first
            for t in (st.x, st.integ, st.t, st.acc, st.target):
                t.fill_(7.0)
        if fresh:
            met = core.rollout_fresh(env, ctl.ctrl, crit, batch, st, nsteps)
        else:
            core.reset(env, batch, st)
            core.rollout(env, ctl.ctrl, crit, batch, st, nsteps)
            met = core.episode_metrics(crit, st)
        torch.cuda.synchronize()
        out.append([t.cpu().numpy() for t in (met, st.x, st.target, st.t, st.acc, st.integ)])
    for a, b in zip(*out):
        np.testing.assert_array_equal(a, b)
    return out[0][0]


CASES = [
    ("lqr_linear", {"target": {"motion_type": "linear"}}, {"dt": 0.01}),
    ("lqi_sinusoidal", {"target": {"motion_type": "sinusoidal"}}, {"dt": 0.01, "use_lqi": True,
                                                                   "q_int": [1e-3, 1e-3, 1e-2]}),
    ("lqr_figure8_ff", {"target": {"motion_type": "figure8"}}, {"dt": 0.01, "feedforward_enabled": True,
                                                               "ff_velocity_gain": 0.5,
                                                               "ff_acceleration_gain": 0.2}),
    ("lqr_circular_euler", {"target": {"motion_type": "circular"}, "simulation": {"integrator": "euler"}},
     {"dt": 0.01}),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("nsteps", [3000, 777])
def test_fresh_pass_bitwise(qt, case, nsteps):
    from quadtrack.controllers import BatchedRiccatiLQR

    _, env_cfg, ctl_cfg = case
    met = _both(BatchedRiccatiLQR(ctl_cfg), env_cfg, 300, nsteps)
    assert np.all(met[-1] > 0)  # every episode stepped


def test_fresh_pass_reused_state_buffer(qt):
    """A fresh pass into a state buffer holding old values stores what
    qt_reset -> qt_rollout would (the integral rows of an LQR pass included)."""
    from quadtrack.controllers import BatchedPID, BatchedRiccatiLQR

    _both(BatchedRiccatiLQR({"dt": 0.01}), {"target": {"motion_type": "linear"}}, 300, 777, dirty=True)
    _both(BatchedRiccatiLQR({"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2]}),
          {"target": {"motion_type": "sinusoidal"}}, 300, 777, dirty=True)
    _both(BatchedPID({"dt": 0.01}), {"target": {"motion_type": "circular"}}, 200, 777, dirty=True)


def test_fresh_pass_pid_and_dense(qt):
    from quadtrack.controllers import BatchedPID, BatchedRiccatiLQR

    _both(BatchedPID({"dt": 0.01}), {"target": {"motion_type": "circular"}}, 200, 3000)
    Q = np.diag([1e-4, 1e-4, 16.0, 0.0036, 0.0036, 4.0])
    Q[0, 3] = Q[3, 0] = 2e-4
    _both(BatchedRiccatiLQR({"dt": 0.01, "Q": Q.tolist()}), {"target": {"motion_type": "linear"}}, 200, 3000)


def test_fresh_pass_deferred_wave(qt):
    """A NaN start offset in wave 2: the fast kernel stores that wave's reset
    state and leaves it to the exact pass (launched without the prologue)."""
    from quadtrack.controllers import BatchedRiccatiLQR

    met = _both(BatchedRiccatiLQR({"dt": 0.01}), {"target": {"motion_type": "circular"}}, 256, 3000, poison=130)
    assert met[-1, 130] < 3000 and np.all(met[-1, :128] == 3000)


@pytest.mark.parametrize("n", [640, 700])
def test_fresh_pass_grouped_mixed(qt, n):
    """640: five groups of two whole waves; 700: 140 per motion, each group
    ending in a partly empty wave."""
    from quadtrack.controllers import BatchedRiccatiLQR

    mass = np.random.default_rng(3).uniform(0.8, 1.2, n)
    motion = np.arange(n) % 5
    ctl = BatchedRiccatiLQR({"dt": 0.01}, mass=torch.as_tensor(mass, device="cuda"))
    _both(ctl, {"target": {"motion_type": "stationary"}}, n, 3000, motion=motion, plant_mass=mass)


@pytest.mark.parametrize("n,nsteps", [(0, 3000), (70, 0)])
def test_fresh_pass_edges(qt, n, nsteps):
    from quadtrack.controllers import BatchedRiccatiLQR

    if n == 0:
        from quadtrack import core
        from quadtrack.env.config import EnvConfig
        from quadtrack.rollout import build_batch

        cfg = EnvConfig.from_dict({"target": {"motion_type": "linear"}})
        ctl = BatchedRiccatiLQR({"dt": 0.01})
        batch = build_batch(ctl, cfg, 0, seeds=np.arange(0))
        met = core.rollout_fresh(cfg.to_params(), ctl.ctrl, core.criteria(), batch,
                                 core.RolloutState.empty(0, batch.device), nsteps)
        assert tuple(met.shape)[1] == 0
        return
    met = _both(BatchedRiccatiLQR({"dt": 0.01}), {"target": {"motion_type": "linear"}}, n, nsteps)
    assert np.all(met == 0.0)
