"""The pair-lane yaw-at-rest flavour (csrc/qt_pair.hpp) against the one-lane
flavour it replaces for small batches: QT_PAIR=1 (default) and QT_PAIR=0 on
the same batch must agree bit for bit — metrics, final state, target
observation, accumulators — for every path the pair kernel takes: fresh
passes, chunked launches (the accumulators and the lagged command-norm sum
carried across launches), the stop vote and the exact finish (speed clamp,
position bounds, time limit), waves deferred to the exact pass, ragged batch
sizes, Euler, the stationary target.  One sample against the oracle as well.
Reference loop: env/quadcopter_env.py:152-232, eval.py:119-165."""

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qt():
    import quadtrack

    quadtrack._abi.require_gpu()
    return quadtrack


def _both(monkeypatch, fn):
    out = {}
    for pair in ("1", "0"):
        monkeypatch.setenv("QT_PAIR", pair)
        out[pair] = fn()
    return out["1"], out["0"]


def _same(a, b):
    assert torch.equal(a.metrics, b.metrics)
    for f in ("x", "t", "acc", "target", "integ"):
        assert torch.equal(getattr(a.state, f), getattr(b.state, f)), f


def _limits(i):
    """Randomised limits (as tests/test_gpu_horizon.py's) that make episodes
    stop inside the loop: the speed clamp's guard, the position bound, the
    time limit."""
    r = np.random.default_rng(2000 + i)
    dt = float(r.choice([0.005, 0.01, 0.02]))
    motion = ["linear", "stationary", "circular", "sinusoidal", "figure8"][i % 5]
    env = {"target": {"motion_type": motion, "speed": float(r.uniform(0.5, 4.0))},
           "simulation": {"dt": dt, "max_velocity": float(r.uniform(1.0, 4.0)),
                          "max_position": float(r.uniform(2.5, 8.0)),
                          "max_episode_time": float(np.round(r.uniform(4.0, 12.0), 3))},
           "quadcopter": {"max_angular_rate": 3.0}}
    if i >= 5:
        env["simulation"]["integrator"] = "euler"
    ctl = {"dt": dt, "max_rate": float(r.uniform(1.0, 3.0)), "q_pos": [float(r.uniform(1e-4, 5.0))] * 2 + [16.0]}
    return env, ctl


@pytest.mark.parametrize("motion,n,sim", [
    ("linear", 8192, {}),
    ("linear", 777, {}),
    ("linear", 1, {}),
    ("stationary", 4096, {}),
    ("linear", 2048, {"integrator": "euler"}),
    ("circular", 4100, {}),
    ("sinusoidal", 3000, {}),
    ("figure8", 3333, {}),
    ("circular", 1500, {"integrator": "euler"}),
])
def test_pair_flavour_bitwise_fresh(qt, monkeypatch, motion, n, sim):
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.rollout import run_closed_loop

    ctl = BatchedRiccatiLQR({"dt": 0.01})
    cfg = {"target": {"motion_type": motion}, "simulation": dict(sim)}
    a, b = _both(monkeypatch, lambda: run_closed_loop(ctl, cfg, n=n, seeds=np.arange(n) + 11))
    _same(a, b)


@pytest.mark.parametrize("i", range(8))
def test_pair_flavour_bitwise_limits(qt, monkeypatch, i):
    from quadtrack._abi import MET
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.rollout import run_closed_loop

    env, ctl_cfg = _limits(i)
    ctl = BatchedRiccatiLQR(ctl_cfg)
    n = 3000
    a, b = _both(monkeypatch, lambda: run_closed_loop(ctl, env, n=n, seeds=np.arange(n)))
    _same(a, b)
    if env["target"]["motion_type"] == "linear":  # the linear sets do stop episodes inside the loop
        assert int((a.metrics[MET["termination_code"]] != 1).sum()) > 0


def test_pair_flavour_bitwise_config4_shard(qt, monkeypatch):
    """Config 4 (the tuner's candidates: per-episode structured gains, circular
    target) on 8 GPUs: a 32,768-episode rank shard runs the pair flavour and
    equals the one-lane run bit for bit (test_gpu_workloads' 384-episode
    config-4 sample against the oracle runs the pair flavour too)."""
    from quadtrack import workloads
    from quadtrack.rollout import run_closed_loop

    total = workloads.EPISODES[4]
    lo, hi = workloads.shard_bounds(total, 5, 8)
    assert hi - lo == 32768
    sh = workloads.build(4, lo, hi)
    a, b = _both(monkeypatch, lambda: run_closed_loop(sh.controller, **sh.run_kwargs()))
    _same(a, b)


def test_pair_flavour_bitwise_chunked(qt, monkeypatch):
    """Launches of 137 steps: the state, accumulators and the pair's lagged sum
    of command norms carried across launches.  (Chunking itself moves the
    last bits in either flavour: a launch starts from the attitude's directly
    evaluated sin / cos, a running loop carries them.)"""
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.rollout import run_closed_loop

    ctl = BatchedRiccatiLQR({"dt": 0.01})
    n = 5000
    lin = {"target": {"motion_type": "linear"}}
    a, b = _both(monkeypatch, lambda: run_closed_loop(ctl, lin, n=n, seeds=np.arange(n), chunk=137))
    _same(a, b)


def test_pair_flavour_deferred_waves(qt, monkeypatch):
    """Episodes outside the yaw-at-rest preconditions (roll beyond the tilt
    clamp): the pair kernel leaves their whole 64-episode waves to the exact
    pass (the exact pass's wave test), which runs them; the same results as
    the one-lane launch set, and as recording the exact step everywhere."""
    from quadtrack import core
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.env.config import EnvConfig
    from quadtrack.rollout import build_batch

    n = 1000
    ctl = BatchedRiccatiLQR({"dt": 0.01})
    lin = {"target": {"motion_type": "linear"}}
    env = EnvConfig.from_dict(lin).to_params()
    crit = core.criteria()

    def run(record=False):
        batch = build_batch(ctl, lin, n, seeds=np.arange(n))
        st = core.RolloutState.empty(n, batch.device)
        core.reset(env, batch, st)
        for slot in (5, 100, 101, 999):  # waves 0, 1 and 15 (the last, partial) defer
            st.x[6, slot] = 1.2
        for k in (150, 450):
            rec = torch.full((k, 16, n), float("nan"), dtype=torch.float64, device=batch.device) if record else None
            core.rollout(env, ctl.ctrl, crit, batch, st, k, rec)
        return core.episode_metrics(crit, st), st

    (ma, sa), (mb, sb) = _both(monkeypatch, run)
    assert torch.equal(ma, mb)
    for f in ("x", "acc", "target", "t"):
        assert torch.equal(getattr(sa, f), getattr(sb, f)), f
    me, se = run(record=True)
    np.testing.assert_allclose(ma.cpu().numpy(), me.cpu().numpy(), rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(sa.x.cpu().numpy(), se.x.cpu().numpy(), rtol=1e-9, atol=1e-9)


def test_pair_flavour_vs_oracle(qt, monkeypatch):
    """Config 2's loop (linear target, Riccati-LQR) at 8,192 episodes through
    the pair flavour: a seeded 256-episode sample against the oracle at the
    north star's 1e-5 / 1e-8."""
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.rollout import run_closed_loop

    monkeypatch.setenv("QT_PAIR", "1")
    n = 8192
    ctl = BatchedRiccatiLQR({"dt": 0.01})
    res = run_closed_loop(ctl, {"target": {"motion_type": "linear"}}, n=n, seeds=np.arange(n))
    idx = np.sort(np.random.default_rng(8).choice(n, 256, replace=False))
    env = O.env_params({"target": {"motion_type": "linear"}})
    pat, off = O.draws(O.MOTIONS.index("linear"), idx)
    x0 = np.array([O.initial_state(env, O.MOTIONS.index("linear"), pat[i], off[i]) for i in range(len(idx))])
    c, K, kc, _, _ = O.controller({"dt": 0.01})
    met, xf, _, _ = O.rollout(env, c, O.criteria(), None, pat, None, None, K, kc, False, x0)
    np.testing.assert_allclose(res.metrics.cpu().numpy()[:, idx].T, met, rtol=1e-8, atol=1e-5)
    np.testing.assert_allclose(res.state.x.cpu().numpy()[:, idx].T, xf, rtol=1e-8, atol=1e-5)


def test_pair_flavour_runs_the_pair_kernel(qt, monkeypatch):
    """The dispatch: a small linear batch launches rollout_pair_kernel, a batch
    beyond one wave per SIMD in pairs (or QT_PAIR=0) the one-lane kernel."""
    from torch.profiler import ProfilerActivity, profile

    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.rollout import run_closed_loop

    ctl = BatchedRiccatiLQR({"dt": 0.01})
    lanes = torch.cuda.get_device_properties(0).multi_processor_count * 4 * 64

    def kernels(n, pair):
        monkeypatch.setenv("QT_PAIR", pair)
        lin = {"target": {"motion_type": "linear"}}
        run_closed_loop(ctl, lin, n=n, seeds=np.arange(n), max_steps=20)  # warm
        with profile(activities=[ProfilerActivity.CUDA]) as p:
            run_closed_loop(ctl, lin, n=n, seeds=np.arange(n), max_steps=20)
            torch.cuda.synchronize()
        return " ".join(e.name for e in p.events())

    small = kernels(4096, "1")
    if "rollout" not in small:
        pytest.skip("the profiler records no kernel names here")
    assert "rollout_pair_kernel" in small
    assert "rollout_pair_kernel" not in kernels(4096, "0")
    assert "rollout_pair_kernel" not in kernels(lanes // 2 + 64, "1")
