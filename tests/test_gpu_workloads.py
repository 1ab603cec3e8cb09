"""BASELINE.json configs 3-5 on the GPU (quadtrack.workloads) against the
oracle on seeded samples, plus shard independence.

Each sample is a shard [lo, lo + n) taken from the middle of the config's
global episode range, so the per-episode inputs exercise the global-index
functions (tuner stream advanced to candidate lo, mass seeds 1e9 + i, motion
i mod 5).  The oracle side derives every per-episode input independently:
Q/R from the reference tuner's sequential draws, K from its own DARE, masses
from numpy default_rng, reset draws from numpy.  Tolerance as in
test_gpu_parity: 1e-5 absolute (north star), 1e-8 relative.
"""

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def qt():
    import quadtrack

    quadtrack._abi.require_gpu()
    return quadtrack


def _tuner_stream(lo, hi):
    """The reference's _generate_random_config (tuning.py:683-735) called hi
    times on default_rng(42), sequential scalar draws; candidates lo..hi-1."""
    r = np.random.default_rng(42)
    out = []
    for _ in range(hi):
        qp = [float(r.uniform(a, b)) for a, b in zip([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0])]
        qv = [float(r.uniform(a, b)) for a, b in zip([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0])]
        rc = [float(r.uniform(0.5, 2.0)) for _ in range(4)]
        out.append({"q_pos": qp, "q_vel": qv, "r_controls": rc})
    return out[lo:]


def _oracle_shard(config, lo, hi, idx=None):
    """(met[n,14], xf[n,12]) of episodes lo..hi-1 (or the global indices idx)
    of `config` by the oracle."""
    idx = np.arange(lo, hi) if idx is None else np.asarray(idx)
    n = len(idx)
    motion = {3: 3, 4: 2}.get(config)
    motions = idx % 5 if config == 5 else np.full(n, motion)
    env = O.env_params({"target": {"motion_type": O.MOTIONS[motions[0]]}})
    pat = np.zeros((n, 4))
    off = np.zeros((n, 3))
    for m in np.unique(motions):
        sel = motions == m
        pat[sel], off[sel] = O.draws(int(m), idx[sel])
    x0 = np.array([O.initial_state(env, int(motions[i]), pat[i], off[i]) for i in range(n)])
    mass = hover = None
    if config == 3:
        c, K, kc, _, _ = O.controller({"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2],
                                       "integral_limit": 10.0, "integral_zero_threshold": 0.01})
        per = False
    elif config == 4:
        Ks = []
        for cand in _tuner_stream(lo, hi):
            c, K, kc, fb, _ = O.controller(dict(cand, dt=0.01))
            assert not fb
            Ks.append(K)
        K, per = np.array(Ks), True
    else:
        mass = np.array([np.random.default_rng(10**9 + int(i)).uniform(0.8, 1.2) for i in idx])
        Ks = []
        for m in mass:
            c, K, kc, fb, _ = O.controller({"dt": 0.01, "mass": float(m)})
            Ks.append(K)
        K, per = np.array(Ks), True
        hover = mass * 9.81
    mo = motions.astype(np.int8) if config == 5 else None
    met, xf, integ, _ = O.rollout(env, c, O.criteria(), mo, pat, mass, hover, K, kc, per, x0)
    return met, xf, mass


# (5, 777777, 700): 140 episodes per motion, so the grouped launch's
# stationary riders fill the other groups' last waves (core.grouped_waves:
# 12 waves, 15 without riders) and rider episodes are in the oracle sample
@pytest.mark.parametrize("config,lo,n", [(3, 40000, 384), (4, 200001, 384), (5, 777777, 640), (5, 777777, 700)])
def test_workload_sample_vs_oracle(qt, config, lo, n):
    from quadtrack import workloads
    from quadtrack.rollout import run_closed_loop

    sh = workloads.build(config, lo, lo + n)
    res = run_closed_loop(sh.controller, **sh.run_kwargs())
    met = res.metrics.cpu().numpy()
    om, oxf, mass = _oracle_shard(config, lo, lo + n)
    if mass is not None:
        np.testing.assert_array_equal(sh.plant_mass.cpu().numpy(), mass)  # device draws == numpy, bit for bit
    np.testing.assert_allclose(met.T, om, rtol=1e-8, atol=TOL)
    np.testing.assert_allclose(res.state.x.cpu().numpy().T, oxf, rtol=1e-8, atol=TOL)


def test_config3_full_size(qt):
    """Config 3 (BASELINE configs[2]) at its full 65,536 episodes in one
    launch: LQI with the reference's weights on the sinusoidal target, which
    diverges (the integral saturates, z falls by hundreds of
    metres; riccati_lqr.py:870-900).  Size-independent properties on every
    episode, a seeded 512-episode sample against the oracle, and two of four
    shards bitwise equal to the full run."""
    from quadtrack import workloads
    from quadtrack._abi import MET
    from quadtrack.rollout import run_closed_loop

    total = workloads.EPISODES[3]
    full = workloads.build(3)
    res = run_closed_loop(full.controller, **full.run_kwargs())
    met = res.metrics.cpu().numpy()
    steps, term = met[MET["steps"]], met[MET["termination_code"]]
    assert np.all(np.isfinite(met)) and bool(torch.isfinite(res.state.x).all())
    # every episode ends: the 3,000-step time limit or the 1,000 m position bound
    assert np.all((term == 1) & (steps == 3000) | (term == 2) & (steps < 3000))
    rms, mean, mx = met[MET["rms_tracking_error"]], met[MET["mean_tracking_error"]], met[MET["max_tracking_error"]]
    assert np.all(rms >= mean - 1e-12) and np.all(mx >= rms - 1e-12)
    assert np.all(np.abs(res.state.integ[:3].cpu().numpy()) <= 10.0)  # integral_limit
    assert float(np.median(mean)) > 10.0  # the reference's divergence, not a tracking run
    sample = np.sort(np.random.default_rng(3).choice(total, 512, replace=False))
    om, oxf, _ = _oracle_shard(3, 0, 0, idx=sample)
    np.testing.assert_allclose(met[:, sample].T, om, rtol=1e-8, atol=TOL)
    np.testing.assert_allclose(res.state.x.cpu().numpy()[:, sample].T, oxf, rtol=1e-8, atol=TOL)
    for r in (1, 2):
        lo, hi = workloads.shard_bounds(total, r, 4)
        sh = workloads.build(3, lo, hi)
        part = run_closed_loop(sh.controller, **sh.run_kwargs())
        assert torch.equal(part.metrics, res.metrics[:, lo:hi])


@pytest.mark.parametrize("config", [4, 5])
def test_workload_full_size_and_shard_independence(qt, config):
    """The whole config on one GPU; then a 4-way sharding of it reproduces
    every per-episode metric bit for bit (results independent of W)."""
    from quadtrack import workloads
    from quadtrack._abi import MET
    from quadtrack.rollout import run_closed_loop

    total = workloads.EPISODES[config]
    full = workloads.build(config)
    res = run_closed_loop(full.controller, **full.run_kwargs())
    met = res.metrics
    assert bool(torch.isfinite(met).all())
    assert int((met[MET["termination_code"]] == 0).sum()) == 0  # every episode terminated
    if config == 5:
        assert full.controller.status.eq(0).all()
    for r in range(4):
        lo, hi = workloads.shard_bounds(total, r, 4)
        if r not in (0, 3):
            continue  # two shards are enough to pin the property; keeps the test short
        sh = workloads.build(config, lo, hi)
        part = run_closed_loop(sh.controller, **sh.run_kwargs())
        assert torch.equal(part.metrics, met[:, lo:hi])
    if config == 5:
        # the 8-GPU layout: every rank's 131,072-episode shard is 2,048 whole
        # waves (stationary riders in the other groups' last waves; 2,050
        # without), and its results are still the full run's bit for bit
        from quadtrack import core

        for r in (0, 3, 7):
            lo, hi = workloads.shard_bounds(total, r, 8)
            sh = workloads.build(config, lo, hi)
            part = run_closed_loop(sh.controller, **sh.run_kwargs())
            assert core.launch_waves(part.batch) == 2048
            assert core.grouped_waves(*part.batch.groups, riders=False) == 2050
            assert torch.equal(part.metrics, met[:, lo:hi])
    del res, full
    torch.cuda.empty_cache()


@pytest.mark.parametrize("case", ["lqi", "pid", "feedforward", "mass"])
def test_riders_bitwise_other_loops(qt, monkeypatch, case):
    """Stationary riders in the other controllers' and options' loops: LQI
    (9-column gains, folded target rotor), PID (3 gains, observation time),
    feed-forward (the target acceleration a rider must see as zero) and
    per-episode plant mass with per-episode gains (config 5's form).  With
    riders and without (QT_RIDERS=0) bit for bit: metrics, state, target
    observation and controller integral."""
    from quadtrack.controllers import BatchedPID, BatchedRiccatiLQR
    from quadtrack.rollout import run_closed_loop

    n = 1100
    motion = [i % 5 for i in range(n)]
    mass = None
    if case == "lqi":
        ctl = BatchedRiccatiLQR({"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2],
                                 "integral_limit": 10.0, "integral_zero_threshold": 0.01})
    elif case == "pid":
        ctl = BatchedPID({})
    elif case == "feedforward":
        ctl = BatchedRiccatiLQR({"dt": 0.01, "feedforward_enabled": True, "ff_velocity_gain": 0.5,
                                 "ff_acceleration_gain": 0.2})
    else:
        mass = 0.8 + 0.4 * np.random.default_rng(5).random(n)
        ctl = BatchedRiccatiLQR({"dt": 0.01}, mass=mass)
    runs = {}
    for riders in ("1", "0"):
        monkeypatch.setenv("QT_RIDERS", riders)
        runs[riders] = run_closed_loop(ctl, {}, n=n, seeds=np.arange(n), motion=motion, plant_mass=mass,
                                       max_steps=700)
    a, b = runs["1"], runs["0"]
    assert a.batch.groups is not None
    assert torch.equal(a.metrics, b.metrics)
    assert torch.equal(a.state.x, b.state.x)
    assert torch.equal(a.state.target, b.state.target)
    assert torch.equal(a.state.integ, b.state.integ)


def test_riders_bitwise_and_deferred(qt, monkeypatch):
    """Stationary riders (qt_rollout_grouped's one-launch layout): a mixed
    batch run with riders equals the same batch with QT_RIDERS=0 bit for bit
    (a rider runs its group's loop with the stationary target selected per
    lane: the stationary loop's numbers), with fewer waves.  Then a rider
    and a host lane of the same wave, and a stationary episode in its own
    group, start outside the fast preconditions (roll beyond the tilt clamp):
    their waves go to the exact pass, which runs each episode with its own
    motion; the results match the exact step everywhere (recording) to 1e-9."""
    from quadtrack import core
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.rollout import build_batch, run_closed_loop

    n = 1100  # 220 per motion: each group's last wave has 36 free lanes
    motion = [i % 5 for i in range(n)]
    ctl = BatchedRiccatiLQR({"dt": 0.01})
    monkeypatch.setenv("QT_PAIR_ROUNDS", "0")  # the plain group layout: the slots named below
    runs = {}
    for riders in ("1", "0"):
        monkeypatch.setenv("QT_RIDERS", riders)
        runs[riders] = run_closed_loop(ctl, {}, n=n, seeds=np.arange(n), motion=motion, max_steps=600)
    g = runs["1"].batch.groups
    assert core.grouped_waves(*g, riders=True) == 18 and core.grouped_waves(*g, riders=False) == 20
    assert torch.equal(runs["1"].metrics, runs["0"].metrics)
    assert torch.equal(runs["1"].state.x, runs["0"].state.x)
    assert torch.equal(runs["1"].state.target, runs["0"].state.target)

    monkeypatch.setenv("QT_RIDERS", "1")
    from quadtrack.env.config import EnvConfig

    env = EnvConfig.from_dict({}).to_params()
    crit = core.criteria()
    out = []
    for record in (False, True):
        batch, perm = build_batch(ctl, {}, n, seeds=np.arange(n), motion=motion).physical_groups()
        st = core.RolloutState.empty(n, batch.device)
        core.reset(env, batch, st)
        # slots in group order sinusoidal, figure-8, circular, linear,
        # stationary (220 each): slot 880 rides in the sinusoidal group's last
        # wave (slots 192..219 + riders), slot 200 is a host lane of that wave,
        # slot 1090 a stationary episode in the stationary group's own waves
        for slot in (880, 200, 1090):
            st.x[6, slot] = 1.2
        for k in (150, 450):
            rec = torch.full((k, 16, n), float("nan"), dtype=torch.float64, device=batch.device) if record else None
            core.rollout(env, ctl.ctrl, crit, batch, st, k, rec)
        out.append((core.episode_metrics(crit, st).cpu().numpy(), st.x.cpu().numpy()))
    (mf, xf), (me, xe) = out
    np.testing.assert_array_equal(mf[O.MET_FIELDS.index("steps")], me[O.MET_FIELDS.index("steps")])
    np.testing.assert_allclose(mf, me, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(xf, xe, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("horizon", [450, 3000])
def test_batched_tuner_vs_sequential_oracle(qt, horizon):
    """BatchedTuner.tune() (all candidates x episodes in one rollout) against
    the reference tuner's loop restated on the oracle: per candidate one
    controller, evaluation_episodes fresh episodes with seeds seed + ep
    (tuning.py:846-928), score = mean ratio - 0.1 mean error."""
    from quadtrack import tuning

    cfg = tuning.TuningConfig(controller_type="riccati_lqr", search_space=tuning.default_search_space(),
                              max_iterations=24, evaluation_episodes=3, target_motion_type="circular",
                              episode_length=5.0, evaluation_horizon=horizon, seed=42)
    res = tuning.BatchedTuner(cfg).tune()
    assert res.iterations_completed == 24
    cands = _tuner_stream(0, 24)
    env = O.env_params({"simulation": {"max_episode_time": 5.0}, "target": {"motion_type": "circular"}})
    crit = O.criteria(0.8, 5.0, 0.5)
    seeds = 42 + np.arange(3)
    pat, off = O.draws("circular", seeds)
    x0 = np.array([O.initial_state(env, 2, pat[i], off[i]) for i in range(3)])
    best = -np.inf
    for k, cand in enumerate(cands):
        assert res.all_results[k]["config"] == cand
        c, K, kc, _, _ = O.controller(dict(cand, dt=0.01))
        met, _, _, _ = O.rollout(env, c, crit, None, pat, None, None, K, kc, False, x0, max_steps=horizon)
        ratio = met[:, O.MET_FIELDS.index("on_target_ratio")]
        err = met[:, O.MET_FIELDS.index("mean_tracking_error")]
        score = np.mean(list(ratio)) - 0.1 * np.mean(list(err))
        got = res.all_results[k]
        assert got["score"] == pytest.approx(score, rel=1e-9, abs=1e-9)
        assert got["metrics"]["mean_on_target_ratio"] == pytest.approx(np.mean(list(ratio)), abs=1e-12)
        best = max(best, score)
    assert res.best_score == pytest.approx(best, rel=1e-9, abs=1e-9)


@pytest.mark.parametrize("case", ["circular", "sinusoidal", "figure8", "pid_circular", "pid_figure8"])
def test_clamping_no_vote_body_is_bitwise_the_voted_loop(qt, monkeypatch, case):
    """run_yaw0's DUAL body (a clamping no-vote horizon for waves whose
    tilt-bounded horizon is short) against the same launches with it turned
    off (QT_DUAL_BELOW=0: those waves take voted steps): every metric and the
    final state bit for bit.  Riccati-LQR on config-4 waves (tuner candidates;
    on the circular target a lane at the tilt clamp makes 46% of the steps
    voted without it) for each target DUAL is compiled for, and a saturating
    PID (the 3-column loop) whose lanes sit at the tilt clamp."""
    from quadtrack import workloads
    from quadtrack.controllers import BatchedPID
    from quadtrack.rollout import run_closed_loop

    sh = workloads.build(4, 100000, 100000 + 2048)
    kw = sh.run_kwargs()
    ctl = sh.controller
    motion = case.split("_")[-1]
    kw["env_config"] = {"target": {"motion_type": motion, "speed": 3.0 if case.startswith("pid") else 1.0}}
    if case.startswith("pid"):
        ctl = BatchedPID({"kp_pos": [2.0, 2.0, 30.0], "kd_pos": [1.0, 1.0, 10.0], "max_thrust": 18.0,
                          "max_rate": 2.0})
        kw["n"] = 2048
    res = []
    for below in ("0", None):
        if below is None:
            monkeypatch.delenv("QT_DUAL_BELOW", raising=False)
        else:
            monkeypatch.setenv("QT_DUAL_BELOW", below)
        r = run_closed_loop(ctl, **kw)
        res.append((r.metrics.clone(), r.state.x.clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
