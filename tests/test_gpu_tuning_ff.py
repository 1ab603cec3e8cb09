"""Batched tuning of the reference's other controller types and per-episode
feed-forward (qt_batch.ff), on the GPU against the oracle.

* BatchedTuner for "pid" and "lqr" with the reference's default search spaces
  (scripts/controller_autotune.py:360-385) plus feed-forward gain ranges, in
  the reference's candidate stream order (_generate_random_config,
  controllers/tuning.py:683-735), scored as _evaluate_config (846-928).
* A Riccati batch with FF enabled where some episodes' DARE fails: those run
  the heuristic fallback WITHOUT feed-forward (riccati_lqr.py:764-776), the
  others with it."""

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qt():
    import quadtrack

    quadtrack._abi.require_gpu("cuda:0")
    return quadtrack


def _stream(space: dict, n: int, seed: int = 42):
    """The reference's random candidates: parameters in _generate_random_config's
    order, one scalar uniform per component from default_rng(seed)."""
    order = ["kp_pos", "ki_pos", "kd_pos", "ff_velocity_gain", "ff_acceleration_gain", "q_pos", "q_vel",
             "r_thrust", "r_rate", "r_controls", "q_int"]
    r = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        cfg = {}
        for name in order:
            if name not in space:
                continue
            lo, hi = space[name]
            if np.ndim(lo) == 0:
                cfg[name] = float(r.uniform(lo, hi))
            else:
                cfg[name] = [float(r.uniform(a, b)) for a, b in zip(lo, hi)]
            if name.startswith("ff_"):
                cfg["feedforward_enabled"] = True
        out.append(cfg)
    return out


SPACES = {
    "pid": {"kp_pos": ([0.005, 0.005, 2.0], [0.05, 0.05, 6.0]), "kd_pos": ([0.02, 0.02, 1.0], [0.15, 0.15, 3.0]),
            "ff_velocity_gain": ([0.0, 0.0, 0.0], [0.5, 0.5, 0.3]),
            "ff_acceleration_gain": ([0.0, 0.0, 0.0], [0.2, 0.2, 0.2])},
    "lqr": {"q_pos": ([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0]), "q_vel": ([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0]),
            "ff_velocity_gain": ([0.0, 0.0, 0.0], [0.5, 0.5, 0.3])},
    "riccati_lqr": {"q_pos": ([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0]),
                    "ff_acceleration_gain": ([0.0, 0.0, 0.0], [0.3, 0.3, 0.3])},
}


@pytest.mark.parametrize("kind", ["pid", "lqr", "riccati_lqr"])
def test_batched_tuner_types_and_ff_ranges_vs_oracle(qt, kind):
    from quadtrack import tuning

    sp = SPACES[kind]
    space = tuning.GainSearchSpace(**{f"{k}_range": v for k, v in sp.items()})
    cfg = tuning.TuningConfig(controller_type=kind, search_space=space, max_iterations=12, evaluation_episodes=3,
                              target_motion_type="circular", episode_length=5.0, evaluation_horizon=450, seed=42)
    res = tuning.BatchedTuner(cfg).tune()
    cands = _stream(sp, 12)
    env = O.env_params({"simulation": {"max_episode_time": 5.0}, "target": {"motion_type": "circular"}})
    crit = O.criteria(0.8, 5.0, 0.5)
    seeds = 42 + np.arange(3)
    pat, off = O.draws("circular", seeds)
    x0 = np.array([O.initial_state(env, 2, pat[i], off[i]) for i in range(3)])
    best = -np.inf
    for k, cand in enumerate(cands):
        got = res.all_results[k]
        assert _same_config(got["config"], cand), (got["config"], cand)
        c, K, kc, _, _ = O.controller(dict(cand, controller=kind, dt=0.01) if kind != "riccati_lqr"
                                      else dict(cand, dt=0.01))
        met, _, _, _ = O.rollout(env, c, crit, None, pat, None, None, K, kc, False, x0, max_steps=450)
        ratio = met[:, O.MET_FIELDS.index("on_target_ratio")]
        err = met[:, O.MET_FIELDS.index("mean_tracking_error")]
        score = np.mean(list(ratio)) - 0.1 * np.mean(list(err))
        assert got["score"] == pytest.approx(score, rel=1e-9, abs=1e-9), (k, cand)
        best = max(best, score)
    assert res.best_score == pytest.approx(best, rel=1e-9, abs=1e-9)


def _same_config(a: dict, b: dict) -> bool:
    if set(a) != set(b):
        return False
    for k in a:
        if np.asarray(a[k], float).tolist() != np.asarray(b[k], float).tolist():
            return False
    return True


def test_failed_dare_episodes_run_without_feedforward(qt):
    """Mixed valid / invalid per-episode R with feed-forward on: the DARE
    fails where R is not positive definite, those episodes take the heuristic
    gains and no feed-forward (riccati_lqr.py:737-777), the rest keep it."""
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.rollout import run_closed_loop

    n = 64
    bad = np.arange(n) % 3 == 1
    rc = np.where(bad[:, None], [1.0, 0.0, 1.0, 1.0], [1.0, 1.0, 1.0, 1.0])
    cfg = {"dt": 0.01, "feedforward_enabled": True, "ff_velocity_gain": [0.3, 0.3, 0.2],
           "ff_acceleration_gain": [0.2, 0.2, 0.4], "ff_max_velocity": 0.8}
    ctl = BatchedRiccatiLQR(cfg, r_controls=rc)
    assert ctl.ff is not None
    assert (ctl.status.cpu().numpy() != 0).tolist() == bad.tolist()
    env_cfg = {"target": {"motion_type": "circular", "speed": 1.5}}
    res = run_closed_loop(ctl, env_cfg, n=n, seeds=np.arange(n), max_steps=600)
    gpu = res.metrics.cpu().numpy().T
    env = O.env_params(env_cfg)
    pat, off = O.draws("circular", range(n))
    x0 = np.array([O.initial_state(env, 2, pat[i], off[i]) for i in range(n)])
    for sel, failed in ((bad, True), (~bad, False)):
        c, K, kc, fb, _ = O.controller(dict(cfg, r_controls=list(rc[np.argmax(sel)])))
        assert fb == failed
        assert c.feedforward_enabled == (0 if fb else 1)
        met, xf, _, _ = O.rollout(env, c, O.criteria(), None, pat[sel], None, None, K, kc, False, x0[sel],
                                  max_steps=600)
        np.testing.assert_allclose(gpu[sel], met, rtol=1e-8, atol=1e-8)
        np.testing.assert_allclose(res.state.x.cpu().numpy().T[sel], xf, rtol=1e-8, atol=1e-8)


def test_per_episode_ff_off_equals_no_ff(qt):
    """A lane whose per-episode feed-forward is off (gains 0, no clamp) runs
    exactly as a batch without feed-forward."""
    from quadtrack import core
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.rollout import build_batch, run_closed_loop

    n = 256
    env_cfg = {"target": {"motion_type": "sinusoidal"}}
    plain = BatchedRiccatiLQR({"dt": 0.01})
    a = run_closed_loop(plain, env_cfg, n=n, seeds=np.arange(n), max_steps=500)
    withff = BatchedRiccatiLQR({"dt": 0.01})
    withff.ff = core.ff_rows(n, withff.device, enabled=False)
    withff.ctrl.feedforward_enabled = 0
    b = run_closed_loop(withff, env_cfg, n=n, seeds=np.arange(n), max_steps=500)
    np.testing.assert_allclose(b.metrics.cpu().numpy(), a.metrics.cpu().numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(b.state.x.cpu().numpy(), a.state.x.cpu().numpy(), rtol=1e-12, atol=1e-12)


CAND_EXTRA = {
    # mass varies per candidate (a per-candidate array: DARE model + hover thrust), max_thrust is common
    "riccati_lqr": [{"q_pos": [2e-4, 2e-4, 14.0], "mass": 1.2, "max_thrust": 18.0},
                    {"q_pos": [1e-4, 1e-4, 20.0], "mass": 0.9, "max_thrust": 18.0}],
    # PIDController's kp / kd aliases (config.get("kp_pos", config.get("kp", ...))) and a common integral limit
    "pid": [{"kp": [0.02, 0.02, 5.0], "kd": [0.1, 0.1, 2.5], "integral_limit": 2.0},
            {"kp": [0.01, 0.01, 3.0], "kd_pos": [0.05, 0.05, 1.5], "kd": [9.0, 9.0, 9.0], "integral_limit": 2.0}],
    "lqr": [{"q_pos": [3e-4, 3e-4, 12.0], "mass": 1.1}, {"r_thrust": 2.0, "mass": 1.0, "max_rate": 2.5}],
}


@pytest.mark.parametrize("kind", ["riccati_lqr", "pid", "lqr"])
def test_tuner_candidate_keys_reach_the_controller(qt, kind):
    """Every key of a candidate config reaches its controller, as the
    reference builds one controller from each whole candidate dict
    (controllers/tuning.py:832-844): per-candidate mass, PID's kp / kd aliases,
    common clamps; _evaluate_config's score equals the oracle's for that config."""
    from quadtrack import tuning

    cands = CAND_EXTRA[kind]
    if kind == "lqr":  # max_rate only on the second candidate: differs -> must raise
        cfg = tuning.TuningConfig(controller_type=kind, max_iterations=2, evaluation_episodes=2,
                                  target_motion_type="circular", episode_length=3.0, evaluation_horizon=300, seed=7)
        with pytest.raises(ValueError, match="max_rate"):
            tuning.BatchedTuner(cfg).evaluate_configs(cands)
        cands = [dict(c, max_rate=2.5) for c in cands]
    cfg = tuning.TuningConfig(controller_type=kind, max_iterations=2, evaluation_episodes=2,
                              target_motion_type="circular", episode_length=3.0, evaluation_horizon=300, seed=7)
    tuner = tuning.BatchedTuner(cfg)
    batch = tuner.evaluate_configs(cands)
    env = O.env_params({"simulation": {"max_episode_time": 3.0}, "target": {"motion_type": "circular"}})
    crit = O.criteria(0.8, 3.0, 0.5)
    seeds = 7 + np.arange(2)
    pat, off = O.draws("circular", seeds)
    x0 = np.array([O.initial_state(env, 2, pat[i], off[i]) for i in range(2)])
    for k, cand in enumerate(cands):
        c, K, kc, _, _ = O.controller(dict(cand, controller=kind, dt=0.01) if kind != "riccati_lqr"
                                      else dict(cand, dt=0.01))
        met, _, _, _ = O.rollout(env, c, crit, None, pat, None, None, K, kc, False, x0, max_steps=300)
        ratio = met[:, O.MET_FIELDS.index("on_target_ratio")]
        err = met[:, O.MET_FIELDS.index("mean_tracking_error")]
        score = np.mean(list(ratio)) - 0.1 * np.mean(list(err))
        one, _ = tuner._evaluate_config(cand)
        assert batch[k][0] == pytest.approx(score, rel=1e-9, abs=1e-9), (k, cand)
        assert one == pytest.approx(score, rel=1e-9, abs=1e-9), (k, cand)
