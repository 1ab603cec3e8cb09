"""Pin the CPU restatement (oracle/) against the reference's own outputs.

The golden fixtures were produced by running the reference itself
(tests/golden/gen_golden.py); this file checks the oracle against every one
of them, so that the GPU parity tests can lean on the oracle at sizes the
fixtures do not cover.  CPU only.
"""

import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

import oracle as O

SCEN = json.load(open(os.path.join(GOLDEN, "scenarios.json")))
CL = np.load(os.path.join(GOLDEN, "closed_loop.npz"))
FIELDS = SCEN["metric_fields"]

# The figure-8 target acceleration is the reference's 1e-6 forward difference
# of positions (target_motion.py:215-229): it amplifies a 1-ulp sin/cos
# difference ~1e12x.  The oracle calls sin and cos separately (not glibc's
# sincos, which rounds differently) and x**2 as libm pow (oracle/Makefile),
# as numpy does, so its figure-8 targets are bitwise the reference's and the
# feed-forward scenario needs no exception.
ATOL = 1e-6
RTOL = 1e-8


def scenario_episodes(s):
    for e, seed in enumerate(s["seeds"]):
        env_cfg = s["env_per_episode"][e] if "env_per_episode" in s else s["env"]
        ctl_cfg = s["ctl_per_episode"][e] if "ctl_per_episode" in s else s["ctl"]
        yield e, seed, env_cfg, ctl_cfg


@pytest.mark.parametrize("s", SCEN["scenarios"], ids=[s["name"] for s in SCEN["scenarios"]])
def test_closed_loop_matches_reference(s):
    atol = ATOL
    for e, seed, env_cfg, ctl_cfg in scenario_episodes(s):
        env = O.env_params(env_cfg)
        c, K, kc, fb, _ = O.controller(ctl_cfg)
        pat, off = O.draws(env.motion, [seed])
        x0 = O.initial_state(env, env.motion, pat[0], off[0])
        np.testing.assert_allclose(x0, CL[s["name"] + "_x0"][e], rtol=0, atol=1e-15)
        met, xf, integ, rec = O.episode(env, c, O.criteria(), env.motion, pat[0], env.mass, c.hover_thrust, K, kc,
                                        x0, record=s["record"])
        ref = CL[s["name"] + "_metrics"][e]
        for i, f in enumerate(FIELDS):
            assert met[i] == pytest.approx(ref[i], rel=RTOL, abs=atol), (s["name"], seed, f)
        fin = CL[s["name"] + "_final"][e]
        np.testing.assert_allclose(xf, fin[:12], rtol=RTOL, atol=atol)
        np.testing.assert_allclose(integ, fin[12:], rtol=RTOL, atol=atol)
        if s["record"]:
            steps = CL["rec_steps"]
            n = int(ref[FIELDS.index("steps")])
            ok = steps < n
            np.testing.assert_allclose(rec[steps[ok], :12], CL[s["name"] + "_rec_state"][e][ok], rtol=RTOL, atol=atol)
            np.testing.assert_allclose(rec[steps[ok], 12:], CL[s["name"] + "_rec_action"][e][ok], rtol=RTOL,
                                       atol=atol)


def test_config1_known_answer():
    """SURVEY §6 config 1 numbers (stationary, Riccati-LQR, seed 0)."""
    env = O.env_params({})
    c, K, kc, _, _ = O.controller({"dt": 0.01})
    pat, off = O.draws(0, [0])
    met, xf, _, _ = O.episode(env, c, O.criteria(), 0, pat[0], 1.0, c.hover_thrust, K, kc,
                              O.initial_state(env, 0, pat[0], off[0]))
    m = dict(zip(FIELDS, met))
    assert m["steps"] == 3000
    assert m["mean_tracking_error"] == pytest.approx(0.1090241018, abs=1e-10)
    assert m["max_tracking_error"] == pytest.approx(0.5314715107, abs=1e-10)
    assert m["rms_tracking_error"] == pytest.approx(0.1385929022, abs=1e-10)
    assert m["on_target_ratio"] == pytest.approx(0.992333, abs=1e-6)
    assert m["env_on_target_ratio"] == pytest.approx(0.992667, abs=1e-6)
    assert m["mean_control_effort"] == pytest.approx(9.81169732, abs=1e-8)
    np.testing.assert_allclose(xf[:3], [0.0673493918, -0.1132311124, 0.9999439135], atol=1e-10)


def test_dare_matches_scipy_fixtures():
    D = np.load(os.path.join(GOLDEN, "dare_cases.npz"))
    cfgs = json.loads(str(D["configs_json"]))
    for i, cfg in enumerate(cfgs):
        n = int(D["n"][i])
        c, K, kc, fb, P = O.controller(cfg)
        assert bool(fb) == bool(D["fallback"][i]), i
        if fb:
            np.testing.assert_allclose(K, D["K"][i][:, :6], rtol=1e-14, atol=0, equal_nan=True)
            continue
        np.testing.assert_allclose(K, D["K"][i][:, :n], rtol=1e-8, atol=1e-10)
        np.testing.assert_allclose(P, D["P"][i][:n, :n], rtol=1e-8, atol=1e-10)


def test_dare_known_gains():
    """SURVEY §8a A12 known answers."""
    _, K, _, _, _ = O.controller({"dt": 0.01})
    assert K[0, 2] == pytest.approx(3.9313145185949483, rel=1e-10)
    assert K[0, 5] == pytest.approx(3.4441016194677427, rel=1e-10)
    assert K[1, 1] == pytest.approx(-0.009963235396734, rel=1e-9)
    assert K[2, 3] == pytest.approx(0.074915170500119, rel=1e-9)
    _, K, _, _, _ = O.controller({"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2]})
    assert K[0, 8] == pytest.approx(0.098270666075, rel=1e-9)
    assert K[1, 7] == pytest.approx(-0.031384128441, rel=1e-9)
    assert K[2, 6] == pytest.approx(0.031384128441, rel=1e-9)


def test_target_states_match_reference():
    T = np.load(os.path.join(GOLDEN, "target_states.npz"))
    variants = json.loads(str(T["variants_json"]))
    for vi, var in enumerate(variants):
        for mi, m in enumerate(O.MOTIONS):
            tgt = dict(var)
            tgt["motion_type"] = m
            env = O.env_params({"target": tgt})
            ref = T[f"v{vi}_{m}"]
            pats, _ = O.draws(m, T["seeds"])
            for si in range(len(T["seeds"])):
                got = np.array([O.target_state(env, mi, pats[si], t) for t in T["times"]])
                # bitwise: same libm sin / cos / pow, same operation order
                np.testing.assert_array_equal(got, ref[si])


def test_compute_action_sequences():
    A = np.load(os.path.join(GOLDEN, "actions.npz"))
    cases = json.loads(str(A["cases_json"]))
    for ci, cfg in enumerate(cases):
        c, K, kc, fb, _ = O.controller(cfg)
        integ = np.zeros(3)
        for k, obs in enumerate(A["obs"]):
            u, integ, _ = O.compute_action(c, K, kc, obs, integ)
            np.testing.assert_allclose(u, A[f"case{ci}_action"][k], rtol=1e-9, atol=1e-9, err_msg=f"case {ci} k {k}")
            if c.use_lqi:
                np.testing.assert_allclose(integ, A[f"case{ci}_integral"][k], rtol=1e-12, atol=1e-14)


def test_pid_and_heuristic_lqr_action_sequences():
    """PIDController / LQRController.compute_action (controllers/__init__.py)
    over an observation sequence with times (repeated and decreasing ones)."""
    A = np.load(os.path.join(GOLDEN, "controller_actions.npz"))
    cases = json.loads(str(A["cases_json"]))
    for ci, cfg in enumerate(cases):
        c, K, kc, _, _ = O.controller(cfg)
        if kc == 6:
            np.testing.assert_allclose(K, A[f"case{ci}_K"], rtol=1e-15)
        state = np.array([0.0, 0.0, 0.0, np.nan])
        for k, obs in enumerate(A["obs"]):
            if kc == 3:
                u, state, _ = O.compute_action_pid(c, K, np.append(obs, A["time"][k]), state)
                np.testing.assert_allclose(state[:3], A[f"case{ci}_integral"][k], rtol=1e-13, atol=1e-15)
            else:
                u, _, _ = O.compute_action(c, K, kc, obs, np.zeros(3))
            np.testing.assert_allclose(u, A[f"case{ci}_action"][k], rtol=1e-12, atol=1e-12,
                                       err_msg=f"case {ci} k {k}")


def test_lqi_integral_known_answer():
    """The reference's one-step integral test (test_env_dynamics.py:3745-3785)."""
    c, K, kc, _, _ = O.controller({"dt": 0.01, "use_lqi": True, "q_int": [0.01, 0.01, 0.1], "integral_limit": 10.0})
    obs = np.zeros(15)
    obs[0:3] = [0.0, 0.0, 1.0]
    obs[6:9] = [1.0, 0.0, 2.0]
    _, integ, _ = O.compute_action(c, K, kc, obs, np.zeros(3))
    np.testing.assert_allclose(integ, [0.01, 0.0, 0.01], atol=1e-12)
    _, integ, _ = O.compute_action(c, K, kc, obs, integ)
    np.testing.assert_allclose(integ, [0.02, 0.0, 0.02], atol=1e-12)


def test_open_loop_steps():
    OL = np.load(os.path.join(GOLDEN, "open_loop.npz"))
    cases = json.loads(str(OL["cases_json"]))
    for ci, case in enumerate(cases):
        cfg = json.loads(json.dumps(case["env"]))
        cfg.setdefault("target", {})["motion_type"] = case["motion"]
        env = O.env_params(cfg)
        pat, off = O.draws(env.motion, [case["seed"]])
        X = OL[f"case{ci}_states"]
        info = OL[f"case{ci}_info"]
        x = X[0].copy()
        np.testing.assert_allclose(x, O.initial_state(env, env.motion, pat[0], off[0]), atol=1e-15)
        t = 0.0
        on = 0
        for k in range(len(OL["actions"])):
            if np.isnan(info[k, 0]):
                break
            x, t, tgt, err, viol, term = O.env_step(env, env.motion, pat[0], env.mass, x, t, OL["actions"][k])
            on += err <= env.target_radius
            np.testing.assert_allclose(x, X[k + 1], rtol=1e-9, atol=1e-9, err_msg=f"case {ci} step {k}")
            assert err == pytest.approx(info[k, 0], rel=1e-9, abs=1e-9)
            assert on / (k + 1) == pytest.approx(info[k, 1])
            assert term == int(info[k, 4]) and (term != 0) == bool(info[k, 3])
            assert t == info[k, 5]


def test_seed_draws_match_reset():
    R = np.load(os.path.join(GOLDEN, "rng_draws.npz"))
    for m in O.MOTIONS:
        pat, off = O.draws(m, R["seeds"])
        env = O.env_params({"target": {"motion_type": m}})
        x0 = np.array([O.initial_state(env, env.motion, pat[i], off[i])[:3] for i in range(len(R["seeds"]))])
        # the draws are bit-exact; x0 adds target(0), where libm and numpy's
        # sin/cos may differ by an ulp
        np.testing.assert_allclose(x0, R[f"{m}_x0"], rtol=0, atol=4.5e-16)
        if m == "linear":
            d = pat[:, :3] / np.linalg.norm(pat[:, :3], axis=1, keepdims=True)
            np.testing.assert_allclose(d / np.linalg.norm(d, axis=1, keepdims=True), R[f"{m}_param"], atol=1e-15)
        if m == "circular":
            np.testing.assert_array_equal(pat[:, 0], R[f"{m}_param"][:, 0])
        elif m == "sinusoidal":
            np.testing.assert_array_equal(pat[:, :3], R[f"{m}_param"])


def test_numpy_order_sums_restated():
    """oracle.np_sum / np_mean_std (numpy's blocked pairwise order, the
    checker of qt_summary_numpy) equal np.add.reduce / np.mean / np.std bit
    for bit, across the leaf (< 8, <= 128), split and block (8,192) edges."""
    rng = np.random.default_rng(11)
    for n in list(range(1, 140)) + [255, 256, 257, 1000, 8191, 8192, 8193, 9000, 16384 + 77, 40000]:
        a = rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 4, n)
        assert O.np_sum(a) == np.add.reduce(a), n
        mu, sd = O.np_mean_std(a)
        assert mu == np.mean(a) and sd == np.std(a), n


def test_numpy_order_summary_fixture():
    """The reference's own EvaluationSummary (tests/golden/evaluator_lqi.npz,
    compute_evaluation_summary over the Evaluator's episodes) from the
    restated means / stds of its per-episode metrics, bitwise."""
    d = np.load(os.path.join(GOLDEN, "evaluator_lqi.npz"))
    fj = json.loads(str(d["fields_json"]))
    fields, summ = fj["metrics"], fj["summary"]
    for name in ("stationary_lqi", "linear_lqi_limit"):
        m = d[f"{name}_metrics"]
        s = dict(zip(summ, d[f"{name}_summary"]))
        r, e, u = (m[:, fields.index(k)] for k in ("on_target_ratio", "mean_tracking_error", "mean_control_effort"))
        mu_r, sd_r = O.np_mean_std(r)
        mu_e, sd_e = O.np_mean_std(e)
        got = [mu_r, sd_r, mu_e, sd_e, O.np_sum(u) / len(u)]
        ref = [s[k] for k in ("mean_on_target_ratio", "std_on_target_ratio", "mean_tracking_error",
                              "std_tracking_error", "mean_control_effort")]
        assert got == ref, name
