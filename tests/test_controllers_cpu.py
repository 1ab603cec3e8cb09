"""Host-side controller logic (no GPU): the heuristic-LQR gain formula of
LQRController._compute_gains (controllers/__init__.py:522-574) in its
broadcast form (one K per episode for BatchedLQR) against the reference's
fixtures and the oracle, and the batched-controller factory's dispatch."""

import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

import oracle as O
from quadtrack.controllers import VALID_CONTROLLER_TYPES, batched_controller, heuristic_gains


def test_heuristic_gains_match_reference_fixtures():
    A = np.load(os.path.join(GOLDEN, "controller_actions.npz"))
    cases = json.loads(str(A["cases_json"]))
    for ci, cfg in enumerate(cases):
        if cfg["controller"] != "lqr" or "K" in cfg:
            continue
        K = heuristic_gains(cfg.get("q_pos", [1e-4, 1e-4, 16.0]), cfg.get("q_vel", [0.0036, 0.0036, 4.0]),
                            cfg.get("r_thrust", 1.0), cfg.get("r_rate", 1.0))
        np.testing.assert_array_equal(K, A[f"case{ci}_K"])


def test_heuristic_gains_broadcast_equals_scalar():
    r = np.random.default_rng(11)
    m = 257
    qp = r.uniform([5e-5, 5e-5, 10], [5e-4, 5e-4, 25], (m, 3))
    qv = r.uniform([1e-3, 1e-3, 2], [1e-2, 1e-2, 8], (m, 3))
    rt, rr = r.uniform(0.5, 2, m), r.uniform(0.5, 2, m)
    Kb = heuristic_gains(qp, qv, rt, rr)
    assert Kb.shape == (m, 4, 6)
    for i in range(0, m, 16):
        np.testing.assert_array_equal(Kb[i], heuristic_gains(qp[i], qv[i], rt[i], rr[i]))
        np.testing.assert_array_equal(Kb[i], O.heuristic_gains(qp[i], qv[i], rt[i], rr[i]))


def test_heuristic_gains_invalid_weights_give_nan_not_error():
    K = heuristic_gains([-1.0, 1e-4, 16.0], [0.0036, 0.0036, 4.0], 1.0, 1.0)
    assert np.isnan(K[2, 0]) and np.isfinite(K[0, 2])


def test_factory_types():
    assert set(VALID_CONTROLLER_TYPES) == {"lqr", "pid", "riccati_lqr", "lqi"}
    with pytest.raises(ValueError, match="Unknown controller type"):
        batched_controller("deep", {})
