"""The batched tuner's host logic (quadtrack.tuning, quadtrack.workloads)
against the reference tuner's candidate streams: random candidates equal the
sequential scalar draws of _generate_random_config (tuning.py:683-735), a
shard's candidates equal the matching slice of the full stream, grid order
follows _generate_grid_configs (737-830).  GPU scoring is in
test_gpu_workloads / test_gpu_tuning."""

from itertools import product

import numpy as np
import pytest

from quadtrack import tuning, workloads


def _sequential(space, n, seed):
    r = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        c = {}
        for name, attr, dim in tuning._PARAM_ORDER:
            rd = getattr(space, attr)
            if rd is None:
                continue
            lo, hi = rd
            c[name] = float(r.uniform(lo, hi)) if dim == 0 else [float(r.uniform(a, b)) for a, b in zip(lo, hi)]
            if name.startswith("ff_"):
                c["feedforward_enabled"] = True
            if name == "q_int":
                c["use_lqi"] = True
        out.append(c)
    return out


def test_random_candidates_match_sequential_stream():
    space = tuning.default_search_space()
    assert tuning.random_configs(space, 500, np.random.default_rng(42)) == _sequential(space, 500, 42)
    full = tuning.GainSearchSpace(q_pos_range=([0, 0, 1], [1, 1, 2]), r_thrust_range=(0.1, 0.5),
                                  r_rate_range=(1.0, 1.0), q_int_range=([0, 0, 0], [1e-3, 1e-3, 1e-2]),
                                  ff_velocity_gain_range=([0, 0, 0], [0.5, 0.5, 0.5]))
    got = tuning.random_configs(full, 50, np.random.default_rng(7))
    assert got == _sequential(full, 50, 7)
    assert got[0]["use_lqi"] and got[0]["feedforward_enabled"]


def test_shard_candidates_are_stream_slices():
    ref = tuning.random_configs(tuning.default_search_space(), 1000, np.random.default_rng(42))
    for lo, hi in [(0, 10), (1, 2), (333, 1000), (999, 1000)]:
        assert workloads.tuner_candidates(lo, hi) == ref[lo:hi]


def test_tuner_batch_continues_stream():
    """Two consecutive generate_random_configs calls == one call (the tuner's rng persists)."""
    cfg = tuning.TuningConfig(controller_type="riccati_lqr", search_space=tuning.default_search_space())
    t = tuning.BatchedTuner.__new__(tuning.BatchedTuner)
    t.config, t.rng = cfg, np.random.default_rng(cfg.seed)
    a = t.generate_random_configs(7) + t.generate_random_configs(5)
    assert a == tuning.random_configs(cfg.search_space, 12, np.random.default_rng(42))


def test_grid_order_and_fixed_axes():
    space = tuning.GainSearchSpace(q_pos_range=([1e-4, 1e-4, 10.0], [1e-4, 2e-4, 20.0]),
                                   r_controls_range=([1.0] * 4, [1.0, 1.0, 1.0, 2.0]), use_lqi=True)
    g = tuning.grid_configs(space, 3)
    qp = [list(c) for c in product([1e-4], list(np.linspace(1e-4, 2e-4, 3)), list(np.linspace(10.0, 20.0, 3)))]
    rc = [list(c) for c in product([1.0], [1.0], [1.0], list(np.linspace(1.0, 2.0, 3)))]
    assert len(g) == len(qp) * len(rc)
    assert [c["q_pos"] for c in g[:: len(rc)]] == qp
    assert [c["r_controls"] for c in g[: len(rc)]] == rc
    assert all(c["use_lqi"] and c["q_int"] == [0.0, 0.0, 0.0] for c in g)


def test_search_space_validation():
    with pytest.raises(ValueError, match="inverted"):
        tuning.GainSearchSpace(q_pos_range=([2, 0, 0], [1, 1, 1])).validate()
    with pytest.raises(ValueError, match="negative"):
        tuning.GainSearchSpace(r_thrust_range=(-1.0, 1.0)).validate()
    with pytest.raises(ValueError, match="exactly 4"):
        tuning.GainSearchSpace(r_controls_range=([1, 1, 1], [2, 2, 2])).validate()
    with pytest.raises(ValueError):
        tuning.TuningConfig(strategy="annealing")
    with pytest.raises(ValueError, match="Invalid controller_type"):
        tuning.TuningConfig(controller_type="deep")


def test_default_search_spaces_match_autotune_script():
    """scripts/controller_autotune.py:360-385 (get_default_search_space)."""
    pid = tuning.default_search_space("pid")
    assert pid.kp_pos_range == ([0.005, 0.005, 2.0], [0.05, 0.05, 6.0])
    assert pid.kd_pos_range == ([0.02, 0.02, 1.0], [0.15, 0.15, 3.0])
    assert pid.get_active_parameters() == ["kp_pos", "kd_pos"]
    lqr = tuning.default_search_space("lqr")
    assert lqr.get_active_parameters() == ["q_pos", "q_vel"]
    ric = tuning.default_search_space("riccati_lqr")
    assert ric.get_active_parameters() == ["q_pos", "q_vel", "r_controls"]
    assert tuning.default_search_space("deep").get_active_parameters() == []


def test_ff_rows_layout():
    """qt_batch.ff rows: velocity gain xyz, acceleration gain xyz, velocity
    clamp; an episode without feed-forward has gains 0 and clamp +inf."""
    import numpy as np
    import torch

    from quadtrack import core

    rows = core.ff_rows(3, torch.device("cpu"), True, [0.1, 0.2, 0.3], 0.5, 7.0, off=[False, True, False])
    r = rows.numpy()
    assert r.shape == (7, 3)
    assert r[:, 0].tolist() == [0.1, 0.2, 0.3, 0.5, 0.5, 0.5, 7.0]
    assert r[:6, 1].tolist() == [0.0] * 6 and np.isinf(r[6, 1])
    per = core.ff_rows(2, torch.device("cpu"), [True, False], np.array([[1, 2, 3], [4, 5, 6]], float))
    assert per.numpy()[:3, 0].tolist() == [1, 2, 3] and per.numpy()[:3, 1].tolist() == [0, 0, 0]


def test_shard_bounds_partition():
    for total in (1, 7, 65536, 1048576):
        for world in (1, 2, 3, 4, 8):
            b = [workloads.shard_bounds(total, r, world) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == total
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))


def test_candidate_arrays_match_dicts():
    qp, qv, rc = workloads.tuner_candidate_arrays(17, 400)
    ref = workloads.tuner_candidates(17, 400)
    assert qp.tolist() == [c["q_pos"] for c in ref]
    assert qv.tolist() == [c["q_vel"] for c in ref]
    assert rc.tolist() == [c["r_controls"] for c in ref]
