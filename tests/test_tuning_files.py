"""Tuner data formats (controllers/tuning.py:363-579, 930-1129) against the
reference's own output (tests/golden/gen_tuning.py): TuningConfig /
TuningResult dictionaries and files, the two files tune() writes, and
resume_from a previous results file."""

import json
import os

import pytest

from conftest import GOLDEN

FIX = json.load(open(os.path.join(GOLDEN, "tuning_results.json")))


def _norm(d):
    return json.loads(json.dumps(d))


def test_tuning_config_dict_form():
    from quadtrack.tuning import TuningConfig

    cfg = TuningConfig.from_dict(FIX["base"])
    d = _norm(cfg.to_dict())
    d.pop("output_dir")
    assert d == FIX["first"]["config"]
    assert TuningConfig.from_dict(cfg.to_dict()).to_dict() == cfg.to_dict()
    for bad in ({"controller_type": "deep"}, {"strategy": "bayes"}, {"max_iterations": 0}, {"cma_sigma0": 0.0},
                {"cma_popsize": 1}, {"evaluation_episodes": 0}):
        with pytest.raises(ValueError):
            TuningConfig.from_dict(dict(FIX["base"], **bad))


def test_tuning_result_file_round_trip(tmp_path):
    from quadtrack.tuning import TuningResult

    res = TuningResult.from_dict(dict(FIX["first_results_file"], timestamp="t"))
    p = res.save(tmp_path / "r" / "x_results.json")
    assert TuningResult.load(p).to_dict() == res.to_dict()
    with pytest.raises(FileNotFoundError):
        TuningResult.load(tmp_path / "missing.json")
    with pytest.raises(ValueError):
        TuningResult.load(tmp_path / ".." / "x.json")


def _check_results(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert _norm(g["config"]) == r["config"]
        assert g["score"] == pytest.approx(r["score"], rel=1e-8, abs=1e-10)
        for k, v in r["metrics"].items():
            assert g["metrics"][k] == pytest.approx(v, rel=1e-8, abs=1e-10), k


@pytest.mark.gpu
def test_tune_files_and_resume(tmp_path):
    import glob

    from quadtrack.tuning import BatchedTuner, TuningConfig, TuningResult

    res = BatchedTuner(TuningConfig.from_dict(dict(FIX["base"], output_dir=str(tmp_path / "a")))).tune()
    _check_results(res.all_results, FIX["first"]["all_results"])
    assert _norm(res.best_config) == FIX["first"]["best_config"]
    assert res.iterations_completed == 3 and res.interrupted is False
    files = sorted(glob.glob(str(tmp_path / "a" / "tuning_riccati_lqr_*")))
    assert len(files) == 2 and files[0].endswith("_best_config.json") and files[1].endswith("_results.json")
    best = json.load(open([f for f in files if f.endswith("_best_config.json")][0]))
    assert sorted(best) == sorted(FIX["first_best_config_file"])
    assert _norm(best["riccati_lqr"]) == FIX["first_best_config_file"]["riccati_lqr"]
    assert TuningResult.load([f for f in files if f.endswith("_results.json")][0]).to_dict() == _norm(res.to_dict())

    # resume from the reference's own results file
    prev = tmp_path / "prev_results.json"
    prev.write_text(json.dumps(dict(FIX["first_results_file"], timestamp="t", config=dict(
        FIX["first_results_file"]["config"], output_dir=str(tmp_path / "a")))))
    res2 = BatchedTuner(TuningConfig.from_dict(dict(FIX["base"], max_iterations=5, resume_from=str(prev),
                                                    output_dir=str(tmp_path / "b")))).tune()
    assert res2.all_results[:3] == FIX["first_results_file"]["all_results"]  # carried over as loaded
    _check_results(res2.all_results, FIX["resumed"]["all_results"])
    assert res2.iterations_completed == FIX["resumed"]["iterations_completed"]
    assert _norm(res2.best_config) == FIX["resumed"]["best_config"]


def test_cma_es_without_cma_raises_import_error():
    """As the reference's ControllerTuner does when `cma` is absent (tuning.py:636-643)."""
    import importlib.util

    from quadtrack.tuning import ControllerTuner, TuningConfig

    if importlib.util.find_spec("cma") is not None:
        pytest.skip("cma installed")
    with pytest.raises(ImportError, match="cma"):
        ControllerTuner(TuningConfig.from_dict(dict(FIX["base"], strategy="cma_es")))


@pytest.mark.gpu
def test_controller_tuner_evaluate_config(tmp_path):
    """The reference's name and single-candidate entry point."""
    from quadtrack.tuning import ControllerTuner, TuningConfig

    t = ControllerTuner(TuningConfig.from_dict(dict(FIX["base"], output_dir=str(tmp_path))))
    for r in FIX["first"]["all_results"]:
        score, metrics = t._evaluate_config(r["config"])
        assert score == pytest.approx(r["score"], rel=1e-8, abs=1e-10)
        assert metrics["mean_on_target_ratio"] == pytest.approx(r["metrics"]["mean_on_target_ratio"], rel=1e-8)


def test_score_rows_equal_per_candidate_means():
    """The vectorised candidate scores equal the reference's per-candidate
    np.mean(list(...)) loop (tuning.py:908-928) bit for bit, for E below and
    above numpy's 8-element pairwise leaf."""
    import numpy as np

    from quadtrack.tuning import score_rows

    rng = np.random.default_rng(9)
    for C, E in [(1, 1), (7, 5), (300, 8), (64, 13), (33, 130)]:
        ratio = rng.integers(0, 3001, (C, E)) / 3000.0
        err = rng.lognormal(size=(C, E))
        succ = rng.integers(0, 2, (C, E)).astype(float)
        got = score_rows(ratio, err, succ)
        for c in range(C):
            mean_on, mean_err, rate = np.mean(list(ratio[c])), np.mean(list(err[c])), np.mean(list(succ[c]))
            assert got[c][0] == float(mean_on - 0.1 * mean_err)
            assert got[c][1] == {"mean_on_target_ratio": float(mean_on), "mean_tracking_error": float(mean_err),
                                 "success_rate": float(rate), "episodes_evaluated": E}
