"""The sequential drop-in Evaluator keeps the LQI integral across episodes, as
the reference's does (eval.py:198-206 never calls controller.reset(); SURVEY
F8): quadtrack.eval.Evaluator against tests/golden/evaluator_lqi.npz, which
the reference's own Evaluator produced (tests/golden/gen_evaluator_lqi.py)."""

import json
import os
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIX = os.path.join(GOLDEN, "evaluator_lqi.npz")


@pytest.fixture(scope="module")
def fx():
    return np.load(FIX, allow_pickle=False)


def _scenarios(fx):
    return json.loads(str(fx["scenarios_json"]))


@pytest.mark.parametrize("idx", [0, 1])
def test_evaluator_lqi_carry_over(fx, idx):
    import quadtrack

    quadtrack._abi.require_gpu("cuda:0")
    from quadtrack.controllers import RiccatiLQRController
    from quadtrack.env.config import EnvConfig
    from quadtrack.eval import Evaluator
    from quadtrack.utils.metrics import compute_episode_metrics

    s = _scenarios(fx)[idx]
    fields = json.loads(str(fx["fields_json"]))
    ctl = RiccatiLQRController(config=dict(s["ctl"]))
    with tempfile.TemporaryDirectory() as tmp:
        ev = Evaluator(ctl, env_config=EnvConfig.from_dict(s["env"]), output_dir=tmp)
        mets, integ = [], []
        for i in range(s["episodes"]):
            data, info = ev.run_episode(seed=s["seed"] + i, max_steps=s["max_steps"])
            m = compute_episode_metrics(data, ev.criteria, info)
            mets.append([float(getattr(m, f)) for f in fields["metrics"]])
            integ.append(ctl.get_integral_state().tolist())
        np.testing.assert_allclose(np.array(mets), fx[f"{s['name']}_metrics"], rtol=1e-8, atol=1e-8)
        np.testing.assert_allclose(np.array(integ), fx[f"{s['name']}_integral"], rtol=1e-8, atol=1e-10)
        # the carry-over matters: fresh controllers give other metrics from episode 1 on
        assert np.abs(fx[f"{s['name']}_metrics"][1:] - fx[f"{s['name']}_metrics_fresh"][1:]).max() > 1e-3
        np.testing.assert_allclose(np.array(mets)[0], fx[f"{s['name']}_metrics_fresh"][0], rtol=1e-8, atol=1e-8)

        # evaluate() itself on a fresh controller: the same episodes, summary and final integral
        ctl2 = RiccatiLQRController(config=dict(s["ctl"]))
        ev2 = Evaluator(ctl2, env_config=EnvConfig.from_dict(s["env"]), output_dir=tmp)
        summary = ev2.evaluate(num_episodes=s["episodes"], base_seed=s["seed"], max_steps_per_episode=s["max_steps"],
                               verbose=False)
        got = np.array([float(getattr(summary, k)) for k in fields["summary"]])
        np.testing.assert_allclose(got, fx[f"{s['name']}_summary"], rtol=1e-8, atol=1e-8)
        np.testing.assert_allclose(ctl2.get_integral_state(), fx[f"{s['name']}_final_integral_evaluate"], rtol=1e-8,
                                   atol=1e-10)
