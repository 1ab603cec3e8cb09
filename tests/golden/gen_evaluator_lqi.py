"""Generate tests/golden/evaluator_lqi.npz from the reference's Evaluator.

Test infrastructure only (build container, reference mounted read-only; the
same no-op `python-dotenv` stand-in as gen_golden.py).  Pins the sequential
Evaluator's LQI carry-over: `Evaluator.evaluate` never calls
`controller.reset()` between episodes (eval.py:198-206), so the LQI integral
of episode i starts where episode i-1 left it.  Records, per
scenario, every episode's EpisodeMetrics fields, the controller's integral
state after each episode, the EvaluationSummary, and the same episodes run
with a fresh controller each (which the carried run must differ from).

Usage:  python tests/golden/gen_evaluator_lqi.py [--out tests/golden]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import import_reference  # noqa: E402

# LQI with a small integral threshold on targets where the integral carries
# real state from one episode into the next (no reset between episodes)
SCENARIOS = [
    {"name": "stationary_lqi", "env": {"target": {"motion_type": "stationary"}},
     "ctl": {"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2], "integral_zero_threshold": 0.001},
     "episodes": 4, "seed": 42, "max_steps": 600},
    {"name": "linear_lqi_limit", "env": {"target": {"motion_type": "linear", "speed": 0.5}},
     "ctl": {"dt": 0.01, "use_lqi": True, "q_int": [5e-3, 5e-3, 2e-2], "integral_limit": 0.5},
     "episodes": 3, "seed": 7, "max_steps": 800},
]

FIELDS = ["episode_duration", "on_target_ratio", "mean_tracking_error", "max_tracking_error",
          "rms_tracking_error", "total_control_effort", "mean_control_effort", "overshoot_count",
          "max_overshoot", "success"]
SUMMARY = ["total_episodes", "successful_episodes", "success_rate", "mean_on_target_ratio", "std_on_target_ratio",
           "mean_tracking_error", "std_tracking_error", "mean_control_effort", "best_episode_idx",
           "worst_episode_idx", "meets_criteria"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    args = ap.parse_args()
    qt = import_reference()
    from quadcopter_tracking.controllers.riccati_lqr import RiccatiLQRController
    from quadcopter_tracking.env.config import EnvConfig
    from quadcopter_tracking.eval import Evaluator

    out = {}
    for s in SCENARIOS:
        ctl = RiccatiLQRController(config=dict(s["ctl"]))
        with tempfile.TemporaryDirectory() as tmp:
            ev = Evaluator(ctl, env_config=EnvConfig.from_dict(s["env"]), output_dir=tmp)
            integ = []
            mets = []
            # evaluate() one episode at a time would re-create nothing: the same
            # controller object runs every episode; record its integral after each
            summary = None
            ev.episode_data_list, ev.episode_info_list = [], []
            from quadcopter_tracking.utils.metrics import compute_episode_metrics, compute_evaluation_summary

            for i in range(s["episodes"]):
                data, info = ev.run_episode(seed=s["seed"] + i, max_steps=s["max_steps"])
                m = compute_episode_metrics(data, ev.criteria, info)
                mets.append([float(getattr(m, f)) for f in FIELDS])
                integ.append(ctl.get_integral_state().tolist())
            # the same episodes each with a fresh controller (what the batched
            # paths and the tuner do): differs from the carried run from episode 1 on
            fresh = []
            for i in range(s["episodes"]):
                ev_f = Evaluator(RiccatiLQRController(config=dict(s["ctl"])), env_config=EnvConfig.from_dict(s["env"]),
                                 output_dir=tmp)
                data, info = ev_f.run_episode(seed=s["seed"] + i, max_steps=s["max_steps"])
                m = compute_episode_metrics(data, ev_f.criteria, info)
                fresh.append([float(getattr(m, f)) for f in FIELDS])
            # the same episodes through evaluate() itself (fresh controller): its summary
            ctl2 = RiccatiLQRController(config=dict(s["ctl"]))
            ev2 = Evaluator(ctl2, env_config=EnvConfig.from_dict(s["env"]), output_dir=tmp)
            summary = ev2.evaluate(num_episodes=s["episodes"], base_seed=s["seed"],
                                   max_steps_per_episode=s["max_steps"], verbose=False)
            ev2_integ = ctl2.get_integral_state().tolist()
        out[f"{s['name']}_metrics"] = np.array(mets)
        out[f"{s['name']}_integral"] = np.array(integ)
        out[f"{s['name']}_metrics_fresh"] = np.array(fresh)
        out[f"{s['name']}_summary"] = np.array([float(getattr(summary, k)) for k in SUMMARY])
        out[f"{s['name']}_final_integral_evaluate"] = np.array(ev2_integ)
    out["scenarios_json"] = np.array(json.dumps(SCENARIOS))
    out["fields_json"] = np.array(json.dumps({"metrics": FIELDS, "summary": SUMMARY}))
    np.savez_compressed(os.path.join(args.out, "evaluator_lqi.npz"), **out)
    print("wrote", os.path.join(args.out, "evaluator_lqi.npz"))


if __name__ == "__main__":
    main()
