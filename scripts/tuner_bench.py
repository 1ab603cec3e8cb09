#!/usr/bin/env python3
"""End-to-end BatchedTuner throughput (GPU box): a random riccati_lqr sweep of
C candidates x E episodes (controllers/tuning.py defaults: circular target,
30 s episodes, scripts/controller_autotune.py's default space), timed from
TuningConfig to the saved result files, with a breakdown.  One JSON line."""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))

import torch  # noqa: E402

from quadtrack import tuning  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--candidates", type=int, default=13107)
ap.add_argument("--episodes", type=int, default=5)
args = ap.parse_args()


def run(out):
    cfg = tuning.TuningConfig(controller_type="riccati_lqr", search_space=tuning.default_search_space("riccati_lqr"),
                              strategy="random", max_iterations=args.candidates,
                              evaluation_episodes=args.episodes, target_motion_type="circular", output_dir=out)
    t = {}
    t0 = time.perf_counter()
    tuner = tuning.BatchedTuner(cfg)
    configs = tuner.generate_random_configs(cfg.max_iterations)
    t["generate_s"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    scored = tuner.evaluate_configs(configs)
    torch.cuda.synchronize()
    t["evaluate_s"] = time.perf_counter() - t1
    t2 = time.perf_counter()
    for c, (s, m) in zip(configs, scored):
        tuner._record(c, s, m)
    res = tuning.TuningResult(best_config=tuner.best_config, best_score=tuner.best_score,
                              best_metrics=tuner.best_metrics, all_results=tuner.results,
                              iterations_completed=len(tuner.results), interrupted=False, timestamp="",
                              config=cfg.to_dict())
    tuner.save_results(res)
    t["record_and_save_s"] = time.perf_counter() - t2
    t["total_s"] = time.perf_counter() - t0
    return res, t


with tempfile.TemporaryDirectory() as d:
    run(d)  # warm-up (kernel loading)
    res, t = run(d)
steps = args.candidates * args.episodes * 3000
print(json.dumps({"candidates": args.candidates, "episodes_per_candidate": args.episodes,
                  **{k: round(v, 4) for k, v in t.items()},
                  "candidates_per_s": round(args.candidates / t["total_s"], 1),
                  "env_steps_per_s_end_to_end": round(steps / t["total_s"], 1),
                  "best_score": res.best_score,
                  "reference_estimate": "one candidate = 5 episodes x 3000 steps at ~7k env-steps/s (SURVEY 6): ~2.1 s"}))
