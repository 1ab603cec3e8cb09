#!/usr/bin/env python3
"""Throughput of the per-step API (include/quadtrack.h ABI 9): a Python loop
of `env.step(ctl.compute_action(obs))` (two launches per step) or
`env.step_closed(ctl)` (one launch per step) over n episodes, the way the
reference's Evaluator drives its plugins (eval.py:119-165).

Prints one JSON line per configuration: env-steps/s of the loop (wall clock
from the first step's launch to the last step's completion), host time per
step (Python + launch issue), the launches per step, and the HBM bytes each
kernel must move per env-step by its contract (DESIGN.md §4 "Per-step API").
Kernel durations and HBM counter bytes come from rocprofv3 runs of this
script (scripts/prof.sh; profiles/r05/step_api_*).

  python scripts/step_api_bench.py --n 65536 1048576 --steps 3000 --mode closed two_call
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-quadcopter-test_amd"))

import quadtrack  # noqa: E402
from quadtrack.controllers import BatchedRiccatiLQR  # noqa: E402

# bytes per env-step each kernel must move by its contract (reads + writes;
# per-episode constants: the pattern draw, 3 doubles for linear / sinusoidal,
# 1 for circular, 0 stationary / figure-8)
FRAME_OUT = 25 * 8 + 3 * 8 + 5  # the frame a step writes


def contract_bytes(mode: str, lqi: bool, pattern_doubles: int, freeze: bool) -> dict:
    integ = 2 * 3 * 8 if lqi else 0
    pat = 8 * pattern_doubles
    step_in = 12 * 8 + 8 + 3 * 8 + (1 if freeze else 0)  # x, t, counters, done flag
    if mode == "closed":
        k = step_in + 6 * 8 + integ + pat + FRAME_OUT + 4 * 8  # + target p, v; writes frame + action
        return {"closed_step": k}
    act = 12 * 8 + integ + 4 * 8  # pos, vel, target p, v; integral r/w; action out
    step = step_in + 4 * 8 + pat + FRAME_OUT  # + the action
    return {"compute_action": act, "frame_step": step}


def run(n, steps, mode, lqi, motion, warm):
    dev = torch.device("cuda", 0)
    cfg = {"target": {"motion_type": motion}}
    ctl = BatchedRiccatiLQR({"dt": 0.01, "use_lqi": lqi, "q_int": [1e-3, 1e-3, 1e-2]} if lqi else {"dt": 0.01})
    env = quadtrack.BatchedQuadcopterEnv(n, cfg)

    def loop(k):
        ctl.reset(n)
        obs = env.reset(np.arange(n))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "closed":
            for _ in range(k):
                obs, r, done, info = env.step_closed(ctl)
        else:
            for _ in range(k):
                obs, r, done, info = env.step(ctl.compute_action(obs))
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        return time.perf_counter() - t0, t_issue, done

    loop(warm)
    wall, issue, done = loop(steps)
    pat = {"linear": 3, "sinusoidal": 3, "circular": 1}.get(motion, 0)
    by = contract_bytes(mode, lqi, pat, True)
    per_step = sum(by.values())
    rate = n * steps / wall
    return {"n": n, "steps": steps, "mode": mode, "controller": "lqi" if lqi else "lqr", "motion": motion,
            "launches_per_step": 1 if mode == "closed" else 2, "wall_s": wall,
            "env_steps_per_s": rate, "ms_per_step": wall / steps * 1e3, "host_us_per_step": issue / steps * 1e6,
            "contract_bytes_per_env_step": by, "contract_GBps": rate * per_step / 1e9,
            "contract_hbm_frac": rate * per_step / 8e12, "all_done": bool(done.all())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[65536, 1048576])
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warm", type=int, default=50)
    ap.add_argument("--mode", nargs="+", default=["closed", "two_call"])
    ap.add_argument("--ctl", nargs="+", default=["lqr"])
    ap.add_argument("--motion", default="linear")
    a = ap.parse_args()
    for n in a.n:
        for mode in a.mode:
            for c in a.ctl:
                print(json.dumps(run(n, a.steps, mode, c == "lqi", a.motion, a.warm)), flush=True)


if __name__ == "__main__":
    main()
