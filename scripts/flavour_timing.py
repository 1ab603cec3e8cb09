#!/usr/bin/env python3
"""Rollout time of one 65,536-episode pass per step flavour, the reference
options that used to leave the fast path included (VERDICT r03 missing #2):

  yaw0        the bench workload (linear target, Riccati-LQR, RK4): the
              yaw-at-rest fast flavour;
  yaw0_euler  the same with integrator: euler (the Euler closed form);
  rewards     qt_rollout_rewards (the trainer's epoch, train.py:578-652) on
              the same batch: the fast flavour with telescoped rewards;
  exact       the exact step: every episode starts with a 1e-300 rad/s yaw
              rate, so no wave passes the yaw-at-rest wave test and all go to
              the exact pass (trajectories differ by ~1e-300);
  exact_euler, exact_rewards  the same for Euler and for rewards;
  fast_yaw    a gain with a yaw-rate row (the heuristic LQR's K plus two yaw
              terms): the full-gain fast flavour (kFast).

HIP events on the launch stream around the reset + rollout launch set,
median of --reps after a 1 s warm-up.  One JSON line per case.

  python scripts/flavour_timing.py [--n 65536] [--reps 5]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--motion", default="linear")
    ap.add_argument("--cases", nargs="*", default=None, help="only these cases (e.g. exact yaw0)")
    ap.add_argument("--warmup-s", type=float, default=1.0)
    args = ap.parse_args()

    import numpy as np
    import torch

    from quadtrack import _abi, core
    from quadtrack.controllers import BatchedLQR, BatchedRiccatiLQR
    from quadtrack.env.config import EnvConfig
    from quadtrack.rollout import build_batch, max_steps_for

    dev = torch.device("cuda", 0)
    n = args.n
    ctl = BatchedRiccatiLQR({"dt": 0.01}, device=dev)
    crit = core.criteria()
    s = torch.cuda.current_stream(dev)
    for integrator in ("rk4", "euler"):
        cfg = EnvConfig.from_dict({"target": {"motion_type": args.motion}, "simulation": {"integrator": integrator}})
        env = cfg.to_params()
        batch = build_batch(ctl, cfg, n, seeds=np.arange(n))
        steps = max_steps_for(env)
        for exact in (False, True):
            for rewards in ((False, True) if integrator == "rk4" else (False,)):
                name = ("exact" if exact else "yaw0") + ("_euler" if integrator == "euler" else "") + \
                    ("_rewards" if rewards else "")
                if args.cases is not None and name not in args.cases:
                    continue
                st = core.RolloutState.empty(n, dev)
                reward = torch.zeros(2, n, dtype=torch.float64, device=dev)

                def one():
                    core.reset(env, batch, st)
                    if exact:
                        st.x[11] = 1e-300
                    if rewards:
                        reward.zero_()
                        core.rollout_rewards(env, ctl.ctrl, crit, batch, st, steps, reward)
                    else:
                        core.rollout(env, ctl.ctrl, crit, batch, st, steps)

                t0 = time.perf_counter()
                while time.perf_counter() - t0 < args.warmup_s:
                    one()
                    torch.cuda.synchronize()
                times = []
                for _ in range(args.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    one()
                    e1.record(s)
                    torch.cuda.synchronize()
                    times.append(e0.elapsed_time(e1))
                ms = float(np.median(times))
                done = float(st.acc[_abi.ACC_STEPS].sum().item())
                print(json.dumps({"case": name, "integrator": integrator, "rewards": rewards, "n": n,
                                  "motion": args.motion, "ms": round(ms, 4), "ms_min": round(min(times), 4),
                                  "env_steps_per_s": round(done / (ms * 1e-3), 1)}), flush=True)
    if args.cases is None or "fast_yaw" in args.cases:
        K = BatchedLQR({}).gains()[0].cpu().numpy().copy()
        K[3, 0], K[3, 4] = 0.02, -0.01
        yctl = BatchedLQR({"K": K}, device=dev)
        cfg = EnvConfig.from_dict({"target": {"motion_type": args.motion}})
        env = cfg.to_params()
        batch = build_batch(yctl, cfg, n, seeds=np.arange(n))
        steps = max_steps_for(env)
        st = core.RolloutState.empty(n, dev)

        def one_yaw():
            core.reset(env, batch, st)
            core.rollout(env, yctl.ctrl, crit, batch, st, steps)

        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.warmup_s:
            one_yaw()
            torch.cuda.synchronize()
        times = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            one_yaw()
            e1.record(s)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        ms = float(np.median(times))
        done = float(st.acc[_abi.ACC_STEPS].sum().item())
        print(json.dumps({"case": "fast_yaw", "integrator": "rk4", "rewards": False, "n": n, "motion": args.motion,
                          "ms": round(ms, 4), "ms_min": round(min(times), 4),
                          "env_steps_per_s": round(done / (ms * 1e-3), 1)}), flush=True)


if __name__ == "__main__":
    main()
