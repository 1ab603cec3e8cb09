#!/usr/bin/env python3
"""Rollout-kernel throughput sweep: env-steps/s per (motion, controller, N).

Times only the fused closed-loop kernel (HIP events on the launch stream),
3,000 steps per episode, inputs resident.  Prints one JSON line per case.
"""

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="16384,65536,262144")
    ap.add_argument("--motions", default="stationary,linear,circular,sinusoidal,figure8,mixed")
    ap.add_argument("--ctl", default="lqr,lqi")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from quadtrack import core
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.env.config import EnvConfig
    from quadtrack.rollout import build_batch, max_steps_for

    dev = torch.device("cuda", 0)
    for ctl_name in args.ctl.split(","):
        cfg_c = {"dt": 0.01} if ctl_name == "lqr" else {"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2]}
        ctl = BatchedRiccatiLQR(cfg_c, device=dev)
        for motion in args.motions.split(","):
            for n in (int(v) for v in args.n.split(",")):
                mix = motion == "mixed"
                cfg = EnvConfig.from_dict({"target": {"motion_type": "stationary" if mix else motion}})
                env = cfg.to_params()
                mo = [i % 5 for i in range(n)] if mix else None
                batch = build_batch(ctl, cfg, n, seeds=np.arange(n), motion=mo,
                                    order=np.argsort(np.array(mo), kind="stable") if mix else None)
                st = core.RolloutState.empty(n, dev)
                steps = max_steps_for(env)
                crit = core.criteria()
                times = []
                s = torch.cuda.current_stream(dev)
                for r in range(args.reps + 1):
                    core.reset(env, batch, st)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    core.rollout(env, ctl.ctrl, crit, batch, st, steps)
                    e1.record(s)
                    torch.cuda.synchronize()
                    if r:
                        times.append(e0.elapsed_time(e1))
                ms = float(np.median(times))
                done = float(st.acc[core._abi.ACC_STEPS].sum().item())
                print(json.dumps({"ctl": ctl_name, "motion": motion, "n": n, "kernel_ms": round(ms, 3),
                                  "env_steps_per_s": round(done / (ms * 1e-3), 1),
                                  "ns_per_env_step": round(ms * 1e6 / done, 4)}), flush=True)


if __name__ == "__main__":
    main()
