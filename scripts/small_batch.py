#!/usr/bin/env python3
"""The fused rollout at small per-GPU batches: config 2's
pass (linear target, shared Riccati-LQR gain, one fresh launch set: reset,
3,000 steps, metrics) at n episodes for each n given, best and median of
--reps passes (HIP events) after a >= 1 s warm-up.  One JSON line per n:
ms per pass, env-steps/s, waves (one lane per episode: n / 64 waves on the
GPU's 1,024 SIMDs) and, for n = 65,536 / W, the strong-scaled "65,536
episodes on W GPUs" reading it implies (65,536 x steps / the per-GPU pass
time).

  python scripts/small_batch.py --n 4096 8192 16384 32768 65536 131072
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-quadcopter-test_amd"))

from quadtrack import core  # noqa: E402
from quadtrack._abi import MET  # noqa: E402
from quadtrack.controllers import BatchedRiccatiLQR  # noqa: E402
from quadtrack.env.config import EnvConfig  # noqa: E402
from quadtrack.rollout import build_batch, max_steps_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[4096, 8192, 16384, 32768, 65536, 131072])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--motion", default="linear")
    ap.add_argument("--warmup-s", type=float, default=1.0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = EnvConfig.from_dict({"target": {"motion_type": a.motion}})
    env = cfg.to_params()
    crit = core.criteria()
    ctl = BatchedRiccatiLQR({"dt": 0.01}, device=dev)
    nsteps = max_steps_for(env)
    stream = torch.cuda.current_stream(dev)
    runs = {}
    for n in a.n:
        batch = build_batch(ctl, cfg, n, seeds=np.arange(n))
        st = core.RolloutState.empty(n, dev)
        core.validate(batch, st)
        runs[n] = (batch, st)
    # clock warm-up on the largest batch
    big = max(a.n)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.warmup_s:
        core.rollout_fresh(env, ctl.ctrl, crit, *runs[big], nsteps)
        torch.cuda.synchronize()
    for n in a.n:
        batch, st = runs[n]
        for _ in range(3):
            core.rollout_fresh(env, ctl.ctrl, crit, batch, st, nsteps)
        times = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            met = core.rollout_fresh(env, ctl.ctrl, crit, batch, st, nsteps)
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        steps = float(met[MET["steps"]].sum().item())
        best, med = min(times), float(np.median(times))
        line = {"n": n, "motion": a.motion, "waves": (n + 63) // 64, "ms_best": round(best, 4),
                "ms_median": round(med, 4), "env_steps": steps, "env_steps_per_s": steps / (best * 1e-3),
                "ns_per_env_step": best * 1e6 / steps}
        if 65536 % n == 0 and n <= 65536:
            w = 65536 // n
            line["strong_scaled"] = {"gpus": w, "episodes_total": 65536,
                                     "env_steps_per_s_total": steps * w / (best * 1e-3)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
