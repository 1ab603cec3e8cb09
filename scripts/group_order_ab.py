#!/usr/bin/env python3
"""Slot orders of config 5's 8-GPU shard (131,072 episodes, 2,048 waves =
the resident set at two waves per SIMD, so each SIMD pairs a wave of the
first 1,024 with one of the second): the committed longest-wave-first group
order against orders that pair long waves with short ones, the motion groups
split into segments (qt_rollout_grouped: <= 8 segments, each a motion).
Alternates the orders --reps times; one JSON line per (order, rep): best and
median of --repeat rollouts after a 1 s warm-up.

  python scripts/group_order_ab.py [--shard 0/8] [--reps 2]
"""

import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))

from quadtrack import core, workloads  # noqa: E402
from quadtrack.rollout import _criteria, build_batch, max_steps_for  # noqa: E402

# name -> list of (motion, fraction of that motion's episodes) segments in slot order
ORDERS = {
    "longest_first": [(3, 1.0), (4, 1.0), (2, 1.0), (1, 1.0), (0, 1.0)],
    # round 1 longest first, round 2 shortest first: sin / fig8 / half circ, then stat / lin / half circ
    "zigzag": [(3, 1.0), (4, 1.0), (2, 0.5), (0, 1.0), (1, 1.0), (2, 0.5)],
    "zigzag_b": [(3, 1.0), (4, 1.0), (2, 0.5), (1, 1.0), (0, 1.0), (2, 0.5)],
}


def order_of(motion: np.ndarray, spec):
    idx = {m: np.nonzero(motion == m)[0] for m in range(5)}
    used = {m: 0 for m in range(5)}
    parts, sm, se, end = [], [], [], 0
    for m, frac in spec:
        cnt = len(idx[m])
        take = cnt - used[m] if frac >= 1.0 or used[m] else int(round(cnt * frac / 64)) * 64
        take = min(take, cnt - used[m])
        parts.append(idx[m][used[m]:used[m] + take])
        used[m] += take
        end += take
        sm.append(m)
        se.append(end)
    assert all(used[m] == len(idx[m]) for m in range(5))
    return np.concatenate(parts).astype(np.int32), sm, se


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard", default="0/8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--repeat", type=int, default=10)
    ap.add_argument("--orders", nargs="*", default=list(ORDERS))
    a = ap.parse_args()
    r, w = (int(v) for v in a.shard.split("/"))
    lo, hi = workloads.shard_bounds(workloads.EPISODES[5], r, w)
    dev = torch.device("cuda", 0)
    sh = workloads.build(5, lo, hi, device=dev)
    base = build_batch(sh.controller, sh.env_config, sh.n, seeds=sh.seeds, motion=sh.motion,
                       plant_mass=sh.plant_mass)
    env = sh.env_config.to_params()
    crit = _criteria(None)
    nsteps = max_steps_for(env)
    stream = torch.cuda.current_stream(dev)
    runs = {}
    for name in a.orders:
        order, sm, se = order_of(np.asarray(sh.motion), ORDERS[name])
        b = dataclasses.replace(base, order=torch.as_tensor(order, device=dev), groups=(sm, se))
        pb, _ = b.physical_groups()
        st = core.RolloutState.empty(sh.n, dev)
        core.validate(pb, st)
        runs[name] = (pb, st, core.grouped_waves(sm, se))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        pb, st, _ = runs[a.orders[0]]
        core.reset(env, pb, st)
        core.rollout(env, sh.controller.ctrl, crit, pb, st, nsteps)
        torch.cuda.synchronize()
    for rep in range(a.reps):
        for name in a.orders:
            pb, st, waves = runs[name]
            times = []
            for _ in range(a.repeat):
                core.reset(env, pb, st)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                core.rollout(env, sh.controller.ctrl, crit, pb, st, nsteps)
                e1.record(stream)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
            print(json.dumps({"order": name, "rep": rep, "shard": a.shard, "waves": waves,
                              "segments": [int(m) for m in pb.groups[0]], "ms_best": round(min(times), 4),
                              "ms_median": round(float(np.median(times)), 4)}), flush=True)


if __name__ == "__main__":
    main()
