#!/usr/bin/env python3
"""Batched DARE throughput: the structured per-axis kernel and the general
dense SDA kernel (qt_dare_batched structured = 1 / 0) on the hover model,
6-state LQR and 9-state LQI, m problems with random diagonal Q and R (the
tuner's ranges).  Prints one JSON line per case (HIP events, median of
--reps).  Run under rocprofv3 --kernel-trace --stats for the kernel table.

  python scripts/dare_bench.py [--m 65536] [--reps 5]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--states", default="6,9", help="state sizes to run (6, 9)")
    ap.add_argument("--kernels", default="structured,dense", help="structured and / or dense")
    args = ap.parse_args()

    import numpy as np
    import torch

    from quadtrack import core

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    m = args.m
    kinds = [k == "structured" for k in args.kernels.split(",")]
    for n in [int(v) for v in args.states.split(",")]:
        qd = np.concatenate([rng.uniform([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0], (m, 3)),
                             rng.uniform([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0], (m, 3))]
                            + ([rng.uniform([1e-4, 1e-4, 1e-3], [1e-3, 1e-3, 1e-2], (m, 3))] if n == 9 else []), axis=1)
        rd = rng.uniform(0.5, 2.0, (m, 4))
        Q = torch.zeros(n * n, m, dtype=torch.float64)
        R = torch.zeros(16, m, dtype=torch.float64)
        for i in range(n):
            Q[i * n + i] = torch.from_numpy(qd[:, i])
        for i in range(4):
            R[i * 4 + i] = torch.from_numpy(rd[:, i])
        Q, R = Q.to(dev), R.to(dev)
        for structured in kinds:
            core.dare_batched(n, 0.01, 9.81, None, Q[:, :256].contiguous(), R[:, :256].contiguous(), structured)
            times = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                K, P, status, iters = core.dare_batched(n, 0.01, 9.81, None, Q, R, structured)
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
            ms = float(np.median(times))
            print(json.dumps({"n_state": n, "structured": structured, "problems": m, "ms": round(ms, 4),
                              "solves_per_s": round(m / (ms * 1e-3), 1), "max_iterations": int(iters.max().item()),
                              "failed": int((status != 0).sum().item())}), flush=True)


if __name__ == "__main__":
    main()
