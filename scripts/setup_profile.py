#!/usr/bin/env python3
"""Where a workload's host-side setup goes (GPU box): cProfile of the second
(warm) workloads.build + build_batch of BASELINE config 4 or 5."""
import argparse
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))

import torch  # noqa: E402

from quadtrack import workloads  # noqa: E402
from quadtrack.rollout import build_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=5)
args = ap.parse_args()
dev = torch.device("cuda", 0)


def once():
    sh = workloads.build(args.config, device=dev)
    build_batch(sh.controller, sh.env_config, sh.n, seeds=sh.seeds, motion=sh.motion, plant_mass=sh.plant_mass,
                group_motion=True)
    torch.cuda.synchronize()


once()
pr = cProfile.Profile()
pr.enable()
once()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
