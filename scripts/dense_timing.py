#!/usr/bin/env python3
"""Rollout time of a dense-gain (coupled Q) batch: 65,536 episodes x 3,000
steps, circular target; k_no_yaw on (yaw-at-rest flavour) vs forced off."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))
from quadtrack import core  # noqa: E402
from quadtrack.controllers import BatchedRiccatiLQR  # noqa: E402
from quadtrack.env.config import EnvConfig  # noqa: E402
from quadtrack.rollout import build_batch, max_steps_for  # noqa: E402

Q = np.diag([1e-4, 1e-4, 16.0, 0.0036, 0.0036, 4.0])
Q[0, 1] = Q[1, 0] = 5e-5
Q[0, 3] = Q[3, 0] = 2e-4
Q[2, 5] = Q[5, 2] = 0.5
dev = torch.device("cuda", 0)
ctl = BatchedRiccatiLQR({"dt": 0.01, "Q": Q.tolist()}, device=dev)
cfg = EnvConfig.from_dict({"target": {"motion_type": "circular"}})
env, crit, n = cfg.to_params(), core.criteria(), 65536
batch = build_batch(ctl, cfg, n, seeds=np.arange(n))
st = core.RolloutState.empty(n, dev)
stream = torch.cuda.current_stream(dev)
for no_yaw in (True, False):
    batch.k_no_yaw = no_yaw
    ts = []
    for _ in range(4):
        core.reset(env, batch, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        core.rollout(env, ctl.ctrl, crit, batch, st, max_steps_for(env))
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"k_no_yaw={no_yaw}: {np.median(ts[1:]):.3f} ms per {n}-episode rollout")
