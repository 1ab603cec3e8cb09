"""Debug: the runtime-motion yaw-at-rest loop (MOTION = -1) against the
motion-specialised loop on single-motion batches, bitwise (GPU)."""
import sys
import numpy as np
import torch
sys.path.insert(0, 'lqr-quadcopter-test_amd')
from quadtrack.controllers import BatchedRiccatiLQR
from quadtrack.rollout import run_closed_loop

n = 4096
ctl = BatchedRiccatiLQR({"dt": 0.01})
names = ["stationary", "linear", "circular", "sinusoidal", "figure8"]
for m, name in enumerate(names):
    env = {"target": {"motion_type": name}}
    a = run_closed_loop(ctl, env, n=n, seeds=np.arange(n))                      # specialised
    b = run_closed_loop(ctl, env, n=n, seeds=np.arange(n), motion=[m] * n)      # runtime motion
    da = (a.metrics - b.metrics).abs().max(dim=1).values.cpu().numpy()
    dx = (a.state.x - b.state.x).abs().max().item()
    print(name, 'metric rows max diff', np.array2string(da, precision=2), 'state', dx, flush=True)
    # the first step only
    a1 = run_closed_loop(ctl, env, n=n, seeds=np.arange(n), max_steps=1)
    b1 = run_closed_loop(ctl, env, n=n, seeds=np.arange(n), motion=[m] * n, max_steps=1)
    print('   1 step: state diff', (a1.state.x - b1.state.x).abs().max().item(), 'target diff',
          (a1.state.target - b1.state.target).abs().max().item(), flush=True)
