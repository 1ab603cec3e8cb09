import sys, os, numpy as np, torch
sys.path.insert(0, 'lqr-quadcopter-test_amd')
from quadtrack import workloads
from quadtrack.rollout import run_closed_loop
total = workloads.EPISODES[5]
full = workloads.build(5)
res = run_closed_loop(full.controller, **full.run_kwargs())
met = res.metrics.cpu().numpy()
kw = full.run_kwargs()
motion_full = np.asarray(kw.get('motion'))
for r in (0, 3):
    lo, hi = workloads.shard_bounds(total, r, 4)
    sh = workloads.build(5, lo, hi)
    part = run_closed_loop(sh.controller, **sh.run_kwargs()).metrics.cpu().numpy()
    d = np.abs(part - met[:, lo:hi])
    bad = np.where(d.max(0) > 0)[0]
    print('shard', r, 'differing episodes', len(bad), 'max diff per row', d.max(1))
    if len(bad):
        idx = lo + bad[:20]
        print(' global idx', idx, 'motion', motion_full[idx])
        # slot positions in the grouped order: stable argsort by motion
        order_full = np.argsort(motion_full, kind='stable')
        pos_full = np.empty(total, int); pos_full[order_full] = np.arange(total)
        ms = motion_full[lo:hi]; order_sh = np.argsort(ms, kind='stable'); pos_sh = np.empty(hi-lo, int); pos_sh[order_sh] = np.arange(hi-lo)
        print(' slot%64 full', pos_full[idx] % 64, 'slot%64 shard', pos_sh[bad[:20]] % 64)
        print(' wave full', pos_full[idx] // 64, 'wave shard', pos_sh[bad[:20]] // 64)
        print(' steps', met[13, idx], 'term', met[10, idx])
