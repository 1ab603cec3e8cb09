"""Measured deviation of the figure-8 feed-forward scenario from the
reference's fixture: the oracle (CPU) and, when a GPU is present, the fused
kernel.  The reference's figure-8 acceleration is a nested 1e-6 forward
difference (target_motion.py:215-229), which turns last-bit sin/cos
differences into ~1e-5-1e-4 noise in the feed-forward term; this prints what
that noise does to the metrics, states and records, per quantity.

    python scripts/ff_fig8_deviation.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "lqr-quadcopter-test_amd")]
import oracle as O  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
SCEN = {s["name"]: s for s in json.load(open(os.path.join(G, "scenarios.json")))["scenarios"]}
CL = np.load(os.path.join(G, "closed_loop.npz"))
FIELDS = json.load(open(os.path.join(G, "scenarios.json")))["metric_fields"]
s = SCEN["ff_figure8"]
ref_m, ref_f = CL["ff_figure8_metrics"], CL["ff_figure8_final"]


def report(tag, met, fin):
    d = np.abs(met - ref_m)
    rel = d / np.maximum(np.abs(ref_m), 1e-300)
    out = {"who": tag, "metrics_max_abs": float(d.max()),
           "worst_field": FIELDS[int(np.argmax(d.max(axis=0)))],
           "per_field_max_abs": {f: float(d[:, i].max()) for i, f in enumerate(FIELDS)},
           "per_field_max_rel": {f: float(rel[:, i].max()) for i, f in enumerate(FIELDS)},
           "final_state_max_abs": float(np.abs(fin[:, :12] - ref_f[:, :12]).max())}
    print(json.dumps(out))
    return out


mets, fins = [], []
for e, seed in enumerate(s["seeds"]):
    env = O.env_params(s["env"])
    c, K, kc, fb, _ = O.controller(s["ctl"])
    pat, off = O.draws(env.motion, [seed])
    x0 = O.initial_state(env, env.motion, pat[0], off[0])
    met, xf, integ, _ = O.episode(env, c, O.criteria(), env.motion, pat[0], env.mass, c.hover_thrust, K, kc, x0)
    mets.append(met)
    fins.append(np.concatenate([xf, integ]))
report("oracle", np.array(mets), np.array(fins))

try:
    import torch
    have_gpu = torch.cuda.is_available()
except Exception:
    have_gpu = False
if have_gpu:
    from quadtrack.controllers import batched_controller
    from quadtrack.rollout import run_closed_loop
    c0 = dict(s["ctl"])
    ctl = batched_controller(c0.pop("controller", "riccati_lqr"), c0)
    for record in (False, True):
        res = run_closed_loop(ctl, s["env"], n=len(s["seeds"]), seeds=s["seeds"], record=record)
        fin = np.concatenate([res.state.x.cpu().numpy().T, res.state.integ[:3].cpu().numpy().T], axis=1)
        report("gpu_exact_step" if record else "gpu_fast_step", res.metrics.cpu().numpy().T, fin)
