#!/usr/bin/env python3
"""In-kernel clock of the bench rollout kernel (MI355X_MICROARCH.md, DVFS
give-back item 6): runs the bench workload back to back for ~`--seconds`
with the diagnostic stamp build (-DQT_CLOCK_STAMP=1, build/stamp/), then
reads the last launch's per-wave s_memtime / s_memrealtime stamps taken
around the step loop.  Prints one JSON line:

  clock_mhz      median over waves of d(memtime) / d(realtime) * 100 MHz
  cycles_per_step median d(memtime) / steps (shader cycles, clock independent)
  loop_ms        median d(realtime) / 100 MHz: the step loop's wall time per wave
  kernel_ms      HIP-event time of the same launches (fast + deferred pass)

  QUADTRACK_LIB=build/stamp/libquadtrack.so python scripts/clock_stamp.py [--motion linear] [--ctl lqr]
"""

from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--motion", default="linear")
    ap.add_argument("--ctl", default="lqr")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--dump", default="", help="write the per-wave stamps to this .npz")
    ap.add_argument("--workload", type=int, default=0,
                    help="a BASELINE workload instead (quadtrack.workloads; 5: the grouped kernel, "
                         "its first --n episodes)")
    args = ap.parse_args()
    if "QUADTRACK_LIB" not in os.environ:
        os.environ["QUADTRACK_LIB"] = os.path.join(ROOT, "build", "stamp", "libquadtrack.so")
    import torch

    from quadtrack import _abi, core
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.env.config import EnvConfig
    from quadtrack.rollout import build_batch, max_steps_for

    lib = _abi.load()
    if not hasattr(lib, "qt_debug_stamps"):
        raise SystemExit(f"{_abi.LIB_PATH} is not a -DQT_CLOCK_STAMP=1 build")
    lib.qt_debug_stamps.argtypes = [C.c_void_p, C.c_int64]
    dev = torch.device("cuda", 0)
    n = args.n
    wave_motion = None
    if args.workload:
        from quadtrack import workloads

        sh = workloads.build(args.workload, 0, n, device=dev)
        ctl, cfg = sh.controller, sh.env_config
        batch = build_batch(ctl, cfg, n, seeds=sh.seeds, motion=sh.motion, plant_mass=sh.plant_mass)
        if batch.groups is not None:
            batch, _ = batch.physical_groups()
            wave_motion = np.concatenate([np.full(-(-(b - a) // 64), m) for m, a, b in
                                          zip(batch.groups[0], [0] + list(batch.groups[1][:-1]), batch.groups[1])])
    else:
        cfg_c = {"dt": 0.01} if args.ctl == "lqr" else {"dt": 0.01, "use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2]}
        ctl = BatchedRiccatiLQR(cfg_c, device=dev)
        cfg = EnvConfig.from_dict({"target": {"motion_type": args.motion}})
        batch = build_batch(ctl, cfg, n, seeds=np.arange(n))
    env = cfg.to_params()
    st = core.RolloutState.empty(n, dev)
    steps = max_steps_for(env)
    crit = core.criteria()
    s = torch.cuda.current_stream(dev)
    ms = []
    t_end = time.perf_counter() + args.seconds
    while time.perf_counter() < t_end:
        core.reset(env, batch, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        core.rollout(env, ctl.ctrl, crit, batch, st, steps)
        e1.record(s)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    waves = (n + 63) // 64 if wave_motion is None else len(wave_motion)
    buf = np.zeros((waves, 6), dtype=np.uint64)
    _abi.check(lib.qt_debug_stamps(buf.ctypes.data, waves), "qt_debug_stamps")
    dt = (buf[:, 1] - buf[:, 0]).astype(np.float64)
    dr = (buf[:, 3] - buf[:, 2]).astype(np.float64)
    ok = (dt > 0) & (dr > 0)
    executed = float(st.acc[_abi.ACC_STEPS].max().item())
    out = {"motion": args.motion, "ctl": args.ctl, "n": n, "launches": len(ms), "waves_stamped": int(ok.sum()),
           "clock_mhz": round(float(np.median(dt[ok] / dr[ok] * 100.0)), 1),
           "clock_mhz_p10_p90": [round(float(v), 1) for v in np.percentile(dt[ok] / dr[ok] * 100.0, [10, 90])],
           "cycles_per_step": round(float(np.median(dt[ok])) / executed, 2),
           "quad_cycles_per_step": round(float(np.median(dt[ok])) / executed / 4, 2),
           "loop_ms_median": round(float(np.median(dr[ok])) / 1e5, 4),
           "loop_ms_max": round(float(np.max(dr[ok])) / 1e5, 4),
           "kernel_ms_last10_median": round(float(np.median(ms[-10:])), 4),
           "kernel_ms_first": round(float(ms[0]), 4)}
    # where the slow waves ran: loop time by XCD and by SIMD-occupancy of their CU
    hw, xcc = buf[:, 4].astype(np.int64), buf[:, 5].astype(np.int64) & 0xF
    cu_key = (xcc << 16) | (((hw >> 13) & 0x7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
    simd_key = (cu_key << 2) | ((hw >> 4) & 3)
    _, simd_inv, simd_cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
    out["waves_per_simd_max"] = int(simd_cnt.max())
    out["simds_used"] = int(len(simd_cnt))
    out["loop_ms_by_xcd"] = {int(x): round(float(np.median(dr[xcc == x])) / 1e5, 4) for x in np.unique(xcc)}
    out["loop_ms_max_by_xcd"] = {int(x): round(float(np.max(dr[xcc == x])) / 1e5, 4) for x in np.unique(xcc)}
    out["clock_mhz_by_xcd"] = {int(x): round(float(np.median((dt / dr * 100.0)[xcc == x])), 1) for x in np.unique(xcc)}
    shared = simd_cnt[simd_inv] > 1
    out["loop_ms_shared_simd_median"] = round(float(np.median(dr[shared])) / 1e5, 4) if shared.any() else None
    start = (buf[:, 2].astype(np.float64) - buf[:, 2].min()) / 1e5
    end = (buf[:, 3].astype(np.float64) - buf[:, 2].min()) / 1e5
    out["start_ms_p50_p99_max"] = [round(float(v), 4) for v in np.percentile(start, [50, 99, 100])]
    out["end_ms_p50_p99_max"] = [round(float(v), 4) for v in np.percentile(end, [50, 99, 100])]
    if wave_motion is not None:  # per motion group: loop time, start and end (ms from the first start)
        out["by_motion"] = {int(m): {"waves": int((wave_motion == m).sum()),
                                     "loop_ms_median": round(float(np.median(dr[wave_motion == m])) / 1e5, 4),
                                     "start_ms_max": round(float(start[wave_motion == m].max()), 4),
                                     "end_ms_max": round(float(end[wave_motion == m].max()), 4)}
                            for m in np.unique(wave_motion)}
        late = start > 0.05
        out["late_waves"] = int(late.sum())
        out["late_start_ms_min"] = round(float(start[late].min()), 4) if late.any() else None
    if args.dump:
        np.savez(args.dump, stamps=buf)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
