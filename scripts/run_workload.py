#!/usr/bin/env python3
"""Run one BASELINE.json workload (quadtrack.workloads, configs 1-5) end to
end and print one JSON line: setup times (per-episode DAREs, device draws),
rollout time (HIP events), env-steps/s and the EvaluationSummary.

  python scripts/run_workload.py --config 5 [--episodes N] [--repeat R]
  python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \
      scripts/run_workload.py --config 4          # episode-sharded, RCCL summary

--episodes runs the first N episodes of the config (global indices 0..N-1);
with W ranks each rank builds only its shard [r N / W, (r + 1) N / W).

Self-checking for multi-GPU runs: --gpus N (default: WORLD_SIZE) must equal
the WORLD_SIZE the launcher started, and rank 0's line carries
world_size_seen, the backend and every rank's shard (global range,
episodes, env-steps, waves of its launch, best shard time).  The shard
time of the slowest rank sets rollout_ms.  --launcher-check runs the same
launch on CPU (gloo): the ranks report their shards without a GPU.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--episodes", type=int, default=None)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--warmup-s", type=float, default=1.0,
                    help="untimed back-to-back rollouts first (the clock ramps up over ~1 s of load)")
    ap.add_argument("--no-group", action="store_true", help="config 5: one runtime-motion launch instead of groups")
    ap.add_argument("--gpus", type=int, default=None, help="ranks expected (default WORLD_SIZE); a mismatch is refused")
    ap.add_argument("--shard", default=None, metavar="R/W",
                    help="one process: run rank R's shard of a W-rank job (the 8-GPU layout timed on one GPU)")
    ap.add_argument("--launcher-check", action="store_true",
                    help="CPU only: join a gloo group and report every rank's shard, no GPU work")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"run_workload.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.launcher_check:
        return launcher_check(args, world, rank)

    import torch
    import torch.distributed as dist

    if torch.cuda.device_count() <= local:
        raise SystemExit(f"run_workload.py: rank {rank} needs GPU {local} but {torch.cuda.device_count()} are visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from quadtrack import core, workloads
    from quadtrack._abi import MET
    from quadtrack.rollout import _criteria, build_batch, max_steps_for

    total = args.episodes or workloads.EPISODES[args.config]
    lo, hi = workloads.shard_bounds(total, rank, world)
    if args.shard:
        if world > 1:
            raise SystemExit("run_workload.py: --shard is a one-process option")
        sr, sw = (int(v) for v in args.shard.split("/"))
        lo, hi = workloads.shard_bounds(total, sr, sw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sh = workloads.build(args.config, lo, hi, device=dev)
    torch.cuda.synchronize()
    t_ctl = time.perf_counter() - t0
    t0 = time.perf_counter()
    batch = build_batch(sh.controller, sh.env_config, sh.n, seeds=sh.seeds, motion=sh.motion,
                        plant_mass=sh.plant_mass, group_motion=not args.no_group)
    torch.cuda.synchronize()
    t_batch = time.perf_counter() - t0
    # the same setup again, warm (kernels loaded, allocator primed): what a
    # tuner pays per sweep after the first
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sh2 = workloads.build(args.config, lo, hi, device=dev)
    torch.cuda.synchronize()
    t_ctl_warm = time.perf_counter() - t0
    t0 = time.perf_counter()
    build_batch(sh2.controller, sh2.env_config, sh2.n, seeds=sh2.seeds, motion=sh2.motion,
                plant_mass=sh2.plant_mass, group_motion=not args.no_group)
    torch.cuda.synchronize()
    t_batch_warm = time.perf_counter() - t0
    del sh2

    # a grouped batch runs on its slot-ordered copy, as run_closed_loop does (coalesced rows)
    perm, t_copy = None, None
    if batch.groups is not None and batch.order is not None:
        batch.physical_groups()  # first call: allocator and kernels warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batch, perm = batch.physical_groups()
        torch.cuda.synchronize()
        t_copy = time.perf_counter() - t0
    env = sh.env_config.to_params()
    crit = _criteria(None)
    st = core.RolloutState.empty(sh.n, dev)
    core.validate(batch, st)
    nsteps = max_steps_for(env)
    stream = torch.cuda.current_stream(dev)
    times = []
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < args.warmup_s:
        core.reset(env, batch, st)
        core.rollout(env, sh.controller.ctrl, crit, batch, st, nsteps)
        torch.cuda.synchronize()
    for _ in range(args.repeat):
        core.reset(env, batch, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        core.rollout(env, sh.controller.ctrl, crit, batch, st, nsteps)
        e1.record(stream)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    met = core.episode_metrics(crit, st)
    if perm is not None:
        met = core.unpermute(met, perm)
    my_steps = float(met[MET["steps"]].sum().item())
    waves = core.launch_waves(batch)
    mine = [float(rank), float(lo), float(hi), my_steps, float(waves), min(times)]
    from quadtrack.parallel import all_gather_rows, reduce_summary

    ranks = all_gather_rows(torch.tensor(mine, dtype=torch.float64, device=dev)) if world > 1 else [mine]
    steps = sum(r[3] for r in ranks)
    kern = max(r[5] for r in ranks)  # the slowest rank's shard sets the job's time

    s = reduce_summary(met, crit, global_offset=lo)
    if rank == 0:
        print(json.dumps({
            "config": args.config, "episodes": total, "world": world, "episodes_per_rank": sh.n,
            "shard": args.shard, "riders": core.riders_on(),
            "world_size_seen": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "ranks": [{"rank": int(r[0]), "lo": int(r[1]), "hi": int(r[2]), "episodes": int(r[2] - r[1]),
                       "env_steps": r[3], "waves": int(r[4]), "shard_ms": round(r[5], 3)} for r in ranks],
            "grouped": batch.groups is not None,
            "setup_s": {"controller_dare_and_params": round(t_ctl, 4), "batch_draws": round(t_batch, 4)},
            "setup_warm_s": {"controller_dare_and_params": round(t_ctl_warm, 4), "batch_draws": round(t_batch_warm, 4),
                             "group_copy": None if t_copy is None else round(t_copy, 4)},
            "dare_max_iterations": int(sh.controller.iters.max().item()),
            "dare_fallbacks": int((sh.controller.status != 0).sum().item()),
            "rollout_ms": round(kern, 3), "rollout_ms_median": round(sorted(times)[len(times) // 2], 3),
            "warmup_s": args.warmup_s, "rollout_ms_all": [round(t, 3) for t in times],
            "env_steps": steps, "env_steps_per_s": round(steps / (kern * 1e-3), 1),
            "summary": {"mean_on_target_ratio": s.mean_on_target_ratio, "std_on_target_ratio": s.std_on_target_ratio,
                        "mean_tracking_error": s.mean_tracking_error, "std_tracking_error": s.std_tracking_error,
                        "success_rate": s.success_rate, "mean_control_effort": s.mean_control_effort,
                        "best_episode_idx": s.best_episode_idx, "worst_episode_idx": s.worst_episode_idx},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def launcher_check(args, world: int, rank: int):
    """The ranks' view of a multi-GPU run, on CPU (gloo): each rank's shard
    of the config as the real run builds it (workloads.shard_bounds); rank 0
    prints one line."""
    import torch
    import torch.distributed as dist

    from quadtrack import workloads

    if world > 1:
        dist.init_process_group("gloo")
    total = args.episodes or workloads.EPISODES[args.config]
    lo, hi = workloads.shard_bounds(total, rank, world)
    mine = torch.tensor([rank, lo, hi], dtype=torch.int64)
    if world > 1:
        out = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(out, mine)
        rows = [o.tolist() for o in out]
    else:
        rows = [mine.tolist()]
    if rank == 0:
        print(json.dumps({"launcher_check": True, "config": args.config, "episodes": total, "world": world,
                          "world_size_seen": dist.get_world_size() if world > 1 else 1,
                          "backend": dist.get_backend() if world > 1 else None,
                          "ranks": [{"rank": r, "lo": a, "hi": b, "episodes": b - a} for r, a, b in rows]}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
