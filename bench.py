#!/usr/bin/env python3
"""Benchmark of the MI355X closed-loop hot path (BASELINE.json metric:
env-steps/s at 65,536 parallel episodes per GPU; mean tracking error vs the
reference).

Workload (BASELINE.json configs[1]): per GPU 65,536
independent 30 s episodes (3,000 steps at dt = 0.01), linear target,
Riccati-LQR with the default weights (one shared DARE gain), seeds = global
episode index.  One bench "step" = one full evaluation pass over the batch,
inputs already in HBM: the fresh launch (qt_rollout_fresh: the fused
closed-loop rollout kernel forms the reset state in its prologue, runs the
3,000 steps of compute_action -> env.step with fused metric accumulation and
writes the per-episode metric rows in its epilogue), the exact-pass launch
after it (returns at once when no wave was deferred), then the summary's two
launches (partials, + one async RCCL all-reduce of the sums when N > 1).
value = all ranks' env-steps / max-over-ranks wall time.

Beside it (rank 0, N = 1, untimed for `value`): the per-step API leg
(`step_api`: 4,194,304 episodes stepped one launch per step from Python by
BatchedQuadcopterEnv.step_closed, the state round-tripping HBM each step —
~1.9 GB per step, far beyond the 256 MB Infinity Cache, so the rate is HBM's;
GB/s against the 8 TB/s HBM peak), the DARE throughput and the CPU baseline.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 runs one process per GPU under torch.distributed.run: when WORLD_SIZE is
unset, bench.py starts `python -m torch.distributed.run --nproc-per-node N`
on itself as a child process (before any GPU call) and exits with its code;
under a launcher, --gpus must equal WORLD_SIZE.  --gpus N with fewer than N
visible GPUs is an error, never a silent 1-GPU run.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lqr-quadcopter-test_amd"))

# Algorithmic FP64 operations per episode-step of the config-2 loop (LQR,
# linear target, RK4), counted from the reference arithmetic with each sin,
# cos, sqrt and fmod as one operation (DESIGN.md §4 has the table):
# controller 58 + Evaluator metric accumulation 22 + env.step 349.
FLOPS_PER_ENV_STEP = 429
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector, spec (half the FP32 vector 157.3 TF/s)
HBM_PEAK_GBS = 8000.0
# the dominant kernel of the bench workload: yaw-at-rest fast flavour, linear target, 6-column structured K
KERNEL_TAG = "rollout_kernel<2, 1, 6, false, true"
# The committed rocprofv3 session this line reads its profile, traffic and
# issued-FP64 numbers from (scripts/profile_session.sh's condensed CSVs):
# one named directory, never "the newest".  --profile-dir overrides it.
PROFILE_DIR = "profiles/r06"
# Warm-up floor: a fresh box's first ~0.5 s of passes run at lower clocks
# (round 2: --warmup 5, 8 ms of GPU work, measured ~7% below --warmup 20), so
# the warm-up runs for at least this long whatever --warmup says.
WARMUP_FLOOR_S = 1.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warmup-seconds", type=float, default=WARMUP_FLOOR_S,
                    help="minimum warm-up time: passes are added after --warmup until this much has run")
    ap.add_argument("--episodes", type=int, default=65536, help="episodes per GPU")
    ap.add_argument("--motion", default="linear")
    ap.add_argument("--cpu-sample", type=int, default=65536, help="episodes in the CPU baseline sample (rank 0, N=1)")
    ap.add_argument("--cpu-sample-1core", type=int, default=4096, help="episodes of the 1-thread CPU sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="threads of the OpenMP CPU leg (0: see cpu_baseline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--step-api-episodes", type=int, default=4194304,
                    help="episodes of the per-step API leg (rank 0, N=1; 0 skips it)")
    ap.add_argument("--step-api-steps", type=int, default=100)
    ap.add_argument("--profile-dir", default=PROFILE_DIR,
                    help="committed rocprofv3 summaries (kernel_stats.csv, pmc_*.csv) the line cites")
    ap.add_argument("--launcher-check", action="store_true",
                    help="CPU plumbing check of the N-rank launch (gloo, no kernels): prints the ranks seen")
    return ap.parse_args()


def visible_gpu_count() -> int:
    """GPUs this process could open, counted without the HIP runtime (the
    launcher parent must not load or initialise it before it starts the ranks):
    KFD topology nodes with SIMDs whose DRM render node exists and is
    accessible — the agents ROCr itself enumerates — narrowed by the
    *_VISIBLE_DEVICES lists.  0 when there is no KFD (no ROCm GPU)."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(base)
    except OSError:
        return 0
    n = 0
    for node in nodes:
        try:
            props = dict(line.split(" ", 1) for line in open(os.path.join(base, node, "properties")).read().splitlines()
                         if " " in line)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue
        render = f"/dev/dri/renderD{int(props.get('drm_render_minor', '-1'))}"
        if os.access(render, os.R_OK | os.W_OK):
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([d for d in v.split(",") if d.strip()]))
    return n


def launch(args) -> int:
    """Re-run this script as N ranks under torch.distributed.run (child
    process, no exec).  Nothing here imports torch or touches the HIP runtime:
    the GPU count comes from the KFD topology (visible_gpu_count), and each
    rank checks its own device again."""
    import socket
    import subprocess

    if not args.launcher_check:
        visible = visible_gpu_count()
        if visible < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) are visible", file=sys.stderr, flush=True)
            return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def launcher_check(world: int, rank: int):
    """The ranks' view of the launch, on CPU (gloo): rank 0 prints one line."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    seen = dist.get_world_size() if world > 1 else 1
    ranks = torch.tensor([rank], dtype=torch.int64)
    if world > 1:
        out = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(out, ranks)
        ranks_all = [int(t.item()) for t in out]
    else:
        ranks_all = [0]
    if rank == 0:
        print(json.dumps({"launcher_check": True, "n_gpus": world, "world_size_seen": seen, "ranks": ranks_all}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.launcher_check:
        return launcher_check(world, rank)
    import torch
    import torch.distributed as dist

    if torch.cuda.device_count() <= local:
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local} but {torch.cuda.device_count()} are visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from quadtrack import core
    from quadtrack.controllers import BatchedRiccatiLQR
    from quadtrack.env.config import EnvConfig
    from quadtrack.rollout import build_batch, max_steps_for

    n = args.episodes
    cfg = EnvConfig.from_dict({"target": {"motion_type": args.motion}})
    env = cfg.to_params()
    crit = core.criteria()

    # ---- setup (untimed): gains, seeded reset draws uploaded to HBM
    t_dare0 = time.perf_counter()
    ctl = BatchedRiccatiLQR({"dt": 0.01}, device=dev)
    torch.cuda.synchronize()
    t_dare = time.perf_counter() - t_dare0
    lo = rank * n
    seeds = lo + np.arange(n)
    batch = build_batch(ctl, cfg, n, seeds=seeds)
    st = core.RolloutState.empty(n, dev)
    core.validate(batch, st)
    nsteps = max_steps_for(env)

    stream = torch.cuda.current_stream(dev)
    ev = []
    pending = []  # in-flight metric all-reduces (async: RCCL's stream, overlapped with the next pass)

    def one_pass(timed: bool):
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        # reset -> rollout -> per-episode metrics as one launch set (qt_rollout_fresh)
        met = core.rollout_fresh(env, ctl.ctrl, crit, batch, st, nsteps)
        if timed:
            e1.record(stream)
            ev.append((e0, e1))
        part = core.summary_partials(met)
        if world > 1:
            # RCCL over xGMI: the one data exchange.  async_op: it runs on
            # RCCL's own stream after this pass's partials and overlaps the next
            # pass's rollout instead of serialising ~tens of us of collective
            # latency into every pass; all are waited for before the clock stops.
            # (the partials tensor is held until the collective is waited for, so the
            # allocator cannot hand its memory to a later pass while RCCL reads it)
            pending.append((dist.all_reduce(part[0:5], async_op=True), part))
        return met

    # warm-up: --warmup passes, then chunks of ~0.1 s until --warmup-seconds
    # have run.  Whether to go on is agreed over ranks (MAX) after each chunk,
    # so every rank issues the same number of per-pass all-reduces.
    tw0 = time.perf_counter()
    warm = 0
    for _ in range(args.warmup):
        one_pass(False)
        warm += 1
    torch.cuda.synchronize()
    chunk = 5
    while args.warmup_seconds > 0:
        go = time.perf_counter() - tw0 < args.warmup_seconds
        if world > 1:
            gt = torch.tensor([int(go)], dtype=torch.int64, device=dev)
            dist.all_reduce(gt, op=dist.ReduceOp.MAX)
            go = bool(gt.item())
        if not go:
            break
        tc = time.perf_counter()
        for _ in range(chunk):
            one_pass(False)
        torch.cuda.synchronize()
        warm += chunk
        chunk = max(1, min(1000, int(0.1 / max((time.perf_counter() - tc) / chunk, 1e-6))))
    for w, _ in pending:
        w.wait()
    pending.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    warmup_s = time.perf_counter() - tw0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        met = one_pass(True)
    for w, _ in pending:
        w.wait()
    pending.clear()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    kern_all = np.array([a.elapsed_time(b) for a, b in ev])
    kern_ms = float(np.mean(kern_all))
    steps_done = met[core._abi.MET["steps"]].sum()
    local_env_steps = float(steps_done.item())  # this rank's executed env-steps per pass
    per_rank = [local_env_steps]
    seen = 1
    if world > 1:
        seen = dist.get_world_size()  # the ranks RCCL saw
        gathered = [torch.zeros_like(steps_done) for _ in range(world)]
        dist.all_gather(gathered, steps_done)
        per_rank = [float(v.item()) for v in gathered]
        dist.all_reduce(steps_done)
    env_steps_per_pass = float(steps_done.item())  # all ranks, executed steps of the last pass
    value = env_steps_per_pass * args.steps / elapsed

    res_summary = None
    from quadtrack.parallel import summary_from_partials
    from quadtrack.utils.metrics import SuccessCriteria

    res_summary = summary_from_partials(met, SuccessCriteria(), global_offset=lo)

    # ---- DARE throughput (per-episode gains, config-4 style), reported beside
    dare = None
    if rank == 0:
        rng = np.random.default_rng(42)
        m = n
        qp = rng.uniform([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0], (m, 3))
        qv = rng.uniform([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0], (m, 3))
        rc = rng.uniform(0.5, 2.0, (m, 4))
        BatchedRiccatiLQR({"dt": 0.01}, device=dev, q_pos=qp[:256], q_vel=qv[:256], r_controls=rc[:256])
        torch.cuda.synchronize()
        td = time.perf_counter()
        b = BatchedRiccatiLQR({"dt": 0.01}, device=dev, q_pos=qp, q_vel=qv, r_controls=rc)
        torch.cuda.synchronize()
        td = time.perf_counter() - td
        dare = {"problems": m, "seconds_incl_host_setup": round(td, 4), "solves_per_s": round(m / td, 1),
                "max_iterations": int(b.iters.max().item()), "shared_gain_solve_s": round(t_dare, 4)}

    step_api = None
    if rank == 0 and world == 1 and args.step_api_episodes > 0:
        step_api = step_api_leg(args, cfg, dev)

    cpu = None
    track = {"mean_tracking_error": res_summary.mean_tracking_error,
             "mean_on_target_ratio": res_summary.mean_on_target_ratio}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, diff = cpu_baseline(args, cfg, seeds[: args.cpu_sample], met[:, : args.cpu_sample])
        track["oracle_sample_episodes"] = int(min(args.cpu_sample, n))
        track["oracle_sample_max_abs_diff"] = diff

    if rank == 0:
        achieved = FLOPS_PER_ENV_STEP * local_env_steps / (kern_ms * 1e-3) / 1e12
        # the dominant kernel: the fast yaw-at-rest flavour (older profiles: the single-flavour kernel)
        traffic, traffic_src = pmc_traffic(args.profile_dir, KERNEL_TAG)
        # algorithmic HBM bytes of one fresh launch: per-episode pattern 3 and start offset 3 doubles
        # in; x 12, target 9, t, acc 14, the 14 metric rows and the 3 integral rows qt_reset would
        # zero out; gains are a broadcast
        algo_bytes = (6 + 53) * 8 * n
        # the same frac from the committed rocprofv3 kernel trace (fast launch alone; its deferred
        # exact pass runs no wave at this workload)
        prof = profiled_kernel(args.profile_dir, KERNEL_TAG)
        prof_line = None
        if prof is not None:
            p_ms, p_min, p_calls, p_dir = prof
            p_ach = FLOPS_PER_ENV_STEP * local_env_steps / (p_ms * 1e-3) / 1e12
            prof_line = {"source": f"{p_dir}/kernel_stats.csv", "kernel_avg_ms": round(p_ms, 4),
                         "kernel_min_ms": round(p_min, 4), "calls": p_calls, "achieved": round(p_ach, 3),
                         "frac": round(p_ach / FP64_PEAK_TFLOPS, 4)}
        # what the hardware issues: FP64 VALU instructions of the dominant kernel from the committed
        # counter pass (64 lanes x (2 FMA + MUL + ADD + TRANS) per wave instruction), over this run's
        # kernel time
        issued = issued_fp64(args.profile_dir, KERNEL_TAG)
        issued_line = None
        if issued is not None:
            i_flops, i_src, i_counts = issued
            i_ach = i_flops / (kern_ms * 1e-3) / 1e12
            issued_line = {"flops_per_launch": i_flops, "per_env_step": round(i_flops / local_env_steps, 2),
                           "source": i_src, "counters_per_launch": i_counts}
        line = {
            "metric": "env-steps/sec at 65 536 parallel episodes per GPU (30 s @ dt=0.01, Riccati-LQR closed loop)",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_passes_run": warm,
            "warmup_s": round(warmup_s, 3),
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: seeded resets, seeds = global episode index; draws made on the GPU by the "
                    "qt_seed_draws restatement of numpy default_rng (SeedSequence + PCG64 + ziggurat)",
            "config": {"workload": f"BASELINE configs[1]: {n} episodes/GPU x {nsteps - 2} steps, {args.motion} "
                                   f"target, Riccati-LQR shared K, RK4 dt=0.01",
                       "episodes_per_gpu": n, "episodes_total": n * world, "parallelism": f"episode-sharded x{world}"},
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": traffic_src, "algorithmic_bytes_per_launch": algo_bytes,
                         "hbm_GBps_achieved": round(algo_bytes / (kern_ms * 1e-3) / 1e9, 3),
                         "kernel": "rollout_kernel<yaw-at-rest fast step, LINEAR, K=6, no-FF, structured K> "
                                   "in a fresh pass (reset prologue, metrics epilogue) + its deferred exact pass "
                                   "(HIP events around both)",
                         "kernel_ms": round(kern_ms, 4),
                         "kernel_ms_min_median_max": [round(float(v), 4) for v in
                                                      (kern_all.min(), np.median(kern_all), kern_all.max())],
                         "flops_per_env_step": FLOPS_PER_ENV_STEP,
                         "issued_tflops": None if issued is None else round(i_ach, 3),
                         "issued_frac": None if issued is None else round(i_ach / FP64_PEAK_TFLOPS, 4),
                         "issued": issued_line,
                         "profiled": prof_line},
            "ranks": {"world_size_seen": seen, "backend": "nccl (RCCL)" if world > 1 else None,
                      "env_steps_per_pass_per_rank": per_rank},
            "cpu_baseline": cpu,
            "tracking": track,
            "dare": dare,
            "step_api": step_api,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# HBM bytes per env-step the per-step API's closed step must move by its
# contract (DESIGN.md §4 "Per-step API"): it reads the previous frame's state
# (12), target position and velocity (6), time (1), the three counters and
# the done flag, and the linear pattern (3); it writes the new frame
# (25 doubles, 3 counters, 5 flags) and the action (4 doubles).
STEP_API_BYTES = (12 + 6 + 1 + 3) * 8 + 1 + 3 * 8 + (25 + 3) * 8 + 5 + 4 * 8
SURVEY_STEP_BYTES = 200  # x[12] read + write + err


def step_api_leg(args, cfg, dev):
    """The per-step API at --step-api-episodes episodes: --step-api-steps
    one-launch closed-loop steps (BatchedQuadcopterEnv.step_closed,
    qt_frame_closed_step) from Python, HIP events on the launch stream around
    the loop (the loop is GPU-bound at this size: host issue < kernel time).
    The HBM roofline of the state round-tripping HBM every step:
    contract bytes / time per step against the 8 TB/s peak; the kernel's own
    rocprofv3 trace and FETCH / WRITE counters are in profiles/."""
    import torch

    from quadtrack import BatchedQuadcopterEnv
    from quadtrack.controllers import BatchedRiccatiLQR

    n, k = args.step_api_episodes, args.step_api_steps
    ctl = BatchedRiccatiLQR({"dt": 0.01}, device=dev)
    env = BatchedQuadcopterEnv(n, cfg, device=dev)
    ctl.reset(n)
    env.reset(np.arange(n))
    for _ in range(10):
        env.step_closed(ctl)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    for _ in range(k):
        env.step_closed(ctl)
    e1.record(s)
    host_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / k
    # what the timed loop computed: the first 1,024 episodes' state after its
    # 10 + k steps against the fused rollout of the same episodes for as many
    # steps (another kernel: the fused loop's closed-form exact step, with
    # recording so that it is not the bench kernel, whose profile averages
    # over its dispatches)
    from quadtrack.rollout import run_closed_loop

    m = min(n, 1024)
    ref = run_closed_loop(BatchedRiccatiLQR({"dt": 0.01}, device=dev), cfg, n=m, seeds=np.arange(m),
                          max_steps=10 + k, record=True)
    got = env.frame.f[0:12, :m]
    check = float((got - ref.state.x).abs().max().item())
    gbps = STEP_API_BYTES * n / (ms * 1e-3) / 1e9
    out = {"episodes": n, "steps": k, "launches_per_step": 1, "ms_per_step": round(ms, 5),
           "env_steps_per_s": round(n / (ms * 1e-3), 1), "host_us_per_step": round(host_s / k * 1e6, 2),
           "contract_bytes_per_env_step": STEP_API_BYTES, "hbm_GBps": round(gbps, 1),
           "hbm_frac": round(gbps / HBM_PEAK_GBS, 4),
           # SURVEY §8(d)'s nominal B_step (state in and out + the error, 200 B for LQR):
           # env-steps/s x 200 B / peak; the frame moves the observation and info besides
           "survey_bytes_per_env_step": SURVEY_STEP_BYTES,
           "survey_hbm_frac": round(SURVEY_STEP_BYTES * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "kernel": "closed_step_kernel<6, no-FF, structured K, freeze> (qt_frame_closed_step)",
           "check_vs_fused_max_abs_diff": check, "check_episodes": m}
    del env, ctl
    torch.cuda.empty_cache()
    return out


def profiled_kernel(profile_dir, tag):
    """Average duration (ms) of the dominant kernel (name containing `tag`) in
    the committed rocprofv3 kernel trace <profile_dir>/kernel_stats.csv:
    (avg_ms, min_ms, calls, profile dir), or None."""
    import csv

    path = os.path.join(ROOT, profile_dir, "kernel_stats.csv")
    if not os.path.exists(path):
        return None
    rows = [r for r in csv.DictReader(open(path)) if tag in r["Name"]]
    if not rows:
        return None
    r = rows[0]
    return float(r["AverageNs"]) * 1e-6, float(r["MinNs"]) * 1e-6, int(r["Calls"]), profile_dir


def _pmc_avg(path, counter, tag):
    """Per-dispatch average of `counter` for the kernel named like `tag` in a
    scripts/pmc_summary.py CSV, or None."""
    import csv

    if not os.path.exists(path):
        return None
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter and tag in r["Kernel_Name"]]
    return float(rows[0]["Average_Per_Dispatch"]) if rows else None


def pmc_traffic(profile_dir, tag):
    """HBM bytes per rollout launch from the committed rocprofv3 PMC passes
    (<profile_dir>/pmc_FETCH_SIZE.csv, pmc_WRITE_SIZE.csv; scripts/profile_session.sh).
    gfx950 FETCH_SIZE counts half the bytes of wide streaming reads
    (MI355X_MICROARCH.md §HBM), so it is doubled; both counters are in KiB."""
    f = _pmc_avg(os.path.join(ROOT, profile_dir, "pmc_FETCH_SIZE.csv"), "FETCH_SIZE", tag)
    w = _pmc_avg(os.path.join(ROOT, profile_dir, "pmc_WRITE_SIZE.csv"), "WRITE_SIZE", tag)
    if f is None or w is None:
        return None, None
    return (2.0 * f + w) * 1024.0, profile_dir


F64_COUNTERS = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")


def issued_fp64(profile_dir, tag):
    """FP64 flops the hardware issues per launch of the kernel named like
    `tag`, from the committed counter pass <profile_dir>/pmc_F64_summary.csv:
    64 lanes x (2 FMA + MUL + ADD + TRANS) per wave instruction (every lane of
    the bench's waves is active).  (flops, source, counts) or None."""
    path = os.path.join(ROOT, profile_dir, "pmc_F64_summary.csv")
    counts = {c: _pmc_avg(path, c, tag) for c in F64_COUNTERS}
    if any(v is None for v in counts.values()):
        return None
    flops = 64.0 * (2.0 * counts["SQ_INSTS_VALU_FMA_F64"] + counts["SQ_INSTS_VALU_MUL_F64"]
                    + counts["SQ_INSTS_VALU_ADD_F64"] + counts["SQ_INSTS_VALU_TRANS_F64"])
    return flops, f"{profile_dir}/pmc_F64_summary.csv", counts


def cpu_baseline(args, cfg, seeds, gpu_met):
    """The oracle (C restatement of the reference loop, oracle/) on the host
    cores over bounded samples of the same episodes: one core on the first
    --cpu-sample-1core episodes, then OpenMP over the host threads on the
    first --cpu-sample; also returns the max |GPU - oracle| over the latter's
    per-episode metrics."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    env = O.env_params({"target": {"motion_type": args.motion}})
    c, K, kc, _, _ = O.controller({"dt": 0.01})
    pat, off = O.draws(args.motion, seeds)
    x0 = np.array([O.initial_state(env, env.motion, pat[i], off[i]) for i in range(len(seeds))])

    def timed(m, threads):
        t0 = time.perf_counter()
        met, _, _, used = O.rollout(env, c, O.criteria(), None, pat[:m], None, None, K, kc, False, x0[:m],
                                    threads=threads)
        return met, time.perf_counter() - t0, used

    m1 = min(args.cpu_sample_1core, len(seeds))
    met1, dt1, _ = timed(m1, 1)
    # threads: --cpu-threads, else OMP_NUM_THREADS (the GPU box sets it to 16, its CPU share per
    # GPU, and asks that pools stay within it), else every CPU this process may run on
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if args.cpu_threads:
        threads, why = args.cpu_threads, "--cpu-threads"
    elif omp:
        threads, why = omp, f"OMP_NUM_THREADS={omp} (the GPU box's CPU share per GPU)"
    else:
        threads, why = affinity, "sched_getaffinity"
    met, dt, used = timed(len(seeds), threads)
    steps = float(met[:, -1].sum())
    diff = float(np.max(np.abs(gpu_met.cpu().numpy().T - met)))
    cpu = {"value": round(steps / dt, 1), "unit": "env-steps/s", "cores": int(used), "kind": "port",
           "sample": f"{len(seeds)} episodes x 3000 steps of the same workload (oracle/qt_oracle.c, FP64, "
                     f"OpenMP over episodes, {int(used)} threads), {dt:.2f} s wall",
           "single_core": {"value": round(float(met1[:, -1].sum()) / dt1, 1), "cores": 1,
                           "sample": f"first {m1} episodes x 3000 steps, 1 thread, {dt1:.2f} s wall"},
           "threads_source": why, "affinity_cpus": affinity, "nproc": os.cpu_count(), "cpu_model": _cpu_model()}
    return cpu, diff


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
