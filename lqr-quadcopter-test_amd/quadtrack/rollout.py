"""The fused batched closed loop: N independent episodes of
`RiccatiLQRController.compute_action` -> `QuadcopterEnv.step` in one kernel.

This is what the reference's per-episode Python loops do one step at a time
(eval.py:95-167 `Evaluator.run_episode`, controllers/tuning.py:874-906
`ControllerTuner._evaluate_config`, train.py:588-638 classical epochs): here
every episode is one GPU lane, the whole 30 s episode runs register-resident
inside `qt_rollout`, and the Evaluator's per-episode metrics are accumulated
in the same pass (no per-step data leaves the chip).

Semantics: each episode uses a fresh controller (integral zeroed at reset),
as the tuner and trainer do (tuning.py:879, train.py:594); see SURVEY F8 for
the Evaluator's carry-over, which `quadtrack.eval.Evaluator` reproduces.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from . import _abi, core
from ._abi import MET, MET_FIELDS, TERM_REASONS
from .controllers.riccati_lqr import BatchedRiccatiLQR  # or BatchedLQR / BatchedPID: same batch interface
from .env import seeding
from .env.batched import motion_indices
from .env.config import as_env_config

F64 = torch.float64


def max_steps_for(env_params) -> int:
    """Upper bound on steps before `t >= max_episode_time` (t accumulates dt)."""
    return int(math.ceil(env_params.max_episode_time / env_params.dt)) + 2


@dataclass
class RolloutResult:
    metrics: torch.Tensor            # [MET_ROWS, n] float64 (EpisodeMetrics fields, include/quadtrack.h)
    state: core.RolloutState
    batch: core.EpisodeBatch
    criteria: object
    record: torch.Tensor | None = None  # [steps, 16, n]: state after step + controller command
    env: object = None                  # EnvParams of the run (trajectory re-runs)
    ctrl: object = None                 # CtrlParams of the run

    @property
    def n(self) -> int:
        return self.metrics.shape[1]

    def metric(self, name: str) -> torch.Tensor:
        return self.metrics[MET[name]]

    def final_state(self) -> torch.Tensor:
        return self.state.x.T.clone()

    def episode_metrics(self):
        """List of utils.metrics.EpisodeMetrics (host copies)."""
        from .utils.metrics import EpisodeMetrics

        m = self.metrics.cpu().numpy()
        out = []
        for e in range(m.shape[1]):
            row = dict(zip(MET_FIELDS, m[:, e]))
            out.append(EpisodeMetrics(
                episode_duration=float(row["episode_duration"]), on_target_ratio=float(row["on_target_ratio"]),
                mean_tracking_error=float(row["mean_tracking_error"]),
                max_tracking_error=float(row["max_tracking_error"]),
                rms_tracking_error=float(row["rms_tracking_error"]),
                total_control_effort=float(row["total_control_effort"]),
                mean_control_effort=float(row["mean_control_effort"]),
                overshoot_count=int(row["overshoot_count"]), max_overshoot=float(row["max_overshoot"]),
                success=bool(row["success"]), termination_reason=TERM_REASONS[int(row["termination_code"])],
                action_violations=int(row["action_violations"])))
        return out

    def summary(self, group=None, global_offset: int = 0):
        """EvaluationSummary over all episodes (utils/metrics.py:341-390); with
        torch.distributed initialised, reduced over every rank's shard."""
        from .parallel import reduce_summary

        return reduce_summary(self.metrics, self.criteria, group=group, global_offset=global_offset)

    # ------------------------------------------------------------ trajectories
    def trajectories(self, episodes=None) -> dict:
        """Per-step arrays of the selected episodes (default: all), for plots and
        reports in the reference's step-record layouts (eval.py:142-158,
        quadcopter_env.py:555-584).

        The fused rollout keeps no per-step data, so the selected episodes are
        re-run from their own inputs with recording on (the exact step: the same
        decisions as the fast step, values equal to ~1e-9).  m = len(episodes),
        S = the longest executed episode among them:

          time            [S]        post-step time (info["time"]; t accumulates dt)
          obs_state       [S, 12, m] state the action was computed on (pre-step)
          obs_target      [S, 9, m]  target observation (p, v, a) at that time
          next_state      [S, 12, m] state after the step
          next_target     [S, 9, m]  target observation after the step
          action          [S, 4, m]  controller command (thrust, roll, pitch, yaw rate)
          applied         [S, 4, m]  command after the env's action parsing (quadcopter_env.py:234-293)
          tracking_error  [S, m]     post-step ‖p − p_T‖ (quadcopter_env.py:498-502); reward = −error
          on_target       [S, m]     bool, error <= the env's target radius
          steps           [m]        executed steps; rows at or beyond them are NaN / False
        """
        if self.env is None or self.ctrl is None:
            raise ValueError("trajectories need the run's env and controller parameters (run_closed_loop)")
        dev = self.batch.device
        if episodes is None:
            idx = torch.arange(self.n, device=dev)
        else:
            idx = torch.as_tensor(np.asarray(episodes, dtype=np.int64).reshape(-1), device=dev)
        if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= self.n):
            raise IndexError(f"episode index out of range for {self.n} episodes")
        env, m = self.env, idx.numel()
        steps = self.metrics[MET["steps"]].index_select(0, idx).to(torch.int64)
        S = int(steps.max().item()) if m else 0
        nan = float("nan")
        rec = torch.full((S, 16, m), nan, dtype=F64, device=dev)
        st = core.RolloutState.empty(m, dev)
        sub = self.batch.select(idx)
        if m:
            core.reset(env, sub, st)
        x0 = st.x.clone()
        if S and m:
            core.rollout(env, self.ctrl, self.criteria, sub, st, S, rec)
        times = np.concatenate([[0.0], np.cumsum(np.full(S, env.dt))])  # t_0 .. t_S, sequential t += dt
        tg = _targets_at(env, sub, torch.as_tensor(times, dtype=F64, device=dev))  # [S + 1, 9, m]
        valid = torch.arange(S, device=dev)[:, None] < steps[None, :]
        obs_state = torch.cat([x0[None], rec[:-1, :12]]) if S else rec[:, :12]
        nxt = rec[:, :12]
        d = nxt[:, 0:3] - tg[1:, 0:3]
        err = torch.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2])
        act = rec[:, 12:16]
        applied = torch.nan_to_num(act, nan=0.0, posinf=0.0, neginf=0.0)
        applied[:, 0].clamp_(env.min_thrust, env.max_thrust)
        applied[:, 1:].clamp_(-env.max_angular_rate, env.max_angular_rate)
        v3 = valid[:, None, :]
        mask = lambda a, v: torch.where(v, a, torch.full_like(a, nan))  # noqa: E731
        return {
            "time": torch.as_tensor(times[1:], dtype=F64, device=dev),
            "obs_state": mask(obs_state, v3), "obs_target": mask(tg[:-1], v3),
            "next_state": mask(nxt, v3), "next_target": mask(tg[1:], v3),
            "action": mask(act, v3), "applied": mask(applied, v3),
            "tracking_error": mask(err, valid), "on_target": (err <= env.target_radius) & valid,
            "steps": steps,
        }

    def episode_data(self, episodes=None) -> list[list[dict]]:
        """The Evaluator's step records of each selected episode (eval.py:142-158):
        pre-step observation, controller command, post-step time / reward /
        tracking error / on-target flag."""
        tr = {k: v.cpu().numpy() for k, v in self.trajectories(episodes).items()}
        out = []
        for j in range(tr["steps"].size):
            rows = []
            for k in range(int(tr["steps"][j])):
                qs, ts = tr["obs_state"][k, :, j], tr["obs_target"][k, :, j]
                rows.append({
                    "time": float(tr["time"][k]), "step": k,
                    "quadcopter_position": qs[0:3].tolist(), "quadcopter_velocity": qs[3:6].tolist(),
                    "target_position": ts[0:3].tolist(), "target_velocity": ts[3:6].tolist(),
                    "action": tr["action"][k, :, j].tolist(),
                    "reward": -float(tr["tracking_error"][k, j]),
                    "tracking_error": float(tr["tracking_error"][k, j]),
                    "on_target": bool(tr["on_target"][k, j]),
                })
            out.append(rows)
        return out

    def history(self, episodes=None, log_interval: int = 10) -> list[list[dict]]:
        """QuadcopterEnv.get_history() of each selected episode
        (quadcopter_env.py:555-584): the steps whose post-step count is a multiple
        of log_interval, with the post-step observation and the applied action."""
        if log_interval < 1:
            raise ValueError("log_interval must be >= 1")
        tr = {k: v.cpu().numpy() for k, v in self.trajectories(episodes).items()}
        out = []
        for j in range(tr["steps"].size):
            rows = []
            for k in range(log_interval - 1, int(tr["steps"][j]), log_interval):
                qs, ts = tr["next_state"][k, :, j], tr["next_target"][k, :, j]
                rows.append({
                    "time": float(tr["time"][k]), "step": k + 1,
                    "quadcopter_position": qs[0:3].tolist(), "quadcopter_velocity": qs[3:6].tolist(),
                    "quadcopter_attitude": qs[6:9].tolist(),
                    "target_position": ts[0:3].tolist(), "target_velocity": ts[3:6].tolist(),
                    "action": tr["applied"][k, :, j].tolist(),
                    "reward": -float(tr["tracking_error"][k, j]),
                    "tracking_error": float(tr["tracking_error"][k, j]),
                    "on_target": bool(tr["on_target"][k, j]),
                })
            out.append(rows)
        return out


def _targets_at(env, batch: core.EpisodeBatch, times: torch.Tensor) -> torch.Tensor:
    """Target observation of every episode of `batch` at every time -> [T, 9, m]
    (qt_target_state on a time-major replicated batch, ~4 M evaluations per launch)."""
    T, m, dev = times.numel(), batch.n, batch.device
    out = torch.empty(T, 9, m, dtype=F64, device=dev)
    if T == 0 or m == 0:
        return out
    rows = max(1, (1 << 22) // m)
    for lo in range(0, T, rows):
        k = min(rows, T - lo)
        rep = core.EpisodeBatch(n=k * m, device=dev, pattern=batch.pattern.repeat(1, k),
                                offset=batch.offset.repeat(1, k), K=batch.K[:, :1], k_cols=batch.k_cols,
                                motion=None if batch.motion is None else batch.motion.repeat(k))
        tg = core.target_state(env, rep, times[lo:lo + k].repeat_interleave(m).contiguous())
        out[lo:lo + k] = tg.view(9, k, m).permute(1, 0, 2)
    return out


def build_batch(controller: BatchedRiccatiLQR, env_config, n: int, seeds=None, motion=None, plant_mass=None,
                draws=None, device=None, order=None, group_motion: bool = True) -> core.EpisodeBatch:
    """Device inputs for `n` episodes.  Mixed motion types are grouped (one
    motion-specialised launch per group, `qt_rollout_grouped`) unless an
    explicit `order` is given or group_motion is False."""
    cfg = as_env_config(env_config)
    dev = _abi.require_gpu(device if device is not None else controller.device)
    if controller.per_episode and controller.num_problems != n:
        raise ValueError(f"controller has {controller.num_problems} gain sets for {n} episodes")
    if draws is None:
        if seeds is None:
            seeds = np.arange(n)
        seeds = np.asarray(seeds, dtype=np.int64).reshape(-1)
        if seeds.size != n:
            raise ValueError(f"{seeds.size} seeds for {n} episodes")
        kinds = motion_indices(motion, n) if motion is not None else cfg.motion_index()
        draws = seeding.draws(kinds, seeds, dev)
    pat, off = draws
    kinds = None if motion is None else motion_indices(motion, n)
    mo = None if kinds is None else torch.as_tensor(kinds, device=dev)
    groups = None
    if kinds is not None and order is None and group_motion and kinds.size and np.any(kinds != kinds.flat[0]):
        # on the device: the order stays there; a batch of one resident set pairs its rounds
        order, seg_motion, seg_end = core.motion_groups(mo, core.resident_grouped_waves(dev))
        groups = (seg_motion, seg_end)
    if plant_mass is None:
        pm = None
    elif isinstance(plant_mass, torch.Tensor) and plant_mass.numel() == n:
        pm = core.to_device(plant_mass.reshape(-1), dev)
    else:
        pm = core.to_device(np.broadcast_to(np.asarray(plant_mass, float), (n,)), dev)
    if order is None:
        od = None
    elif isinstance(order, torch.Tensor):
        od = order.to(device=dev, dtype=torch.int32)
    else:
        od = torch.as_tensor(np.asarray(order, dtype=np.int32), device=dev)
    b = core.EpisodeBatch(n=n, device=dev, pattern=core.to_device(pat, dev), offset=core.to_device(off, dev),
                          K=controller.K, k_cols=controller.k_cols, motion=mo, plant_mass=pm, hover=controller.hover,
                          order=od, k_structured=controller.k_structured,
                          k_no_yaw=core.gains_no_yaw(controller.K, controller.k_cols), groups=groups,
                          ff=getattr(controller, "ff", None))
    return b


def run_closed_loop(controller: BatchedRiccatiLQR, env_config=None, n: int | None = None, seeds=None, motion=None,
                    plant_mass=None, criteria=None, draws=None, max_steps: int | None = None, chunk: int | None = None,
                    record: bool = False, batch: core.EpisodeBatch | None = None) -> RolloutResult:
    """Run `n` closed-loop episodes to termination (or `max_steps`).

    seeds     per-episode reset seeds (default 0..n-1); draws=(pattern, offset) overrides them
    motion    per-episode motion types (default: the config's)
    plant_mass per-episode plant mass (controller masses are the controller's)
    criteria  the Evaluator's SuccessCriteria (default utils.metrics defaults)
    chunk     steps per kernel launch (default: the whole episode in one launch)
    record    keep every step's state and action ([steps, 16, n]; for parity tests)
    """
    cfg = as_env_config(env_config)
    env = cfg.to_params()
    if n is None:
        n = controller.num_problems if controller.per_episode else (len(seeds) if seeds is not None else 1)
    if batch is None:
        batch = build_batch(controller, cfg, n, seeds=seeds, motion=motion, plant_mass=plant_mass, draws=draws)
    crit = _criteria(criteria)
    # a motion-grouped batch runs on its slot-ordered copy (coalesced rows);
    # state, metrics and records come back in episode order below
    run, perm = batch.physical_groups() if batch.groups is not None and batch.order is not None else (batch, None)
    st = core.RolloutState.empty(n, batch.device)
    core.validate(run, st)
    total = max_steps if max_steps is not None else max_steps_for(env)
    step = chunk or total
    rec = torch.full((total, 16, n), float("nan"), dtype=F64, device=batch.device) if record else None
    if rec is None and step >= total:
        # one launch set: reset in the rollout's prologue, metrics in its epilogue
        met = core.rollout_fresh(env, controller.ctrl, crit, run, st, total)
    else:
        core.reset(env, run, st)
        done = 0
        while done < total:
            k = min(step, total - done)
            core.rollout(env, controller.ctrl, crit, run, st, k, None if rec is None else rec[done:done + k])
            done += k
        met = core.episode_metrics(crit, st)
    if perm is not None:
        met = core.unpermute(met, perm)
        st = core.RolloutState(x=core.unpermute(st.x, perm), integ=core.unpermute(st.integ, perm),
                               t=core.unpermute(st.t, perm), acc=core.unpermute(st.acc, perm),
                               target=core.unpermute(st.target, perm))
        if rec is not None:
            rec = core.unpermute(rec, perm)
    return RolloutResult(metrics=met, state=st, batch=batch, criteria=crit, record=rec, env=env,
                         ctrl=controller.ctrl)


def _criteria(criteria):
    if criteria is None:
        return core.criteria()
    if isinstance(criteria, _abi.Criteria):
        return criteria
    return core.criteria(criteria.min_on_target_ratio, criteria.min_episode_duration, criteria.target_radius)
