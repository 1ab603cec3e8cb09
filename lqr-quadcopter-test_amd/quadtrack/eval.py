"""Evaluation drivers — drop-in `Evaluator` / `load_controller` of the
reference's `quadcopter_tracking.eval` (eval.py:59-513) plus the batched
evaluator that replaces its per-episode loop.

* `Evaluator.run_episode` / `evaluate` keep the reference semantics exactly,
  including the controller NOT being reset between episodes (eval.py:95-206;
  SURVEY F8: the LQI integral carries over), stepping the GPU-backed
  `QuadcopterEnv` and controller one step at a time.
* `evaluate_batched` runs all episodes at once in the fused closed-loop
  kernel with a fresh controller per episode (the tuner / trainer semantics,
  controllers/tuning.py:879, train.py:594) and returns the same
  `EvaluationSummary`.
"""

from __future__ import annotations

import json
import logging
from copy import deepcopy
from datetime import datetime, timezone
from pathlib import Path
from typing import Callable

import numpy as np

from ._abi import MET
from .controllers import (
    BaseController,
    LQRController,
    PIDController,
    RiccatiLQRController,
    batched_controller,
)
from .env import EnvConfig, QuadcopterEnv
from .env.config import as_env_config
from .rollout import run_closed_loop
from .utils.metrics import (
    EvaluationSummary,
    SuccessCriteria,
    compute_episode_metrics,
    compute_evaluation_summary,
    format_metrics_report,
)

logger = logging.getLogger(__name__)


class Evaluator:
    """Controller evaluation pipeline (eval.py:59-268, plots excluded)."""

    def __init__(self, controller: BaseController, env_config: EnvConfig | None = None,
                 criteria: SuccessCriteria | None = None, output_dir: str | Path = "reports"):
        self.controller = controller
        self.env_config = env_config or EnvConfig()
        self.criteria = criteria or SuccessCriteria()
        self.output_dir = Path(output_dir)
        self.output_dir.mkdir(parents=True, exist_ok=True)
        (self.output_dir / "plots").mkdir(exist_ok=True)
        self.episode_data_list: list[list[dict]] = []
        self.episode_info_list: list[dict] = []

    def run_episode(self, seed: int, max_steps: int | None = None,
                    progress_callback: Callable | None = None) -> tuple[list[dict], dict]:
        env = QuadcopterEnv(config=self.env_config)
        obs = env.reset(seed=seed)
        episode_data: list[dict] = []
        done = False
        step = 0
        info: dict = {}
        while not done:
            if max_steps is not None and step >= max_steps:
                break
            try:
                action = self.controller.compute_action(obs)
            except Exception as e:  # eval.py:124-136
                logger.error("Controller error at step %d: %s", step, e)
                info = {"termination_reason": "controller_error", "time": step * env.dt, "tracking_error": 0.0,
                        "on_target": False, "on_target_ratio": 0.0, "action_violations": 0}
                break
            next_obs, reward, done, info = env.step(action)
            episode_data.append({
                "time": info.get("time", step * env.dt), "step": step,
                "quadcopter_position": obs["quadcopter"]["position"].tolist(),
                "quadcopter_velocity": obs["quadcopter"]["velocity"].tolist(),
                "target_position": obs["target"]["position"].tolist(),
                "target_velocity": obs["target"]["velocity"].tolist(),
                "action": [action["thrust"], action["roll_rate"], action["pitch_rate"], action["yaw_rate"]],
                "reward": reward, "tracking_error": info.get("tracking_error", 0.0),
                "on_target": info.get("on_target", False),
            })
            obs = next_obs
            step += 1
            if progress_callback and step % 100 == 0:
                progress_callback(step, info)
        return episode_data, info

    def evaluate(self, num_episodes: int = 10, base_seed: int = 42, max_steps_per_episode: int | None = None,
                 verbose: bool = True) -> EvaluationSummary:
        self.episode_data_list, self.episode_info_list = [], []
        metrics = []
        for i in range(num_episodes):
            data, info = self.run_episode(seed=base_seed + i, max_steps=max_steps_per_episode)
            self.episode_data_list.append(data)
            self.episode_info_list.append(info)
            m = compute_episode_metrics(data, self.criteria, info)
            metrics.append(m)
            if verbose:
                logger.info("  %s | on-target: %.1f%% | error: %.3fm | duration: %.1fs",
                            "SUCCESS" if m.success else "FAILED", m.on_target_ratio * 100, m.mean_tracking_error,
                            m.episode_duration)
        summary = compute_evaluation_summary(metrics, self.criteria)
        if verbose:
            print("\n" + format_metrics_report(summary))
        return summary

    def save_report(self, summary: EvaluationSummary, experiment_name: str | None = None) -> dict[str, Path]:
        """metrics.json + text report (eval.py:233-268)."""
        if experiment_name is None:
            stamp = datetime.now(timezone.utc).strftime("%Y%m%d_%H%M%S")
            experiment_name = f"eval_{self.controller.name}_{stamp}"
        paths = {"metrics": self.output_dir / "metrics.json", "report": self.output_dir / f"{experiment_name}_report.txt"}
        paths["metrics"].write_text(json.dumps(summary.to_dict(), indent=2))
        paths["report"].write_text(format_metrics_report(summary))
        return paths


def load_controller(controller_type: str, checkpoint_path=None, config: dict | None = None) -> BaseController:
    """Controller factory (eval.py:472-513) for the controllers on this path."""
    config = config or {}
    if controller_type == "lqr":
        return LQRController(config=config)
    if controller_type == "pid":
        return PIDController(config=config)
    if controller_type == "riccati_lqr":
        return RiccatiLQRController(config=config)
    if controller_type == "lqi":
        cfg = deepcopy(config)
        cfg["use_lqi"] = True
        cfg.setdefault("q_int", [0.01, 0.01, 0.1])
        return RiccatiLQRController(config=cfg)
    if controller_type == "deep":
        raise NotImplementedError(f"controller type '{controller_type}' is outside the MI355X hot path")
    raise ValueError(f"Unknown controller type: {controller_type}")


def evaluate_batched(controller, env_config=None, num_episodes: int = 10, base_seed: int = 42,
                     criteria: SuccessCriteria | None = None, motion=None, plant_mass=None,
                     max_steps_per_episode: int | None = None, with_episode_metrics: bool = True,
                     group=None, global_offset: int = 0) -> EvaluationSummary:
    """All episodes in one fused closed-loop launch (fresh controller each).

    `controller` is a drop-in controller (RiccatiLQRController, LQRController,
    PIDController: shared gains), a batched one (BatchedRiccatiLQR,
    BatchedLQR, BatchedPID: shared or per-episode gains) or a config dict
    (its "controller" key picks the type, default riccati_lqr)."""
    cfg = as_env_config(env_config)
    controller = _as_batched(controller)
    seeds = base_seed + global_offset + np.arange(num_episodes)
    res = run_closed_loop(controller, cfg, n=num_episodes, seeds=seeds, motion=motion, plant_mass=plant_mass,
                          criteria=criteria, max_steps=max_steps_per_episode)
    summary = res.summary(group=group, global_offset=global_offset)
    if with_episode_metrics:
        summary.episode_metrics = res.episode_metrics()
    return summary


def _as_batched(controller):
    if isinstance(controller, dict):
        c = dict(controller)
        return batched_controller(c.pop("controller", "riccati_lqr"), c)
    if isinstance(controller, (RiccatiLQRController, LQRController, PIDController)):
        return controller.to_batched()
    return controller


class BatchedEvaluator:
    """The Evaluator pipeline (eval.py:59-268) with every episode in one fused
    launch and a fresh controller per episode (the tuner / trainer semantics,
    SURVEY F8).  `evaluate` fills `episode_data_list` / `episode_info_list` in
    the reference's formats (eval.py:142-158, the env's final info dict,
    quadcopter_env.py:209-226) for the episodes in `record_episodes` (default:
    all of them up to 64), recorded by a re-run of just those episodes."""

    def __init__(self, controller, env_config=None, criteria: SuccessCriteria | None = None,
                 output_dir: str | Path = "reports"):
        self.controller = controller
        self.env_config = as_env_config(env_config)
        self.criteria = criteria or SuccessCriteria()
        self.output_dir = Path(output_dir)
        self.output_dir.mkdir(parents=True, exist_ok=True)
        self.episode_data_list: list[list[dict]] = []
        self.episode_info_list: list[dict] = []
        self.result = None

    def evaluate(self, num_episodes: int = 10, base_seed: int = 42, max_steps_per_episode: int | None = None,
                 verbose: bool = True, record_episodes=None, group=None, global_offset: int = 0) -> EvaluationSummary:
        seeds = base_seed + global_offset + np.arange(num_episodes)
        res = run_closed_loop(_as_batched(self.controller), self.env_config, n=num_episodes, seeds=seeds,
                              criteria=self.criteria, max_steps=max_steps_per_episode)
        self.result = res
        if record_episodes is None:
            record_episodes = range(num_episodes) if num_episodes <= 64 else []
        rec = [int(i) for i in record_episodes]
        self.episode_data_list = res.episode_data(rec) if rec else []
        self.episode_info_list = self._final_info(res, rec, self.episode_data_list) if rec else []
        summary = res.summary(group=group, global_offset=global_offset)
        summary.episode_metrics = res.episode_metrics()
        if verbose:
            print("\n" + format_metrics_report(summary))
        return summary

    def _final_info(self, res, episodes, data) -> list[dict]:
        """The info dict env.step returned on each episode's last step."""
        from ._abi import TERM_REASONS

        met = res.metrics.cpu().numpy()
        env = res.env
        out = []
        for j, e in enumerate(episodes):
            steps = int(met[MET["steps"], e])
            if steps == 0:
                out.append({})
                continue
            last = data[j][-1]
            ratio = float(met[MET["env_on_target_ratio"], e])
            info = {"time": last["time"], "step": steps, "tracking_error": last["tracking_error"],
                    "on_target": last["on_target"], "on_target_ratio": ratio,
                    "action_violations": int(met[MET["action_violations"], e])}
            term = int(met[MET["termination_code"], e])
            if term:
                info["termination_reason"] = TERM_REASONS[term]
                info["episode_length"] = last["time"]
                info["success"] = bool(last["time"] >= env.min_episode_duration and ratio >= env.min_on_target_ratio)
            out.append(info)
        return out

    def save_report(self, summary: EvaluationSummary, experiment_name: str | None = None) -> dict[str, Path]:
        """metrics.json + text report (eval.py:233-268)."""
        if experiment_name is None:
            stamp = datetime.now(timezone.utc).strftime("%Y%m%d_%H%M%S")
            experiment_name = f"eval_{getattr(self.controller, 'name', 'batched')}_{stamp}"
        paths = {"metrics": self.output_dir / "metrics.json", "report": self.output_dir / f"{experiment_name}_report.txt"}
        paths["metrics"].write_text(json.dumps(summary.to_dict(), indent=2))
        paths["report"].write_text(format_metrics_report(summary))
        return paths


def _stateless(controller) -> bool:
    """True when compute_action keeps no state from one episode to the next,
    so a fresh controller per episode (batched) gives the sequential
    Evaluator's episodes: LQR, and Riccati-LQR without its LQI integral (or on
    its heuristic fallback, riccati_lqr.py:764-776, which ignores LQI)."""
    if isinstance(controller, LQRController):
        return True
    if isinstance(controller, RiccatiLQRController):
        return not controller.use_lqi or controller.fallback_controller is not None
    return False


def run_hyperparameter_sweep(sweep_config_path: str | Path, output_dir: str | Path = "reports/sweeps",
                             batched: bool | str = "auto") -> list[dict]:
    """Evaluation sweep over controller configurations (eval.py:516-628):
    each entry of the YAML's `configurations` builds a controller
    (`controller_type`, `controller_config`), an EnvConfig (`env_config`) and
    SuccessCriteria (`criteria`), is evaluated over `num_episodes` seeded
    episodes (`seed`), and the valid results are ranked by mean on-target
    ratio and written to `output_dir/sweep_results.json`; a configuration that
    raises is logged and left out of the ranking, as the reference does.

    batched: "auto" (default) runs a configuration whose controller carries
    no state between episodes (`_stateless`) as one fused launch
    (evaluate_batched) and the others through the sequential Evaluator, whose
    controller is never reset; True runs every configuration
    batched (a fresh controller per episode); False runs all sequentially."""
    import yaml

    with open(sweep_config_path) as f:
        entries = (yaml.safe_load(f) or {}).get("configurations", [])
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    logger.info("Running sweep with %d configurations", len(entries))
    outcomes = []
    for i, entry in enumerate(entries):
        logger.info("Configuration %d/%d: %s", i + 1, len(entries), entry.get("name"))
        outcomes.append(_sweep_entry(entry, entry.get("name", f"config_{i}"), out, batched))
    ranked = sorted((r for r in outcomes if "error" not in r), key=lambda r: r["mean_on_target_ratio"], reverse=True)
    path = out / "sweep_results.json"
    path.write_text(json.dumps(ranked, indent=2))
    logger.info("Saved sweep results: %s", path)
    bar = "=" * 60
    lines = [f"{k}. {r['name']}: on-target={r['mean_on_target_ratio']:.1%}, success={r['success_rate']:.1%}"
             for k, r in enumerate(ranked, 1)]
    print("\n".join(["", bar, "HYPERPARAMETER SWEEP RESULTS (Ranked)", bar, *lines, bar]))
    return ranked


def _sweep_criteria(entry: dict) -> SuccessCriteria:
    """A sweep entry's `criteria` block over the SuccessCriteria defaults."""
    crit = entry.get("criteria")
    if crit is None:
        return SuccessCriteria()
    return SuccessCriteria(min_on_target_ratio=crit.get("min_on_target_ratio", 0.8),
                           min_episode_duration=crit.get("min_episode_duration", 30.0),
                           target_radius=crit.get("target_radius", 0.5))


def _sweep_entry(entry: dict, name: str, out: Path, batched) -> dict:
    """One sweep configuration: its result row, or an `error` row when building
    or evaluating it raises (eval.py:592-601 logs and keeps going)."""
    try:
        controller = load_controller(controller_type=entry.get("controller_type", "deep"),
                                     checkpoint_path=entry.get("checkpoint_path"),
                                     config=entry.get("controller_config"))
        env_config = EnvConfig.from_dict(entry["env_config"]) if "env_config" in entry else EnvConfig()
        criteria = _sweep_criteria(entry)
        episodes, seed = entry.get("num_episodes", 5), entry.get("seed", 42)
        if batched is True or (batched == "auto" and _stateless(controller)):
            (out / name / "plots").mkdir(parents=True, exist_ok=True)  # the directories Evaluator() makes
            summary = evaluate_batched(controller, env_config, num_episodes=episodes, base_seed=seed,
                                       criteria=criteria, with_episode_metrics=False)
        else:
            summary = Evaluator(controller=controller, env_config=env_config, criteria=criteria,
                                output_dir=out / name).evaluate(num_episodes=episodes, base_seed=seed, verbose=False)
    except Exception as e:
        logger.error("Configuration %s failed: %s", entry.get("name"), e)
        return {"name": name, "config": entry, "error": str(e)}
    logger.info("  Result: on-target=%.1f%%, success=%.1f%%", summary.mean_on_target_ratio * 100,
                summary.success_rate * 100)
    return {"name": name, "config": entry, "mean_on_target_ratio": summary.mean_on_target_ratio,
            "success_rate": summary.success_rate, "mean_tracking_error": summary.mean_tracking_error,
            "meets_criteria": summary.meets_criteria}
