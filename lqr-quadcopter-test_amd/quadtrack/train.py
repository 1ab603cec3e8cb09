"""The trainer's classical evaluation epoch on the fused device rollout.

Reference: `Trainer._evaluate_epoch` (train.py:578-652), which the trainer
runs instead of a training epoch for the classical controllers (PID, LQR,
Riccati-LQR; train.py:394-429): episodes_per_epoch episodes, reset seeds
`env_seed + epoch * 1000 + episode`, `controller.reset()` before each (a fresh
controller per episode), at most max_steps_per_episode env steps, and per
episode the sum of env.step's rewards (-post-step tracking error,
quadcopter_env.py:198-199, 504-511) and the last step's info on-target ratio
and tracking error (quadcopter_env.py:205-220); the epoch returns their
np.mean and difficulty 1.0.

Here every episode of the epoch runs in one exact-step rollout launch
(`qt_rollout_rewards`, which keeps the reward sum and the last post-step error
per episode) and the three means are numpy's, bit for bit, from the
block-pairwise summary kernel (`qt_summary_numpy`).  The env is built as the
Trainer builds it (train.py:306-312): EnvConfig defaults with the
TrainingConfig's seed, episode length, motion type and target radius.
Deep-policy training (the rest of train.py) is outside the hot path.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _abi, core
from .controllers import batched_controller
from .env.config import EnvConfig

F64 = torch.float64

CLASSICAL = ("pid", "lqr", "riccati_lqr")


@dataclass
class EpochResult:
    """`_evaluate_epoch`'s dict plus the per-episode values it averages."""

    mean_reward: float
    mean_on_target_ratio: float
    mean_tracking_error: float
    difficulty: float
    episode_reward: torch.Tensor           # [E] sum of rewards
    episode_on_target_ratio: torch.Tensor  # [E] last step's info["on_target_ratio"]
    episode_tracking_error: torch.Tensor   # [E] last step's info["tracking_error"]
    episode_steps: torch.Tensor            # [E] env steps taken

    def as_dict(self) -> dict:
        return {"mean_reward": self.mean_reward, "mean_on_target_ratio": self.mean_on_target_ratio,
                "mean_tracking_error": self.mean_tracking_error, "difficulty": self.difficulty}


def env_config_for(env_seed=42, target_motion_type="circular", episode_length=30.0, target_radius=0.5) -> EnvConfig:
    """The Trainer's env (train.py:306-312)."""
    return EnvConfig.from_dict({"seed": env_seed, "simulation": {"max_episode_time": episode_length},
                                "target": {"motion_type": target_motion_type},
                                "success_criteria": {"target_radius": target_radius}})


def _np_means(rows: torch.Tensor) -> list[float]:
    """np.mean of each of three [3, E] device rows, bit for bit: the
    qt_summary_numpy kernel sums (numpy's block-pairwise order) of a
    metrics-shaped tensor carrying the rows in its three summed slots."""
    n = rows.shape[1]
    met = torch.zeros(_abi.MET_ROWS, n, dtype=F64, device=rows.device)
    met[_abi.MET["on_target_ratio"]] = rows[0]
    met[_abi.MET["mean_tracking_error"]] = rows[1]
    met[_abi.MET["mean_control_effort"]] = rows[2]
    blocks = core.summary_numpy_blocks(met, 0).cpu().numpy()
    return [core.np_fold(blocks[i]) / n for i in range(3)]


def evaluate_epoch(config=None, epoch: int = 0, *, controller: str = "riccati_lqr",
                   controller_config: dict | None = None, episodes_per_epoch: int = 10,
                   max_steps_per_episode: int = 3000, env_seed: int = 42, target_motion_type: str = "circular",
                   episode_length: float = 30.0, target_radius: float = 0.5, device=None) -> EpochResult:
    """One classical evaluation epoch (train.py:578-652) in one launch.

    `config` may be a TrainingConfig-like object (attributes controller,
    episodes_per_epoch, max_steps_per_episode, env_seed, target_motion_type,
    episode_length, target_radius and optionally full_config, whose entry
    under the controller type holds its settings, train.py:394-429); the
    keyword arguments are used otherwise."""
    if config is not None:
        controller = config.controller
        episodes_per_epoch = config.episodes_per_epoch
        max_steps_per_episode = config.max_steps_per_episode
        env_seed, target_motion_type = config.env_seed, config.target_motion_type
        episode_length, target_radius = config.episode_length, config.target_radius
        controller_config = dict(getattr(config, "full_config", {}) or {}).get(controller, {})
    if controller not in CLASSICAL:
        raise ValueError(f"evaluation epochs run the classical controllers {CLASSICAL}, not '{controller}'")
    if episodes_per_epoch < 1 or max_steps_per_episode < 1:
        raise ValueError("episodes_per_epoch and max_steps_per_episode must be >= 1")
    dev = _abi.require_gpu(device)
    cfg = env_config_for(env_seed, target_motion_type, episode_length, target_radius)
    env = cfg.to_params()
    ctl = batched_controller(controller, dict(controller_config or {}), device=dev)
    seeds = env_seed + epoch * 1000 + np.arange(episodes_per_epoch)
    from .rollout import build_batch

    batch = build_batch(ctl, cfg, episodes_per_epoch, seeds=seeds)
    st = core.RolloutState.empty(episodes_per_epoch, dev)
    core.validate(batch, st)
    core.reset(env, batch, st)
    reward = torch.zeros(2, episodes_per_epoch, dtype=F64, device=dev)
    crit = core.criteria(target_radius=target_radius)
    core.rollout_rewards(env, ctl.ctrl, crit, batch, st, int(max_steps_per_episode), reward)
    steps = st.acc[_abi.ACC_STEPS]
    ratio = st.acc[_abi.ACC_ON_POST] / steps  # on_target_count / total_steps (quadcopter_env.py:215-219)
    mean_ratio, mean_err, mean_reward = _np_means(torch.stack([ratio, reward[1], reward[0]]))
    return EpochResult(mean_reward=mean_reward, mean_on_target_ratio=mean_ratio, mean_tracking_error=mean_err,
                       difficulty=1.0, episode_reward=reward[0].clone(), episode_on_target_ratio=ratio,
                       episode_tracking_error=reward[1].clone(), episode_steps=steps.to(torch.int64))
