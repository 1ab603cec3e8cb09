"""Batched quadcopter environment on the GPU.

`BatchedQuadcopterEnv(n, config)` holds n independent episodes in HBM
(structure-of-arrays float64) and exposes the reference's reset/step API
(env/quadcopter_env.py:111-232) on tensors: `reset(seeds)` runs the reset
kernel on the per-seed draws, `step(actions)` runs the open-loop step kernel
(action validation, RK4/Euler, state constraints, post-step tracking error,
termination) for every episode at once.  Returned tensors are fresh copies
owned by the caller, like the reference's observation arrays
(quadcopter_env.py:481-486).
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _abi, core
from .._abi import ACC_ON_POST, ACC_STEPS, ACC_VIOLATIONS, MOTIONS
from . import seeding
from .config import as_env_config

F64 = torch.float64


def motion_indices(motion, n: int) -> np.ndarray:
    """Per-episode motion names / indices -> int8 array of enum qt_motion."""
    if isinstance(motion, (np.ndarray, torch.Tensor)) and not (isinstance(motion, np.ndarray)
                                                                and motion.dtype.kind in "UOS"):
        a = np.asarray(motion.cpu() if isinstance(motion, torch.Tensor) else motion).reshape(-1)
        if a.size != n:
            raise ValueError(f"{a.size} motion types for {n} episodes")
        if a.size and (a.min() < 0 or a.max() >= len(MOTIONS)):
            raise ValueError(f"Invalid motion type index in {sorted(set(a.tolist()))[:8]}")
        return a.astype(np.int8)
    out = np.empty(n, dtype=np.int8)
    vals = list(motion)
    if len(vals) != n:
        raise ValueError(f"{len(vals)} motion types for {n} episodes")
    for i, m in enumerate(vals):
        if isinstance(m, str):
            if m.lower() not in MOTIONS:
                raise ValueError(f"Invalid motion type: {m}. Valid types: {set(MOTIONS)}")
            out[i] = MOTIONS.index(m.lower())
        else:
            if not 0 <= int(m) < len(MOTIONS):
                raise ValueError(f"Invalid motion type index: {m}")
            out[i] = int(m)
    return out


class BatchedQuadcopterEnv:
    STATE_DIM = 12
    ACTION_DIM = 4

    def __init__(self, num_envs: int, config=None, device=None, motion=None, mass=None):
        if num_envs < 1:
            raise ValueError("num_envs must be >= 1")
        self.config = as_env_config(config)
        self.params = self.config.to_params()
        self.num_envs = int(num_envs)
        self.device = _abi.require_gpu(device)
        n, dev = self.num_envs, self.device
        self.motion = None
        if motion is not None:
            self.motion = torch.as_tensor(motion_indices(motion, n), device=dev)
        self.plant_mass = None if mass is None else core.to_device(np.broadcast_to(np.asarray(mass, float), (n,)), dev)
        self.state = core.RolloutState.empty(n, dev)
        self.batch: core.EpisodeBatch | None = None
        self._dummy_K = torch.zeros(24, 1, dtype=F64, device=dev)

    # ---------------------------------------------------------------- reset
    def reset_from_draws(self, pattern, offset):
        """Reset every episode from explicit draws: pattern [4, n], offset [3, n]."""
        n, dev = self.num_envs, self.device
        self.batch = core.EpisodeBatch(n=n, device=dev, pattern=core.to_device(pattern, dev),
                                       offset=core.to_device(offset, dev), K=self._dummy_K, k_cols=6,
                                       motion=self.motion, plant_mass=self.plant_mass)
        core.validate(self.batch, self.state)
        core.reset(self.params, self.batch, self.state)
        return self.observation()

    def reset(self, seeds=None):
        """QuadcopterEnv.reset(seed) for every episode: seeds [n] (default
        config.seed + arange(n))."""
        if seeds is None:
            seeds = self.config.seed + np.arange(self.num_envs)
        seeds = np.asarray(seeds.cpu() if isinstance(seeds, torch.Tensor) else seeds, dtype=np.int64).reshape(-1)
        if seeds.size != self.num_envs:
            raise ValueError(f"{seeds.size} seeds for {self.num_envs} episodes")
        kinds = self.motion if self.motion is not None else self.config.motion_index()
        pat, off = seeding.draws(kinds, seeds, self.device)
        return self.reset_from_draws(pat, off)

    # ----------------------------------------------------------------- step
    def step(self, actions):
        """actions [n, 4] (thrust, roll, pitch, yaw rates) -> (obs, reward [n],
        done [n] bool, info dict of tensors)."""
        if self.batch is None:
            raise RuntimeError("Environment not initialized. Call reset() first.")
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions, dtype=np.float64))
        if a.dim() != 2 or a.shape != (self.num_envs, 4):
            raise ValueError(f"Action array must have shape ({self.num_envs}, 4), got {tuple(a.shape)}")
        a = a.to(device=self.device, dtype=F64).T.contiguous()
        err, on, done, term, viol = core.env_step(self.params, self.batch, a, self.state)
        acc = self.state.acc
        steps = acc[ACC_STEPS]
        info = {
            "time": self.state.t.clone(),
            "step": steps.to(torch.int64),
            "tracking_error": err,
            "on_target": on,
            "on_target_ratio": torch.where(steps > 0, acc[ACC_ON_POST] / steps.clamp(min=1), torch.zeros_like(steps)),
            "action_violations": acc[ACC_VIOLATIONS].to(torch.int64),
            "termination_code": term,
            "violation": viol,
        }
        return self.observation(), -err, done, info

    # ---------------------------------------------------------- observation
    def observation(self) -> dict:
        x, tg = self.state.x, self.state.target
        return {
            "quadcopter": {"position": x[0:3].T.clone(), "velocity": x[3:6].T.clone(),
                           "attitude": x[6:9].T.clone(), "angular_velocity": x[9:12].T.clone()},
            "target": {"position": tg[0:3].T.clone(), "velocity": tg[3:6].T.clone(),
                       "acceleration": tg[6:9].T.clone()},
            "time": self.state.t.clone(),
        }

    def get_state_vector(self) -> torch.Tensor:
        return self.state.x.T.clone()

    def set_state_vector(self, x) -> None:
        x = torch.as_tensor(x, dtype=F64, device=self.device)
        if x.shape != (self.num_envs, self.STATE_DIM):
            raise ValueError(f"State must have shape ({self.num_envs}, {self.STATE_DIM}), got {tuple(x.shape)}")
        self.state.x.copy_(x.T)

    @property
    def time(self) -> torch.Tensor:
        return self.state.t.clone()

    @property
    def dt(self) -> float:
        return self.config.simulation.dt
