"""The BASELINE.json workloads as shard builders.

Every per-episode input is a function of the GLOBAL episode index i, so a
rank that owns episodes [lo, hi) builds exactly its slice and results do not
depend on the world size:

  1  1 episode, stationary target, Riccati-LQR defaults, seed 0
  2  65,536 episodes, linear target, Riccati-LQR defaults (one shared K), seed i
  3  65,536 episodes, sinusoidal target, LQI q_int [1e-3, 1e-3, 1e-2],
     integral_limit 10, integral_zero_threshold 0.01 (shared 4x9 K), seed i
  4  262,144 episodes, circular target, Riccati-LQR with per-episode
     q_pos / q_vel / r_controls = the i-th candidate of the reference tuner's
     random stream default_rng(42) over the controller_autotune.py:375-383
     ranges (tuning.py:683-735), seed i  -> one DARE per episode
  5  1,048,576 episodes, motion type i mod 5 over (stationary, linear,
     circular, sinusoidal, figure8), per-episode mass
     default_rng(10**9 + i).uniform(0.8, 1.2) used by plant and controller
     (hover thrust, B[5,0] = 1/m; inertia is never read by the dynamics,
     SURVEY F4), seed i  -> one DARE per episode

A shard is (controller, env_config, seeds, motion, plant_mass); hand it to
`rollout.run_closed_loop` or `rollout.build_batch`.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import core
from .controllers.riccati_lqr import BatchedRiccatiLQR
from .env.config import EnvConfig
from .tuning import default_search_space, random_configs

EPISODES = {1: 1, 2: 65536, 3: 65536, 4: 262144, 5: 1048576}
MOTION = {1: "stationary", 2: "linear", 3: "sinusoidal", 4: "circular", 5: None}
LQI_CONFIG = {"use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2], "integral_limit": 10.0, "integral_zero_threshold": 0.01}
TUNER_SEED = 42
MASS_SEED_BASE = 10**9
MASS_RANGE = (0.8, 1.2)
TUNER_DRAWS_PER_CANDIDATE = 10  # q_pos 3 + q_vel 3 + r_controls 4


@dataclass
class Shard:
    config: int
    lo: int
    hi: int
    controller: BatchedRiccatiLQR
    env_config: EnvConfig
    seeds: np.ndarray
    motion: np.ndarray | None = None
    plant_mass: torch.Tensor | None = None

    @property
    def n(self) -> int:
        return self.hi - self.lo

    def run_kwargs(self) -> dict:
        return dict(env_config=self.env_config, n=self.n, seeds=self.seeds, motion=self.motion,
                    plant_mass=self.plant_mass)


def shard_bounds(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous global ranges [r*N/W, (r+1)*N/W)."""
    return rank * total // world, (rank + 1) * total // world


def tuner_candidates(lo: int, hi: int, seed: int = TUNER_SEED) -> list[dict]:
    """Candidates lo..hi-1 of the reference tuner's random stream: the stream
    is advanced past the lo earlier candidates' draws (PCG64.advance, one
    64-bit output per uniform) so a shard needs none of them."""
    rng = np.random.default_rng(seed)
    rng.bit_generator.advance(TUNER_DRAWS_PER_CANDIDATE * lo)
    return random_configs(default_search_space("riccati_lqr"), hi - lo, rng)


def tuner_candidate_arrays(lo: int, hi: int, seed: int = TUNER_SEED) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """tuner_candidates as arrays (q_pos [n,3], q_vel [n,3], r_controls [n,4]),
    same stream, no per-candidate dicts."""
    space = default_search_space("riccati_lqr")
    lo_v = np.array(list(space.q_pos_range[0]) + list(space.q_vel_range[0]) + list(space.r_controls_range[0]))
    hi_v = np.array(list(space.q_pos_range[1]) + list(space.q_vel_range[1]) + list(space.r_controls_range[1]))
    rng = np.random.default_rng(seed)
    rng.bit_generator.advance(TUNER_DRAWS_PER_CANDIDATE * lo)
    u = rng.uniform(lo_v, hi_v, size=(hi - lo, TUNER_DRAWS_PER_CANDIDATE))
    return u[:, 0:3].copy(), u[:, 3:6].copy(), u[:, 6:10].copy()


def tuner_candidate_tensors(lo: int, hi: int, device, seed: int = TUNER_SEED):
    """tuner_candidate_arrays drawn on the device (qt_stream_uniform: each
    candidate's lane jumps the one stream to its own draws), as [n, 3], [n, 3],
    [n, 4] views of one [10, n] array; bitwise the same values."""
    space = default_search_space("riccati_lqr")
    lo_v = list(space.q_pos_range[0]) + list(space.q_vel_range[0]) + list(space.r_controls_range[0])
    hi_v = list(space.q_pos_range[1]) + list(space.q_vel_range[1]) + list(space.r_controls_range[1])
    u = core.stream_uniform(seed, lo, hi - lo, lo_v, hi_v, device)
    return u[0:3].T, u[3:6].T, u[6:10].T


def episode_masses(lo: int, hi: int, device) -> torch.Tensor:
    """default_rng(10**9 + i).uniform(0.8, 1.2) for i in [lo, hi), drawn on the
    device (qt_seed_uniform)."""
    seeds = torch.arange(MASS_SEED_BASE + lo, MASS_SEED_BASE + hi, dtype=torch.int64, device=device)
    return core.seed_uniform(seeds, [MASS_RANGE[0]], [MASS_RANGE[1]])[0].contiguous()


def motion_of(lo: int, hi: int) -> np.ndarray:
    """Motion type i mod 5 of episodes [lo, hi) (the 5-cycle tiled, no 64-bit modulo)."""
    n = max(0, hi - lo)
    return np.tile(((np.arange(5) + lo) % 5).astype(np.int8), -(-n // 5))[:n]


def build(config: int, lo: int | None = None, hi: int | None = None, device=None) -> Shard:
    if config not in EPISODES:
        raise ValueError(f"unknown workload {config}; BASELINE.json has configs 1-5")
    lo = 0 if lo is None else int(lo)
    hi = EPISODES[config] if hi is None else int(hi)
    if not 0 <= lo <= hi:
        raise ValueError("need 0 <= lo <= hi")
    seeds = np.arange(lo, hi, dtype=np.int64)
    env = EnvConfig.from_dict({"target": {"motion_type": MOTION[config] or "stationary"}})
    motion = None
    mass = None
    if config in (1, 2):
        ctl = BatchedRiccatiLQR({"dt": 0.01}, device=device)
    elif config == 3:
        ctl = BatchedRiccatiLQR(dict(LQI_CONFIG, dt=0.01), device=device)
    elif config == 4:
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        qp, qv, rc = tuner_candidate_tensors(lo, hi, dev)
        ctl = BatchedRiccatiLQR({"dt": 0.01}, device=dev, q_pos=qp, q_vel=qv, r_controls=rc)
    else:
        motion = motion_of(lo, hi)
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        mass = episode_masses(lo, hi, dev)
        ctl = BatchedRiccatiLQR({"dt": 0.01}, device=device, mass=mass)
    return Shard(config, lo, hi, ctl, env, seeds, motion, mass)


__all__ = ["EPISODES", "MOTION", "LQI_CONFIG", "Shard", "shard_bounds", "tuner_candidates", "tuner_candidate_arrays",
           "tuner_candidate_tensors",
           "episode_masses",
           "motion_of", "build"]
