"""Per-episode random draws of `QuadcopterEnv.reset(seed)`, on the GPU.

The reference re-creates two `numpy.random.default_rng(seed)` streams on every
seeded reset (env/quadcopter_env.py:122-127): the target stream draws the
pattern parameters (target_motion.py:318-366: linear `standard_normal(3)`,
circular `uniform(0, 2*pi)`, sinusoidal `uniform(0, 2*pi, 3)`, figure8 and
stationary nothing) and the env stream draws the start offset
`uniform(-0.5, 0.5, 3)` (quadcopter_env.py:137).  `qt_seed_draws`
(csrc/qt_seed.hip, csrc/qt_rng.hpp) reproduces numpy's SeedSequence + PCG64 +
ziggurat on the device, one lane per episode, so a batched reset needs no
host random numbers.  (The single-episode drop-in `QuadcopterEnv` keeps the
reference's own numpy generators because an unseeded reset continues their
streams, quadcopter_env.py:122-137.)
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _abi, core
from .._abi import MOTIONS


def draws(motion, seeds, device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """Return (pattern [4, n], offset [3, n]) float64 device tensors.

    `motion`: one motion name/index for every episode, or a per-episode
    sequence / int8 tensor of indices.  `seeds`: non-negative integers."""
    dev = _abi.require_gpu(device)
    if isinstance(seeds, torch.Tensor):
        s = seeds.to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
    else:
        s = torch.as_tensor(np.asarray(seeds, dtype=np.int64).reshape(-1), device=dev)
    n = s.numel()
    if isinstance(motion, (str, int, np.integer)):
        m = MOTIONS.index(motion) if isinstance(motion, str) else int(motion)
        return core.seed_draws(s, None, m)
    mt = motion if isinstance(motion, torch.Tensor) else torch.as_tensor(np.asarray(motion, dtype=np.int8))
    mt = mt.to(device=dev, dtype=torch.int8).reshape(-1).contiguous()
    if mt.numel() != n:
        raise ValueError(f"per-episode motion has {mt.numel()} entries for {n} seeds")
    return core.seed_draws(s, mt, 0)
