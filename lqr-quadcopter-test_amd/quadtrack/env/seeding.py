"""Per-episode random draws of `QuadcopterEnv.reset(seed)`.

The reference re-creates two `numpy.random.default_rng(seed)` streams on every
seeded reset (env/quadcopter_env.py:122-127): the target stream draws the
pattern parameters (target_motion.py:318-366: linear `standard_normal(3)`,
circular `uniform(0, 2*pi)`, sinusoidal `uniform(0, 2*pi, 3)`, figure8 and
stationary nothing) and the env stream draws the start offset
`uniform(-0.5, 0.5, 3)` (quadcopter_env.py:137).  Reproducing those values
bit for bit needs numpy's own generator (PCG64 + SeedSequence + ziggurat), so
the draws are made with numpy on the host — setup work of a few µs per
episode, outside the closed loop — and uploaded once; everything downstream
of the draws (the t = 0 target, the initial state) is computed by the reset
kernel.
"""

from __future__ import annotations

import math

import numpy as np

from .._abi import MOTIONS

_TWO_PI = 2 * math.pi


def draws(motion, seeds) -> tuple[np.ndarray, np.ndarray]:
    """Return (pattern[4, n], offset[3, n]) float64 for the given seeds.

    `motion` is one motion name/index for all episodes or a per-episode
    sequence of indices.
    """
    seeds = np.asarray(seeds, dtype=np.int64).reshape(-1)
    n = seeds.size
    if isinstance(motion, (str, int, np.integer)):
        m = MOTIONS.index(motion) if isinstance(motion, str) else int(motion)
        kinds = np.full(n, m, dtype=np.int64)
    else:
        kinds = np.asarray(motion, dtype=np.int64).reshape(-1)
        if kinds.size != n:
            raise ValueError(f"per-episode motion has {kinds.size} entries for {n} seeds")
    pat = np.zeros((4, n))
    off = np.empty((3, n))
    rng = np.random.default_rng
    for i in range(n):
        s = int(seeds[i])
        k = kinds[i]
        if k == 1:
            pat[:3, i] = rng(s).standard_normal(3)
        elif k == 2:
            pat[0, i] = rng(s).uniform(0, _TWO_PI)
        elif k == 3:
            pat[:3, i] = rng(s).uniform(0, _TWO_PI, 3)
        off[:, i] = rng(s).uniform(-0.5, 0.5, 3)
    return pat, off
