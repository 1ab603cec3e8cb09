"""Target trajectories — drop-in for the reference's
`quadcopter_tracking.env.target_motion` (env/target_motion.py:1-429).

The pattern classes and `TargetMotion` keep their constructors and
`get_state` signatures; the position / velocity / (clamped) acceleration are
evaluated by the HIP target kernel (`qt_target_state`) for a one-episode
batch.  `TargetMotion` draws its pattern parameters from its own
`numpy.random.default_rng(seed)` stream exactly like the reference
(target_motion.py:285-369), so the same seed gives the same trajectory.
"""

from __future__ import annotations

import math

import numpy as np
import torch

from .. import _abi, core
from .._abi import MOTIONS
from .config import TargetParams

F64 = torch.float64


def _evaluate(params: TargetParams, motion: int, raw, t: float, max_acceleration=None):
    dev = _abi.require_gpu()
    ep = _env_params(params, motion, max_acceleration)
    pat = np.zeros((4, 1))
    raw = np.asarray(raw, float).reshape(-1)
    pat[: raw.size, 0] = raw
    b = core.EpisodeBatch(n=1, device=dev, pattern=core.to_device(pat, dev), offset=torch.zeros(3, 1, dtype=F64, device=dev),
                          K=torch.zeros(24, 1, dtype=F64, device=dev), k_cols=6)
    out = core.target_state(ep, b, torch.tensor([float(t)], dtype=F64, device=dev)).cpu().numpy()[:, 0]
    return out[0:3].copy(), out[3:6].copy(), out[6:9].copy()


def _env_params(params: TargetParams, motion: int, max_acceleration=None):
    from .config import EnvConfig

    cfg = EnvConfig(target=params)
    p = cfg.to_params() if params.motion_type.lower() in MOTIONS else EnvConfig().to_params()
    p.motion = motion
    p.speed, p.amplitude, p.frequency, p.radius = params.speed, params.amplitude, params.frequency, params.radius
    for i in range(3):
        p.center[i] = float(params.center[i])
    p.max_acceleration = math.inf if max_acceleration is None else float(max_acceleration)
    return p


class _Pattern:
    """Base of the pattern classes: get_state(t) -> (position, velocity, acceleration)."""

    motion = 0

    def _params(self) -> TargetParams:
        raise NotImplementedError

    def _raw(self):
        return np.zeros(3)

    def get_state(self, t: float):
        return _evaluate(self._params(), self.motion, self._raw(), t)


class LinearMotion(_Pattern):
    """target_motion.py:29-56"""

    motion = 1

    def __init__(self, start: np.ndarray, direction: np.ndarray, speed: float):
        self.start = np.array(start, dtype=float).copy()
        self.direction = np.asarray(direction, float) / np.linalg.norm(direction)
        self.speed = speed
        self.velocity = self.direction * self.speed

    def _params(self):
        return TargetParams(motion_type="linear", speed=self.speed, center=tuple(self.start))

    def _raw(self):
        return self.direction


class CircularMotion(_Pattern):
    """target_motion.py:59-115"""

    motion = 2

    def __init__(self, center: np.ndarray, radius: float, speed: float, initial_angle: float = 0.0):
        self.center = np.array(center, dtype=float).copy()
        self.radius = radius
        self.speed = speed
        self.omega = speed / radius
        self.initial_angle = initial_angle

    def _params(self):
        return TargetParams(motion_type="circular", speed=self.speed, radius=self.radius, center=tuple(self.center))

    def _raw(self):
        return np.array([self.initial_angle])


class SinusoidalMotion(_Pattern):
    """target_motion.py:118-150 with the (A, A/2, A/4) amplitudes and (f, 1.3f,
    0.7f) frequencies TargetMotion gives it (337-359)."""

    motion = 3

    def __init__(self, center: np.ndarray, amplitude: np.ndarray, frequency: np.ndarray, phase: np.ndarray = None):
        self.center = np.array(center, dtype=float).copy()
        self.amplitude = np.array(amplitude, dtype=float).copy()
        self.frequency = np.array(frequency, dtype=float)
        self.omega = 2 * np.pi * self.frequency
        self.phase = phase if phase is not None else np.zeros(3)
        a, f = self.amplitude, self.frequency
        if not (np.allclose(a, [a[0], a[0] * 0.5, a[0] * 0.25], rtol=0, atol=0)
                and np.allclose(f, [f[0], f[0] * 1.3, f[0] * 0.7], rtol=0, atol=0)):
            raise ValueError("device SinusoidalMotion supports the TargetMotion amplitude/frequency ratios "
                             "(A, A/2, A/4) and (f, 1.3f, 0.7f)")

    def _params(self):
        return TargetParams(motion_type="sinusoidal", amplitude=float(self.amplitude[0]),
                            frequency=float(self.frequency[0]), center=tuple(self.center))

    def _raw(self):
        return np.asarray(self.phase, float)


class Figure8Motion(_Pattern):
    """target_motion.py:153-231 (lemniscate; acceleration by the reference's
    1e-6 forward difference)."""

    motion = 4

    def __init__(self, center: np.ndarray, scale: float, speed: float):
        self.center = np.array(center, dtype=float).copy()
        self.scale = scale
        self.omega = speed / scale
        self.speed = speed

    def _params(self):
        return TargetParams(motion_type="figure8", amplitude=self.scale, speed=self.speed, center=tuple(self.center))


class StationaryMotion(_Pattern):
    """target_motion.py:234-248"""

    motion = 0

    def __init__(self, position: np.ndarray):
        self.position = np.array(position, dtype=float).copy()

    def _params(self):
        return TargetParams(motion_type="stationary", center=tuple(self.position))


class TargetMotion:
    """Seeded target generator (target_motion.py:251-429)."""

    VALID_MOTION_TYPES = set(MOTIONS)

    def __init__(self, params: TargetParams | None = None, seed: int | None = None):
        self.params = params or TargetParams()
        self.rng = np.random.default_rng(seed)
        self._pattern = None
        self._raw = np.zeros(3)
        self._time = 0.0
        self._last_position = None
        self._last_velocity = None

    def reset(self, seed: int | None = None) -> None:
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self._time = 0.0
        self._last_position = None
        self._last_velocity = None
        self._pattern = self._create_pattern()

    def _create_pattern(self):
        """Draw the pattern parameters from this generator's stream (306-369)."""
        m = self.params.motion_type.lower()
        if m not in self.VALID_MOTION_TYPES:
            raise ValueError(f"Invalid motion type: {m}. Valid types: {self.VALID_MOTION_TYPES}")
        center = np.array(self.params.center)
        p = self.params
        if m == "linear":
            d = self.rng.standard_normal(3)
            self._raw = d.copy()
            d /= np.linalg.norm(d)
            return LinearMotion(start=center, direction=d, speed=p.speed)
        if m == "circular":
            a = self.rng.uniform(0, 2 * math.pi)
            self._raw = np.array([a])
            return CircularMotion(center=center, radius=p.radius, speed=p.speed, initial_angle=a)
        if m == "sinusoidal":
            ph = self.rng.uniform(0, 2 * math.pi, 3)
            self._raw = ph.copy()
            return SinusoidalMotion(center=center, amplitude=np.array([p.amplitude, p.amplitude * 0.5,
                                                                       p.amplitude * 0.25]),
                                    frequency=np.array([p.frequency, p.frequency * 1.3, p.frequency * 0.7]),
                                    phase=ph)
        self._raw = np.zeros(3)
        if m == "figure8":
            return Figure8Motion(center=center, scale=p.amplitude, speed=p.speed)
        return StationaryMotion(position=center)

    @property
    def motion_index(self) -> int:
        return MOTIONS.index(self.params.motion_type.lower())

    @property
    def raw_draws(self) -> np.ndarray:
        """The pattern draws in qt_batch.pattern form (raw normal draw, theta0 or phases)."""
        if self._pattern is None:
            self.reset()
        out = np.zeros(4)
        out[: self._raw.size] = self._raw
        return out

    def get_position(self, time: float) -> tuple[float, float, float]:
        p, _, _ = self._state(time)
        return tuple(p)

    def _state(self, time: float):
        if self._pattern is None:
            self.reset()
        return _evaluate(self.params, self.motion_index, self._raw, time, self.params.max_acceleration)

    def get_state(self, time: float) -> dict:
        p, v, a = self._state(time)
        return {"position": p, "velocity": v, "acceleration": a}

    def step(self, dt: float) -> dict:
        self._time += dt
        return self.get_state(self._time)

    @property
    def current_time(self) -> float:
        return self._time
