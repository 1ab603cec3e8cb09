"""Environment parameter schema — drop-in for the reference's
`quadcopter_tracking.env.config` (env/config.py:11-222): same dataclass names,
field names, defaults and dict round trip (`from_dict` / `to_dict`, including
the legacy flat `dt` / `episode_length` keys and the
`target.radius_requirement` -> `success_criteria.target_radius` mapping).

`EnvConfig.to_params()` packs the fields the hot path reads into the C ABI
struct `qt_env_params` (include/quadtrack.h).  Inertia, arm length and the
thrust/torque coefficients are carried for API compatibility only; the
reference dynamics never read them.
"""

from __future__ import annotations

from dataclasses import asdict, dataclass, field, fields

from .._abi import MOTIONS, EnvParams


@dataclass
class QuadcopterParams:
    mass: float = 1.0
    arm_length: float = 0.25
    Ixx: float = 0.0082
    Iyy: float = 0.0082
    Izz: float = 0.0149
    k_thrust: float = 1.0e-5
    k_torque: float = 1.0e-7
    max_thrust: float = 20.0
    min_thrust: float = 0.0
    max_angular_rate: float = 3.0
    gravity: float = 9.81
    drag_coeff_linear: float = 0.1
    drag_coeff_angular: float = 0.01


@dataclass
class SimulationParams:
    dt: float = 0.01
    max_episode_time: float = 30.0
    integrator: str = "rk4"
    max_velocity: float = 50.0
    max_angular_velocity: float = 10.0
    max_position: float = 1000.0


@dataclass
class TargetParams:
    motion_type: str = "stationary"
    speed: float = 1.0
    amplitude: float = 2.0
    frequency: float = 0.5
    radius: float = 2.0
    center: tuple[float, float, float] = (0.0, 0.0, 1.0)
    max_acceleration: float = 5.0
    radius_requirement: float = 0.5


@dataclass
class SuccessCriteria:
    min_on_target_ratio: float = 0.8
    min_episode_duration: float = 30.0
    target_radius: float = 0.5


@dataclass
class LoggingParams:
    enabled: bool = True
    log_interval: int = 10
    output_dir: str = "experiments"


def _pick(cls, src: dict):
    """Instantiate dataclass `cls` from the keys of `src` it knows (others ignored)."""
    names = {f.name for f in fields(cls)}
    return cls(**{k: v for k, v in src.items() if k in names})


@dataclass
class EnvConfig:
    seed: int = 42
    quadcopter: QuadcopterParams = field(default_factory=QuadcopterParams)
    simulation: SimulationParams = field(default_factory=SimulationParams)
    target: TargetParams = field(default_factory=TargetParams)
    success_criteria: SuccessCriteria = field(default_factory=SuccessCriteria)
    logging: LoggingParams = field(default_factory=LoggingParams)

    @classmethod
    def from_dict(cls, config_dict: dict) -> "EnvConfig":
        sim = dict(config_dict.get("simulation", {}))
        succ = dict(config_dict.get("success_criteria", {}))
        tgt = dict(config_dict.get("target", {}))
        # legacy flat keys (config.py:114-118)
        if "dt" in config_dict and "dt" not in sim:
            sim["dt"] = config_dict["dt"]
        if "episode_length" in config_dict:
            sim["max_episode_time"] = config_dict["episode_length"]
        # one on-target radius for motion and evaluation (config.py:120-126)
        if "radius_requirement" in tgt:
            succ.setdefault("target_radius", tgt["radius_requirement"])
        if "center" in tgt:
            tgt["center"] = tuple(tgt["center"])
        return cls(
            seed=config_dict.get("seed", 42),
            quadcopter=_pick(QuadcopterParams, config_dict.get("quadcopter", {})),
            simulation=_pick(SimulationParams, sim),
            target=_pick(TargetParams, tgt),
            success_criteria=_pick(SuccessCriteria, succ),
            logging=_pick(LoggingParams, config_dict.get("logging", {})),
        )

    def to_dict(self) -> dict:
        return asdict(self)

    # ------------------------------------------------------------ C ABI

    def motion_index(self) -> int:
        m = self.target.motion_type.lower()
        if m not in MOTIONS:
            # TargetMotion._create_pattern (target_motion.py:310-314)
            raise ValueError(f"Invalid motion type: {m}. Valid types: {set(MOTIONS)}")
        return MOTIONS.index(m)

    def to_params(self) -> EnvParams:
        q, s, t, sc = self.quadcopter, self.simulation, self.target, self.success_criteria
        p = EnvParams()
        p.mass, p.gravity = q.mass, q.gravity
        p.drag_linear, p.drag_angular = q.drag_coeff_linear, q.drag_coeff_angular
        p.min_thrust, p.max_thrust, p.max_angular_rate = q.min_thrust, q.max_thrust, q.max_angular_rate
        p.dt, p.max_episode_time = s.dt, s.max_episode_time
        p.max_velocity, p.max_angular_velocity, p.max_position = s.max_velocity, s.max_angular_velocity, s.max_position
        # anything but "euler" integrates with RK4 (quadcopter_env.py:309-312)
        p.integrator = 1 if s.integrator == "euler" else 0
        p.motion = self.motion_index()
        p.speed, p.amplitude, p.frequency, p.radius = t.speed, t.amplitude, t.frequency, t.radius
        for i in range(3):
            p.center[i] = float(t.center[i])
        p.max_acceleration = t.max_acceleration
        p.target_radius = sc.target_radius
        p.min_on_target_ratio = sc.min_on_target_ratio
        p.min_episode_duration = sc.min_episode_duration
        return p


def as_env_config(config) -> EnvConfig:
    if config is None:
        return EnvConfig()
    if isinstance(config, dict):
        return EnvConfig.from_dict(config)
    return config
