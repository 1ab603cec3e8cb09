"""Environment: drop-in QuadcopterEnv / TargetMotion / EnvConfig of the
reference's `quadcopter_tracking.env` (env/__init__.py:48-83), GPU-backed,
plus the batched `BatchedQuadcopterEnv`."""

from .batched import BatchedQuadcopterEnv
from .config import EnvConfig, LoggingParams, QuadcopterParams, SimulationParams, SuccessCriteria, TargetParams
from .quadcopter_env import QuadcopterEnv
from .target_motion import (
    CircularMotion,
    Figure8Motion,
    LinearMotion,
    SinusoidalMotion,
    StationaryMotion,
    TargetMotion,
)

__all__ = ["QuadcopterEnv", "BatchedQuadcopterEnv", "TargetMotion", "EnvConfig", "QuadcopterParams",
           "SimulationParams", "TargetParams", "SuccessCriteria", "LoggingParams", "LinearMotion", "CircularMotion",
           "SinusoidalMotion", "Figure8Motion", "StationaryMotion"]
