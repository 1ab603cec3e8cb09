"""Batched controller-tuner evaluation (BASELINE config 4).

The reference's `ControllerTuner` (controllers/tuning.py:581-1442) evaluates
one candidate gain configuration at a time: `_evaluate_config` (846-928)
builds one controller (one DARE), then runs `evaluation_episodes` fresh
environments with seeds `seed + ep` (874-906), calling `controller.reset()`
before each, and scores the candidate as
`mean(on_target_ratio) - 0.1 * mean(mean_tracking_error)` (915-919).

`BatchedTuner` evaluates every candidate of a sweep at once: all candidate
DAREs in one batched SDA launch (`BatchedRiccatiLQR` with per-candidate
q_pos / q_vel / r_controls / q_int), then candidates x episodes closed-loop
episodes in one fused rollout, then per-candidate scores.  Candidate
generation follows the reference's random stream exactly
(`_generate_random_config` 683-735: `default_rng(seed)`, parameters in its
fixed order, one `uniform(lo, hi)` per component) and its grid order
(`_generate_grid_configs` 737-830).  Its data formats come along: TuningConfig
/ TuningResult dictionaries, `resume_from` a previous results file, and the
two files `tune()` writes (`_save_results`, 1103-1129).  CMA-ES needs the
`cma` package's sequential ask / tell loop (absent here, as the reference
itself then raises ImportError) and stays out of scope.

Supported controller_type: "riccati_lqr" (per-candidate q_pos / q_vel /
r_controls / q_int -> one DARE each), "pid" (kp_pos / ki_pos / kd_pos, the
PIDController of controllers/__init__.py:116-396) and "lqr" (q_pos / q_vel /
r_thrust / r_rate -> the heuristic gains of LQRController, 522-574), each with
per-candidate feed-forward gain ranges (qt_batch.ff).  As in the reference,
a candidate's controller is built from the candidate's keys alone (plus
`base_controller_config`); keys the controller type does not read are
ignored, as the reference's controllers ignore them.
"""

from __future__ import annotations

import json
import logging
import os
from dataclasses import dataclass, field, fields
from datetime import datetime, timezone
from itertools import product
from pathlib import Path

import numpy as np
import torch

from .controllers.lqr import BatchedLQR
from .controllers.pid import BatchedPID
from .controllers.riccati_lqr import BatchedRiccatiLQR
from .env.config import EnvConfig
from .rollout import run_closed_loop
from .utils.metrics import SuccessCriteria

logger = logging.getLogger(__name__)


# substrings a result / resume path may not contain, with the reference's
# messages (tuning.py:64-106)
_PATH_REFUSED = (
    ("..", "Path contains path traversal sequence '..': {p}. "
           "Use absolute paths or paths without parent directory references."),
    ("\x00", "Path contains null byte: {p}"),
)


def _validate_path(path: Path) -> None:
    """Path checks of tuning.py:64-106: no '..' or NUL; resolvable; a relative
    path may leave the working directory only to somewhere below the root."""
    for token, message in _PATH_REFUSED:
        if token in str(path):
            raise ValueError(message.format(p=path))
    try:
        resolved = path.resolve()
        if path.is_absolute() or len(resolved.parts) >= 2:
            return
        inside = True
        try:
            resolved.relative_to(Path.cwd().resolve())
        except ValueError:
            inside = False
    except (OSError, RuntimeError) as e:
        raise ValueError(f"Cannot resolve path {path}: {e}")
    if not inside:
        raise ValueError(f"Relative path resolves outside working directory: {path}")


# parameter name -> (range attribute, components); the order of
# _generate_random_config (tuning.py:689-733)
_PARAM_ORDER = (
    ("kp_pos", "kp_pos_range", 3),
    ("ki_pos", "ki_pos_range", 3),
    ("kd_pos", "kd_pos_range", 3),
    ("ff_velocity_gain", "ff_velocity_gain_range", 3),
    ("ff_acceleration_gain", "ff_acceleration_gain_range", 3),
    ("q_pos", "q_pos_range", 3),
    ("q_vel", "q_vel_range", 3),
    ("r_thrust", "r_thrust_range", 0),
    ("r_rate", "r_rate_range", 0),
    ("r_controls", "r_controls_range", 4),
    ("q_int", "q_int_range", 3),
)


@dataclass
class GainSearchSpace:
    """Search ranges (tuning.py:146-360): (min_values, max_values) per vector
    parameter, (min, max) for the scalar r_thrust / r_rate; None = not tuned."""

    kp_pos_range: tuple | None = None
    ki_pos_range: tuple | None = None
    kd_pos_range: tuple | None = None
    ff_velocity_gain_range: tuple | None = None
    ff_acceleration_gain_range: tuple | None = None
    q_pos_range: tuple | None = None
    q_vel_range: tuple | None = None
    r_thrust_range: tuple | None = None
    r_rate_range: tuple | None = None
    r_controls_range: tuple | None = None
    q_int_range: tuple | None = None
    use_lqi: bool = False

    def validate(self) -> None:
        """Inverted or negative ranges and wrong lengths raise ValueError (tuning.py:194-298)."""
        for name, attr, dim in _PARAM_ORDER:
            rng = getattr(self, attr)
            if rng is None:
                continue
            lo, hi = rng
            if dim == 0:
                lo, hi = [lo], [hi]
            elif len(lo) != dim or len(hi) != dim:
                raise ValueError(f"{attr} must have exactly {dim} values, got min={len(lo)}, max={len(hi)}")
            for i, (a, b) in enumerate(zip(lo, hi)):
                if a > b:
                    raise ValueError(f"{attr}[{i}] has inverted range: min={a} > max={b}")
                if a < 0:
                    raise ValueError(f"{attr}[{i}] has negative minimum: {a}")

    def get_active_parameters(self) -> list[str]:
        out = [name for name, attr, _ in _PARAM_ORDER if getattr(self, attr) is not None]
        if self.use_lqi and "q_int" not in out:
            out.append("use_lqi")
        return out

    @classmethod
    def from_dict(cls, d: dict) -> "GainSearchSpace":
        return cls(**{f.name: d.get(f.name, f.default) for f in fields(cls)})

    def to_dict(self) -> dict:
        return {f.name: getattr(self, f.name) for f in fields(self)}


def default_search_space(controller_type: str = "riccati_lqr") -> GainSearchSpace:
    """The default ranges of scripts/controller_autotune.py:360-385 (`get_default_search_space`):
    PID kp / kd, heuristic-LQR q_pos / q_vel, Riccati-LQR q_pos / q_vel / r_controls (config 4)."""
    if controller_type == "pid":
        return GainSearchSpace(kp_pos_range=([0.005, 0.005, 2.0], [0.05, 0.05, 6.0]),
                               kd_pos_range=([0.02, 0.02, 1.0], [0.15, 0.15, 3.0]))
    if controller_type == "lqr":
        return GainSearchSpace(q_pos_range=([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0]),
                               q_vel_range=([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0]))
    if controller_type == "riccati_lqr":
        return GainSearchSpace(q_pos_range=([5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0]),
                               q_vel_range=([1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0]),
                               r_controls_range=([0.5] * 4, [2.0] * 4))
    return GainSearchSpace()


@dataclass
class TuningConfig:
    """Tuner settings (tuning.py:363-478); same defaults and dictionary form."""

    controller_type: str = "pid"
    search_space: GainSearchSpace = field(default_factory=GainSearchSpace)
    strategy: str = "random"
    max_iterations: int = 50
    grid_points_per_dim: int = 3
    evaluation_episodes: int = 5
    evaluation_horizon: int = 3000
    seed: int = 42
    target_motion_type: str = "stationary"
    episode_length: float = 30.0
    target_radius: float = 0.5
    output_dir: str = "reports/tuning"
    resume_from: str | None = None
    feedforward_enabled: bool = False
    cma_sigma0: float = 0.3
    cma_popsize: int | None = None

    def __post_init__(self):
        if self.controller_type not in ("pid", "lqr", "riccati_lqr"):
            raise ValueError(f"Invalid controller_type: '{self.controller_type}'. "
                             "Valid choices are: pid, lqr, riccati_lqr")
        if self.strategy not in ("grid", "random", "cma_es"):
            raise ValueError(f"Invalid strategy: '{self.strategy}'. Valid choices are: grid, random, cma_es")
        if self.max_iterations < 1:
            raise ValueError(f"max_iterations must be >= 1, got {self.max_iterations}")
        if self.evaluation_episodes < 1:
            raise ValueError(f"evaluation_episodes must be >= 1, got {self.evaluation_episodes}")
        if self.cma_sigma0 <= 0:
            raise ValueError(f"cma_sigma0 must be > 0, got {self.cma_sigma0}")
        if self.cma_popsize is not None and self.cma_popsize < 2:
            raise ValueError(f"cma_popsize must be >= 2, got {self.cma_popsize}")

    @classmethod
    def from_dict(cls, config: dict) -> "TuningConfig":
        kw = {f.name: config.get(f.name, f.default) for f in fields(cls) if f.name != "search_space"}
        return cls(search_space=GainSearchSpace.from_dict(config.get("search_space", {})), **kw)

    def to_dict(self) -> dict:
        d = {f.name: getattr(self, f.name) for f in fields(self)}
        d["search_space"] = self.search_space.to_dict()
        return d


@dataclass
class TuningResult:
    """tuning.py:480-579: the result and its JSON file."""

    best_config: dict
    best_score: float
    best_metrics: dict
    all_results: list
    iterations_completed: int
    interrupted: bool
    timestamp: str
    config: dict

    def to_dict(self) -> dict:
        return {f.name: getattr(self, f.name) for f in fields(self)}

    @classmethod
    def from_dict(cls, data: dict) -> "TuningResult":
        return cls(**{f.name: data[f.name] for f in fields(cls)})

    def save(self, path: str | Path) -> Path:
        path = Path(path)
        _validate_path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=2)
        return path

    @classmethod
    def load(cls, path: str | Path) -> "TuningResult":
        path = Path(path)
        _validate_path(path)
        if not path.exists():
            raise FileNotFoundError(f"Tuning results file not found: {path}")
        if not path.is_file():
            raise ValueError(f"Path is not a file: {path}")
        with open(path) as f:
            return cls.from_dict(json.load(f))


def random_configs(space: GainSearchSpace, n: int, rng: np.random.Generator) -> list[dict]:
    """n consecutive `_generate_random_config` results from `rng` (tuning.py:683-735).

    One vectorised draw of [n, D] uniforms: numpy fills it in C order from
    the same stream, lo + (hi - lo) * next_double per element, which is what
    the reference's D scalar `rng.uniform(lo, hi)` calls per candidate do."""
    cols, spec = [], []
    for name, attr, dim in _PARAM_ORDER:
        rng_def = getattr(space, attr)
        if rng_def is None:
            continue
        lo, hi = rng_def
        lo, hi = ([lo], [hi]) if dim == 0 else (list(lo), list(hi))
        spec.append((name, len(cols), dim))
        cols.extend(zip(lo, hi))
    if not cols:
        u = np.empty((n, 0))
    else:
        lo = np.array([c[0] for c in cols], float)
        hi = np.array([c[1] for c in cols], float)
        u = rng.uniform(lo, hi, size=(n, len(cols)))
    out = []
    for i in range(n):
        cfg = {}
        for name, j, dim in spec:
            cfg[name] = float(u[i, j]) if dim == 0 else [float(v) for v in u[i, j:j + dim]]
            if name in ("ff_velocity_gain", "ff_acceleration_gain"):
                cfg["feedforward_enabled"] = True
            if name == "q_int":
                cfg["use_lqi"] = True
        if space.q_int_range is None and space.use_lqi:
            cfg["use_lqi"] = True
            cfg["q_int"] = [0.0, 0.0, 0.0]
        out.append(cfg)
    return out


def grid_configs(space: GainSearchSpace, points: int) -> list[dict]:
    """The reference's grid (tuning.py:737-830): per-axis linspace (a single
    point where lo == hi), Cartesian products in parameter order."""

    def axis(lo, hi):
        return [lo] if np.isclose(lo, hi) else list(np.linspace(lo, hi, points))

    grids = {}
    for name, attr, dim in _PARAM_ORDER:
        rng_def = getattr(space, attr)
        if rng_def is None:
            if name == "q_int" and space.use_lqi:
                grids[name] = [[0.0, 0.0, 0.0]]
            continue
        lo, hi = rng_def
        if dim == 0:
            grids[name] = axis(lo, hi)
        else:
            grids[name] = [list(c) for c in product(*[axis(a, b) for a, b in zip(lo, hi)])]
    if not grids:
        return []
    names = list(grids)
    out = []
    for combo in product(*[grids[k] for k in names]):
        cfg = dict(zip(names, combo))
        if "ff_velocity_gain" in cfg or "ff_acceleration_gain" in cfg:
            cfg["feedforward_enabled"] = True
        if "q_int" in cfg or space.use_lqi:
            cfg["use_lqi"] = True
        out.append(cfg)
    return out


def score_rows(ratio: np.ndarray, err: np.ndarray, succ: np.ndarray) -> list[tuple[float, dict]]:
    """Per-candidate (score, metrics) from [C, E] episode metrics
    (tuning.py:908-928): np.mean of each candidate's E values, score =
    mean ratio - 0.1 * mean error.  One reduction per array: numpy reduces
    each contiguous row of a C-ordered array exactly as it reduces that row
    alone, so the values equal the reference's per-candidate np.mean."""
    E = ratio.shape[1]
    mean_on, mean_err, rate = (np.ascontiguousarray(a, dtype=np.float64).mean(axis=1) for a in (ratio, err, succ))
    score = mean_on - 0.1 * mean_err
    return [(s, {"mean_on_target_ratio": r, "mean_tracking_error": e, "success_rate": q, "episodes_evaluated": E})
            for s, r, e, q in zip(score.tolist(), mean_on.tolist(), mean_err.tolist(), rate.tolist())]


class BatchedTuner:
    """`ControllerTuner` with every candidate evaluated in one batch.

    evaluate_configs(configs) -> [(score, metrics)] in candidate order, the
    values `_evaluate_config` returns for each (tuning.py:846-928)."""

    def __init__(self, config: TuningConfig, device=None, base_controller_config: dict | None = None):
        config.search_space.validate()
        if config.strategy == "cma_es":  # tuning.py:636-643
            try:
                import cma  # noqa: F401
            except ImportError:
                raise ImportError("CMA-ES strategy requires the 'cma' package. Install it with: pip install cma")
            # with cma installed the reference runs its sequential ask / tell loop; that
            # search strategy is not batched here, so refuse it up front
            raise NotImplementedError("CMA-ES is a sequential search; the batched tuner runs grid and random")
        self.config = config
        self.device = device
        self.base = dict(base_controller_config or {})
        self.rng = np.random.default_rng(config.seed)
        self.results: list[dict] = []
        self.best_config: dict = {}
        self.best_score = float("-inf")
        self.best_metrics: dict = {}
        self.output_dir = Path(os.environ.get("TUNING_OUTPUT_DIR", config.output_dir))  # tuning.py:627-628
        _validate_path(self.output_dir)

    # ---- candidate generation (reference stream order)
    def generate_random_configs(self, n: int) -> list[dict]:
        return random_configs(self.config.search_space, n, self.rng)

    def generate_grid_configs(self) -> list[dict]:
        return grid_configs(self.config.search_space, self.config.grid_points_per_dim)

    # ---- evaluation
    def env_config(self) -> EnvConfig:
        """tuning.py:859-863."""
        env = EnvConfig()
        env.simulation.max_episode_time = self.config.episode_length
        env.target.motion_type = self.config.target_motion_type
        env.success_criteria.target_radius = self.config.target_radius
        return env

    def criteria(self) -> SuccessCriteria:
        """tuning.py:865-869."""
        return SuccessCriteria(min_on_target_ratio=0.8, min_episode_duration=self.config.episode_length,
                               target_radius=self.config.target_radius)

    # per-candidate keys each controller type reads (its batched constructor's per-episode arrays)
    _PER_CANDIDATE = {
        "riccati_lqr": ("q_pos", "q_vel", "r_controls", "q_int", "mass"),
        "pid": ("kp_pos", "ki_pos", "kd_pos", "mass"),
        "lqr": ("q_pos", "q_vel", "r_thrust", "r_rate", "mass"),
    }
    _FF_KEYS = ("ff_velocity_gain", "ff_acceleration_gain")
    # PIDController reads config.get("kp_pos", config.get("kp", default)) (controllers/__init__.py)
    _ALIASES = {"pid": {"kp": "kp_pos", "ki": "ki_pos", "kd": "kd_pos"}}

    @classmethod
    def _canonical(cls, kind: str, cfg: dict) -> dict:
        """A candidate with the controller's key aliases resolved as its
        constructor resolves them (the canonical key wins over its alias)."""
        out = dict(cfg)
        for alias, key in cls._ALIASES.get(kind, {}).items():
            if alias in out:
                v = out.pop(alias)
                out.setdefault(key, v)
        return out

    def controller(self, configs: list[dict]):
        """One batched controller over the candidates, one gain set (one DARE
        for riccati_lqr) per candidate, built from each candidate's whole
        config as the reference builds one controller per candidate
        (tuning.py:832-844): keys with a per-candidate form become arrays,
        any other key must be the same for every candidate and joins the
        shared config (a key that varies without a per-candidate form
        raises)."""
        kind = self.config.controller_type
        base = self._canonical(kind, self.base)
        configs = [self._canonical(kind, c) for c in configs]
        keys = set().union(*[c.keys() for c in configs]) if configs else set()
        shared = dict(base)
        if kind == "riccati_lqr":
            lqi = {bool(c.get("use_lqi", base.get("use_lqi", False))) for c in configs}
            if len(lqi) > 1:
                raise ValueError("candidates mix LQR and LQI")
            shared["use_lqi"] = lqi.pop() if lqi else False
        if any(c.get("feedforward_enabled", base.get("feedforward_enabled")) for c in configs):
            shared["feedforward_enabled"] = True
        per = set(self._PER_CANDIDATE[kind]) | set(self._FF_KEYS)
        _missing = object()
        for key in sorted(keys - per - {"use_lqi", "feedforward_enabled"}):
            vals = [c.get(key, base.get(key, _missing)) for c in configs]
            first = vals[0]
            same = all(v is not _missing for v in vals) and all(
                np.array_equal(np.asarray(v, dtype=object), np.asarray(first, dtype=object)) for v in vals[1:])
            if not same:
                raise ValueError(f"candidate key '{key}' differs between candidates and has no per-candidate "
                                 f"form in the batched {kind} controller")
            shared[key] = first

        defaults = {"q_pos": [1e-4, 1e-4, 16.0], "q_vel": [0.0036, 0.0036, 4.0], "r_controls": [1.0] * 4,
                    "q_int": [0.0, 0.0, 0.0], "r_thrust": 1.0, "r_rate": 1.0,
                    "ff_velocity_gain": [0.0, 0.0, 0.0], "ff_acceleration_gain": [0.0, 0.0, 0.0]}
        scalar_keys = ("r_thrust", "r_rate", "mass")

        def col(key):
            if kind == "pid" and key in ("kp_pos", "ki_pos", "kd_pos"):
                from .controllers.pid import _DEFAULT_KD, _DEFAULT_KI, _DEFAULT_KP
                d = {"kp_pos": _DEFAULT_KP, "ki_pos": _DEFAULT_KI, "kd_pos": _DEFAULT_KD}[key]
                base_v = shared.get(key, d)
            elif key == "mass":
                base_v = shared.get("mass", 1.0)
            else:
                base_v = shared.get(key, defaults[key])

            def vec(v):
                v = np.asarray(v, float)
                return np.full(3, float(v)) if v.ndim == 0 and key not in scalar_keys else v
            vals = [c.get(key, base_v) for c in configs]
            try:  # one conversion of the whole column (every candidate the same shape)
                arr = np.array(vals, dtype=float)
            except ValueError:
                arr = None
            if arr is None or arr.ndim not in (1, 2) or (arr.ndim == 1 and key not in scalar_keys):
                return np.stack([vec(v) for v in vals])
            return arr

        kw = {k: col(k) for k in self._PER_CANDIDATE[kind] if k in keys}
        if kind == "riccati_lqr" and shared["use_lqi"]:
            kw["q_int"] = col("q_int")
        if keys & set(self._FF_KEYS):
            kw.update({k: col(k) for k in self._FF_KEYS})
        if not kw:  # nothing per candidate: one shared gain set repeated (still one row per candidate)
            kw = {"mass": np.full(len(configs), float(shared.get("mass", 1.0)))}
        cls = {"riccati_lqr": BatchedRiccatiLQR, "pid": BatchedPID, "lqr": BatchedLQR}[kind]
        return cls(shared, device=self.device, **kw)

    def evaluate_configs(self, configs: list[dict], chunk: int | None = None):
        """Scores and metrics of every candidate (tuning.py:846-928)."""
        if not configs:
            return []
        E = self.config.evaluation_episodes
        ctl = self.controller(configs).repeat_episodes(E)
        seeds = np.tile(self.config.seed + np.arange(E, dtype=np.int64), len(configs))
        res = run_closed_loop(ctl, self.env_config(), n=len(seeds), seeds=seeds, criteria=self.criteria(),
                              max_steps=self.config.evaluation_horizon, chunk=chunk)
        m = res.metrics.cpu().numpy()
        from ._abi import MET

        C = len(configs)
        return score_rows(m[MET["on_target_ratio"]].reshape(C, E), m[MET["mean_tracking_error"]].reshape(C, E),
                          m[MET["success"]].reshape(C, E))

    def _evaluate_config(self, controller_config: dict) -> tuple[float, dict]:
        """One candidate's (score, metrics), as tuning.py:846-928 returns them."""
        return self.evaluate_configs([controller_config])[0]

    def _record(self, cfg, score, metrics):
        """tuning.py:1075-1088 (strictly-greater best update)."""
        self.results.append({"config": cfg, "score": score, "metrics": metrics})
        if score > self.best_score:
            self.best_score, self.best_config, self.best_metrics = score, cfg, metrics

    def tune(self) -> TuningResult:
        """Random or grid search (tuning.py:930-1001) with all candidates
        evaluated in one batch: resume from `resume_from` (previous results and
        best kept; a random search draws the remaining candidates from the
        seed's stream, as the reference's fresh generator does), then the
        results files of `_save_results`."""
        if self.config.strategy == "cma_es":
            raise NotImplementedError("CMA-ES is sequential; out of scope for the batched tuner")
        if self.config.resume_from:
            prev = TuningResult.load(self.config.resume_from)
            self.results = prev.all_results
            self.best_config, self.best_score, self.best_metrics = prev.best_config, prev.best_score, prev.best_metrics
        if self.config.strategy == "grid":
            configs = self.generate_grid_configs()[:self.config.max_iterations]
        else:
            configs = self.generate_random_configs(max(0, self.config.max_iterations - len(self.results)))
        for cfg, (score, metrics) in zip(configs, self.evaluate_configs(configs) if configs else []):
            self._record(cfg, score, metrics)
        result = TuningResult(best_config=self.best_config, best_score=self.best_score,
                              best_metrics=self.best_metrics, all_results=self.results,
                              iterations_completed=len(self.results), interrupted=False,
                              timestamp=datetime.now(timezone.utc).isoformat(), config=self.config.to_dict())
        self.save_results(result)
        return result

    def save_results(self, result: TuningResult) -> dict[str, Path]:
        """`<output_dir>/tuning_<type>_<UTC stamp>_results.json` (the full
        result) and `..._best_config.json` (tuning.py:1103-1129)."""
        self.output_dir.mkdir(parents=True, exist_ok=True)
        stamp = datetime.now(timezone.utc).strftime("%Y%m%d_%H%M%S")
        base = f"tuning_{self.config.controller_type}_{stamp}"
        paths = {"results": result.save(self.output_dir / f"{base}_results.json"),
                 "best_config": self.output_dir / f"{base}_best_config.json"}
        with open(paths["best_config"], "w") as f:
            json.dump({"controller_type": self.config.controller_type,
                       self.config.controller_type: result.best_config,
                       "metrics": result.best_metrics, "score": result.best_score}, f, indent=2)
        logger.info("Saved tuning results to %s", self.output_dir)
        return paths


# the reference's class name (controllers/tuning.py:581): same constructor and tune()
# for grid and random search.  Differences: strategy "cma_es"
# raises (ImportError without `cma`, as the reference; NotImplementedError with
# it), and there is no SIGINT / SIGTERM partial save (the whole search is one
# batch), so TuningResult.interrupted is always False.
ControllerTuner = BatchedTuner

__all__ = ["GainSearchSpace", "TuningConfig", "TuningResult", "BatchedTuner", "ControllerTuner", "score_rows", "random_configs", "grid_configs",
           "default_search_space"]
