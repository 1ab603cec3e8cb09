"""ctypes binding of the C ABI in include/quadtrack.h (libquadtrack.so).

The library is the product: every numeric operation of the quadtrack package
runs in its HIP kernels on the GPU.  There is no CPU fallback — if the shared
object is missing, or no GPU is visible, the calls raise.
"""

from __future__ import annotations

import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# QUADTRACK_LIB points timing experiments (scripts/ablate.sh) at another build
LIB_PATH = os.environ.get("QUADTRACK_LIB") or os.path.join(_HERE, "_lib", "libquadtrack.so")
ABI_VERSION = 9

# enums (include/quadtrack.h)
MOTIONS = ("stationary", "linear", "circular", "sinusoidal", "figure8")
TERM_REASONS = ("", "time_limit", "position_bounds", "numerical_instability")
DARE_OK, DARE_Q_NOT_PSD, DARE_R_NOT_PD, DARE_NO_CONVERGE, DARE_SINGULAR = range(5)

ACC_ROWS = 14
(ACC_SUM_ERR, ACC_SUM_ERR2, ACC_MAX_ERR, ACC_ON_PRE, ACC_ON_POST, ACC_SUM_EFFORT, ACC_OS_COUNT, ACC_OS_MAX,
 ACC_OS_CUR, ACC_OS_STREAK, ACC_PREV_ON, ACC_STEPS, ACC_VIOLATIONS, ACC_TERM) = range(ACC_ROWS)

MET_FIELDS = ("episode_duration", "on_target_ratio", "mean_tracking_error", "max_tracking_error",
              "rms_tracking_error", "total_control_effort", "mean_control_effort", "overshoot_count",
              "max_overshoot", "success", "termination_code", "action_violations",
              "env_on_target_ratio", "steps")
MET_ROWS = len(MET_FIELDS)
MET = {k: i for i, k in enumerate(MET_FIELDS)}


class EnvParams(C.Structure):
    """qt_env_params"""

    _fields_ = [(k, C.c_double) for k in ("mass", "gravity", "drag_linear", "drag_angular", "min_thrust",
                                           "max_thrust", "max_angular_rate", "dt", "max_episode_time",
                                           "max_velocity", "max_angular_velocity", "max_position")] + [
        ("integrator", C.c_int32), ("motion", C.c_int32)] + [
        (k, C.c_double) for k in ("speed", "amplitude", "frequency", "radius")] + [
        ("center", C.c_double * 3), ("max_acceleration", C.c_double)] + [
        (k, C.c_double) for k in ("target_radius", "min_on_target_ratio", "min_episode_duration")]


class CtrlParams(C.Structure):
    """qt_ctrl_params"""

    _fields_ = [(k, C.c_double) for k in ("dt", "hover_thrust", "min_thrust", "max_thrust", "max_rate")] + [
        ("use_lqi", C.c_int32), ("feedforward_enabled", C.c_int32),
        ("integral_limit", C.c_double), ("integral_zero_threshold", C.c_double),
        ("ff_velocity_gain", C.c_double * 3), ("ff_acceleration_gain", C.c_double * 3),
        ("ff_max_velocity", C.c_double), ("ff_max_acceleration", C.c_double)]


class Criteria(C.Structure):
    """qt_criteria"""

    _fields_ = [("min_on_target_ratio", C.c_double), ("min_episode_duration", C.c_double),
                ("target_radius", C.c_double), ("overshoot_window", C.c_int32), ("pad_", C.c_int32)]


class Batch(C.Structure):
    """qt_batch"""

    _fields_ = [("n", C.c_int64), ("motion", C.c_void_p), ("pattern", C.c_void_p), ("plant_mass", C.c_void_p),
                ("hover_thrust", C.c_void_p), ("K", C.c_void_p), ("k_cols", C.c_int32),
                ("k_per_episode", C.c_int32), ("k_structured", C.c_int32), ("k_no_yaw", C.c_int32),
                ("order", C.c_void_p), ("ff", C.c_void_p)]


class State(C.Structure):
    """qt_state"""

    _fields_ = [("x", C.c_void_p), ("integ", C.c_void_p), ("t", C.c_void_p), ("acc", C.c_void_p),
                ("target", C.c_void_p)]


class View(C.Structure):
    """qt_view (ABI 9): element (row r, episode e) at p[r * rs + e * es]"""

    _fields_ = [("p", C.c_void_p), ("rs", C.c_int64), ("es", C.c_int64)]


class ObsView(C.Structure):
    """qt_obs_view (ABI 9)"""

    _fields_ = [(k, View) for k in ("pos", "vel", "tpos", "tvel", "tacc", "time")]


# observation frame (qt_frame_row / qt_frame_count / qt_frame_flag, ABI 9)
FR_ROWS, FC_ROWS, FB_ROWS = 25, 3, 5
FR_X, FR_TARGET, FR_TIME, FR_ERR, FR_REWARD, FR_RATIO = 0, 12, 21, 22, 23, 24
FC_STEP, FC_VIOLATIONS, FC_ON_TARGET = range(FC_ROWS)
FB_DONE, FB_ON_TARGET, FB_VIOLATION, FB_SUCCESS, FB_TERM = range(FB_ROWS)


def frame_bytes(n: int) -> int:
    """QT_FRAME_BYTES(n)"""
    return n * (FR_ROWS * 8 + FC_ROWS * 8 + FB_ROWS)


EXPORTS = ("qt_abi_version", "qt_host_alloc", "qt_host_free", "qt_stream_sync", "qt_seed_draws", "qt_seed_uniform", "qt_reset", "qt_rollout", "qt_rollout_rewards", "qt_rollout_grouped", "qt_rollout_fresh",
           "qt_env_step", "qt_compute_action", "qt_target_state",
           "qt_episode_metrics", "qt_metrics_from_arrays", "qt_dare_batched", "qt_dare_dense", "qt_summary",
           "qt_summary_parts", "qt_summary_numpy", "qt_stream_uniform", "qt_frame_reset", "qt_frame_step",
           "qt_compute_action_obs", "qt_frame_closed_step")

_lib = None


class QuadtrackError(RuntimeError):
    pass


def load():
    """Load libquadtrack.so (raises ImportError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"quadtrack HIP library not built: {LIB_PATH} missing "
                          "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    L = C.CDLL(LIB_PATH)
    P, vp, i32, i64, dbl = C.POINTER, C.c_void_p, C.c_int32, C.c_int64, C.c_double
    L.qt_abi_version.restype = C.c_int
    L.qt_host_alloc.argtypes = [i64, P(vp), P(vp)]
    L.qt_host_free.argtypes = [vp]
    L.qt_stream_sync.argtypes = [vp]
    L.qt_seed_draws.argtypes = [i64, vp, vp, i32, vp, vp, vp]
    L.qt_reset.argtypes = [P(EnvParams), P(Batch), vp, State, vp]
    L.qt_rollout.argtypes = [P(EnvParams), P(CtrlParams), P(Criteria), P(Batch), State, i32, vp, vp]
    L.qt_rollout_rewards.argtypes = [P(EnvParams), P(CtrlParams), P(Criteria), P(Batch), State, i32, vp, vp]
    L.qt_rollout_grouped.argtypes = [P(EnvParams), P(CtrlParams), P(Criteria), P(Batch), State, i32, vp, i32,
                                     P(C.c_int32), P(C.c_int64), vp]
    L.qt_rollout_fresh.argtypes = [P(EnvParams), P(CtrlParams), P(Criteria), P(Batch), vp, State, i32, vp, i32,
                                   P(C.c_int32), P(C.c_int64), vp]
    L.qt_seed_uniform.argtypes = [i64, vp, i32, vp, vp, vp, vp]
    L.qt_env_step.argtypes = [P(EnvParams), P(Batch), vp, State, vp, vp, vp, vp, vp, vp]
    L.qt_compute_action.argtypes = [P(CtrlParams), P(Batch), vp, vp, vp, vp, vp, vp]
    L.qt_target_state.argtypes = [P(EnvParams), P(Batch), vp, vp, vp]
    L.qt_episode_metrics.argtypes = [P(Criteria), i64, vp, vp, vp, vp]
    L.qt_metrics_from_arrays.argtypes = [P(Criteria), i64, i32, vp, vp, vp, vp, vp, vp, vp]
    L.qt_dare_batched.argtypes = [i32, i64, dbl, dbl, vp, vp, vp, i32, vp, vp, vp, vp, vp]
    L.qt_dare_dense.argtypes = [i32, i32, i64, vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]
    L.qt_summary.argtypes = [i64, vp, dbl, dbl, vp, vp]
    L.qt_summary_parts.argtypes = [i64, vp, dbl, dbl, vp, vp, i32, vp]
    L.qt_summary_numpy.argtypes = [i64, vp, i32, dbl, dbl, vp, vp]
    L.qt_stream_uniform.argtypes = [C.c_uint64, i64, i64, i32, vp, vp, vp, vp]
    L.qt_frame_reset.argtypes = [P(EnvParams), P(Batch), vp, vp, vp]
    L.qt_frame_step.argtypes = [P(EnvParams), P(Batch), vp, View, vp, i32, vp]
    L.qt_compute_action_obs.argtypes = [P(CtrlParams), P(Batch), P(ObsView), vp, vp, vp, vp]
    L.qt_frame_closed_step.argtypes = [P(EnvParams), P(CtrlParams), P(Batch), vp, vp, vp, vp, i32, vp]
    for name in EXPORTS[1:]:
        getattr(L, name).restype = C.c_int
    v = L.qt_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"libquadtrack ABI {v} != expected {ABI_VERSION}")
    _lib = L
    return L


def require_gpu(device=None) -> torch.device:
    """The HIP path needs a visible GPU; there is no CPU fallback."""
    if not torch.cuda.is_available():
        raise QuadtrackError("quadtrack runs on MI355X (HIP) only: no GPU is visible")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        raise QuadtrackError(f"quadtrack tensors must live on a GPU, got device {dev}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_of(dev: torch.device):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


try:  # the current stream's handle without building a torch.cuda.Stream object (per-step calls)
    _raw_stream = torch._C._cuda_getCurrentRawStream
except AttributeError:  # pragma: no cover
    _raw_stream = None


def raw_stream(dev: torch.device) -> int:
    """stream_of as a plain int (the per-step API's hot path)."""
    if _raw_stream is not None:
        return _raw_stream(dev.index)
    return torch.cuda.current_stream(dev).cuda_stream


try:  # the current device's ordinal without torch.cuda.current_device()'s lazy-init checks
    _get_device = torch._C._cuda_getDevice
except AttributeError:  # pragma: no cover
    _get_device = None


class _Current:
    """A no-op context: the launch's device is already the current one."""

    __slots__ = ()

    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_CURRENT = _Current()


def on_device(dev: torch.device):
    """`torch.cuda.device(dev)`, or a no-op context when dev is already the
    current device: the per-step API enters it once per launch, and entering
    and leaving torch's context costs ~1.5 us of host time per step
    (profiles/r06/step_host_parts.jsonl), more than the kernel of a
    65,536-episode step takes on the GPU."""
    if _get_device is not None and dev.index is not None and _get_device() == dev.index:
        return _CURRENT
    return torch.cuda.device(dev)


def check(rc: int, what: str):
    if rc != 0:
        raise QuadtrackError(f"{what} failed with status {rc} ({'invalid argument' if rc == -1 else 'HIP launch error'})")
