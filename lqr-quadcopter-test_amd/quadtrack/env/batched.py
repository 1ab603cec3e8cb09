"""Batched quadcopter environment on the GPU.

`BatchedQuadcopterEnv(n, config)` holds n independent episodes in HBM and
exposes the reference's reset / step API (env/quadcopter_env.py:111-232) on
tensors.  Each call is one kernel launch (include/quadtrack.h ABI 9):

  reset(seeds)   qt_seed_draws + qt_frame_reset (numpy default_rng(seed)'s
                 draws on the device, quadcopter_env.py:111-150)
  step(actions)  qt_frame_step: action validation, RK4 / Euler, state
                 constraints, post-step tracking error, reward, termination,
                 info, for every episode (quadcopter_env.py:152-293)
  step_closed(controller)
                 qt_frame_closed_step: the controller's compute_action on the
                 current observation, then the step, in one launch

Every step writes an observation frame (quadtrack.step.Frame); the returned
observation / reward / done / info tensors are views of it.  No later step
writes a frame whose tensors the caller still holds (Frame.recyclable), so
what the caller keeps stays as it was, as the reference's observation arrays
are fresh copies (quadcopter_env.py:481-486); a loop that drops them cycles
through a small pool of frames.  The next step reads its state from the last
frame, so writing into the returned tensors in place would change the
environment: the env detects that (the views share one version counter) and
raises instead.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .. import _abi, core
from .._abi import FB_DONE, FR_X, MOTIONS, check, on_device, raw_stream
from ..step import Frame, FramePool, action_tensor
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
    """n QuadcopterEnv episodes stepped together.

    motion      per-episode motion types (names or enum indices; default the config's)
    mass        per-episode plant mass (default the config's)
    freeze_done True (default): an episode that is done is not stepped again,
                its observation and info stay those of its last step (the
                Evaluator stops stepping at done, eval.py:119-165); False:
                every episode is stepped on every call, as the reference's
                env steps after done.
    """

    STATE_DIM = 12
    ACTION_DIM = 4

    def __init__(self, num_envs: int, config=None, device=None, motion=None, mass=None, freeze_done: bool = True):
        if num_envs < 0:
            raise ValueError("num_envs must be >= 0")
        self.config = as_env_config(config)
        self.params = self.config.to_params()
        self.num_envs = int(num_envs)
        self.device = _abi.require_gpu(device)
        self.freeze_done = bool(freeze_done)
        n, dev = self.num_envs, self.device
        self.motion = None
        if motion is not None:
            self.motion = torch.as_tensor(motion_indices(motion, n), device=dev)
        self.plant_mass = None if mass is None else core.to_device(np.broadcast_to(np.asarray(mass, float), (n,)), dev)
        self.pattern: torch.Tensor | None = None
        self.offset: torch.Tensor | None = None
        self._frame: Frame | None = None
        self._pool = FramePool(self.num_envs, self.device)  # the frames steps write
        self._env_ref = C.byref(self.params)
        self._batch = None
        self._closed = None  # (controller, its qt_batch, byref) of step_closed

    # ---------------------------------------------------------------- reset
    def reset_from_draws(self, pattern, offset):
        """Reset every episode from explicit draws: pattern [4, n], offset [3, n]."""
        n, dev = self.num_envs, self.device
        self.pattern = core.to_device(pattern, dev)
        self.offset = core.to_device(offset, dev)
        core._check_cols("pattern", self.pattern, 4, n)
        core._check_cols("offset", self.offset, 3, n)
        b = _abi.Batch()
        b.n = n
        b.motion = None if self.motion is None else self.motion.data_ptr()
        b.pattern = self.pattern.data_ptr()
        b.plant_mass = None if self.plant_mass is None else self.plant_mass.data_ptr()
        self._batch = b
        self._batch_ref = C.byref(b)
        self._closed = None
        self._frame = None
        fr = self._next_frame()
        with torch.cuda.device(dev):
            check(_abi.load().qt_frame_reset(self._env_ref, self._batch_ref, self.offset.data_ptr(), fr.ptr,
                                             raw_stream(dev)), "qt_frame_reset")
        self._frame = fr.seal()
        return fr.observation()

    def reset(self, seeds=None):
        """QuadcopterEnv.reset(seed) for every episode: seeds [n] (default
        config.seed + arange(n)).  Returns the observation dict ([n, 3] tensors)."""
        if seeds is None:
            seeds = self.config.seed + np.arange(self.num_envs)
        seeds = np.asarray(seeds.cpu() if isinstance(seeds, torch.Tensor) else seeds, dtype=np.int64).reshape(-1)
        if seeds.size != self.num_envs:
            raise ValueError(f"{seeds.size} seeds for {self.num_envs} episodes")
        kinds = self.motion if self.motion is not None else self.config.motion_index()
        pat, off = seeding.draws(kinds, seeds, self.device)
        return self.reset_from_draws(pat, off)

    # ----------------------------------------------------------------- step
    def _next_frame(self) -> Frame:
        """The frame the next step writes (FramePool.take: never one the caller
        holds, nor the current one, which the step reads)."""
        return self._pool.take(self._frame)

    def _current(self) -> Frame:
        fr = self._frame
        if fr is None:
            raise RuntimeError("Environment not initialized. Call reset() first.")
        fr.check_intact()
        return fr

    def step(self, actions):
        """actions [n, 4] (thrust, roll, pitch, yaw rates; any strides, e.g. a
        controller's output) or a dict of [n] tensors -> (obs, reward [n],
        done [n] bool, info dict of [n] tensors)."""
        fr = self._current()
        n, dev = self.num_envs, self.device
        a = action_tensor(actions, n, dev)
        out = self._next_frame()
        with on_device(dev):
            check(_abi.load().qt_frame_step(self._env_ref, self._batch_ref, fr.ptr,
                                            _abi.View(a.data_ptr(), a.stride(1), a.stride(0)), out.ptr,
                                            int(self.freeze_done), raw_stream(dev)), "qt_frame_step")
        self._frame = out.seal()
        return out.step_result()

    def step_closed(self, controller):
        """One closed-loop step in ONE launch: `controller.compute_action` on
        the current observation, then `step` with its command
        (qt_frame_closed_step).  Same results as
        `env.step(controller.compute_action(obs))`; info["action"] holds the
        command ([n, 4]).  With freeze_done, a done episode's controller state
        is not advanced."""
        fr = self._current()
        n, dev = self.num_envs, self.device
        if controller.device != dev:
            raise ValueError(f"the controller is on {controller.device}, the environment on {dev}")
        cb = self._closed_batch(controller)
        integ = controller._state_for(n)
        out = self._next_frame()
        with on_device(dev):
            check(_abi.load().qt_frame_closed_step(
                self._env_ref, controller._ctrl_ref, cb, fr.ptr, None if integ is None else integ.data_ptr(),
                out.ptr, out.act_ptr, int(self.freeze_done), raw_stream(dev)), "qt_frame_closed_step")
        self._frame = out.seal()
        return out.step_result(with_action=True)

    def _closed_batch(self, controller):
        """qt_batch of the env's episodes with the controller's gains (cached)."""
        controller.c_batch(self.num_envs)
        key = (controller, controller._cb)
        if self._closed is None or self._closed[0] != key:
            b = _abi.Batch()
            C.memmove(C.addressof(b), C.addressof(controller._cb), C.sizeof(b))  # gains, hover, feed-forward
            b.n = self.num_envs
            b.motion, b.pattern, b.plant_mass = self._batch.motion, self._batch.pattern, self._batch.plant_mass
            self._closed = (key, b, C.byref(b))
        return self._closed[2]

    # ---------------------------------------------------------- observation
    def observation(self) -> dict:
        """The current observation (views of the last frame)."""
        return self._current().observation()

    @property
    def done(self) -> torch.Tensor:
        return self._current().b[FB_DONE].view(torch.bool)

    def get_state_vector(self) -> torch.Tensor:
        return self._current().f[FR_X:FR_X + 12].T.clone()

    def set_state_vector(self, x) -> None:
        """Replace every episode's 12-state (the observation after this call sees it)."""
        fr = self._current()
        x = torch.as_tensor(x, dtype=F64, device=self.device)
        if x.shape != (self.num_envs, self.STATE_DIM):
            raise ValueError(f"State must have shape ({self.num_envs}, {self.STATE_DIM}), got {tuple(x.shape)}")
        out = Frame(self.num_envs, self.device)
        out.buf.copy_(fr.buf)
        out.f[FR_X:FR_X + 12].copy_(x.T)
        self._frame = out.seal()

    @property
    def frame(self) -> Frame:
        return self._current()

    @property
    def time(self) -> torch.Tensor:
        return self._current().f[_abi.FR_TIME].clone()

    @property
    def dt(self) -> float:
        return self.config.simulation.dt
