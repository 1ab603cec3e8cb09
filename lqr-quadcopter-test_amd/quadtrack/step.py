"""The per-step API on tensors (include/quadtrack.h ABI 9).

The reference drives its plugins one step at a time from Python
(`action = ctrl.compute_action(obs); obs, r, done, info = env.step(action)`,
eval.py:119-165, controllers/tuning.py:885-906, train.py:600-619).  The fused
rollout (quadtrack.rollout) replaces that whole loop by one kernel launch;
this module serves callers that keep the loop: every step is ONE kernel
launch over the batch, and what it returns is views, not copies.

* A `Frame` is one step's output (quadtrack.h qt_frame_row): the state, the
  target observation and the info values of every episode in one contiguous
  SoA block.  The observation dict holds [n, 3] views of it (strides (1, n)),
  the info dict [n] views.  A step never writes a frame any of whose
  tensors the caller still holds (Frame.recyclable), so an observation the
  caller keeps never changes, as the reference's fresh-copy arrays do not
  (quadcopter_env.py:481-486); a loop that drops them cycles through two
  frames whose views are built once.
* Views, not transposes: `qt_view` passes any [n, k] tensor layout to the
  kernels by its strides, so the controller reads an observation in place
  and the env reads an action in place (an [n, 4] transpose of the
  controller's [4][n] output, or a caller's contiguous [n, 4] array).

A closed-loop step through the two plugin calls is two launches
(qt_compute_action_obs, qt_frame_step); `BatchedQuadcopterEnv.step_closed`
is one (qt_frame_closed_step).
"""

from __future__ import annotations

import ctypes as C
import sys

import numpy as np
import torch

from . import _abi
from ._abi import (FB_DONE, FB_ROWS, FB_TERM, FC_ROWS, FR_ROWS, FR_TIME, Batch, ObsView, View, check, on_device,
                   raw_stream)

F64 = torch.float64


def frame_words(n: int) -> int:
    """float64 elements of a frame of n episodes (QT_FRAME_BYTES rounded up)."""
    return (FR_ROWS + FC_ROWS) * n + (FB_ROWS * n + 7) // 8


class Observation(dict):
    """The observation dict of a batched step (quadcopter_env.py:472-496 with
    [n, 3] / [n] tensors): a plain dict that also knows the frame it views,
    so a batched controller can pass the frame to its kernel directly."""

    __slots__ = ("frame",)


_CAN_RECYCLE = hasattr(torch._C, "_storage_Use_Count")


def _stor_uses(stor) -> int:
    """Tensors (views included) sharing the storage `stor` — an object the
    caller keeps for this count (Frame._stor, _Out._stor), so it includes
    that object; 0 on a torch build without the (private) use count, whose
    frames and action buffers are then never recycled (_CAN_RECYCLE)."""
    if not _CAN_RECYCLE:
        return 0
    return torch._C._storage_Use_Count(stor._cdata)


class Frame:
    """One step's observation + info block (qt_frame_row): f [25, n] float64,
    c [3, n] int64, b [5, n] int8 views of one device allocation, followed
    by the [4, n] command rows of a closed-loop step (`act`).

    The tensors a step hands out are built once per frame (`_views`).  A
    frame is `recyclable` — a later step may write it again — only when
    nothing outside holds any of it: every handed-out view is back to the
    Python reference count the frame itself holds, and no other tensor
    (a slice, a reshape) shares its storage.  So a caller that keeps an
    observation, a reward, an info value or a view derived from one keeps
    it unchanged, as with a fresh frame; a loop that drops them lets the
    env cycle through two frames without allocating or building views.

    What a held tensor pins: every reward, done, info or observation tensor
    is a view of the whole frame, so holding one keeps the frame's
    QT_FRAME_BYTES(n) (229 B per episode) plus its 32 B of command rows alive
    and out of the recycling cycle.  A loop that keeps a value of every step
    (the reference Evaluator keeps each step's reward and info,
    eval.py:139-159) should keep `value.clone()` (8 B per episode), not the
    view: 65,536 episodes x 3,000 steps of held views would pin ~51 GB where
    clones take ~1.5 GB."""

    __slots__ = ("n", "buf", "f", "c", "b", "act", "ptr", "act_ptr", "version", "_q", "_obs_view", "_views",
                 "_refs", "_uses", "_info", "_stor")

    def __init__(self, n: int, device):
        self.n = n
        fw = frame_words(n)
        self.buf = torch.empty(fw + 4 * n, dtype=F64, device=device)
        f, c, b, a = self.buf.split([FR_ROWS * n, FC_ROWS * n, fw - (FR_ROWS + FC_ROWS) * n, 4 * n])
        self.f = f.view(FR_ROWS, n)
        self.c = c.view(torch.int64).view(FC_ROWS, n)
        self.b = b.view(torch.int8)[:FB_ROWS * n].view(FB_ROWS, n)
        self.act = a.view(4, n)
        self.ptr = self.buf.data_ptr()
        self.act_ptr = self.act.data_ptr()
        # the buffer's storage object, held for its use count (_stor_uses)
        self._stor = self.buf.untyped_storage() if _CAN_RECYCLE else None
        self.version = None  # buf._version once a kernel has written it (seal)
        self._q = None
        self._obs_view = None
        self._views = None
        self._info = None

    def seal(self) -> "Frame":
        """Mark the frame as written: a later in-place change of any of its views
        (which share the buffer's version counter) is detected by `check_intact`."""
        self.version = self.buf._version
        return self

    def check_intact(self) -> None:
        if self.buf._version != self.version:
            raise RuntimeError("the observation of the last step was modified in place; its tensors are views of "
                               "the environment state (clone() them before writing into them)")

    # --------------------------------------------------------------- views
    def _quantities(self):
        if self._q is None:
            # rows 0..20 as seven [n, 3] views: position, velocity, attitude,
            # angular velocity, target position, velocity, acceleration; then time
            self._q = self.f[:21].view(7, 3, self.n).transpose(1, 2).unbind(0) + (self.f[FR_TIME],)
        return self._q

    def observation(self) -> Observation:
        if self._views is None:
            self._build_views()
            self._snapshot()
        q = self._q
        obs = Observation(quadcopter={"position": q[0], "velocity": q[1], "attitude": q[2],
                                      "angular_velocity": q[3]},
                          target={"position": q[4], "velocity": q[5], "acceleration": q[6]},
                          time=q[7])
        obs.frame = self
        return obs

    def _build_views(self):
        q = self._quantities()
        t, err, rew, ratio = self.f[FR_TIME:FR_TIME + 4].unbind(0)
        step, viol, on_count = self.c.unbind(0)
        done, on, violation, success = self.b[:FB_TERM].view(torch.bool).unbind(0)
        self._info = (("time", t), ("step", step), ("tracking_error", err), ("on_target", on),
                      ("on_target_ratio", ratio), ("action_violations", viol), ("termination_code", self.b[FB_TERM]),
                      ("episode_length", t), ("success", success), ("violation", violation),
                      ("on_target_count", on_count))
        # every tensor a step hands out: reward, done, the command, the observation, the info values
        self._views = (rew, done, self.act.T) + q + tuple(v for _, v in self._info)

    def _counts(self):
        return list(map(sys.getrefcount, self._views))

    def _snapshot(self):
        # what the frame itself holds (called with no other reference alive)
        self._refs = self._counts()
        self._uses = _stor_uses(self._stor)

    def recyclable(self) -> bool:
        """True when no view of this frame is held outside it (see the class doc)."""
        return (self._views is not None and _CAN_RECYCLE and _stor_uses(self._stor) == self._uses
                and self._counts() == self._refs)

    def step_result(self, with_action: bool = False):
        """(obs, reward [n], done [n] bool, info) of QuadcopterEnv.step
        (quadcopter_env.py:152-232).  info holds every key the reference's
        info has, as [n] tensors; termination_code / success / episode_length
        are meaningful where done (the reference adds them only then).
        with_action: info["action"] is the [n, 4] command of a closed-loop step."""
        obs = self.observation()
        v = self._views
        info = dict(self._info)
        if with_action:
            info["action"] = v[2]
        return obs, v[0], v[1], info

    def obs_view(self) -> ObsView:
        """The qt_obs_view of this frame's observation (built once)."""
        if self._obs_view is None:
            n, p, es = self.n, self.ptr, 1
            v = ObsView()
            for k, row in (("pos", 0), ("vel", 3), ("tpos", 12), ("tvel", 15), ("tacc", 18)):
                setattr(v, k, View(p + row * n * 8, n, es))
            v.time = View(p + FR_TIME * n * 8, n, es)
            self._obs_view = v
        return self._obs_view

    def views_of(self, obs) -> bool:
        """True when `obs` holds exactly this frame's observation tensors."""
        q = self._quantities()
        try:
            oq, ot = obs["quadcopter"], obs["target"]
            return (oq["position"] is q[0] and oq["velocity"] is q[1] and ot["position"] is q[4]
                    and ot["velocity"] is q[5] and ot.get("acceleration") is q[6] and obs.get("time") is q[7])
        except (KeyError, TypeError):
            return False


class FramePool:
    """The frames an env's steps write (BatchedQuadcopterEnv): `take(cur)`
    returns a frame that nothing outside the pool holds — neither the Frame
    object (e.g. `env.frame`, `obs.frame`) nor any tensor it handed out
    (Frame.recyclable) — other than `cur`, the frame the step reads; else a
    new one.  The pool keeps `size` frames and forgets the oldest held one
    past that (its holder owns it)."""

    def __init__(self, n: int, device, size: int = 3):
        self.n, self.device, self.size = n, device, size
        self.frames: list[Frame] = []

    @staticmethod
    def _own_refs(items) -> int:
        # the reference count of an item nothing else holds, seen from take()'s
        # loop (the list, the loop variable, getrefcount's argument: 3 on CPython)
        for it in items:
            return sys.getrefcount(it)
        return 0

    _OWN = None

    def take(self, cur: Frame | None) -> Frame:
        if FramePool._OWN is None:
            FramePool._OWN = self._own_refs([object()])
        own = FramePool._OWN
        for fr in self.frames:
            if fr is not cur and sys.getrefcount(fr) == own and fr.recyclable():
                return fr
        fr = Frame(self.n, self.device)
        if len(self.frames) >= self.size:
            self.frames.remove(next(f for f in self.frames if f is not cur))
        self.frames.append(fr)
        return fr


class _Out:
    """A [rows, n] output buffer handed out as its [n, rows] transpose;
    reusable once released (no reference to the view, no other tensor on
    the storage), as Frame.recyclable."""

    __slots__ = ("buf", "view", "_ref", "_uses", "_stor")

    def __init__(self, rows: int, n: int, device):
        self.buf = torch.empty(rows, n, dtype=F64, device=device)
        self.view = self.buf.T
        self._stor = self.buf.untyped_storage() if _CAN_RECYCLE else None  # as Frame._stor
        self._ref = sys.getrefcount(self.view)
        self._uses = _stor_uses(self._stor)

    def free(self) -> bool:
        return _CAN_RECYCLE and sys.getrefcount(self.view) == self._ref and _stor_uses(self._stor) == self._uses


def tensor_view(t: torch.Tensor, rows: int, n: int, name: str, device) -> View:
    """qt_view of an [n, rows] float64 tensor on `device` (any strides)."""
    if not isinstance(t, torch.Tensor) or t.dtype != F64 or t.device != device or tuple(t.shape) != (n, rows):
        raise ValueError(f"{name} must be a float64 [{n}, {rows}] tensor on {device}")
    return View(t.data_ptr(), t.stride(1), t.stride(0))


def action_tensor(actions, n: int, device) -> torch.Tensor:
    """env.step's action argument as an [n, 4] float64 tensor on the device:
    a tensor of that shape passes as it is (any strides); a dict of
    {thrust, roll_rate, pitch_rate, yaw_rate} ([n] each, missing keys 0, as
    quadcopter_env.py:249-257) or an array is gathered once."""
    if isinstance(actions, torch.Tensor) and actions.dtype == F64 and actions.device == device:
        a = actions
    elif isinstance(actions, dict):
        z = torch.zeros(n, dtype=F64, device=device)
        cols = [actions.get(k) for k in ("thrust", "roll_rate", "pitch_rate", "yaw_rate")]
        a = torch.stack([z if v is None else torch.as_tensor(v, dtype=F64, device=device).reshape(n)
                         for v in cols], dim=1)
    else:
        a = torch.as_tensor(actions.cpu() if isinstance(actions, torch.Tensor) else np.asarray(actions, np.float64),
                            dtype=F64).to(device)
    if a.dim() != 2 or tuple(a.shape) != (n, 4):
        raise ValueError(f"Action array must have shape ({n}, 4), got {tuple(a.shape)}")
    return a


def obs_view_of(obs, n: int, device, with_time: bool):
    """qt_obs_view of any observation dict of [n, 3] float64 device tensors."""
    q, tg = obs["quadcopter"], obs["target"]
    v = ObsView()
    v.pos = tensor_view(q["position"], 3, n, "position", device)
    v.vel = tensor_view(q["velocity"], 3, n, "velocity", device)
    v.tpos = tensor_view(tg["position"], 3, n, "target position", device)
    v.tvel = tensor_view(tg["velocity"], 3, n, "target velocity", device)
    acc = tg.get("acceleration")
    v.tacc = View(None, 0, 0) if acc is None else tensor_view(acc, 3, n, "target acceleration", device)
    if with_time:
        t = obs["time"]
        if not isinstance(t, torch.Tensor):
            t = torch.full((n,), float(t), dtype=F64, device=device)
        if t.dtype != F64 or t.device != device or t.numel() != n:
            raise ValueError(f"time must be a float64 [{n}] tensor on {device}")
        t = t.reshape(n)
        v.time = View(t.data_ptr(), 0, t.stride(0))
        return v, t
    v.time = View(None, 0, 0)
    return v, None


class BatchedControlMixin:
    """`compute_action(obs)` / `reset(n)` on tensors for the batched
    controllers (BatchedRiccatiLQR, BatchedLQR, BatchedPID): the plugin call
    of controllers/base.py:83-135 for n episodes at once, one launch
    (qt_compute_action_obs).  Returns the actions as an [n, 4] tensor (a view
    of the kernel's [4][n] output, owned by the caller).  Controller state
    (LQI integral, PID integral and last observation time) is kept per
    episode in `integral_state` and cleared by `reset` (riccati_lqr.py:1073-1086,
    controllers/__init__.py:389-393)."""

    integral_state: torch.Tensor | None = None

    def _integ_rows(self) -> int:
        return 4 if self.k_cols == 3 else (3 if self.k_cols == 9 else 0)

    def reset(self, n: int | None = None) -> None:
        n = n or self.num_problems
        rows = max(self._integ_rows(), 3)
        st = torch.zeros(rows, n, dtype=F64, device=self.device)
        if self.k_cols == 3:
            st[3] = float("nan")  # PID: no previous observation time (None)
        self.integral_state = st

    def c_batch(self, n: int) -> Batch:
        """The controller half of a qt_batch (gains, hover thrust, feed-forward)."""
        if self.per_episode and n != self.num_problems:
            raise ValueError(f"{n} observations for {self.num_problems} per-episode gain sets")
        cb = getattr(self, "_cb", None)
        hover, ff = self.hover, getattr(self, "ff", None)
        if cb is None or cb.n != n or cb.K != self.K.data_ptr() or self._cb_key != (
                id(self.ctrl), None if hover is None else hover.data_ptr(), None if ff is None else ff.data_ptr()):
            cb = Batch()
            cb.n = n
            cb.K = self.K.data_ptr()
            cb.k_cols = self.k_cols
            cb.k_per_episode = int(self.K.shape[1] != 1)
            cb.k_structured = int(bool(getattr(self, "k_structured", False)))
            cb.k_no_yaw = 0
            cb.hover_thrust = None if hover is None else hover.data_ptr()
            cb.ff = None if ff is None else ff.data_ptr()
            self._cb = cb
            self._cb_key = (id(self.ctrl), cb.hover_thrust, cb.ff)
            self._cb_ref = C.byref(cb)
            self._ctrl_ref = C.byref(self.ctrl)
        return cb

    def _state_for(self, n: int):
        if self.k_cols == 6:
            return None
        if self.integral_state is None or self.integral_state.shape[1] != n:
            self.reset(n)
        return self.integral_state

    def compute_action(self, obs) -> torch.Tensor:
        """Batched compute_action: obs from BatchedQuadcopterEnv (or any dict
        of [n, 3] float64 device tensors).  Returns actions [n, 4]."""
        n = obs["quadcopter"]["position"].shape[0]
        self.c_batch(n)
        fr = getattr(obs, "frame", None)
        keep = None
        if fr is not None and fr.n == n and fr.views_of(obs):
            if fr.buf.device != self.device:
                raise ValueError(f"the observation is on {fr.buf.device}, the controller on {self.device}")
            v = fr.obs_view()
        else:
            v, keep = obs_view_of(obs, n, self.device, self.k_cols == 3)
        integ = self._state_for(n)
        out = self._action_out(n)
        with on_device(self.device):  # the launch's stream and pointers are this device's
            check(_abi.load().qt_compute_action_obs(self._ctrl_ref, self._cb_ref, C.byref(v),
                                                    None if integ is None else integ.data_ptr(), out.buf.data_ptr(),
                                                    None, raw_stream(self.device)), "qt_compute_action_obs")
        del keep
        return out.view

    def _action_out(self, n: int) -> _Out:
        """An action buffer the caller no longer holds (the last step's command
        once env.step has taken it), else a new one; at most three are kept."""
        outs = self.__dict__.setdefault("_outs", [])
        if outs and outs[0].buf.shape[1] != n:
            outs.clear()
        for o in outs:
            if o.free():
                return o
        o = _Out(4, n, self.device)
        if len(outs) >= 3:
            outs.pop(0)
        outs.append(o)
        return o


def frame_done(fr: Frame) -> torch.Tensor:
    return fr.b[FB_DONE].view(torch.bool)
