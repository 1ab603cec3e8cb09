"""Device-side batch containers and thin launchers over the C ABI.

All arrays are structure-of-arrays float64 tensors in HBM ([rows][n], one
column per episode), the layout the kernels read coalesced (one lane per
episode).  Every launcher is asynchronous on the current torch stream of the
batch's device.
"""

from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _abi
from ._abi import ACC_ROWS, MET_ROWS, Batch, Criteria, CtrlParams, EnvParams, State, check, ptr, stream_of

F64 = torch.float64


def criteria(min_on_target_ratio=0.8, min_episode_duration=30.0, target_radius=0.5, window=10) -> Criteria:
    """utils/metrics.py SuccessCriteria defaults (26-39) + detect_overshoots window (208)."""
    return Criteria(float(min_on_target_ratio), float(min_episode_duration), float(target_radius), int(window), 0)


@dataclass
class EpisodeBatch:
    """Per-episode inputs (qt_batch)."""

    n: int
    device: torch.device
    pattern: torch.Tensor                     # [4, n] raw draws
    offset: torch.Tensor                      # [3, n]
    K: torch.Tensor                           # [4*k_cols, n] or [4*k_cols, 1] ([9, .] for PID)
    k_cols: int                               # 6 LQR | 9 LQI | 3 PID (gains kp, ki, kd)
    motion: torch.Tensor | None = None        # [n] int8
    plant_mass: torch.Tensor | None = None    # [n]
    hover: torch.Tensor | None = None         # [n]
    order: torch.Tensor | None = None         # [n] int32
    k_structured: bool = False                # every off-axis K entry is exactly zero
    k_no_yaw: bool = False                    # the yaw-rate row of K is exactly zero
    groups: tuple | None = None               # (seg_motion, seg_end): `order` groups slots by motion
    ff: torch.Tensor | None = None            # [7, n] per-episode feed-forward (qt_batch.ff, ff_rows)

    def c_batch(self, with_k=True) -> Batch:
        b = Batch()
        b.n = self.n
        b.motion = ptr(self.motion)
        b.pattern = ptr(self.pattern)
        b.plant_mass = ptr(self.plant_mass)
        b.hover_thrust = ptr(self.hover)
        b.K = ptr(self.K) if with_k else None
        b.k_cols = self.k_cols
        b.k_per_episode = int(self.K.shape[1] != 1)
        b.k_structured = int(self.k_structured)
        b.k_no_yaw = int(self.k_no_yaw)
        b.order = ptr(self.order)
        b.ff = ptr(self.ff)
        return b

    def select(self, idx: torch.Tensor) -> "EpisodeBatch":
        """The sub-batch of episodes `idx` (int64 on the device), in that order:
        the same inputs column for column, runtime motion (no grouping)."""
        idx = idx.to(device=self.device, dtype=torch.int64)
        col = lambda t: None if t is None else t.index_select(-1, idx).contiguous()  # noqa: E731
        K = self.K if self.K.shape[1] == 1 else col(self.K)
        return EpisodeBatch(n=idx.numel(), device=self.device, pattern=col(self.pattern), offset=col(self.offset), K=K,
                            k_cols=self.k_cols, motion=col(self.motion), plant_mass=col(self.plant_mass),
                            hover=col(self.hover), k_structured=self.k_structured,
                            k_no_yaw=self.k_no_yaw, ff=col(self.ff))

    def physical_groups(self) -> tuple["EpisodeBatch", torch.Tensor]:
        """For a motion-grouped batch (`order` + `groups`): a copy whose
        per-episode arrays are stored in slot order (the groups contiguous, order
        = None), so the grouped rollout and every kernel around it read and write
        whole coalesced rows instead of gathering through `order` (config 5: the
        gathered state traffic was ~5x the algorithmic bytes).  Returns (copy,
        perm) with perm[slot] = episode; results of the copy map back with
        `unpermute`."""
        if self.order is None or self.groups is None:
            raise ValueError("physical_groups needs a grouped batch (order and groups)")
        validate(self)  # the gather below trusts `order`: a permutation of 0..n-1, checked first
        perm = self.order.to(torch.int64)
        col = lambda t: None if t is None else t.index_select(-1, perm).contiguous()  # noqa: E731
        K = self.K if self.K.shape[1] == 1 else col(self.K)
        return EpisodeBatch(n=self.n, device=self.device, pattern=col(self.pattern), offset=col(self.offset), K=K,
                            k_cols=self.k_cols, motion=col(self.motion), plant_mass=col(self.plant_mass),
                            hover=col(self.hover), order=None, k_structured=self.k_structured,
                            k_no_yaw=self.k_no_yaw, groups=self.groups, ff=col(self.ff)), perm


def unpermute(t: torch.Tensor, perm: torch.Tensor) -> torch.Tensor:
    """Columns (last axis) of a slot-ordered result back to episode order:
    out[..., perm[slot]] = t[..., slot]."""
    out = torch.empty_like(t)
    out.index_copy_(t.dim() - 1, perm, t)
    return out


@dataclass
class RolloutState:
    """Mutable per-episode state (qt_state)."""

    x: torch.Tensor       # [12, n]
    integ: torch.Tensor   # [4, n]: LQI integral (rows 0-2) | PID integral error + last observation time
    t: torch.Tensor       # [n]
    acc: torch.Tensor     # [ACC_ROWS, n]
    target: torch.Tensor  # [9, n]

    @classmethod
    def empty(cls, n: int, device) -> "RolloutState":
        z = lambda *s: torch.zeros(*s, dtype=F64, device=device)  # noqa: E731
        return cls(z(12, n), z(INTEG_ROWS, n), z(n), z(ACC_ROWS, n), z(9, n))

    def c_state(self) -> State:
        s = State()
        s.x, s.integ, s.t, s.acc, s.target = (ptr(v) for v in (self.x, self.integ, self.t, self.acc, self.target))
        return s


INTEG_ROWS = 4
FF_ROWS = 7


def ff_rows(m: int, device, enabled=True, velocity_gain=0.0, acceleration_gain=0.0, max_velocity=10.0,
            off=None) -> torch.Tensor:
    """Per-episode feed-forward parameters (qt_batch.ff, [7, m]): velocity gain
    xyz, acceleration gain xyz, target-velocity clamp.  velocity_gain /
    acceleration_gain: scalar, [3] or [m, 3]; enabled: bool or [m]; off: [m]
    bool (or None) of episodes that run without feed-forward — gains 0 and no
    clamp, the identity (the heuristic fallback of a failed DARE,
    riccati_lqr.py:764-776)."""
    vg = np.broadcast_to(np.asarray(velocity_gain, float).reshape(-1, 3) if np.ndim(velocity_gain) else
                         np.full(3, float(velocity_gain)), (m, 3))
    ag = np.broadcast_to(np.asarray(acceleration_gain, float).reshape(-1, 3) if np.ndim(acceleration_gain) else
                         np.full(3, float(acceleration_gain)), (m, 3))
    rows = np.empty((FF_ROWS, m))
    rows[0:3] = vg.T
    rows[3:6] = ag.T
    rows[6] = np.broadcast_to(np.asarray(max_velocity, float), (m,))
    dis = ~np.broadcast_to(np.asarray(enabled, bool), (m,))
    if off is not None:
        dis = dis | np.asarray(off, bool).reshape(m)
    rows[:, dis] = 0.0
    rows[6, dis] = np.inf
    return torch.as_tensor(rows, dtype=F64, device=device).contiguous()


def gain_rows(k_cols: int) -> int:
    """Rows of the SoA gain array: 4 x k_cols, or kp/ki/kd (9) for PID."""
    return 9 if k_cols == 3 else 4 * k_cols


_AXIS_PATTERN = {6: [(0, 2), (0, 5), (1, 1), (1, 4), (2, 0), (2, 3)]}
_AXIS_PATTERN[9] = _AXIS_PATTERN[6] + [(0, 8), (1, 7), (2, 6)]


def gains_structured(K: torch.Tensor, k_cols: int) -> bool:
    """True when every entry of K ([4*k_cols, m]) outside the per-axis pattern
    is exactly zero (qt_batch.k_structured).  PID gains (k_cols 3) are
    per-axis by construction."""
    if k_cols == 3:
        return True
    mask = torch.ones(4 * k_cols, dtype=torch.bool, device=K.device)
    for r, c in _AXIS_PATTERN[k_cols]:
        mask[r * k_cols + c] = False
    return bool((K[mask] == 0).all().item())


def gains_no_yaw(K: torch.Tensor, k_cols: int) -> bool:
    """True when the yaw-rate row of K ([4*k_cols, m], row 3) is exactly zero
    (qt_batch.k_no_yaw): the DARE gains always (B has no yaw column), the
    heuristic LQR always (controllers/__init__.py:560-574), PID by design."""
    if k_cols == 3:
        return True
    return bool((K[3 * k_cols:4 * k_cols] == 0).all().item())


class MappedBlock:
    """Page-locked host memory mapped into the device address space
    (qt_host_alloc): numpy views on the host side, device pointers for the
    kernels, no copies.  `take` carves 64-byte aligned arrays out of it.
    Used by the batch-1 drop-in objects, whose every call is one launch and
    one stream sync (QuadcopterEnv, the one-episode controllers)."""

    def __init__(self, nbytes: int):
        self._lib = _abi.load()
        host, dev = C.c_void_p(), C.c_void_p()
        check(self._lib.qt_host_alloc(int(nbytes), C.byref(host), C.byref(dev)), "qt_host_alloc")
        self.host, self.dev, self.nbytes, self._off = host.value, dev.value, int(nbytes), 0
        self._raw = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.host))

    def take(self, shape, dtype=np.float64):
        """A zeroed array of `shape` and its device address."""
        dt = np.dtype(dtype)
        size = int(np.prod(shape)) * dt.itemsize
        off = self._off
        if off + size > self.nbytes:
            raise ValueError("MappedBlock exhausted")
        self._off = (off + size + 63) & ~63
        return self._raw[off:off + size].view(dt).reshape(shape), C.c_void_p(self.dev + off)

    def __del__(self, _vp=C.c_void_p):  # bound at definition: module globals may be gone at interpreter exit
        if getattr(self, "host", None):
            self._lib.qt_host_free(_vp(self.host))
            self.host = None


def sync(stream) -> None:
    check(_abi.load().qt_stream_sync(stream), "qt_stream_sync")


def to_device(a, device, dtype=F64) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.require(a, requirements=["C", "W"]), dtype=dtype, device=device).contiguous()


def _check_cols(name, t, rows, n):
    if t is not None and (t.dim() != 2 or t.shape[0] != rows or t.shape[1] != n or not t.is_contiguous()):
        raise ValueError(f"{name} must be a contiguous [{rows}, {n}] tensor, got {tuple(t.shape)}")


def validate(batch: EpisodeBatch, st: RolloutState | None = None):
    """Host-side shape checks before any launch (the kernels index [rows][n])."""
    n = batch.n
    _check_cols("pattern", batch.pattern, 4, n)
    _check_cols("offset", batch.offset, 3, n)
    _check_cols("ff", batch.ff, FF_ROWS, n)
    if batch.k_cols not in (3, 6, 9):
        raise ValueError("k_cols must be 3 (PID), 6 (LQR) or 9 (LQI)")
    rows = gain_rows(batch.k_cols)
    if batch.K.dim() != 2 or batch.K.shape[0] != rows or batch.K.shape[1] not in (1, n):
        raise ValueError(f"K must be [{rows}, 1 or {n}], got {tuple(batch.K.shape)}")
    for name in ("motion", "plant_mass", "hover", "order"):
        t = getattr(batch, name)
        if t is not None and (t.numel() != n or not t.is_contiguous()):
            raise ValueError(f"{name} must have {n} contiguous entries")
    if batch.motion is not None and (int(batch.motion.min()) < 0 or int(batch.motion.max()) > 4):
        raise ValueError("motion types must be in 0..4")
    if st is not None:
        _check_cols("x", st.x, 12, n)
        _check_cols("integ", st.integ, INTEG_ROWS, n)
        _check_cols("acc", st.acc, ACC_ROWS, n)
        _check_cols("target", st.target, 9, n)
        if st.t.numel() != n:
            raise ValueError("t must have n entries")
    for t in (batch.pattern, batch.offset, batch.K, batch.plant_mass, batch.hover, batch.ff):
        if t is not None and (t.device != batch.device or t.dtype != F64):
            raise ValueError("batch tensors must be float64 on the batch device")
    # the kernels read these through raw pointers: dtypes are part of the ABI
    if batch.motion is not None and (batch.motion.dtype != torch.int8 or batch.motion.device != batch.device):
        raise ValueError("motion must be an int8 tensor on the batch device")
    if batch.order is not None:
        if batch.order.dtype != torch.int32 or batch.order.device != batch.device:
            raise ValueError("order must be an int32 tensor on the batch device")
        if n:
            # the kernels index st.x[i * n + order[slot]]: a permutation of 0..n-1, checked
            # with one bincount (no sort) and one host read
            o = batch.order.to(torch.int64)
            lo, hi = o.min(), o.max()
            ok = (lo >= 0) & (hi < n)
            perm = ok & (torch.bincount(o.clamp(0, n - 1), minlength=n) == 1).all()
            ok, perm = (bool(v) for v in torch.stack([ok, perm]).tolist())
            if not ok:
                raise ValueError("order entries out of range")
            if not perm:
                raise ValueError("order must be a permutation of the episodes")


def seed_draws(seeds: torch.Tensor, motion: torch.Tensor | None, motion_default: int):
    """Device reset draws: seeds int64 [n] -> (pattern [4, n], offset [3, n])."""
    lib = _abi.load()
    n, dev = seeds.numel(), seeds.device
    if seeds.dtype != torch.int64 or not seeds.is_contiguous():
        raise ValueError("seeds must be a contiguous int64 tensor")
    if n and int(seeds.min()) < 0:
        raise ValueError("seeds must be non-negative (numpy SeedSequence)")
    pat = torch.empty(4, n, dtype=F64, device=dev)
    off = torch.empty(3, n, dtype=F64, device=dev)
    with torch.cuda.device(dev):
        check(lib.qt_seed_draws(n, ptr(seeds), ptr(motion), int(motion_default), ptr(pat), ptr(off),
                                stream_of(dev)), "qt_seed_draws")
    return pat, off


def reset(env: EnvParams, batch: EpisodeBatch, st: RolloutState):
    lib = _abi.load()
    with torch.cuda.device(batch.device):
        check(lib.qt_reset(C.byref(env), C.byref(batch.c_batch(with_k=False)), ptr(batch.offset), st.c_state(),
                           stream_of(batch.device)), "qt_reset")


def rollout(env: EnvParams, ctrl: CtrlParams, crit: Criteria, batch: EpisodeBatch, st: RolloutState, nsteps: int,
            rec: torch.Tensor | None = None):
    lib = _abi.load()
    if rec is not None and (rec.numel() < nsteps * 16 * batch.n or rec.dtype != F64):
        raise ValueError("rec must hold nsteps * 16 * n float64")
    with torch.cuda.device(batch.device):
        if batch.groups is not None:
            seg_motion, seg_end = batch.groups
            nseg = len(seg_motion)
            sm = (C.c_int32 * nseg)(*[int(v) for v in seg_motion])
            se = (C.c_int64 * nseg)(*[int(v) for v in seg_end])
            check(lib.qt_rollout_grouped(C.byref(env), C.byref(ctrl), C.byref(crit), C.byref(batch.c_batch()),
                                         st.c_state(), int(nsteps), ptr(rec), nseg, sm, se,
                                         stream_of(batch.device)), "qt_rollout_grouped")
        else:
            check(lib.qt_rollout(C.byref(env), C.byref(ctrl), C.byref(crit), C.byref(batch.c_batch()), st.c_state(),
                                 int(nsteps), ptr(rec), stream_of(batch.device)), "qt_rollout")


def rollout_fresh(env: EnvParams, ctrl: CtrlParams, crit: Criteria, batch: EpisodeBatch, st: RolloutState,
                  nsteps: int, met: torch.Tensor | None = None) -> torch.Tensor:
    """reset -> rollout(nsteps) -> episode_metrics as one launch set
    (qt_rollout_fresh, ABI 8): the rollout kernel forms the reset state from
    batch.offset in its prologue and writes the metrics rows in its epilogue.
    Same results as the three calls, bit for bit.  Returns met [MET_ROWS, n]."""
    lib = _abi.load()
    n = batch.n
    if met is None:
        met = torch.empty(MET_ROWS, n, dtype=F64, device=batch.device)
    elif met.dtype != F64 or not met.is_contiguous() or tuple(met.shape) != (MET_ROWS, n):
        raise ValueError("met must be a contiguous float64 [MET_ROWS, n] tensor")
    nseg, sm, se = 0, None, None
    if batch.groups is not None:
        seg_motion, seg_end = batch.groups
        nseg = len(seg_motion)
        sm = (C.c_int32 * nseg)(*[int(v) for v in seg_motion])
        se = (C.c_int64 * nseg)(*[int(v) for v in seg_end])
    with torch.cuda.device(batch.device):
        check(lib.qt_rollout_fresh(C.byref(env), C.byref(ctrl), C.byref(crit), C.byref(batch.c_batch()),
                                   ptr(batch.offset), st.c_state(), int(nsteps), ptr(met), nseg, sm, se,
                                   stream_of(batch.device)), "qt_rollout_fresh")
    return met


def rollout_rewards(env: EnvParams, ctrl: CtrlParams, crit: Criteria, batch: EpisodeBatch, st: RolloutState,
                    nsteps: int, reward: torch.Tensor):
    """qt_rollout_rewards: the exact-step rollout that also accumulates
    reward[0] += -(post-step tracking error) per step and keeps the last one in
    reward[1] (reward: float64 [2, n], zeroed before the first chunk)."""
    lib = _abi.load()
    if reward.dtype != F64 or not reward.is_contiguous() or tuple(reward.shape) != (2, batch.n):
        raise ValueError("reward must be a contiguous float64 [2, n] tensor")
    if batch.groups is not None:
        raise ValueError("rollout_rewards takes an ungrouped batch (motion per episode is fine)")
    with torch.cuda.device(batch.device):
        check(lib.qt_rollout_rewards(C.byref(env), C.byref(ctrl), C.byref(crit), C.byref(batch.c_batch()),
                                     st.c_state(), int(nsteps), ptr(reward), stream_of(batch.device)),
              "qt_rollout_rewards")


# Slot order of the motion groups in a grouped rollout: longest wave first
# (sinusoidal, figure-8, circular, linear, stationary: the per-motion loops'
# wave times in config 5, profiles/r04/cfg5_stamps.json), so that the long
# waves start first and the short ones fill the end of the launch (config 5:
# 131,072 episodes 4.35 -> 3.93 ms, 1,048,576 23.5 -> 23.1 ms,
# profiles/r04/grouping_ab.jsonl).  QT_GROUP_ORDER (a comma list of the five
# motion types) is an A/B knob, read and validated when a grouping is made.
DEFAULT_GROUP_ORDER = (3, 4, 2, 1, 0)


def group_order() -> tuple:
    """The motion groups' slot order: QT_GROUP_ORDER if set, else
    DEFAULT_GROUP_ORDER; a malformed value raises here (not at import)."""
    raw = os.environ.get("QT_GROUP_ORDER")
    if raw is None or raw.strip() == "":
        return DEFAULT_GROUP_ORDER
    try:
        order = tuple(int(v) for v in raw.split(","))
    except ValueError:
        raise ValueError(f"QT_GROUP_ORDER={raw!r} is not a comma list of the motion types 0..4") from None
    if sorted(order) != [0, 1, 2, 3, 4]:
        raise ValueError(f"QT_GROUP_ORDER={raw!r} is not an order of the motion types 0..4")
    return order


def motion_groups(motion, resident_waves: int | None = None):
    """Grouping for qt_rollout_grouped: (order int32 [n], seg_motion, seg_end).
    A device tensor of motion types is grouped on the device (stable sort, one
    5-element read back); a numpy array on the host.  Groups follow
    group_order(); within a group, episodes keep their index order.

    resident_waves (the waves the grouped kernel holds at once on the device:
    2 per SIMD): a batch of at most that many waves runs as one resident set,
    its first half of the waves the first on their SIMDs and the second half
    beside them; the group straddling the middle is then split at it and its
    second part moved to the end (pair_rounds), so that the second half opens
    with the short groups instead of the rest of a long one (config 5's 8-GPU
    shard, 2,048 waves: 2.91-2.95 -> 2.85-2.86 ms, profiles/r06/order_ab.jsonl)."""
    order, kinds, ends = _motion_groups(motion)
    if resident_waves:
        order, kinds, ends = pair_rounds(order, kinds, ends, resident_waves)
    return order, kinds, ends


def pair_rounds(order, kinds, ends, resident_waves: int):
    """motion_groups' layout for a batch that fits one resident set: the
    group holding the middle wave (grouped_waves' layout, riders included)
    split there at a wave boundary and its second part moved to the end
    (<= 8 segments, each a whole motion; the stationary group is not split,
    its riders keep filling the other groups' last waves)."""
    total = grouped_waves(kinds, ends)
    if total > resident_waves or len(kinds) >= 8 or total < 4:
        return order, kinds, ends
    half, w, start = total // 2, 0, 0
    for i, (k, e) in enumerate(zip(kinds, ends)):
        cnt = e - start
        own = (cnt + 63) // 64
        if w + own > half:
            if k == 0 or w == half:
                return order, kinds, ends
            cut = start + (half - w) * 64  # whole waves of this group before the middle
            if cut <= start or cut >= e:
                return order, kinds, ends
            if isinstance(order, torch.Tensor):
                new = torch.cat([order[:cut], order[e:], order[cut:e]])
            else:
                new = np.concatenate([order[:cut], order[e:], order[cut:e]])
            counts = [b - a for a, b in zip([0] + list(ends[:-1]), ends)]
            seq = list(zip(kinds[:i], counts[:i])) + [(k, cut - start)] + list(zip(kinds[i + 1:], counts[i + 1:])) \
                + [(k, e - cut)]
            return new, [m for m, _ in seq], [int(v) for v in np.cumsum([c for _, c in seq])]
        w += own
        start = e
    return order, kinds, ends


def _motion_groups(motion):
    GROUP_ORDER = group_order()
    pos = np.empty(5, np.int64)
    pos[list(GROUP_ORDER)] = np.arange(5)
    if isinstance(motion, torch.Tensor):
        m = motion.reshape(-1).to(torch.int64)
        order = torch.argsort(torch.as_tensor(pos, device=m.device)[m], stable=True).to(torch.int32)
        counts = torch.bincount(m, minlength=5).cpu().numpy()
    else:
        m = np.asarray(motion).reshape(-1).astype(np.intp)
        order = np.argsort(pos[m], kind="stable").astype(np.int32)
        counts = np.bincount(m, minlength=5)  # motion types 0..4: O(n), no sort
    kinds = [k for k in GROUP_ORDER if counts[k]]
    return order, kinds, [int(v) for v in np.cumsum(counts[kinds])]


def resident_grouped_waves(device) -> int | None:
    """Waves the grouped kernel holds at once on `device`: 2 per SIMD
    (QT_GROUPED_WAVES), 4 SIMDs per compute unit.  None (no round pairing in
    motion_groups) with QT_PAIR_ROUNDS=0, an A/B knob."""
    if os.environ.get("QT_PAIR_ROUNDS") == "0":
        return None
    return torch.cuda.get_device_properties(device).multi_processor_count * 4 * 2


def riders_on() -> bool:
    """Stationary riders in the one-launch grouped rollout (qt_rollout.hip
    riders_on): on unless QT_RIDERS=0."""
    return os.environ.get("QT_RIDERS") != "0"


def grouped_waves(seg_motion, seg_end, riders: bool | None = None) -> int:
    """The waves of the one-launch grouped rollout of a batch grouped as
    (seg_motion, seg_end) — qt_rollout.hip grouped_waves restated: with
    riders, the first episodes of the stationary group fill the free lanes of
    every other group's last wave, so the stationary group's own waves hold
    only the rest.  (For reports and tests; the kernel's layout is the C
    side's.)"""
    riders = riders_on() if riders is None else riders
    cnt, prev = [], 0
    for m, e in zip(seg_motion, seg_end):
        if e - prev > 0:
            cnt.append([int(m), int(e - prev), 0])  # motion, own episodes, riders
        prev = e
    stat = next((i for i, c in enumerate(cnt) if c[0] == 0), None)
    if len(cnt) > 8:  # more groups than the one-launch form takes: one launch set per group, no riders
        riders = False
    if riders and stat is not None:
        avail = cnt[stat][1]
        for i, c in enumerate(cnt):
            if i != stat:
                take = min((64 - c[1] % 64) % 64, avail)
                c[2], avail = take, avail - take
        cnt[stat][1] = avail
    return sum((own + rid + 63) // 64 for _, own, rid in cnt)


def launch_waves(batch: EpisodeBatch) -> int:
    """Waves of a rollout launch over `batch`: the grouped layout's
    (grouped_waves) for a motion-grouped batch with per-episode motions,
    ceil(n / 64) otherwise."""
    if batch.groups is not None:
        return grouped_waves(*batch.groups, riders=None if batch.motion is not None else False)
    return (batch.n + 63) // 64


def seed_uniform(seeds: torch.Tensor, lo, hi) -> torch.Tensor:
    """First k draws of default_rng(seed).uniform(lo[j], hi[j]) per seed -> [k, n]."""
    lib = _abi.load()
    n, dev = seeds.numel(), seeds.device
    if seeds.dtype != torch.int64 or not seeds.is_contiguous():
        raise ValueError("seeds must be a contiguous int64 tensor")
    if n and int(seeds.min()) < 0:
        raise ValueError("seeds must be non-negative (numpy SeedSequence)")
    lo_t = to_device(np.atleast_1d(np.asarray(lo, float)), dev)
    hi_t = to_device(np.atleast_1d(np.asarray(hi, float)), dev)
    if lo_t.numel() != hi_t.numel() or lo_t.numel() > 64:
        raise ValueError("lo and hi must have the same length k <= 64")
    out = torch.empty(lo_t.numel(), n, dtype=F64, device=dev)
    with torch.cuda.device(dev):
        check(lib.qt_seed_uniform(n, ptr(seeds), lo_t.numel(), ptr(lo_t), ptr(hi_t), ptr(out), stream_of(dev)),
              "qt_seed_uniform")
    return out


def stream_uniform(seed: int, first: int, n: int, lo, hi, device) -> torch.Tensor:
    """Draw vectors first .. first+n-1 of default_rng(seed).uniform(lo, hi,
    size=(., k)) -> [k, n] on the device (qt_stream_uniform)."""
    lib = _abi.load()
    if seed < 0 or first < 0 or n < 0:
        raise ValueError("seed, first and n must be non-negative")
    lo_t = to_device(np.atleast_1d(np.asarray(lo, float)), device)
    hi_t = to_device(np.atleast_1d(np.asarray(hi, float)), device)
    if lo_t.numel() != hi_t.numel() or lo_t.numel() > 64:
        raise ValueError("lo and hi must have the same length k <= 64")
    out = torch.empty(lo_t.numel(), n, dtype=F64, device=device)
    with torch.cuda.device(device):
        check(lib.qt_stream_uniform(int(seed), int(first), int(n), lo_t.numel(), ptr(lo_t), ptr(hi_t), ptr(out),
                                    stream_of(device)), "qt_stream_uniform")
    return out


def episode_metrics(crit: Criteria, st: RolloutState) -> torch.Tensor:
    lib = _abi.load()
    n = st.t.numel()
    met = torch.empty(MET_ROWS, n, dtype=F64, device=st.t.device)
    with torch.cuda.device(st.t.device):
        check(lib.qt_episode_metrics(C.byref(crit), n, ptr(st.acc), ptr(st.t), ptr(met), stream_of(st.t.device)),
              "qt_episode_metrics")
    return met


def summary_parts_for(n: int) -> int:
    """Workgroups of the summary reduction: ~1,024 episodes each, at most 1,024."""
    return max(1, min(1024, -(-n // 1024)))


def summary_partials(met: torch.Tensor, mu_ratio=0.0, mu_err=0.0, nparts: int | None = None) -> torch.Tensor:
    """[sum ratio, sum err, sum effort, sum success, count, M2 ratio, M2 err, max, argmax, min, argmin]
    (qt_summary_parts; nparts = 1 is the single-workgroup qt_summary)."""
    lib = _abi.load()
    n = met.shape[1]
    nparts = summary_parts_for(n) if nparts is None else int(nparts)
    out = torch.empty(11, dtype=F64, device=met.device)  # the final reduction writes all 11
    with torch.cuda.device(met.device):
        if nparts == 1:
            check(lib.qt_summary(n, ptr(met), float(mu_ratio), float(mu_err), ptr(out), stream_of(met.device)),
                  "qt_summary")
        else:
            work = torch.empty(nparts * 11, dtype=F64, device=met.device)
            check(lib.qt_summary_parts(n, ptr(met), float(mu_ratio), float(mu_err), ptr(out), ptr(work), nparts,
                                       stream_of(met.device)), "qt_summary_parts")
    return out


NP_BLOCK = 8192  # numpy's reduction block (elements), qt_summary_numpy


def summary_numpy_blocks(met: torch.Tensor, pass_: int, mu_ratio=0.0, mu_err=0.0) -> torch.Tensor:
    """Per-block pairwise sums in numpy's order (qt_summary_numpy): pass 0 ->
    [3, nblocks] (ratio, mean_err, mean_effort), pass 1 -> [2, nblocks] of the
    squared deviations from (mu_ratio, mu_err).  Folding a row in block order
    from 0.0 gives np.add.reduce of it bit for bit (np_fold)."""
    lib = _abi.load()
    if met.dim() != 2 or met.shape[0] != _abi.MET_ROWS or met.dtype != F64 or not met.is_contiguous():
        raise ValueError("met must be a contiguous float64 [MET_ROWS, n] tensor")
    if pass_ not in (0, 1):
        raise ValueError("pass_ must be 0 (sums) or 1 (squared deviations)")
    n = met.shape[1]
    nb = -(-n // NP_BLOCK)
    out = torch.empty(3 if pass_ == 0 else 2, nb, dtype=F64, device=met.device)
    if n:
        with torch.cuda.device(met.device):
            check(lib.qt_summary_numpy(n, ptr(met), int(pass_), float(mu_ratio), float(mu_err), ptr(out),
                                       stream_of(met.device)), "qt_summary_numpy")
    return out


def np_fold(blocks) -> float:
    """numpy's running total over block sums (in order, from 0.0)."""
    s = 0.0
    for v in blocks:
        s += float(v)
    return s


def dare_batched(n_state: int, dt: float, gravity: float, mass: torch.Tensor | None, Q: torch.Tensor,
                 R: torch.Tensor, structured: bool):
    """Q [n_state*n_state, m], R [16, m] SoA -> (K [4*n_state, m], P [n_state^2, m], status int8 [m], iters int32 [m])."""
    lib = _abi.load()
    m = Q.shape[1]
    dev = Q.device
    if Q.shape[0] != n_state * n_state or R.shape != (16, m):
        raise ValueError("Q must be [n*n, m] and R [16, m]")
    if mass is not None and mass.numel() != m:
        raise ValueError("mass must have m entries")
    K = torch.empty(4 * n_state, m, dtype=F64, device=dev)
    P = torch.empty(n_state * n_state, m, dtype=F64, device=dev)
    status = torch.empty(m, dtype=torch.int8, device=dev)
    iters = torch.empty(m, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        check(lib.qt_dare_batched(n_state, m, float(dt), float(gravity), ptr(mass), ptr(Q), ptr(R), int(structured),
                                  ptr(K), ptr(P), ptr(status), ptr(iters), stream_of(dev)), "qt_dare_batched")
    return K, P, status, iters


def dare_dense(A: torch.Tensor, B: torch.Tensor, Q: torch.Tensor, R: torch.Tensor, ab_per_problem: bool):
    """General DARE: A [n*n, m'], B [n*p, m'], Q [n*n, m], R [p*p, m] SoA (m' = m or 1)."""
    lib = _abi.load()
    m = Q.shape[1]
    n = int(round(Q.shape[0] ** 0.5))
    p = int(round(R.shape[0] ** 0.5))
    dev = Q.device
    K = torch.empty(p * n, m, dtype=F64, device=dev)
    P = torch.empty(n * n, m, dtype=F64, device=dev)
    status = torch.empty(m, dtype=torch.int8, device=dev)
    iters = torch.empty(m, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        check(lib.qt_dare_dense(n, p, m, ptr(A), ptr(B), int(ab_per_problem), ptr(Q), ptr(R), ptr(K), ptr(P),
                                ptr(status), ptr(iters), stream_of(dev)), "qt_dare_dense")
    return K, P, status, iters


def target_state(env: EnvParams, batch: EpisodeBatch, t: torch.Tensor) -> torch.Tensor:
    lib = _abi.load()
    out = torch.empty(9, batch.n, dtype=F64, device=batch.device)
    with torch.cuda.device(batch.device):
        check(lib.qt_target_state(C.byref(env), C.byref(batch.c_batch(with_k=False)), ptr(t), ptr(out),
                                  stream_of(batch.device)), "qt_target_state")
    return out


def env_step(env: EnvParams, batch: EpisodeBatch, action: torch.Tensor, st: RolloutState):
    """Open-loop step; returns (err[n], on_target[n] bool, done[n] bool, term[n] int8, violation[n] bool)."""
    lib = _abi.load()
    n, dev = batch.n, batch.device
    _check_cols("action", action, 4, n)
    err = torch.empty(n, dtype=F64, device=dev)
    on = torch.empty(n, dtype=torch.int8, device=dev)
    done = torch.empty(n, dtype=torch.int8, device=dev)
    term = torch.empty(n, dtype=torch.int8, device=dev)
    viol = torch.empty(n, dtype=torch.int8, device=dev)
    with torch.cuda.device(dev):
        check(lib.qt_env_step(C.byref(env), C.byref(batch.c_batch(with_k=False)), ptr(action), st.c_state(), ptr(err),
                              ptr(on), ptr(done), ptr(term), ptr(viol), stream_of(dev)), "qt_env_step")
    return err, on.bool(), done.bool(), term, viol.bool()


def compute_action(ctrl: CtrlParams, K: torch.Tensor, k_cols: int, obs: torch.Tensor, integ: torch.Tensor,
                   hover: torch.Tensor | None = None, diag: torch.Tensor | None = None,
                   ff: torch.Tensor | None = None):
    """obs [15, n] -> (action [4, n], saturated [n] bool); integ [3, n] updated in place (LQI);
    diag [16, n] (optional) receives the control components.  PID (k_cols 3): obs [16, n] with the
    observation time in row 15, integ [4, n] (integral error, last time), diag [18, n]."""
    lib = _abi.load()
    n, dev = obs.shape[1], obs.device
    _check_cols("obs", obs, 16 if k_cols == 3 else 15, n)
    if K.dim() != 2 or K.shape[0] != gain_rows(k_cols) or K.shape[1] not in (1, n):
        raise ValueError(f"K must be [{gain_rows(k_cols)}, 1 or {n}], got {tuple(K.shape)}")
    if k_cols != 6 and (integ is None or integ.shape[0] < (4 if k_cols == 3 else 3) or integ.shape[-1] != n):
        raise ValueError("integ must be [3, n] (LQI) or [4, n] (PID)")
    if diag is not None:
        _check_cols("diag", diag, 18 if k_cols == 3 else 16, n)
    b = Batch()
    b.n = n
    b.K = ptr(K)
    b.k_cols = k_cols
    b.k_per_episode = int(K.shape[1] != 1)
    b.hover_thrust = ptr(hover)
    if ff is not None:
        _check_cols("ff", ff, FF_ROWS, n)
    b.ff = ptr(ff)
    act = torch.empty(4, n, dtype=F64, device=dev)
    sat = torch.empty(n, dtype=torch.int8, device=dev)
    with torch.cuda.device(dev):
        check(lib.qt_compute_action(C.byref(ctrl), C.byref(b), ptr(obs), ptr(integ), ptr(act), ptr(sat), ptr(diag),
                                    stream_of(dev)), "qt_compute_action")
    return act, sat.bool()


def metrics_from_arrays(crit: Criteria, qpos: torch.Tensor, tpos: torch.Tensor, actions: torch.Tensor,
                        steps: torch.Tensor, last_time: torch.Tensor) -> torch.Tensor:
    """qpos/tpos [S, 3, n], actions [S, 4, n], steps int32 [n], last_time [n] -> met [MET_ROWS, n]."""
    lib = _abi.load()
    S, _, n = qpos.shape
    dev = qpos.device
    met = torch.empty(MET_ROWS, n, dtype=F64, device=dev)
    with torch.cuda.device(dev):
        check(lib.qt_metrics_from_arrays(C.byref(crit), n, S, ptr(qpos), ptr(tpos), ptr(actions), ptr(steps),
                                         ptr(last_time), ptr(met), stream_of(dev)), "qt_metrics_from_arrays")
    return met
