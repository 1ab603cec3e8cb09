"""Host-side checks of the per-step API's frame layout (quadtrack.step,
include/quadtrack.h qt_frame_row): the views the Python side hands out sit
exactly where the kernels write (QT_FRAME_BYTES), no GPU needed."""

import numpy as np
import pytest
import torch

from quadtrack import _abi
from quadtrack.step import Frame, FramePool, _Out, action_tensor, frame_words, obs_view_of


@pytest.mark.parametrize("n", [0, 1, 7, 64, 1001])
def test_frame_views_follow_the_c_layout(n):
    fr = Frame(n, torch.device("cpu"))
    assert fr.buf.numel() * 8 >= _abi.frame_bytes(n) and frame_words(n) * 8 - _abi.frame_bytes(n) < 8
    base = fr.buf.data_ptr()
    if n == 0:
        return
    # f rows, then the int64 counters, then the int8 flags (QT_FRAME_BYTES order)
    assert fr.f.data_ptr() == base and fr.f.shape == (_abi.FR_ROWS, n)
    assert fr.c.data_ptr() == base + _abi.FR_ROWS * n * 8 and fr.c.dtype == torch.int64
    assert fr.b.data_ptr() == base + (_abi.FR_ROWS + _abi.FC_ROWS) * n * 8 and fr.b.dtype == torch.int8
    # write through raw row offsets, read through the observation / info views
    raw = fr.buf.numpy().view(np.uint8)
    f = raw[:_abi.FR_ROWS * n * 8].view(np.float64).reshape(_abi.FR_ROWS, n)
    f[:] = np.arange(_abi.FR_ROWS * n, dtype=float).reshape(_abi.FR_ROWS, n)
    c = raw[_abi.FR_ROWS * n * 8:(_abi.FR_ROWS + _abi.FC_ROWS) * n * 8].view(np.int64).reshape(_abi.FC_ROWS, n)
    c[:] = np.arange(_abi.FC_ROWS * n).reshape(_abi.FC_ROWS, n)
    b = raw[(_abi.FR_ROWS + _abi.FC_ROWS) * n * 8:_abi.frame_bytes(n)].reshape(_abi.FB_ROWS, n)
    b[:] = 0
    b[_abi.FB_DONE, ::2] = 1
    b[_abi.FB_TERM] = 3
    obs, rew, done, info = fr.step_result()
    np.testing.assert_array_equal(obs["quadcopter"]["position"].numpy(), f[0:3].T)
    np.testing.assert_array_equal(obs["quadcopter"]["angular_velocity"].numpy(), f[9:12].T)
    np.testing.assert_array_equal(obs["target"]["acceleration"].numpy(), f[18:21].T)
    np.testing.assert_array_equal(obs["time"].numpy(), f[_abi.FR_TIME])
    np.testing.assert_array_equal(rew.numpy(), f[_abi.FR_REWARD])
    np.testing.assert_array_equal(info["on_target_ratio"].numpy(), f[_abi.FR_RATIO])
    np.testing.assert_array_equal(info["step"].numpy(), c[_abi.FC_STEP])
    np.testing.assert_array_equal(info["action_violations"].numpy(), c[_abi.FC_VIOLATIONS])
    np.testing.assert_array_equal(done.numpy(), np.arange(n) % 2 == 0)
    assert np.all(info["termination_code"].numpy() == 3)
    # the frame's own qt_obs_view names the same rows as the generic one
    v = fr.obs_view()
    g, _ = obs_view_of(obs, n, torch.device("cpu"), True)
    for k in ("pos", "vel", "tpos", "tvel", "tacc", "time"):
        a, bb = getattr(v, k), getattr(g, k)
        assert (a.p, a.es) == (bb.p, bb.es), k
        if k != "time":
            assert a.rs == bb.rs, k
    assert fr.views_of(obs)
    obs2 = dict(obs)
    obs2["quadcopter"] = dict(obs["quadcopter"], position=obs["quadcopter"]["position"].clone())
    assert not fr.views_of(obs2)


def test_in_place_change_of_an_observation_is_detected():
    fr = Frame(5, torch.device("cpu")).seal()
    obs = fr.observation()
    fr.check_intact()
    obs["target"]["velocity"].mul_(2.0)
    with pytest.raises(RuntimeError, match="modified in place"):
        fr.check_intact()


def test_frame_recyclable_only_when_nothing_is_held():
    """Frame.recyclable (the env's frame pool): true once every tensor a step
    handed out is dropped, false while the caller holds any of them, a dict
    holding them, or a view derived from one."""
    fr = Frame(6, torch.device("cpu")).seal()
    assert not fr.recyclable()  # never handed out: its views are not built yet
    assert fr.act.data_ptr() == fr.buf.data_ptr() + frame_words(6) * 8 and fr.act.shape == (4, 6)

    def hold(pick):
        r = fr.step_result(with_action=True)
        return pick(*r)

    hold(lambda o, r, d, i: None)
    assert fr.recyclable() is True
    for pick in (lambda o, r, d, i: o, lambda o, r, d, i: r, lambda o, r, d, i: d, lambda o, r, d, i: i,
                 lambda o, r, d, i: o["target"], lambda o, r, d, i: o["time"], lambda o, r, d, i: i["action"],
                 lambda o, r, d, i: i["termination_code"], lambda o, r, d, i: o["quadcopter"]["attitude"][:, 1],
                 lambda o, r, d, i: r.view(2, 3), lambda o, r, d, i: [d]):
        kept = hold(pick)
        assert not fr.recyclable()
        del kept
        assert fr.recyclable()
    # a tensor copied out holds nothing
    c = hold(lambda o, r, d, i: o["quadcopter"]["position"].clone())
    assert fr.recyclable() and c.shape == (6, 3)


def test_frame_pool_cycles_released_frames_only():
    """FramePool.take: a loop that drops each step's results cycles through
    two frames; a held Frame object or a held result keeps its frame out."""
    pool = FramePool(4, torch.device("cpu"), size=3)
    cur = None
    seen = []
    for _ in range(6):  # the env's loop: write a frame, hand out its results, drop the last ones
        fr = pool.take(cur)
        out = fr.step_result()
        cur = fr
        seen.append(id(fr))
        del fr, out
    assert len(set(seen)) == 2 and len(pool.frames) == 2
    held = pool.take(cur)  # the caller keeps the Frame object itself
    held.step_result()
    nxt = pool.take(held)
    assert nxt is not held and nxt is not cur
    keep = nxt.step_result()[0]  # ... or an observation
    a = pool.take(nxt)
    assert a is not held and a is not nxt
    assert len(pool.frames) <= 3
    del keep, held, a


def test_action_buffer_reused_only_when_released():
    o = _Out(4, 5, torch.device("cpu"))
    assert o.free() and o.view.shape == (5, 4) and o.view.data_ptr() == o.buf.data_ptr()
    v = o.view
    assert not o.free()
    del v
    w = o.view[:, 0]  # a view derived from the handed-out one
    assert not o.free()
    del w
    assert o.free()


def test_action_tensor_forms():
    dev = torch.device("cpu")
    a = torch.arange(12, dtype=torch.float64).view(4, 3).T  # [3, 4] transpose view
    assert action_tensor(a, 3, dev) is a
    d = action_tensor({"thrust": [1.0, 2.0, 3.0], "yaw_rate": torch.ones(3, dtype=torch.float64)}, 3, dev)
    np.testing.assert_array_equal(d.numpy(), [[1, 0, 0, 1], [2, 0, 0, 1], [3, 0, 0, 1]])
    np.testing.assert_array_equal(action_tensor(np.ones((3, 4)), 3, dev).numpy(), np.ones((3, 4)))
    with pytest.raises(ValueError, match="shape"):
        action_tensor(np.ones((3, 3)), 3, dev)


def test_frame_pool_without_the_storage_use_count(monkeypatch):
    """A torch build without the private torch._C._storage_Use_Count: the
    frame pool and the action buffers fall back to fresh allocations (never
    recycled) instead of failing, and every handed-out view still works."""
    import quadtrack.step as S

    monkeypatch.setattr(S, "_CAN_RECYCLE", False)
    monkeypatch.delattr(torch._C, "_storage_Use_Count")
    pool = FramePool(4, torch.device("cpu"), size=3)
    cur, seen = None, []
    for k in range(5):
        fr = pool.take(cur)
        fr.f.fill_(float(k))
        obs, rew, done, info = fr.seal().step_result(with_action=True)
        assert not fr.recyclable()
        assert torch.equal(obs["quadcopter"]["position"], torch.full((4, 3), float(k), dtype=torch.float64))
        cur = fr
        seen.append(fr)
        del fr, obs, rew, done, info
    assert len({id(f) for f in seen}) == 5  # a new frame every step
    # what an earlier step handed out keeps its values
    for k, f in enumerate(seen):
        assert torch.equal(f.f, torch.full_like(f.f, float(k)))
    o = _Out(4, 3, torch.device("cpu"))
    assert not o.free()


def test_dlpack_export_keeps_the_frame():
    """A DLPack capsule (or a numpy array) of an observation tensor holds the
    frame's storage: the frame is not recycled while the export lives, even
    after the Python view itself is dropped."""
    from torch.utils.dlpack import to_dlpack

    fr = Frame(6, torch.device("cpu")).seal()
    obs = fr.observation()
    cap = to_dlpack(obs["quadcopter"]["velocity"])
    del obs
    assert not fr.recyclable()
    del cap
    assert fr.recyclable()
    arr = fr.step_result()[1].numpy()
    assert not fr.recyclable()
    del arr
    assert fr.recyclable()


def test_on_device_enters_torch_context_only_for_another_device(monkeypatch):
    """_abi.on_device: a no-op context when the launch's device is the current
    one (the per-step hot path), torch.cuda.device otherwise (a
    controller or env on another GPU than the current one)."""
    monkeypatch.setattr(_abi, "_get_device", lambda: 1)
    ctx = _abi.on_device(torch.device("cuda", 1))
    assert ctx is _abi._CURRENT
    with ctx as v:  # enters and leaves without touching the device
        assert v is None
    other = _abi.on_device(torch.device("cuda", 0))
    assert isinstance(other, torch.cuda.device) and other.idx == 0
    # no ordinal query available: always torch's context
    monkeypatch.setattr(_abi, "_get_device", None)
    assert isinstance(_abi.on_device(torch.device("cuda", 1)), torch.cuda.device)


def test_frame_keeps_its_command_pointer_and_storage():
    """Frame.act_ptr is the command rows' address (after the frame words) and
    the kept storage object serves the recycling test."""
    fr = Frame(64, "cpu")
    assert fr.act_ptr == fr.act.data_ptr() == fr.ptr + frame_words(64) * 8
    obs = fr.observation()
    assert not fr.recyclable()  # the observation is held
    del obs
    assert fr.recyclable()
    view = fr.f[0, :8]  # a derived view shares the storage: not recyclable
    assert not fr.recyclable()
    del view
    assert fr.recyclable()
