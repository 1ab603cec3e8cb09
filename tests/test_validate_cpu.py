"""core.validate's host-side checks of a batch before any launch (CPU
tensors: the checks are device-independent).  `order` indexes the state
columns inside the kernels, so anything but a permutation of 0..n-1 must be
refused before a launch."""

import pytest
import torch

from quadtrack import core

F64 = torch.float64


def _batch(n, order=None):
    dev = torch.device("cpu")
    return core.EpisodeBatch(n=n, device=dev, pattern=torch.zeros(4, n, dtype=F64),
                             offset=torch.zeros(3, n, dtype=F64), K=torch.zeros(24, 1, dtype=F64), k_cols=6,
                             order=None if order is None else torch.tensor(order, dtype=torch.int32))


def test_order_permutation_accepted():
    core.validate(_batch(5, [4, 0, 3, 1, 2]))
    core.validate(_batch(3))


@pytest.mark.parametrize("order,msg", [([0, 1, 5], "out of range"), ([0, -1, 2], "out of range"),
                                       ([0, 1, 1], "permutation"), ([2, 2, 2], "permutation")])
def test_order_rejected(order, msg):
    with pytest.raises(ValueError, match=msg):
        core.validate(_batch(3, order))


@pytest.mark.parametrize("order,msg", [([0, 1, 7], "out of range"), ([0, 0, 2], "permutation")])
def test_physical_groups_checks_order(order, msg):
    """A grouped batch is gathered through `order` before any launch: a bad
    order is refused there too (not a device-side index_select assert)."""
    b = _batch(3, order)
    b.groups = (torch.tensor([0], dtype=torch.int32), torch.tensor([3], dtype=torch.int64))
    b.motion = torch.zeros(3, dtype=torch.int8)
    with pytest.raises(ValueError, match=msg):
        b.physical_groups()



@pytest.mark.parametrize("counts", [(640, 128, 0, 64, 192), (400, 400, 400, 400, 400), (65, 0, 0, 0, 0),
                                    (0, 70, 70, 0, 0), (26215, 26215, 26214, 26214, 26214)])
def test_motion_groups_layout(counts):
    """core.motion_groups: one segment per motion present, in GROUP_ORDER
    (longest wave first), each holding exactly that motion's episodes in index
    order; numpy and torch inputs give the same grouping."""
    import numpy as np

    m = np.concatenate([np.full(c, k, np.int8) for k, c in enumerate(counts)])
    m = m[np.random.default_rng(0).permutation(m.size)]
    order, sm, se = core.motion_groups(m)
    assert sm == [k for k in core.group_order() if counts[k]]
    assert se[-1] == m.size and sorted(order.tolist()) == list(range(m.size))
    for k, a, b in zip(sm, [0] + se[:-1], se):
        assert np.array_equal(order[a:b], np.nonzero(m == k)[0])
    to, tsm, tse = core.motion_groups(torch.as_tensor(m))
    assert np.array_equal(to.numpy(), order) and tsm == sm and tse == se


def test_grouped_waves_with_stationary_riders(monkeypatch):
    """core.grouped_waves (qt_rollout.hip grouped_waves): stationary riders
    fill every other group's last wave, so a batch needs ceil(n / 64) waves
    when the stationary group can cover the gaps — config 5's 8-GPU shards
    2,048 (2,050 without riders), the whole config 16,384 (16,385) — and no
    fewer than the groups' own waves otherwise.  QT_RIDERS=0 turns them off."""
    import numpy as np

    from quadtrack import workloads

    def waves(lo, hi, riders=None):
        _, sm, se = core.motion_groups(workloads.motion_of(lo, hi))
        return core.grouped_waves(sm, se, riders)

    for r in range(8):
        lo, hi = workloads.shard_bounds(1048576, r, 8)
        assert (waves(lo, hi, True), waves(lo, hi, False)) == (2048, 2050)
    assert (waves(0, 1048576, True), waves(0, 1048576, False)) == (16384, 16385)
    rng = np.random.default_rng(1)
    for _ in range(200):
        counts = rng.integers(0, 300, size=5)
        sm = [k for k in core.group_order() if counts[k]]
        se = list(np.cumsum([counts[k] for k in sm]))
        own = sum(-(-int(counts[k]) // 64) for k in sm)
        gaps = sum((-int(counts[k])) % 64 for k in sm if k != 0)
        w = core.grouped_waves(sm, se, True)
        assert w >= -(-int(counts.sum()) // 64) and w <= own
        if counts[0] >= gaps:
            assert w == -(-int(counts.sum()) // 64)
    monkeypatch.setenv("QT_RIDERS", "0")
    assert core.grouped_waves(*core.motion_groups(workloads.motion_of(0, 131072))[1:]) == 2050


def test_pair_rounds_layout():
    """core.motion_groups with resident_waves (core.pair_rounds): a batch of
    one resident set has the group holding its middle wave split there at a
    wave boundary, the second part moved to the end; every segment is one
    motion, the order a permutation, the wave count unchanged; a batch beyond
    one resident set, or whose middle falls on a group boundary or in the
    stationary group, keeps the plain layout."""
    import numpy as np

    from quadtrack import workloads

    for lo, hi, split in ((0, 131072, True), (917504, 1048576, True), (0, 1048576, False), (0, 1100, True),
                          (777777, 778477, False), (0, 64, False)):
        m = workloads.motion_of(lo, hi)
        order, sm, se = core.motion_groups(m, 2048)
        po, psm, pse = core.motion_groups(m)
        assert sorted(order.tolist()) == list(range(hi - lo))
        start = 0
        for k, e in zip(sm, se):
            assert np.all(m[order[start:e]] == k)
            start = e
        assert core.grouped_waves(sm, se) == core.grouped_waves(psm, pse)
        assert (len(sm) == len(psm) + 1) == split, (lo, hi, sm)
        if split:
            assert sm[-1] == sm[len(psm) // 2] and sm[:len(psm)] == psm  # [3, 4, 2, 1, 0] + [2]
            half = core.grouped_waves(psm, pse) // 2
            first = sum(-(-(b - a) // 64) for a, b in zip([0] + se[:len(psm) // 2], se[:len(psm) // 2 + 1]))
            assert first == half
    counts = [5000, 0, 0, 300, 0]  # the middle in the stationary group, which is never split
    m = np.concatenate([np.full(c, k, np.int8) for k, c in enumerate(counts)])
    order, sm, se = core.motion_groups(m, 2048)
    assert sm == [3, 0]
    counts = [300, 0, 0, 5000, 0]  # the middle inside the long group: its second part after the stationary one
    m = np.concatenate([np.full(c, k, np.int8) for k, c in enumerate(counts)])
    order, sm, se = core.motion_groups(m, 2048)
    assert sm == [3, 0, 3] and se[0] == 41 * 64


def test_group_order_knob_is_validated_when_used(monkeypatch):
    """QT_GROUP_ORDER (an A/B knob) is read when a grouping is made: a
    malformed value raises there with the variable named, and never breaks
    the import of quadtrack.core."""
    import os
    import subprocess
    import sys

    import numpy as np

    from conftest import ROOT

    env = dict(os.environ, QT_GROUP_ORDER="3,,4",
               PYTHONPATH=os.path.join(ROOT, "lqr-quadcopter-test_amd") + os.pathsep + os.environ.get("PYTHONPATH", ""))
    subprocess.run([sys.executable, "-c", "import quadtrack.core"], env=env, check=True)
    monkeypatch.setenv("QT_GROUP_ORDER", "3,,4")
    with pytest.raises(ValueError, match="QT_GROUP_ORDER"):
        core.motion_groups(np.array([0, 1, 2], dtype=np.int8))
    monkeypatch.setenv("QT_GROUP_ORDER", "0,1,2,3,3")
    with pytest.raises(ValueError, match="QT_GROUP_ORDER"):
        core.group_order()
    monkeypatch.setenv("QT_GROUP_ORDER", "0,1,2,3,4")
    assert core.group_order() == (0, 1, 2, 3, 4)
    monkeypatch.delenv("QT_GROUP_ORDER")
    assert core.group_order() == core.DEFAULT_GROUP_ORDER
