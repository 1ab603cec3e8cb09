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


def _check_groups(m, order, seg_motion, seg_end):
    import numpy as np

    o = np.asarray(order.cpu() if isinstance(order, torch.Tensor) else order)
    assert sorted(o.tolist()) == list(range(m.size))
    starts = [0] + list(seg_end[:-1])
    for k, a, b in zip(seg_motion, starts, seg_end):
        if k >= 0:
            assert np.all(m[o[a:b]] == k)
            if seg_motion[-1] == -1:
                assert (b - a) % core.WAVE == 0
    assert seg_end[-1] == m.size
    assert all(k >= 0 for k in seg_motion[:-1])


@pytest.mark.parametrize("counts,tail", [((640, 128, 0, 64, 192), False),   # whole waves only
                                         ((400, 400, 400, 400, 400), True),  # 5 remainders of 16: 2 tail waves
                                         ((65, 0, 0, 0, 0), False),          # one motion
                                         ((70, 70, 0, 0, 0), True),          # 2 remainders of 6 -> 1 wave: packed
                                         ((100, 60, 0, 0, 0), False),        # 36 + 60 -> 2 waves: no gain
                                         ((26215, 26214, 26214, 26214, 26214), True)])
def test_motion_groups_layout(counts, tail):
    """core.motion_groups: stable per-motion groups; when the groups'
    remainders pack into fewer waves than one per motion, each group keeps
    its whole waves and the remainders form a mixed tail (seg_motion -1,
    last).  numpy and torch inputs give the same grouping."""
    import numpy as np

    m = np.concatenate([np.full(c, k, np.int8) for k, c in enumerate(counts)])
    m = m[np.random.default_rng(0).permutation(m.size)]
    order, sm, se = core.motion_groups(m)
    _check_groups(m, order, sm, se)
    to, tsm, tse = core.motion_groups(torch.as_tensor(m))
    assert np.array_equal(np.asarray(to), order) and tsm == sm and tse == se
    assert (sm[-1] == -1) == tail
    if sm[-1] == -1:
        rem = sum(c % core.WAVE for c in counts)
        assert se[-1] - (se[-2] if len(se) > 1 else 0) == rem
