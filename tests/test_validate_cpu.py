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
