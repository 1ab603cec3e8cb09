"""Episode sharding with the real kernels: two ranks (gloo) on the one GPU of
the box each run their shard of a batched evaluation; the reduced summary
must equal a single-process run over all episodes."""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N = 3000
CFG = {"target": {"motion_type": "circular"}, "simulation": {"max_episode_time": 5.0}}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "lqr-quadcopter-test_amd"))
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadtrack import evaluate_batched
        from quadtrack.parallel import shard_range

        lo, hi = shard_range(N, rank, world)
        s = evaluate_batched({"dt": 0.01}, CFG, num_episodes=hi - lo, base_seed=0, global_offset=lo,
                             with_episode_metrics=False)
        if rank == 0:
            q.put(s.to_dict())
    finally:
        dist.destroy_process_group()


def test_two_rank_summary_equals_single():
    from quadtrack import evaluate_batched

    ref = evaluate_batched({"dt": 0.01}, CFG, num_episodes=N, base_seed=0, with_episode_metrics=False).to_dict()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    for k in ("total_episodes", "successful_episodes", "best_episode_idx", "worst_episode_idx", "meets_criteria"):
        assert got[k] == ref[k], k
    # numpy-order sums (qt_summary_numpy): shards of 1,500 are not aligned to
    # numpy's 8,192-element blocks, so the rows are gathered and reduced whole
    for k in ("mean_on_target_ratio", "std_on_target_ratio", "mean_tracking_error", "std_tracking_error",
              "mean_control_effort"):
        assert got[k] == ref[k], k
    assert np.isfinite(got["mean_tracking_error"])


# synthetic per-episode metrics: shard layouts aligned to numpy's blocks
# (block sums gathered) and not (rows gathered), 3 ranks
LAYOUTS = {"aligned": [(0, 8192), (8192, 16384), (16384, 19384)], "unaligned": [(0, 6000), (6000, 13001), (13001, 19384)]}


def _synthetic_met(n):
    from quadtrack._abi import MET, MET_ROWS

    rng = np.random.default_rng(3)
    met = np.zeros((MET_ROWS, n))
    met[MET["on_target_ratio"]] = rng.integers(0, 3001, n) / 3000.0
    met[MET["mean_tracking_error"]] = rng.lognormal(size=n)
    met[MET["mean_control_effort"]] = rng.uniform(5, 15, n)
    met[MET["success"]] = rng.integers(0, 2, n)
    return met


def _summary_rank(rank, world, port, layout, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "lqr-quadcopter-test_amd"))
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadtrack.parallel import summary_from_partials
        from quadtrack.utils.metrics import SuccessCriteria

        lo, hi = LAYOUTS[layout][rank]
        met = torch.as_tensor(_synthetic_met(LAYOUTS[layout][-1][1])[:, lo:hi].copy(), device="cuda")
        s = summary_from_partials(met, SuccessCriteria(), global_offset=lo)
        if rank == 0:
            q.put(s.to_dict())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("layout", sorted(LAYOUTS))
def test_sharded_summary_numpy_bitwise(layout):
    from quadtrack._abi import MET

    met = _synthetic_met(LAYOUTS[layout][-1][1])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_summary_rank, args=(r, 3, port, layout, q)) for r in range(3)]
    for p in ps:
        p.start()
    got = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    r, e, u = (met[MET[k]] for k in ("on_target_ratio", "mean_tracking_error", "mean_control_effort"))
    assert (got["mean_on_target_ratio"], got["std_on_target_ratio"]) == (np.mean(r), np.std(r))
    assert (got["mean_tracking_error"], got["std_tracking_error"]) == (np.mean(e), np.std(e))
    assert got["mean_control_effort"] == np.mean(u)
    assert got["best_episode_idx"] == int(np.argmax(r)) and got["worst_episode_idx"] == int(np.argmin(r))


def _rccl_rank(port, q):
    """One rank over RCCL (backend "nccl") on the box's GPU: the summary's
    device all-reduces and all-gather run through RCCL itself."""
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "lqr-quadcopter-test_amd"))
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from quadtrack import evaluate_batched

        assert dist.get_backend() == "nccl"
        s = evaluate_batched({"dt": 0.01}, CFG, num_episodes=N, base_seed=0, with_episode_metrics=False)
        q.put(s.to_dict())
    finally:
        dist.destroy_process_group()


def test_rccl_single_rank_summary_equals_local():
    """The RCCL code path of the metric reduction (one rank: a full RCCL
    communicator on the GPU, collectives on device tensors) gives the
    single-process summary; multi-GPU runs use the same calls."""
    from quadtrack import evaluate_batched

    ref = evaluate_batched({"dt": 0.01}, CFG, num_episodes=N, base_seed=0, with_episode_metrics=False).to_dict()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank, args=(_port(), q))
    p.start()
    got = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    for k, v in ref.items():
        np.testing.assert_allclose(got[k], v, rtol=1e-12, atol=1e-12, err_msg=k)
