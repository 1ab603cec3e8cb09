"""Multi-process (gloo, world_size 2 and 3) checks of the episode sharding and
the metric exchange, on CPU.  The per-rank partial statistics are computed
with numpy here (the GPU kernel that produces them is covered by the gpu
tests); what is tested is that sharding + the collectives reproduce the
single-process EvaluationSummary (utils/metrics.py:341-390) exactly."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from quadtrack.parallel import all_gather_rows, all_reduce_sum, pick_extremes, shard_range, summary_from_stats


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n):
    rng = np.random.default_rng(11)
    ratio = np.round(rng.uniform(0, 1, n), 2)  # many ties -> exercises first-occurrence argmax
    err = rng.uniform(0, 5, n)
    eff = rng.uniform(9, 11, n)
    succ = (ratio >= 0.8).astype(float)
    return ratio, err, eff, succ


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ratio, err, eff, succ = _data(n)
        lo, hi = shard_range(n, rank, world)
        r, e = ratio[lo:hi], err[lo:hi]
        sums = torch.tensor([r.sum(), e.sum(), eff[lo:hi].sum(), succ[lo:hi].sum(), hi - lo], dtype=torch.float64)
        all_reduce_sum(sums)
        count = sums[4].item()
        mu_r, mu_e = sums[0].item() / count, sums[1].item() / count
        m2 = torch.tensor([((r - mu_r) ** 2).sum(), ((e - mu_e) ** 2).sum()], dtype=torch.float64)
        all_reduce_sum(m2)
        if hi > lo:
            ext = torch.tensor([r.max(), lo + int(np.argmax(r)), r.min(), lo + int(np.argmin(r))], dtype=torch.float64)
        else:
            ext = torch.tensor([-np.inf, -1, np.inf, -1], dtype=torch.float64)
        best, worst = pick_extremes(all_gather_rows(ext))
        s = summary_from_stats(sums.tolist(), m2.tolist(), best, worst, 0.8)
        if rank == 0:
            q.put(s.to_dict())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (3, 1001), (2, 1)])
def test_sharded_summary_equals_single_process(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ratio, err, eff, succ = _data(n)
    assert got["total_episodes"] == n
    assert got["successful_episodes"] == int(succ.sum())
    assert got["mean_on_target_ratio"] == pytest.approx(ratio.mean(), rel=1e-12)
    assert got["std_on_target_ratio"] == pytest.approx(ratio.std(), rel=1e-9, abs=1e-15)
    assert got["mean_tracking_error"] == pytest.approx(err.mean(), rel=1e-12)
    assert got["std_tracking_error"] == pytest.approx(err.std(), rel=1e-9)
    assert got["mean_control_effort"] == pytest.approx(eff.mean(), rel=1e-12)
    assert got["best_episode_idx"] == int(np.argmax(ratio))
    assert got["worst_episode_idx"] == int(np.argmin(ratio))
    assert got["meets_criteria"] == bool(ratio.mean() >= 0.8)


def test_shard_range_partitions():
    for n in (0, 1, 7, 65536, 1048576 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - lo for lo, h in spans]
            assert max(sizes) - min(sizes) <= 1
