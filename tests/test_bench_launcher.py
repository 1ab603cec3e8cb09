"""bench.py's N-rank entry point (the driver's `bench.py --gpus N`), on CPU.

`--launcher-check` runs the same launch path as a real multi-GPU bench —
bench.py re-starts itself under torch.distributed.run with N ranks when
WORLD_SIZE is unset — but each rank only joins a gloo group and reports the
ranks it saw, so the plumbing is tested without a GPU.  The real bench must
refuse to run N ranks on fewer visible GPUs instead of benchmarking one."""

import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, gpu_available

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    return env


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.parametrize("n", [1, 2, 4])
def test_launcher_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launcher-check"], capture_output=True, text=True,
                       env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == n
    assert line["world_size_seen"] == n
    assert line["ranks"] == list(range(n))


def test_gpus_must_match_world_size():
    env = _env()
    env.update({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launcher-check"], capture_output=True, text=True,
                       env=env, timeout=60)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def _visible_gpus() -> int:
    import torch

    return torch.cuda.device_count() if gpu_available() else 0


def test_more_gpus_than_visible_is_an_error():
    want = max(2, _visible_gpus() + 1)  # more than this host has (2 on a 1-GPU box)
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(want), "--steps", "1", "--warmup", "0"], capture_output=True,
                       text=True, env=_env(), timeout=60)
    assert r.returncode == 2
    assert "GPU(s) are visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
