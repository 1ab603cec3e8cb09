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


_PARENT_PROBE = r"""
import json, subprocess, sys
sys.path.insert(0, {root!r})
import bench

def fake_call(cmd, env=None):
    maps = open("/proc/self/maps").read()
    print(json.dumps({{"hip_mapped": "libamdhip64" in maps, "torch_loaded": "torch" in sys.modules,
                      "cmd_has_run": "torch.distributed.run" in cmd}}), flush=True)
    return 0

subprocess.call = fake_call
bench.visible_gpu_count = lambda: {fake_gpus}
sys.argv = ["bench.py"] + {argv!r}
bench.main()
"""


@pytest.mark.parametrize("argv", [["--gpus", "2", "--launcher-check"], ["--gpus", "8", "--steps", "1"]])
def test_launcher_parent_never_loads_hip(argv):
    """The parent that starts the ranks reads no HIP: at the moment it would
    spawn torch.distributed.run, libamdhip64 is not mapped and torch is not
    imported (the GPU count comes from the KFD topology)."""
    code = _PARENT_PROBE.format(root=ROOT, fake_gpus=8, argv=argv)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=_env(), timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line == {"hip_mapped": False, "torch_loaded": False, "cmd_has_run": True}


def test_visible_gpu_count_without_hip():
    """visible_gpu_count reads sysfs only: no torch import, and it honours
    HIP_VISIBLE_DEVICES narrowing."""
    code = ("import sys, os; sys.path.insert(0, %r); import bench; n = bench.visible_gpu_count(); "
            "os.environ['HIP_VISIBLE_DEVICES'] = '0'; m = bench.visible_gpu_count(); "
            "print(n, m, 'torch' in sys.modules)") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=_env(), timeout=60)
    n, m, torch_loaded = r.stdout.split()
    assert torch_loaded == "False"
    assert int(m) == min(int(n), 1)
    if not gpu_available():
        assert int(n) == 0


def test_profile_readers_use_one_named_directory(tmp_path):
    """bench.py cites the committed rocprofv3 summaries of ONE directory
    (--profile-dir, default PROFILE_DIR): kernel average, HBM traffic and the
    issued FP64 flops (64 x (2 FMA + MUL + ADD + TRANS) per launch) come from
    that directory's files, and a directory without them gives None (never
    another round's files)."""
    sys.path.insert(0, ROOT)
    import bench

    tag = bench.KERNEL_TAG
    name = f"void qtk::{tag}, false>(args)"
    d = tmp_path / "prof"
    d.mkdir()
    (d / "kernel_stats.csv").write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"\n'
                                        f'"{name}",10,13000000,1300000.0,99.0,1290000,1310000\n')
    hdr = "Kernel_Name,Counter_Name,Dispatches,Average_Per_Dispatch\n"
    (d / "pmc_FETCH_SIZE.csv").write_text(hdr + f'"{name}",FETCH_SIZE,3,100.0\n')
    (d / "pmc_WRITE_SIZE.csv").write_text(hdr + f'"{name}",WRITE_SIZE,3,50.0\n')
    (d / "pmc_F64_summary.csv").write_text(hdr + "".join(
        f'"{name}",{c},3,{v}\n' for c, v in zip(bench.F64_COUNTERS, (10.0, 4.0, 3.0, 1.0))))
    rel = os.path.relpath(d, ROOT)
    ms, mn, calls, src = bench.profiled_kernel(rel, tag)
    assert (ms, mn, calls, src) == (1.3, 1.29, 10, rel)
    assert bench.pmc_traffic(rel, tag) == ((2 * 100.0 + 50.0) * 1024.0, rel)
    flops, src, counts = bench.issued_fp64(rel, tag)
    assert flops == 64.0 * (2 * 10.0 + 4.0 + 3.0 + 1.0) and src == f"{rel}/pmc_F64_summary.csv"
    empty = tmp_path / "none"
    empty.mkdir()
    rel2 = os.path.relpath(empty, ROOT)
    assert bench.profiled_kernel(rel2, tag) is None
    assert bench.pmc_traffic(rel2, tag) == (None, None)
    assert bench.issued_fp64(rel2, tag) is None


RUN_WORKLOAD = os.path.join(ROOT, "scripts", "run_workload.py")


@pytest.mark.parametrize("config,world", [(5, 2), (4, 3)])
def test_run_workload_launcher_check(config, world):
    """scripts/run_workload.py under torch.distributed.run (the configs 4 / 5
    multi-GPU driver), on CPU: every rank joins (gloo) and rank 0 reports
    world_size_seen, the backend and each rank's shard of the config, which
    tile the global range."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", RUN_WORKLOAD, "--config", str(config),
           "--gpus", str(world), "--launcher-check"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["world_size_seen"] == world and line["backend"] == "gloo"
    ranks = line["ranks"]
    assert [x["rank"] for x in ranks] == list(range(world))
    total = {4: 262144, 5: 1048576}[config]
    assert ranks[0]["lo"] == 0 and ranks[-1]["hi"] == total
    assert all(a["hi"] == b["lo"] for a, b in zip(ranks, ranks[1:]))


def test_run_workload_refuses_world_mismatch():
    env = _env()
    env.update({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    r = subprocess.run([sys.executable, RUN_WORKLOAD, "--config", "5", "--gpus", "8", "--launcher-check"],
                       capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
