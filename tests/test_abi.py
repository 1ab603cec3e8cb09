"""C-ABI checks that need no GPU: the library loads, exports every entry point
include/quadtrack.h declares, and the ctypes structs have the C layout."""

import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

from quadtrack import _abi

HEADER = os.path.join(ROOT, "include", "quadtrack.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^int (qt_\w+)\(", src, flags=re.M)))


def test_header_declares_expected_entry_points():
    assert set(declared_functions()) == set(_abi.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _abi.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.qt_abi_version() == _abi.ABI_VERSION
    nm = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r" T (qt_\w+)", nm.stdout))
    assert set(declared_functions()) <= exported


PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "quadtrack.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("qt_env_params %zu\nqt_ctrl_params %zu\nqt_criteria %zu\nqt_batch %zu\nqt_state %zu\n",
         sizeof(qt_env_params), sizeof(qt_ctrl_params), sizeof(qt_criteria), sizeof(qt_batch), sizeof(qt_state));
  F(qt_env_params, integrator) F(qt_env_params, motion) F(qt_env_params, speed) F(qt_env_params, center)
  F(qt_env_params, min_episode_duration) F(qt_ctrl_params, use_lqi) F(qt_ctrl_params, integral_limit)
  F(qt_ctrl_params, ff_max_acceleration) F(qt_criteria, overshoot_window) F(qt_batch, K) F(qt_batch, k_cols)
  F(qt_batch, order) F(qt_batch, ff) F(qt_state, target)
  printf("QT_ACC_ROWS %d\nQT_MET_ROWS %d\n", QT_ACC_ROWS, QT_MET_ROWS);
  printf("qt_view %zu\nqt_obs_view %zu\n", sizeof(qt_view), sizeof(qt_obs_view));
  F(qt_view, rs) F(qt_view, es) F(qt_obs_view, tacc) F(qt_obs_view, time)
  printf("QT_FR_ROWS %d\nQT_FC_ROWS %d\nQT_FB_ROWS %d\nQT_FR_TIME %d\nQT_FR_RATIO %d\nQT_FB_TERM %d\n",
         QT_FR_ROWS, QT_FC_ROWS, QT_FB_ROWS, QT_FR_TIME, QT_FR_RATIO, QT_FB_TERM);
  printf("QT_FRAME_BYTES_1000 %lld\n", (long long)QT_FRAME_BYTES(1000));
  return 0;
}
"""


def test_struct_layout_matches_c(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                              check=True).stdout.strip().splitlines())
    cls = {"qt_env_params": _abi.EnvParams, "qt_ctrl_params": _abi.CtrlParams, "qt_criteria": _abi.Criteria,
           "qt_batch": _abi.Batch, "qt_state": _abi.State, "qt_view": _abi.View, "qt_obs_view": _abi.ObsView}
    for k, v in out.items():
        if k in cls:
            assert C.sizeof(cls[k]) == int(v), k
        elif k.startswith("QT_"):
            continue
        elif "." in k:
            s, f = k.split(".")
            assert getattr(cls[s], f).offset == int(v), k
    assert int(out["QT_ACC_ROWS"]) == _abi.ACC_ROWS
    assert int(out["QT_MET_ROWS"]) == _abi.MET_ROWS
    assert (int(out["QT_FR_ROWS"]), int(out["QT_FC_ROWS"]), int(out["QT_FB_ROWS"])) == \
        (_abi.FR_ROWS, _abi.FC_ROWS, _abi.FB_ROWS)
    assert (int(out["QT_FR_TIME"]), int(out["QT_FR_RATIO"]), int(out["QT_FB_TERM"])) == \
        (_abi.FR_TIME, _abi.FR_RATIO, _abi.FB_TERM)
    assert int(out["QT_FRAME_BYTES_1000"]) == _abi.frame_bytes(1000)


def test_no_gpu_means_loud_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_abi.QuadtrackError):
        _abi.require_gpu()
    from quadtrack import BatchedQuadcopterEnv, RiccatiLQRController

    with pytest.raises(_abi.QuadtrackError):
        BatchedQuadcopterEnv(4)
    with pytest.raises(_abi.QuadtrackError):
        RiccatiLQRController({"dt": 0.01})


def test_kernels_built_for_gfx950():
    """The shipped library's offload bundle holds gfx950 code objects and no
    other target: the bundle entry ids read from the file itself (roc-obj-ls
    as well where it runs)."""
    data = open(_abi.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}, targets
    try:
        out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", _abi.LIB_PATH], capture_output=True, text=True)
    except OSError:
        return
    if out.returncode == 0:
        assert "gfx950" in out.stdout
