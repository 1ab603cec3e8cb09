#!/usr/bin/env python3
"""Build the per-step kernel variants of round 5's A/B (profiles/r05/step_kernel_ab.jsonl)
as whole libraries under build/ab_step/<variant>/ (run here, after `make`; the
GPU side is scripts/ab_step.sh):

  head  csrc/qt_step.hip as committed (160 VGPRs, 3 waves per SIMD)
  w4    closed_step_kernel capped at 4 waves per SIMD (amdgpu_waves_per_eu(4): 128 VGPRs, scratch spills)
  cf    env_step_into with the fused exact step's closed-form RK4 (integrate_closed) for states of
        moderate magnitude, the staged RK4 otherwise (180 VGPRs: 2 waves per SIMD)
  cfw3  cf capped at 3 waves per SIMD
  early the frame rows that depend on time only (target observation, time, step count) computed
        and stored before the integration, so their stores drain while the step computes (round 6)

Each variant recompiles qt_step.hip only and links it with the in-tree objects of the other
translation units."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "lqr-quadcopter-test_amd")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-ffp-contract=on"]
KERNEL = "__global__ __launch_bounds__(kBlock) void closed_step_kernel"

CLOSED_FORM_OLD = """  const bool viol = parse_action(e, u, ua);
  integrate(e, pl, x, ua);
"""
CLOSED_FORM_NEW = """  const bool viol = parse_action(e, u, ua);
  double m = 0.0;
#pragma unroll
  for (int i = 0; i < 12; ++i) m = fmax(m, fabs(x[i]));
  if (m <= 1e100) {
    Trig ta, t4;
    double d4[3];
    trig_of(x + 6, ta);
    integrate_closed(e, make_rate_lin(e), make_vel_lin(e, pl), pl, ta, x, ua, d4, t4);
  } else {
    integrate(e, pl, x, ua);
  }
"""


EARLY_OLD = """  double ua[4];
  const bool viol = parse_action(e, u, ua);
  integrate(e, pl, x, ua);
  t += e.dt;
  // np.clip's NaN propagation kept: a caller's action may drive the state anywhere
  const int term = constrain_terminate<true>(e, x, t);
  Target tg;
  target_state<true>(e, motion, pt, t, tg);
"""
EARLY_NEW = """  double ua[4];
  t += e.dt;
  Target tg;
  target_state<true>(e, motion, pt, t, tg);
  store_target(O, n, ep, tg);
  O.f[QT_FR_TIME * n + ep] = t;
  O.c[QT_FC_STEP * n + ep] = k.step + 1;
  const bool viol = parse_action(e, u, ua);
  integrate(e, pl, x, ua);
  // np.clip's NaN propagation kept: a caller's action may drive the state anywhere
  const int term = constrain_terminate<true>(e, x, t);
"""
EARLY_STORES_OLD = """  store_target(O, n, ep, tg);
  O.f[QT_FR_TIME * n + ep] = t;
  O.f[QT_FR_ERR * n + ep] = err;"""
EARLY_STORES_NEW = """  O.f[QT_FR_ERR * n + ep] = err;"""
EARLY_STEP_OLD = """  O.c[QT_FC_STEP * n + ep] = k.step;
  O.c[QT_FC_VIOLATIONS"""
EARLY_STEP_NEW = """  O.c[QT_FC_VIOLATIONS"""


def early(src):
    for a, b in ((EARLY_OLD, EARLY_NEW), (EARLY_STORES_OLD, EARLY_STORES_NEW), (EARLY_STEP_OLD, EARLY_STEP_NEW)):
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    return src


def waves(src, w):
    return src.replace(KERNEL, KERNEL.replace("__global__ __launch_bounds__(kBlock)",
                                              f"__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu({w})))"))


def main():
    head = open(os.path.join(PKG, "csrc", "qt_step.hip")).read()
    assert CLOSED_FORM_OLD in head and KERNEL in head
    cf = head.replace(CLOSED_FORM_OLD, CLOSED_FORM_NEW)
    variants = {"head": head, "w4": waves(head, 4), "cf": cf, "cfw3": waves(cf, 3), "early": early(head)}
    objs = [os.path.join(PKG, "build", f) for f in ("qt_dare.o", "qt_rollout.o", "qt_rollout_fast.o", "qt_seed.o")]
    for name, src in variants.items():
        if len(sys.argv) > 1 and name not in sys.argv[1:]:
            continue
        out = os.path.join(ROOT, "build", "ab_step", name)
        os.makedirs(out, exist_ok=True)
        path = os.path.join(PKG, "csrc", f"_ab_{name}.hip")  # beside its headers
        try:
            open(path, "w").write(src)
            subprocess.run([HIPCC, *FLAGS, "-c", path, "-o", os.path.join(out, "qt_step.o")], check=True)
        finally:
            os.remove(path)
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libquadtrack.so"),
                        *objs, os.path.join(out, "qt_step.o")], check=True)
        print("built", name)


if __name__ == "__main__":
    main()
