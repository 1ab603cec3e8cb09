"""The kernels' elementary functions (csrc/qt_math.hpp), compiled for the
host, against numpy: sin/cos within 2 ulp over the domain the loop uses, and
the fmod-free angle wrap bit-identical to numpy's float remainder."""

import os
import subprocess

import numpy as np
import pytest

from conftest import PKG

SRC = r"""
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "qt_math.hpp"
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  std::vector<double> x;
  double v;
  while (fread(&v, 8, 1, f) == 1) x.push_back(v);
  fclose(f);
  FILE* o = fopen(argv[2], "wb");
  for (double a : x) {
    double s, c;
    qt::fast_sincos(a, &s, &c);
    double m = qt::py_mod_2pi(a, 6.283185307179586);
    double ss, cs, st, ct, sr, cr;
    qt::small_sincos(a, &ss, &cs);
    qt::sincos_tilt(a, &st, &ct);
    qt::rate_sincos(a, &sr, &cr);
    double sq, cq;
    qt::resid_sincos(a, &sq, &cq);
    fwrite(&s, 8, 1, o);
    fwrite(&c, 8, 1, o);
    fwrite(&m, 8, 1, o);
    fwrite(&ss, 8, 1, o);
    fwrite(&cs, 8, 1, o);
    fwrite(&st, 8, 1, o);
    fwrite(&ct, 8, 1, o);
    fwrite(&sr, 8, 1, o);
    fwrite(&cr, 8, 1, o);
    fwrite(&sq, 8, 1, o);
    fwrite(&cq, 8, 1, o);
  }
  fclose(o);
  return 0;
}
"""


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    d = tmp_path_factory.mktemp("math")
    (d / "p.cpp").write_text(SRC)
    exe = d / "p"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(PKG, "csrc"),
                    str(d / "p.cpp"), "-o", str(exe)], check=True)

    def run(x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        (d / "in.bin").write_bytes(x.tobytes())
        subprocess.run([str(exe), str(d / "in.bin"), str(d / "out.bin")], check=True)
        return np.frombuffer((d / "out.bin").read_bytes(), dtype=np.float64).reshape(-1, 11)

    return run


def ulp_err(a, ref):
    return np.abs(a - ref) / np.spacing(np.maximum(np.abs(ref), 1e-300))


def test_sincos_accuracy(probe):
    rng = np.random.default_rng(0)
    x = np.concatenate([
        rng.uniform(-np.pi - 0.2, np.pi + 0.2, 200000),       # attitude angles + RK4 stage offsets
        rng.uniform(-2000.0, 2000.0, 100000),                  # target phases
        np.arange(-64, 65) * (np.pi / 2),                      # quadrant boundaries
        np.arange(-64, 65) * (np.pi / 4),
        [0.0, -0.0, 1e-300, -1e-20, 5e-9],
    ])
    out = probe(x)
    s, c = out[:, 0], out[:, 1]
    # near the zeros of sin / cos the relative measure is meaningless: use absolute 2^-53 there
    tol_s = np.maximum(2 * np.spacing(np.abs(np.sin(x))), 1.2e-16 * np.maximum(1, np.abs(x) / 1e3))
    tol_c = np.maximum(2 * np.spacing(np.abs(np.cos(x))), 1.2e-16 * np.maximum(1, np.abs(x) / 1e3))
    assert np.all(np.abs(s - np.sin(x)) <= tol_s)
    assert np.all(np.abs(c - np.cos(x)) <= tol_c)
    small = np.abs(x) <= np.pi + 0.2
    assert np.max(ulp_err(s[small], np.sin(x[small]))[np.abs(np.sin(x[small])) > 1e-3]) <= 2.0
    assert np.max(ulp_err(c[small], np.cos(x[small]))[np.abs(np.cos(x[small])) > 1e-3]) <= 2.0


def test_small_angle_sincos_and_rotation(probe):
    """The RK4 stage trig: small_sincos on |d| <= 0.25 and the angle-addition
    rotation used for stages 2-4 (qt_device.hpp trig_shift)."""
    rng = np.random.default_rng(2)
    d = np.concatenate([rng.uniform(-0.125, 0.125, 200000), [0.0, -0.0, 1e-12, 0.125, -0.125]])
    out = probe(d)
    ss, cs = out[:, 3], out[:, 4]
    assert np.max(ulp_err(ss, np.sin(d))[np.abs(d) > 1e-300]) <= 1.0
    assert np.max(ulp_err(cs, np.cos(d))) <= 1.0
    a = rng.uniform(-np.pi, np.pi, d.size)
    base = probe(a)
    s = np.fma(base[:, 0], cs, base[:, 1] * ss) if hasattr(np, "fma") else base[:, 0] * cs + base[:, 1] * ss
    c = base[:, 1] * cs - base[:, 0] * ss
    assert np.max(np.abs(s - np.sin(a + d))) <= 4.5e-16
    assert np.max(np.abs(c - np.cos(a + d))) <= 4.5e-16


def test_sincos_nonfinite(probe):
    out = probe([np.nan, np.inf, -np.inf])
    assert np.all(np.isnan(out[:, :2]))


def test_angle_wrap_bit_identical_to_numpy(probe):
    rng = np.random.default_rng(1)
    a = np.concatenate([rng.uniform(-4 * np.pi, 4 * np.pi, 200000) + np.pi, rng.uniform(-100, 100, 20000),
                        np.array([0.0, -0.0, 2 * np.pi, -2 * np.pi, 4 * np.pi, -4 * np.pi, np.nan, np.inf])])
    out = probe(a)[:, 2]
    ref = a % (2 * np.pi)
    same = (out == ref) | (np.isnan(out) & np.isnan(ref))
    assert np.all(same)
    assert not np.any(np.signbit(out[out == 0]))


def test_tilt_sincos_accuracy(probe):
    """sincos_tilt (no argument reduction) on the roll / pitch range of the
    yaw-at-rest fast step: |a| <= pi/3 (every step starts inside the tilt clamp)."""
    rng = np.random.default_rng(3)
    lim = np.pi / 3
    a = np.concatenate([rng.uniform(-lim, lim, 300000), [0.0, -0.0, 1e-300, np.pi / 3, -np.pi / 3, lim, -lim]])
    out = probe(a)
    st, ct = out[:, 5], out[:, 6]
    assert np.max(ulp_err(st, np.sin(a))[np.abs(a) > 1e-300]) <= 1.0
    assert np.max(ulp_err(ct, np.cos(a))) <= 2.0  # as fast_sincos: the last step 1 + z*q rounds at ulp(1)/2
    assert st[300002] == 1e-300 and ct[300000] == 1.0 and st[300001] == 0.0


def test_rate_sincos_accuracy(probe):
    """rate_sincos: the stage offsets of the rate-bounded fast step,
    |d| <= kRateAngle = 0.031 (dt * max commanded rate), and the rotation."""
    rng = np.random.default_rng(4)
    d = np.concatenate([rng.uniform(-0.031, 0.031, 200000), [0.0, -0.0, 1e-12, 0.031, -0.031]])
    out = probe(d)
    sr, cr = out[:, 7], out[:, 8]
    assert np.max(ulp_err(sr, np.sin(d))[np.abs(d) > 1e-300]) <= 1.0
    assert np.max(ulp_err(cr, np.cos(d))) <= 1.0
    a = rng.uniform(-np.pi / 3, np.pi / 3, d.size)
    base = probe(a)
    s = base[:, 5] * cr + base[:, 6] * sr
    c = base[:, 6] * cr - base[:, 5] * sr
    assert np.max(np.abs(s - np.sin(a + d))) <= 4.5e-16
    assert np.max(np.abs(c - np.cos(a + d))) <= 4.5e-16


def test_residual_sincos_accuracy(probe, col=9, lim=4e-3):
    """resid_sincos (|d| <= kStage3Angle: the yaw-at-rest step's third stage
    from its second), which returns sin d and cos d - 1, and the rotation
    rotate_cm built on it."""
    rng = np.random.default_rng(5 + col)
    d = np.concatenate([rng.uniform(-lim, lim, 200000), [0.0, -0.0, 1e-12, lim, -lim]])
    out = probe(d)
    sd, cm = out[:, col], out[:, col + 1]
    assert np.max(ulp_err(sd, np.sin(d))[np.abs(d) > 1e-300]) <= 1.0
    cm_ref = -2.0 * np.sin(0.5 * d) ** 2  # cos d - 1 without cancellation
    # cos d - 1 is truncated (d^6 / 6!): absolute error, what the rotation sees
    assert np.max(np.abs(cm - cm_ref) - 2 * np.spacing(np.abs(cm_ref))) <= 6e-18
    a = rng.uniform(-np.pi / 3, np.pi / 3, d.size)
    base = probe(a)
    s0, c0 = base[:, 5], base[:, 6]
    s = np.fma(c0, sd, np.fma(s0, cm, s0)) if hasattr(np, "fma") else s0 + (s0 * cm + c0 * sd)
    c = np.fma(-s0, sd, np.fma(c0, cm, c0)) if hasattr(np, "fma") else c0 + (c0 * cm - s0 * sd)
    assert np.max(np.abs(s - np.sin(a + d))) <= 3.4e-16
    assert np.max(np.abs(c - np.cos(a + d))) <= 3.4e-16


CR_SRC = r"""
#include <cstdio>
#include <vector>
#include "qt_crtrig.hpp"
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  std::vector<double> x;
  double v;
  while (fread(&v, 8, 1, f) == 1) x.push_back(v);
  fclose(f);
  FILE* o = fopen(argv[2], "wb");
  for (double a : x) {
    double s, c;
    qt::cr_sincos(a, &s, &c);
    fwrite(&s, 8, 1, o);
    fwrite(&c, 8, 1, o);
  }
  fclose(o);
  return 0;
}
"""


@pytest.fixture(scope="module")
def cr_probe(tmp_path_factory):
    d = tmp_path_factory.mktemp("crtrig")
    (d / "p.cpp").write_text(CR_SRC)
    exe = d / "p"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(PKG, "csrc"),
                    str(d / "p.cpp"), "-o", str(exe)], check=True)

    def run(x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        (d / "in.bin").write_bytes(x.tobytes())
        subprocess.run([str(exe), str(d / "in.bin"), str(d / "out.bin")], check=True)
        return np.fromfile(d / "out.bin").reshape(-1, 2).T

    return run


def _angles(n, seed):
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.uniform(-60, 60, n // 2), rng.uniform(-1e4, 1e4, n // 4), rng.uniform(-1, 1, n // 8),
                           np.arange(1, n // 8 + 1) * (np.pi / 4), [0.0, -0.0, 1e-300, 5e-324, np.pi / 2, np.pi]])


def test_cr_sincos_vs_mpmath(cr_probe):
    """qt_crtrig.hpp's cr_sincos (the figure-8 feed-forward target's trig)
    against mpmath at 200 bits: correctly rounded on every sample, including
    multiples of pi/4 (the reduction's quadrant boundaries)."""
    mpmath = pytest.importorskip("mpmath")
    x = _angles(24000, 11)
    s, c = cr_probe(x)
    with mpmath.workprec(200):
        rs = np.array([float(mpmath.sin(mpmath.mpf(float(v)))) for v in x])
        rc = np.array([float(mpmath.cos(mpmath.mpf(float(v)))) for v in x])
    np.testing.assert_array_equal(s, rs)
    np.testing.assert_array_equal(c, rc)


def test_cr_sincos_vs_glibc(cr_probe):
    """Against numpy (= glibc sin / cos here), which rounds incorrectly in
    ~0.15% of arguments: the two agree everywhere else."""
    x = _angles(2_000_000, 12)
    s, c = cr_probe(x)
    ms, mc = np.mean(s != np.sin(x)), np.mean(c != np.cos(x))
    assert ms < 3e-3 and mc < 3e-3, (ms, mc)
    fin = np.isfinite(x)
    assert np.all(np.abs(s - np.sin(x))[fin] <= np.spacing(np.abs(np.sin(x)))[fin])
    assert np.isnan(cr_probe(np.array([np.inf, -np.inf, np.nan]))).all()


# ------------------------------------------------ glibc sin / cos / pow(x, 2)
# qt_glibc.hpp restates glibc 2.35's __sin_fma / __cos_fma / __ieee754_pow_fma
# (the variants numpy's scalar np.sin / np.cos / x**2 reach on an FMA host) for
# the figure-8 feed-forward target.  The probe evaluates both the host libm and
# the restatement on the same arguments and counts bit mismatches.

GLIBC_SRC = r"""
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "qt_glibc.hpp"
extern "C" double sin(double);
extern "C" double cos(double);
extern "C" double pow(double, double);
static bool same(double a, double b) {
  uint64_t x, y;
  memcpy(&x, &a, 8);
  memcpy(&y, &b, 8);
  return x == y || (a != a && b != b);
}
// splitmix64: arguments are generated here (1e7+ is too many to pass through files)
static uint64_t sm(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
int main(int argc, char** argv) {
  long n = atol(argv[1]);
  uint64_t seed = strtoull(argv[2], 0, 10);
  long bad[3] = {0, 0, 0}, checked = 0;
  std::vector<double> xs;
  if (argc > 3) {  // explicit arguments from a file
    FILE* f = fopen(argv[3], "rb");
    double v;
    while (fread(&v, 8, 1, f) == 1) xs.push_back(v);
    fclose(f);
    n = (long)xs.size();
  }
  for (long i = 0; i < n; ++i) {
    double x;
    if (!xs.empty()) {
      x = xs[i];
    } else {
      const uint64_t r = sm(seed);
      const double u = (double)(r >> 11) * 0x1p-53;
      switch (i % 8) {
        case 0: x = (2 * u - 1) * 8.0; break;             // a few periods: every quadrant / table entry
        case 1: x = (2 * u - 1) * 200.0; break;           // figure-8 angles omega t over long episodes
        case 2: x = std::ldexp(1.0 + u, -30 + (int)(u * 30)); break;  // small: Taylor / tiny branches
        case 3: x = 0.8 + u * 1.7; break;                 // the hp0 - |x| branch
        case 4: x = (2 * u - 1) * 1e7; break;             // large reduce_sincos arguments
        case 5: { const uint64_t b = sm(seed); memcpy(&x, &b, 8); break; }  // any bit pattern
        case 6: x = (2 * u - 1) * 2.0; break;             // sin_t and 1 + sin_t^2 of the figure-8
        default: x = std::ldexp(u, -1074 + (int)(u * 2100)); break;   // subnormals .. huge (pow)
      }
    }
    const bool trig = std::fabs(x) < 105414350.0 || !std::isfinite(x);
    if (trig) {
      bad[0] += !same(sin(x), qt::glibc::sin(x));
      bad[1] += !same(cos(x), qt::glibc::cos(x));
      ++checked;
    }
    bad[2] += !same(pow(x, 2.0), qt::glibc::pow2(x));
  }
  printf("%ld %ld %ld %ld %ld\n", n, checked, bad[0], bad[1], bad[2]);
  return 0;
}
"""


def _host_has_fma():
    try:
        return " fma " in open("/proc/cpuinfo").read().replace("\n", " ")
    except OSError:
        return False


@pytest.fixture(scope="module")
def glibc_probe(tmp_path_factory):
    if not _host_has_fma():
        pytest.skip("host libm would run its non-FMA variants, which qt_glibc.hpp does not restate")
    d = tmp_path_factory.mktemp("glibc")
    (d / "p.cpp").write_text(GLIBC_SRC)
    exe = d / "p"
    # -fno-builtin: every sin / cos / pow call goes to libm (no folding, no sincos merge, no pow(x, 2) -> x * x)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-builtin", "-I", os.path.join(PKG, "csrc"),
                    str(d / "p.cpp"), "-o", str(exe), "-lm"], check=True)

    def run(n=0, seed=1, x=None):
        args = [str(exe), str(n), str(seed)]
        if x is not None:
            (d / "in.bin").write_bytes(np.ascontiguousarray(x, dtype=np.float64).tobytes())
            args.append(str(d / "in.bin"))
        out = subprocess.run(args, check=True, capture_output=True, text=True).stdout.split()
        return [int(v) for v in out]

    return run


def test_glibc_sin_cos_pow2_bitwise_vs_host_libm(glibc_probe):
    """1.2e7 arguments over every branch of sin / cos (Taylor, table, hp0 - |x|,
    reduce_sincos) and pow(x, 2) (subnormal to overflow, negative, +-0,
    inf / nan): bitwise equal to the host glibc."""
    n, checked, bs, bc, bp = glibc_probe(12_000_000, seed=20261017)
    assert checked > 0.85 * n
    assert (bs, bc, bp) == (0, 0, 0)


def test_glibc_edge_arguments(glibc_probe):
    """Branch boundaries (2^-27, 2^-26, 0.126, 0.855469, 2.426265, 105414350),
    multiples of pi/4 and pi/2 (quadrant edges), the table grid i/128 and its
    midpoints, and pow's special inputs."""
    edges = []
    for b in (2.0 ** -27, 2.0 ** -26, 0.126, 0.85546875, 2.426265, 105414349.0, 1.0, 0.5):
        for v in (b, np.nextafter(b, 0), np.nextafter(b, np.inf)):
            edges += [v, -v]
    k = np.arange(-4000, 4001)
    grid = np.arange(0, 112) / 128.0
    x = np.concatenate([edges, k * (np.pi / 4), k * (np.pi / 2), np.nextafter(k * (np.pi / 2), np.inf),
                        grid, grid + 1 / 256.0, -grid,
                        [0.0, -0.0, 5e-324, -5e-324, 2.2250738585072014e-308, 1.7976931348623157e308,
                         -1.7976931348623157e308, 1e154, 1.4e154, 1e-160, 1e-170, np.inf, -np.inf, np.nan]])
    n, checked, bs, bc, bp = glibc_probe(x=x)
    assert n == x.size and (bs, bc, bp) == (0, 0, 0)


def test_glibc_is_what_numpy_scalars_call(glibc_probe):
    """The reference's call forms themselves: np.sin / np.cos of a Python float
    and np.float64 ** 2 (target_motion.py:178-180) agree with the host libm,
    so the probe above compares against the right functions."""
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(-60, 60, 3000), rng.uniform(-1.5, 1.5, 3000)])
    import math  # math.sin / math.cos / math.pow call the host libm directly

    for x in xs:
        xf = float(x)
        assert np.cos(xf) == math.cos(xf) and np.sin(xf) == math.sin(xf)
        v = np.float64(xf)
        assert v ** 2 == math.pow(xf, 2.0)
