"""The device RNG restatement (csrc/qt_rng.hpp, host build) against numpy's
default_rng: raw PCG64 words, doubles and ziggurat normals bit for bit,
including multi-word seeds; and the device reset draws (qt_seed_draws, GPU)
against the oracle's numpy draws."""

import os
import subprocess

import numpy as np
import pytest

from conftest import PKG

import oracle as O

SRC = r"""
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "qt_rng.hpp"
int main(int argc, char** argv) {
  if (argc > 3 && !strcmp(argv[3], "log1p")) {  // restated log1p vs this libm, n arguments in (-1, 3)
    uint64_t st = strtoull(argv[1], 0, 10) | 1;
    long bad = 0;
    const long n = atol(argv[2]);
    for (long i = 0; i < n; ++i) {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      const double u = (double)(st >> 11) * (1.0 / 9007199254740992.0);
      const double x = (i % 4 == 0) ? -u : (i % 4 == 1) ? -u * 1e-3 : (i % 4 == 2) ? 3.0 * u : -u * u * u * u;
      const double a = log1p(x), b = qt::fdlibm_log1p(x);
      if (memcmp(&a, &b, 8)) ++bad;
    }
    printf("%ld\n", bad);
    return 0;
  }
  if (argc > 3 && !strcmp(argv[3], "normals")) {  // n normals of one stream, raw doubles to stdout
    qt::Pcg64 g = qt::pcg64_from_seed(strtoull(argv[1], 0, 10));
    const long n = atol(argv[2]);
    for (long i = 0; i < n; ++i) {
      const double v = qt::pcg_standard_normal(g);
      fwrite(&v, 8, 1, stdout);
    }
    return 0;
  }
  const unsigned long long seed = strtoull(argv[1], 0, 10);
  const int n = atoi(argv[2]);
  qt::Pcg64 g = qt::pcg64_from_seed(seed);
  for (int i = 0; i < n; ++i) printf("%llu\n", (unsigned long long)qt::pcg_next64(g));
  g = qt::pcg64_from_seed(seed);
  for (int i = 0; i < n; ++i) printf("%a\n", qt::pcg_next_double(g));
  g = qt::pcg64_from_seed(seed);
  for (int i = 0; i < n; ++i) printf("%a\n", qt::pcg_standard_normal(g));
  return 0;
}
"""


@pytest.fixture(scope="module")
def rng_probe(tmp_path_factory):
    d = tmp_path_factory.mktemp("rng")
    (d / "r.cpp").write_text(SRC)
    exe = d / "r"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(PKG, "csrc"),
                    str(d / "r.cpp"), "-o", str(exe)], check=True)

    def run(seed, n):
        out = subprocess.run([str(exe), str(seed), str(n)], capture_output=True, text=True, check=True).stdout.split()
        raw = np.array([int(v) for v in out[:n]], dtype=np.uint64)
        dbl = np.array([float.fromhex(v) for v in out[n:2 * n]])
        nrm = np.array([float.fromhex(v) for v in out[2 * n:]])
        return raw, dbl, nrm

    run.exe = str(exe)
    return run


def test_log1p_restatement_matches_libm(rng_probe):
    # qt::fdlibm_log1p is glibc's s_log1p restated; the ziggurat tail uses it
    # on host and device so tail normals round as numpy's do
    out = subprocess.run([rng_probe.exe, "7", "20000000", "log1p"], capture_output=True, text=True, check=True)
    assert int(out.stdout) == 0


def test_normals_million_draws_match_numpy(rng_probe):
    n = 1_500_000
    out = subprocess.run([rng_probe.exe, "2024", str(n), "normals"], capture_output=True, check=True).stdout
    got = np.frombuffer(out, dtype=np.float64)
    np.testing.assert_array_equal(got, np.random.default_rng(2024).standard_normal(n))


@pytest.mark.parametrize("seed", [0, 1, 42, 12345, 2**31 - 1, 2**32, 2**40 + 7, 2**63 - 1])
def test_pcg64_seedsequence_matches_numpy(rng_probe, seed):
    raw, dbl, nrm = rng_probe(seed, 3000)
    np.testing.assert_array_equal(raw, np.random.PCG64(seed).random_raw(3000))
    np.testing.assert_array_equal(dbl, np.random.default_rng(seed).random(3000))
    np.testing.assert_array_equal(nrm, np.random.default_rng(seed).standard_normal(3000))


@pytest.mark.gpu
@pytest.mark.parametrize("motion", O.MOTIONS)
def test_device_reset_draws_match_numpy(motion):
    import sys

    sys.path.insert(0, PKG)
    from quadtrack.env import seeding

    seeds = np.concatenate([np.arange(20000), [2**40 + 7, 2**63 - 1, 10**9]])
    pat, off = seeding.draws(motion, seeds)
    ref_pat, ref_off = O.draws(motion, seeds)
    np.testing.assert_array_equal(off.cpu().numpy().T, ref_off)
    # bit-exact, normals included: the ziggurat tail's log1p is glibc's
    # restated (qt::fdlibm_log1p), not the device libm's
    np.testing.assert_array_equal(pat.cpu().numpy().T, ref_pat)


@pytest.mark.gpu
def test_device_normals_million_draws_bit_exact():
    """>= 1M device ziggurat normals (linear reset draws, 3 per seed) bitwise
    equal to numpy's default_rng(seed).standard_normal(3); the batch holds
    many base-strip tail draws (the log1p path)."""
    import sys

    sys.path.insert(0, PKG)
    from quadtrack.env import seeding

    seeds = np.arange(350_000, dtype=np.int64) * 7919 + 3
    pat, _ = seeding.draws("linear", seeds)
    got = pat.cpu().numpy()[:3].T
    ref = np.stack([np.random.default_rng(int(s)).standard_normal(3) for s in seeds])
    assert got.size >= 1_000_000
    np.testing.assert_array_equal(got, ref)


@pytest.mark.gpu
def test_device_reset_draws_mixed_motion():
    import sys

    sys.path.insert(0, PKG)
    from quadtrack.env import seeding

    n = 5000
    motion = np.arange(n) % 5
    pat, off = seeding.draws(motion, np.arange(n) + 10**9)
    for m in range(5):
        idx = np.nonzero(motion == m)[0]
        rp, ro = O.draws(m, idx + 10**9)
        np.testing.assert_array_equal(pat.cpu().numpy().T[idx], rp)
        np.testing.assert_array_equal(off.cpu().numpy().T[idx], ro)


ADV_SRC = r"""
#include <cstdio>
#include <cstdlib>
#include "qt_rng.hpp"
int main(int argc, char** argv) {
  const unsigned long long seed = strtoull(argv[1], 0, 10), d = strtoull(argv[2], 0, 10);
  qt::Pcg64 g = qt::pcg64_from_seed(seed);
  qt::pcg_advance(g, (qt::u128)d);
  for (int i = 0; i < 4; ++i) printf("%llu\n", (unsigned long long)qt::pcg_next64(g));
  return 0;
}
"""


@pytest.mark.parametrize("seed,delta", [(42, 0), (42, 1), (7, 10 * 131071), (12345, 2**40 + 3), (2**63 - 1, 2**62)])
def test_pcg64_advance_matches_numpy(tmp_path, seed, delta):
    """qt::pcg_advance (the jump-ahead qt_stream_uniform uses) = numpy's PCG64.advance."""
    (tmp_path / "a.cpp").write_text(ADV_SRC)
    exe = tmp_path / "a"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(PKG, "csrc"), str(tmp_path / "a.cpp"), "-o",
                    str(exe)], check=True)
    out = subprocess.run([str(exe), str(seed), str(delta)], capture_output=True, text=True, check=True).stdout.split()
    bg = np.random.default_rng(seed).bit_generator
    bg.advance(delta)
    np.testing.assert_array_equal(np.array([int(v) for v in out], dtype=np.uint64), bg.random_raw(4))


@pytest.mark.gpu
@pytest.mark.parametrize("first,n", [(0, 1), (0, 1000), (131071, 4097), (262143, 1)])
def test_device_stream_uniform_matches_numpy(first, n):
    """qt_stream_uniform: draw vectors first.. of one default_rng stream, bitwise
    numpy's uniform(lo, hi, size=(first + n, k))[first:]; the config-4 candidate
    tensors equal the host candidate arrays."""
    import torch

    from quadtrack import core, workloads

    lo, hi = [5e-5, 1e-3, 0.5, -2.0], [5e-4, 1e-2, 2.0, 3.0]
    got = core.stream_uniform(42, first, n, lo, hi, torch.device("cuda", 0)).cpu().numpy()
    bg = np.random.default_rng(42)
    bg.bit_generator.advance(4 * first)
    np.testing.assert_array_equal(got, bg.uniform(lo, hi, size=(n, 4)).T)
    dev = [t.cpu().numpy() for t in workloads.tuner_candidate_tensors(first, first + n, torch.device("cuda", 0))]
    for a, b in zip(dev, workloads.tuner_candidate_arrays(first, first + n)):
        np.testing.assert_array_equal(a, b)
