// qt_rng.hpp — numpy's default_rng(seed) stream, restated for the device.
//
// The reference seeds every reset with numpy.random.default_rng(seed)
// (env/quadcopter_env.py:122-137, env/target_motion.py:285-353): SeedSequence
// entropy mixing -> PCG64 (XSL-RR 128/64) -> doubles as (u64 >> 11) * 2^-53,
// uniform(lo, hi) = lo + (hi - lo) * u, standard_normal by numpy's 256-layer
// ziggurat.  Reproducing those draws on the GPU lets reset run without any
// host-side random number generation.  Published algorithms: O'Neill's
// SeedSequence / PCG64 (pcg-random.org) as numpy implements them
// (numpy/random/bit_generator.pyx, _pcg64.pyx, src/pcg64/pcg64.h,
// src/distributions/distributions.c).
//
// Plain C++ (host + device) so tests/test_rng.py can check it against numpy.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define QT_RNG_HD __device__ __forceinline__
#else
#include <cmath>
#define QT_RNG_HD inline
#endif

#include "qt_ziggurat.hpp"

namespace qt {

typedef unsigned __int128 u128;

// ---------------------------------------------------------------- SeedSequence

constexpr uint32_t kInitA = 0x43b0d7e5u, kMultA = 0x931e8875u, kInitB = 0x8b51f9ddu, kMultB = 0x58f38dedu;
constexpr uint32_t kMixMultL = 0xca01f9ddu, kMixMultR = 0x4973f715u;

QT_RNG_HD uint32_t ss_hashmix(uint32_t value, uint32_t& hash_const) {
  value ^= hash_const;
  hash_const *= kMultA;
  value *= hash_const;
  value ^= value >> 16;
  return value;
}

QT_RNG_HD uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = kMixMultL * x - kMixMultR * y;
  r ^= r >> 16;
  return r;
}

// SeedSequence(seed).generate_state(4, uint64) for a non-negative seed
// (< 2^64: at most two 32-bit entropy words, always fewer than the pool of 4).
QT_RNG_HD void seed_sequence_state(uint64_t seed, uint64_t out[4]) {
  uint32_t ent[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  const int nent = (seed >> 32) ? 2 : 1;
  uint32_t pool[4];
  uint32_t hc = kInitA;
  for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i < nent ? ent[i] : 0u, hc);
  for (int src = 0; src < 4; ++src)
    for (int dst = 0; dst < 4; ++dst)
      if (src != dst) pool[dst] = ss_mix(pool[dst], ss_hashmix(pool[src], hc));
  uint32_t hb = kInitB;
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i & 3];
    v ^= hb;
    hb *= kMultB;
    v *= hb;
    v ^= v >> 16;
    w[i] = v;
  }
  for (int i = 0; i < 4; ++i) out[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

// ---------------------------------------------------------------------- PCG64

struct Pcg64 {
  u128 state, inc;
};

constexpr uint64_t kPcgMultHi = 0x2360ED051FC65DA4ull, kPcgMultLo = 0x4385DF649FCCF645ull;

QT_RNG_HD void pcg_step(Pcg64& g) {
  const u128 mult = ((u128)kPcgMultHi << 64) | kPcgMultLo;
  g.state = g.state * mult + g.inc;
}

// PCG64(SeedSequence(seed)): pcg64_set_seed(state, val[0..1], val[2..3]) ->
// pcg_setseq_128_srandom_r (state = 0; inc = (initseq << 1) | 1; step;
// state += initstate; step).
QT_RNG_HD Pcg64 pcg64_from_seed(uint64_t seed) {
  uint64_t v[4];
  seed_sequence_state(seed, v);
  const u128 initstate = ((u128)v[0] << 64) | v[1];
  const u128 initseq = ((u128)v[2] << 64) | v[3];
  Pcg64 g;
  g.state = 0;
  g.inc = (initseq << 1) | 1;
  pcg_step(g);
  g.state += initstate;
  pcg_step(g);
  return g;
}

// Jump the generator `delta` outputs ahead (numpy's PCG64.advance:
// pcg_setseq_128_advance_r, the LCG's jump-ahead by squaring, O(log delta)).
QT_RNG_HD void pcg_advance(Pcg64& g, u128 delta) {
  u128 cur_mult = ((u128)kPcgMultHi << 64) | kPcgMultLo, cur_plus = g.inc;
  u128 acc_mult = 1, acc_plus = 0;
  while (delta > 0) {
    if (delta & 1) {
      acc_mult *= cur_mult;
      acc_plus = acc_plus * cur_mult + cur_plus;
    }
    cur_plus = (cur_mult + 1) * cur_plus;
    cur_mult *= cur_mult;
    delta >>= 1;
  }
  g.state = acc_mult * g.state + acc_plus;
}

QT_RNG_HD uint64_t pcg_next64(Pcg64& g) {
  pcg_step(g);
  const uint64_t x = (uint64_t)(g.state >> 64) ^ (uint64_t)g.state;
  const unsigned rot = (unsigned)(g.state >> 122);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

QT_RNG_HD double pcg_next_double(Pcg64& g) { return (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0); }

// log1p as glibc 2.35 computes it (sysdeps/ieee754/dbl-64/s_log1p.c: the fdlibm
// algorithm with its polynomial regrouped as R1 + z^2 R2 + z^4 R3 + z^6 R4),
// restated with the same operations in the same order and no contraction, so
// the ziggurat tail below rounds exactly as numpy's npy_log1p -> libm does on
// the device too (the device libm's log1p differs by an ulp in ~1 of 2,000
// arguments).  Bitwise equal to the host glibc over 2e8 arguments in
// (-1, 3), tests/test_rng.py.  Domain used here: x = -u, u in [0, 1).
QT_RNG_HD double fdlibm_log1p(double x) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  constexpr double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                   Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                   Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                   Lp7 = 1.479819860511658591e-01;
  const uint64_t xb = __builtin_bit_cast(uint64_t, x);
  const int32_t hx = (int32_t)(xb >> 32);
  const int32_t ax = hx & 0x7fffffff;
  double f = 0.0, c = 0.0, u;
  int32_t k = 1, hu = 0;
  if (hx < 0x3FDA827A) {  // x < 0.41422
    if (ax >= 0x3ff00000) return x == -1.0 ? -__builtin_huge_val() : __builtin_nan("");  // x <= -1
    if (ax < 0x3e200000) return ax < 0x3c900000 ? x : x - x * x * 0.5;                 // |x| < 2^-29
    if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {  // -0.2929 < x < 0.41422
      k = 0;
      f = x;
      hu = 1;
    }
  }
  if (hx >= 0x7ff00000) return x + x;
  if (k != 0) {
    if (hx < 0x43400000) {
      u = 1.0 + x;
      hu = (int32_t)(__builtin_bit_cast(uint64_t, u) >> 32);
      k = (hu >> 20) - 1023;
      c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);  // correction term
      c /= u;
    } else {
      u = x;
      hu = (int32_t)(__builtin_bit_cast(uint64_t, u) >> 32);
      k = (hu >> 20) - 1023;
      c = 0.0;
    }
    hu &= 0x000fffff;
    const uint64_t lo = __builtin_bit_cast(uint64_t, u) & 0xffffffffull;
    if (hu < 0x6a09e) {  // normalise u
      u = __builtin_bit_cast(double, lo | ((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32));
    } else {  // normalise u / 2
      k += 1;
      u = __builtin_bit_cast(double, lo | ((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32));
      hu = (0x00100000 - hu) >> 2;
    }
    f = u - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  if (hu == 0) {  // |f| < 2^-20
    if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + (c + dk * ln2_lo);
    const double R = hfsq * (1.0 - 0.66666666666666666 * f);
    return k == 0 ? f - R : dk * ln2_hi - ((R - (dk * ln2_lo + c)) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double R1 = z * Lp1, z2 = z * z, R2 = Lp2 + z * Lp3, z4 = z2 * z2, R3 = Lp4 + z * Lp5, z6 = z4 * z2,
               R4 = Lp6 + z * Lp7;
  const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + (dk * ln2_lo + c))) - f);
}

// random_standard_normal (distributions.c): 256-layer ziggurat
QT_RNG_HD double pcg_standard_normal(Pcg64& g) {
#if defined(__clang__)
#pragma clang fp contract(off)  // numpy evaluates these as separate mul / add
#endif
  for (;;) {
    uint64_t r = pcg_next64(g);
    const int idx = (int)(r & 0xff);
    r >>= 8;
    const int sign = (int)(r & 1);
    const uint64_t rabs = (r >> 1) & 0x000fffffffffffffull;
    double x = (double)rabs * kZigWi[idx];
    if (sign) x = -x;
    if (rabs < kZigKi[idx]) return x;
    if (idx == 0) {
      for (;;) {
        const double xx = -kZigNorInvR * fdlibm_log1p(-pcg_next_double(g));
        const double yy = -fdlibm_log1p(-pcg_next_double(g));
        if (yy + yy > xx * xx) return ((rabs >> 8) & 1) ? -(kZigNorR + xx) : kZigNorR + xx;
      }
    } else {
      if ((kZigFi[idx - 1] - kZigFi[idx]) * pcg_next_double(g) + kZigFi[idx] < exp(-0.5 * x * x)) return x;
    }
  }
}

}  // namespace qt
