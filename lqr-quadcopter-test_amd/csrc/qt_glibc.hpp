// qt_glibc.hpp — glibc 2.35's double sin, cos and pow(x, 2), restated
// operation for operation, for the device (and the host, for the tests).
//
// Why: the reference's figure-8 target (target_motion.py:173-229) evaluates
// np.sin / np.cos of a Python float — glibc `sin` / `cos` — and `x**2` of an
// np.float64 — glibc `pow(x, 2.0)` — and then forms the acceleration as a
// nested 1e-6 forward difference, a ~1e12 gain on the positions' last bit,
// which the feed-forward term feeds into the thrust (riccati_lqr.py:853-861).
// glibc rounds sin / cos incorrectly for ~0.15% of arguments and pow(x, 2)
// differs from x * x for ~0.2%, so only glibc's own arithmetic reproduces the
// reference's acceleration.
//
// What is restated: the x86-64 multiarch variants numpy runs on an FMA-capable
// host (this image's CPUs and the GPU box's): `__sin_fma`, `__cos_fma`
// (sysdeps/ieee754/dbl-64/s_sin.c compiled with -mfma, so GCC contracted
// a * b + c into FMAs) and `__ieee754_pow_fma` (e_pow.c, __FP_FAST_FMA
// branches plus contraction).  Every FMA below sits where the compiled glibc
// has one (read from its disassembly); every other operation is a separately
// rounded add / sub / mul, so this header is compiled with contraction off.
// Tables: qt_glibc_tables.hpp (generated from libm-2.35.a by
// scripts/gen_glibc_tables.py).  Checked bitwise against the host libm over
// >= 1e7 arguments (tests/test_math.py::test_glibc_*).
//
// Domain: sin / cos for |x| < 105414350 (glibc's `reduce_sincos` range; above
// it glibc calls `__branred`, not restated: qt::cr_sincos, correctly
// rounded, stands in, and such arguments are outside any configured episode);
// pow(x, 2.0) for every double x.
#pragma once

#include <stdint.h>

#include "qt_crtrig.hpp"
#include "qt_glibc_tables.hpp"

#if defined(__HIPCC__)
#define QT_GL_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define QT_GL_HD inline
#endif

#if defined(__clang__)
#define QT_GL_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define QT_GL_NOCONTRACT
#endif

namespace qt {
namespace glibc {

QT_GL_HD uint64_t as_u64(double x) { return __builtin_bit_cast(uint64_t, x); }
QT_GL_HD double as_f64(uint64_t u) { return __builtin_bit_cast(double, u); }

// s_sin.c / usncs.h constants (as compiled into __sin_fma's constant pool)
constexpr double kS1 = -0x1.5555555555555p-3, kS2 = 0x1.1111111110ecep-7, kS3 = -0x1.a01a019db08b8p-13,
                 kS4 = 0x1.71de27b9a7ed9p-19, kS5 = -0x1.addffc2fcdf59p-26;
constexpr double kSn3 = -0x1.5555555555515p-3, kSn5 = 0x1.11110e829872fp-7;
constexpr double kCs2 = 0x1p-1, kCs4 = -0x1.5555555555535p-5, kCs6 = 0x1.6c16bedd9e239p-10;
constexpr double kBig = 0x1.8p45;  // ulp 2^-7: big + |x| rounds |x| to the table grid i/128
constexpr double kHp0 = 0x1.921fb54442d18p0, kHp1 = 0x1.1a62633145c07p-54;  // pi/2 = hp0 + hp1
constexpr double kHpInv = 0x1.45f306dc9c883p-1, kToInt = 0x1.8p52;
constexpr double kMp1 = 0x1.921fb58p0, kMp2 = -0x1.dde973cp-27;  // pi/2 split for reduce_sincos
constexpr double kPp3 = -0x1.cb3b398p-55, kPp4 = -0x1.d747f23e32ed7p-83;

// TAYLOR_SIN (s_sin.c): sin(a + da) for |a| < 0.126
QT_GL_HD double taylor_sin(double a, double da) {
  QT_GL_NOCONTRACT
  const double xx = a * a;
  const double p = fma(fma(fma(fma(kS5, xx, kS4), xx, kS3), xx, kS2), xx, kS1);
  const double t = fma(xx, fma(p, a, -(da * 0.5)), da);
  return t + a;
}

// do_sin (s_sin.c): sin(x + dx), table step
QT_GL_HD double do_sin(double x, double dx) {
  QT_GL_NOCONTRACT
  if (fabs(x) < 0.126) return taylor_sin(x, dx);
  if (!(x > 0.0)) dx = -dx;
  const double ax = fabs(x);
  const double u = kBig + ax;
  const int k = (int)(uint32_t)as_u64(u) << 2;
  const double xr = ax - (u - kBig);
  const double xx = xr * xr;
  const double s = xr + fma(xr * xx, fma(xx, kSn5, kSn3), dx);
  const double c = fma(xr, dx, xx * fma(xx, fma(xx, kCs6, kCs4), kCs2));
  const double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
  const double cor = fma(s, cs, fma(-c, sn, fma(s, ccs, ssn)));
  return copysign(sn + cor, x);
}

// do_cos (s_sin.c): cos(x + dx), table step
QT_GL_HD double do_cos(double x, double dx) {
  QT_GL_NOCONTRACT
  if (x < 0.0) dx = -dx;
  const double ax = fabs(x);
  const double u = kBig + ax;
  const int k = (int)(uint32_t)as_u64(u) << 2;
  const double xr = (ax - (u - kBig)) + dx;
  const double xx = xr * xr;
  const double s = fma(xr * xx, fma(xx, kSn5, kSn3), xr);
  const double c = xx * fma(xx, fma(xx, kCs6, kCs4), kCs2);
  const double sn = kSinCosTab[k], ssn = kSinCosTab[k + 1], cs = kSinCosTab[k + 2], ccs = kSinCosTab[k + 3];
  const double cor = fma(-s, sn, fma(-c, cs, fma(-s, ssn, ccs)));
  return cs + cor;
}

// reduce_sincos (s_sin.c): x = n pi/2 + a + da, |x| < 105414350
QT_GL_HD int reduce_sincos(double x, double* a, double* da) {
  QT_GL_NOCONTRACT
  const double t = fma(x, kHpInv, kToInt);
  const double xn = t - kToInt;
  const double y = fma(-xn, kMp2, fma(-xn, kMp1, x));
  const int n = (int)(as_u64(t) & 3);
  const double t2 = fma(-xn, kPp3, y);
  double db = fma(-kPp3, xn, y - t2);
  const double b = fma(-xn, kPp4, t2);
  db = db + fma(-xn, kPp4, t2 - b);
  *a = b;
  *da = db;
  return n;
}

QT_GL_HD double do_sincos(double a, double da, int n) {
  const double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
  return (n & 2) ? -r : r;
}

// __sin (s_sin.c)
QT_GL_HD double sin(double x) {
  QT_GL_NOCONTRACT
  const uint32_t k = (uint32_t)(as_u64(x) >> 32) & 0x7fffffffu;
  if (k < 0x3e500000u) return x;                          // |x| < 2^-26
  if (k < 0x3feb6000u) return do_sin(x, 0.0);             // |x| < 0.855469
  if (k < 0x400368fdu) return copysign(do_cos(kHp0 - fabs(x), kHp1), x);  // |x| < 2.426265
  if (k < 0x419921fbu) {                                  // |x| < 105414350
    double a, da;
    const int n = reduce_sincos(x, &a, &da);
    return do_sincos(a, da, n);
  }
  if (k >= 0x7ff00000u) return x - x;  // inf / nan -> nan
  double s, c;
  qt::cr_sincos(x, &s, &c);  // __branred range: not restated (see header)
  return s;
}

// __cos (s_sin.c)
QT_GL_HD double cos(double x) {
  QT_GL_NOCONTRACT
  const uint32_t k = (uint32_t)(as_u64(x) >> 32) & 0x7fffffffu;
  if (k < 0x3e400000u) return 1.0;                        // |x| < 2^-27
  if (k < 0x3feb6000u) return do_cos(x, 0.0);
  if (k < 0x400368fdu) {
    const double y = kHp0 - fabs(x);
    const double a = y + kHp1;
    const double da = (y - a) + kHp1;
    return do_sin(a, da);
  }
  if (k < 0x419921fbu) {
    double a, da;
    const int n = reduce_sincos(x, &a, &da);
    return do_sincos(a, da, n + 1);
  }
  if (k >= 0x7ff00000u) return x - x;
  double s, c;
  qt::cr_sincos(x, &s, &c);
  return c;
}

// ------------------------------------------------------------- pow(x, 2)
// e_pow.c (Szabolcs Nagy's pow): log_inline -> y * log -> exp_inline, with
// the __FP_FAST_FMA branches, specialised to y = 2.0 (an even integer: the
// sign of x drops out; y itself never takes a special path).
constexpr uint64_t kPowOff = 0x3fe6955500000000ull;

// log_inline: log(x) = hi + *tail for the bit pattern ix of a positive normal x
QT_GL_HD double log_inline(uint64_t ix, double* tail) {
  QT_GL_NOCONTRACT
  const double* D = kPowLogData;  // ln2hi, ln2lo, A[0..6], tab[128][4]
  const uint64_t tmp = ix - kPowOff;
  const int i = (int)((tmp >> 45) & 127);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = as_f64(iz), kd = (double)k;
  const double invc = D[9 + 4 * i], logc = D[9 + 4 * i + 2], logctail = D[9 + 4 * i + 3];
  const double r = fma(z, invc, -1.0);
  const double t1 = fma(kd, D[0], logc);
  const double t2 = t1 + r;
  const double lo1 = fma(kd, D[1], logctail);
  const double lo2 = (t1 - t2) + r;
  const double ar = r * D[2];
  const double ar2 = r * ar;
  const double ar3 = r * ar2;
  const double hi = t2 + ar2;
  const double lo3 = fma(ar, r, -ar2);
  const double lo4 = (t2 - hi) + ar2;
  const double q = fma(ar2, fma(r, D[8], D[7]), fma(r, D[6], D[5]));
  const double pin = fma(ar2, q, fma(r, D[4], D[3]));
  const double lo = fma(ar3, pin, ((lo1 + lo2) + lo3) + lo4);
  const double y = hi + lo;
  *tail = (hi - y) + lo;
  return y;
}

// exp_inline's specialcase: scale * (1 + tmp) near the over/underflow range
QT_GL_HD double exp_specialcase(double tmp, uint64_t sbits, uint64_t ki) {
  QT_GL_NOCONTRACT
  if ((ki & 0x80000000ull) == 0) {
    const double scale = as_f64(sbits - (1009ull << 52));
    return fma(tmp, scale, scale) * 0x1p1009;
  }
  sbits += 1022ull << 52;
  const double scale = as_f64(sbits);
  const double st = tmp * scale;
  double y = scale + st;
  if (fabs(y) < 1.0) {
    const double one = y < 0.0 ? -1.0 : 1.0;
    double lo = (scale - y) + st;
    const double hi = y + one;
    lo = ((one - hi) + y) + lo;
    y = (lo + hi) - one;
    if (y == 0.0) y = as_f64(sbits & 0x8000000000000000ull);
  }
  return y * 0x1p-1022;
}

// exp_inline (sign_bias 0): exp(x + xtail)
QT_GL_HD double exp_inline(double x, double xtail) {
  QT_GL_NOCONTRACT
  const uint64_t* E = kExpData;  // invln2N, shift, negln2hiN, negln2loN, C2..C5, ..., tab at 14
  uint32_t abstop = (uint32_t)(as_u64(x) >> 52) & 0x7ff;
  if (abstop - 0x3c9u >= 0x3fu) {
    if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;
    if (abstop >= 0x409u) return (as_u64(x) >> 63) ? 0x1p-767 * 0x1p-767 : 0x1p769 * 0x1p769;
    abstop = 0;
  }
  double kd = fma(x, as_f64(E[0]), as_f64(E[1]));
  const uint64_t ki = as_u64(kd);
  kd = kd - as_f64(E[1]);
  double r = fma(kd, as_f64(E[2]), x);
  r = fma(kd, as_f64(E[3]), r);
  const uint64_t idx = 2 * (ki & 127);
  const uint64_t top = ki << 45;
  const uint64_t sbits = E[14 + idx + 1] + top;
  r = xtail + r;
  const double tail = as_f64(E[14 + idx]);
  const double a1 = fma(r, as_f64(E[5]), as_f64(E[4]));
  const double b = tail + r;
  const double r2 = r * r;
  const double a2 = fma(r, as_f64(E[7]), as_f64(E[6]));
  double tmp = fma(a1, r2, b);
  tmp = fma(a2, r2 * r2, tmp);
  if (abstop == 0) return exp_specialcase(tmp, sbits, ki);
  const double scale = as_f64(sbits);
  return fma(tmp, scale, scale);
}

// __ieee754_pow_fma(x, 2.0)
QT_GL_HD double pow2(double x) {
  QT_GL_NOCONTRACT
  uint64_t ix = as_u64(x);
  const uint32_t topx = (uint32_t)(ix >> 52);
  if (topx - 1u >= 0x7feu) {  // x <= 0, subnormal, inf or nan
    if (2 * ix - 1 >= 0xffdfffffffffffffull) return x * x;  // +-0, +-inf, nan
    ix &= 0x7fffffffffffffffull;                                // x < 0, y even
    if ((topx & 0x7ff) == 0) {                                  // subnormal: normalise
      ix = as_u64(x * 0x1p52) & 0x7fffffffffffffffull;
      ix -= 52ull << 52;
    }
  }
  double lo;
  const double hi = log_inline(ix, &lo);
  const double ehi = 2.0 * hi;
  const double elo = fma(2.0, lo, fma(hi, 2.0, -ehi));
  return exp_inline(ehi, elo);
}

}  // namespace glibc
}  // namespace qt
