// qt_crtrig.hpp — sin / cos correctly rounded (double-double evaluation).
//
// The reference evaluates np.sin / np.cos, i.e. glibc's sin / cos, which are
// correctly rounded for all but ~0.15% of arguments (measured against mpmath
// at 200 bits, tests/test_math.py).  The device's fast_sincos (qt_math.hpp,
// <= 2 ulp) is enough everywhere except where the reference amplifies the
// last bit: the figure-8 acceleration is a nested 1e-6 forward difference of
// positions (target_motion.py:215-229), a 1e12 gain on the sin / cos
// rounding, which the feed-forward term then feeds into the thrust
// (riccati_lqr.py:853-861).  There this header's cr_sincos is used, so the
// device's figure-8 acceleration equals the reference's whenever glibc
// rounds correctly.
//
// Method: Cody-Waite reduction r = x - k pi/2 with pi/2 in four parts
// (k pi/2_1 exact by FMA, x - k pi/2_1 exact by Sterbenz), r kept as a
// double-double; sin / cos of |r| <= pi/4 (+ rounding slack) by Taylor series
// whose leading terms run in double-double and whose tail (r^9 / 9! and
// beyond, r^10 / 10! for cos) runs in double: total relative error < 2^-72,
// so the result rounds correctly unless the exact value lies within 2^-19
// ulp of a rounding midpoint.  |x| >= 2^30 or non-finite x: not used here
// (the caller's angles are omega t); returns NaN for non-finite x.
//
// Plain C++ (host + device) so tests/test_math.py can check it on the host.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define QT_CR_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define QT_CR_HD inline
#endif

namespace qt {
namespace cr {

#if defined(__clang__)
#define QT_CR_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define QT_CR_NOCONTRACT
#endif

struct DD {
  double h, l;
};

QT_CR_HD DD two_sum(double a, double b) {
  QT_CR_NOCONTRACT
  const double s = a + b;
  const double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}

QT_CR_HD DD quick_two_sum(double a, double b) {  // |a| >= |b|
  QT_CR_NOCONTRACT
  const double s = a + b;
  return {s, b - (s - a)};
}

QT_CR_HD DD two_prod(double a, double b) {
  QT_CR_NOCONTRACT
  const double p = a * b;
  return {p, fma(a, b, -p)};
}

QT_CR_HD DD add(DD a, DD b) {
  QT_CR_NOCONTRACT
  DD s = two_sum(a.h, b.h);
  const DD t = two_sum(a.l, b.l);
  s.l += t.h;
  s = quick_two_sum(s.h, s.l);
  s.l += t.l;
  return quick_two_sum(s.h, s.l);
}

QT_CR_HD DD mul(DD a, DD b) {
  QT_CR_NOCONTRACT
  DD p = two_prod(a.h, b.h);
  p.l += a.h * b.l + a.l * b.h;
  return quick_two_sum(p.h, p.l);
}

QT_CR_HD DD mul_d(DD a, double b) {
  QT_CR_NOCONTRACT
  DD p = two_prod(a.h, b);
  p.l += a.l * b;
  return quick_two_sum(p.h, p.l);
}

// pi/2 = P1 + P2 + P3 + P4 (each the rounding of the remainder)
constexpr double kP1 = 1.5707963267948966, kP2 = 6.123233995736766e-17, kP3 = -1.4973849048591698e-33,
                 kP4 = 5.562271104316826e-50, kTwoOverPi = 0.6366197723675814;

// x - k pi/2 as a double-double (k integral, |k| < 2^30)
QT_CR_HD DD reduce(double x, double k) {
  QT_CR_NOCONTRACT
  const DD p1 = two_prod(k, kP1);
  DD r = {x - p1.h, 0.0};  // exact: x and k P1 within a factor 2 (or k = 0)
  r = add(r, DD{-p1.l, 0.0});
  r = add(r, two_prod(-k, kP2));
  r = add(r, two_prod(-k, kP3));
  return add(r, DD{-k * kP4, 0.0});
}

// sin(r), cos(r) for |r| <= pi/4 + slack, r double-double
QT_CR_HD void sincos_reduced(DD r, DD* s, DD* c) {
  QT_CR_NOCONTRACT
  const DD r2 = mul(r, r);
  const double z = r2.h;
  // sin: r + r r2 (-1/3! + r2 (1/5! + r2 (-1/7! + r2 T))), T = 1/9! - z/11! + ... + z^8/25!
  double T = 6.446950284384474e-26;
  T = -3.868170170630684e-23 + z * T;
  T = 1.9572941063391263e-20 + z * T;
  T = -8.22063524662433e-18 + z * T;
  T = 2.8114572543455206e-15 + z * T;
  T = -7.647163731819816e-13 + z * T;
  T = 1.6059043836821613e-10 + z * T;
  T = -2.505210838544172e-08 + z * T;
  T = 2.7557319223985893e-06 + z * T;
  DD a = add(DD{-0.0001984126984126984, -1.7209558293420705e-22}, mul_d(r2, T));
  a = add(DD{0.008333333333333333, 1.1564823173178714e-19}, mul(r2, a));
  a = add(DD{-0.16666666666666666, -9.25185853854297e-18}, mul(r2, a));
  *s = add(r, mul(r, mul(r2, a)));
  // cos: 1 + r2 (-1/2 + r2 (1/4! + r2 (-1/6! + r2 (1/8! + r2 U)))), U = -1/10! + z/12! - ... + z^7/24!
  double U = 1.6117375710961184e-24;
  U = -8.896791392450574e-22 + z * U;
  U = 4.110317623312165e-19 + z * U;
  U = -1.5619206968586225e-16 + z * U;
  U = 4.779477332387385e-14 + z * U;
  U = -1.1470745597729725e-11 + z * U;
  U = 2.08767569878681e-09 + z * U;
  U = -2.755731922398589e-07 + z * U;
  DD b = add(DD{2.48015873015873e-05, 2.1511947866775882e-23}, mul_d(r2, U));
  b = add(DD{-0.001388888888888889, 5.300543954373577e-20}, mul(r2, b));
  b = add(DD{0.041666666666666664, 2.3129646346357427e-18}, mul(r2, b));
  b = add(DD{-0.5, 0.0}, mul(r2, b));
  *c = add(DD{1.0, 0.0}, mul(r2, b));
}

}  // namespace cr

// sin(x), cos(x) correctly rounded except within 2^-19 ulp of a midpoint
QT_CR_HD void cr_sincos(double x, double* sp, double* cp) {
  QT_CR_NOCONTRACT
  if (!(fabs(x) < 1073741824.0)) {  // 2^30; NaN / inf
    *sp = *cp = __builtin_bit_cast(double, 0x7ff8000000000000ull);  // NaN
    return;
  }
  const double k = rint(x * cr::kTwoOverPi);
  cr::DD s, c;
  cr::sincos_reduced(cr::reduce(x, k), &s, &c);
  const int q = (int)((long long)k & 3);
  const double sv = s.h + s.l, cv = c.h + c.l;
  *sp = q == 0 ? sv : q == 1 ? cv : q == 2 ? -sv : -cv;
  *cp = q == 0 ? cv : q == 1 ? -sv : q == 2 ? -cv : sv;
}

}  // namespace qt
