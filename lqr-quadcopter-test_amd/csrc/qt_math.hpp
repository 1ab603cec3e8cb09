// qt_math.hpp — FP64 elementary functions for the closed-loop kernels.
//
// The library sin/cos carry a Payne-Hanek path for huge arguments that costs
// registers and branches in every call; on this path every argument is small
// (attitude angles are wrapped to [-pi, pi] each step and move <= 0.11 rad
// inside an RK4 step; target phases stay below ~2e3 rad), so a Cody-Waite
// reduction by pi/2 with a 3-part constant and the classic minimax kernels on
// [-pi/4, pi/4] give <= ~1 ulp results in ~30 straight-line operations.
//
// Plain C++ so that the same header builds for the host (tests/test_math.py
// checks it against numpy) and for gfx950.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define QT_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define QT_HD inline
#endif

namespace qt {

// pi/2 = P1 + P2 + P3 (each the double nearest the remaining tail)
constexpr double kPio2_1 = 1.5707963267948966;
constexpr double kPio2_2 = 6.123233995736766e-17;
constexpr double kPio2_3 = -1.4973849048591698e-33;
constexpr double kTwoOverPi = 0.6366197723675814;

// minimax polynomials on [-pi/4, pi/4] (the fdlibm kernel coefficients)
constexpr double kS1 = -1.66666666666666324348e-01, kS2 = 8.33333333332248946124e-03,
                 kS3 = -1.98412698298579493134e-04, kS4 = 2.75573137070700676789e-06,
                 kS5 = -2.50507602534068634195e-08, kS6 = 1.58969099521155010221e-10;
constexpr double kC1 = 4.16666666666666019037e-02, kC2 = -1.38888888888741095749e-03,
                 kC3 = 2.48015872894767294178e-05, kC4 = -2.75573143513906633035e-07,
                 kC5 = 2.08757232129817482790e-09, kC6 = -1.13596475577881948265e-11;

QT_HD void sincos_kernel(double r, double* s, double* c) {
  const double z = r * r;
  const double v = z * r;
  const double ps = kS2 + z * (kS3 + z * (kS4 + z * (kS5 + z * kS6)));
  *s = r + v * (kS1 + z * ps);
  const double pc = z * (kC1 + z * (kC2 + z * (kC3 + z * (kC4 + z * (kC5 + z * kC6)))));
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  *c = w + (((1.0 - w) - hz) + z * pc);
}

// sin and cos of x.  Accurate (<= ~1 ulp) for |x| < 2^40; NaN and Inf give
// NaN.  Domain on this path: |x| < 2e3 (see the header comment).
QT_HD void fast_sincos(double x, double* s, double* c) {
  const double k = rint(x * kTwoOverPi);
  double r = fma(-k, kPio2_1, x);
  r = fma(-k, kPio2_2, r);
  r = fma(-k, kPio2_3, r);
  double sr, cr;
  sincos_kernel(r, &sr, &cr);
  const int q = static_cast<int>(k) & 3;
  const double s01 = (q & 1) ? cr : sr;
  const double c01 = (q & 1) ? -sr : cr;
  *s = (q & 2) ? -s01 : s01;
  *c = (q & 2) ? -c01 : c01;
}

// sin / cos of a small angle, |d| <= kSmallAngle, by Taylor polynomials whose
// truncation error is below 3e-17 relative on that range (next terms
// d^11/11! and d^12/12!).  RK4 stage offsets are dt * body rate <= ~0.113 rad
// at the default limits.
constexpr double kSmallAngle = 0.125;

// The Taylor coefficients of small_sincos, resid_sincos and tiny_sincos as
// values (defaults: the literals, which the optimiser folds as before).  A
// loop short of scalar registers (the exact step) pins them in vector
// registers once (pin: no instruction emitted) instead of re-materialising
// each 64-bit constant with two s_mov per use.
struct SmallCoef {
  double s9 = 2.7557319223985893e-06;   // 1/9!
  double s7 = -1.9841269841269841e-04;  // -1/7!
  double s5 = 8.3333333333333332e-03;   // 1/5!
  double s3 = -1.6666666666666666e-01;  // -1/3!
  double c10 = -2.7557319223985888e-07;  // -1/10!
  double c8 = 2.4801587301587302e-05;   // 1/8!
  double c6 = -1.3888888888888889e-03;  // -1/6!
  double c4 = 4.1666666666666664e-02;   // 1/4!
  double third = 3.3333333333333331e-01;  // tiny_sincos' 1/3
#if defined(__HIP_DEVICE_COMPILE__)
  __device__ __forceinline__ void pin() {
    asm("" : "+v"(s9), "+v"(s7), "+v"(s5), "+v"(s3), "+v"(c10), "+v"(c8), "+v"(c6), "+v"(c4), "+v"(third));
  }
#else
  void pin() {}
#endif
};

QT_HD void small_sincos(double d, double* s, double* c, const SmallCoef& k = SmallCoef{}) {
  const double z = d * d;
  double p = k.s9;  // 1/9!
  p = fma(z, p, k.s7);  // -1/7!
  p = fma(z, p, k.s5);  // 1/5!
  p = fma(z, p, k.s3);  // -1/3!
  *s = fma(d * z, p, d);
  double q = k.c10;  // -1/10!
  q = fma(z, q, k.c8);  // 1/8!
  q = fma(z, q, k.c6);  // -1/6!
  q = fma(z, q, k.c4);  // 1/4!
  q = fma(z, q, -0.5);
  *c = fma(z, q, 1.0);
}

// sin / cos of an attitude inside the tilt clamp, |a| <= pi/3 (roll / pitch
// at the start of a fast step: clamped to +-pi/3 every step, checked at
// kernel entry), without argument reduction or quadrant selects: Taylor
// polynomials to a^17 / a^18, whose truncation error is below 2e-17 (sin,
// the a^19 / 19! term) and 1.1e-18 (cos) there; <= 1 ulp (sin) / 2 ulp (cos:
// its last step 1 + z q rounds at ulp(1) / 2).
QT_HD void sincos_tilt(double a, double* s, double* c) {
  const double z = a * a;
  double p = 2.8114572543455206e-15;      // 1/17!
  p = fma(z, p, -7.647163731819816e-13);  // -1/15!
  p = fma(z, p, 1.6059043836821613e-10);  // 1/13!
  p = fma(z, p, -2.505210838544172e-08);  // -1/11!
  p = fma(z, p, 2.7557319223985893e-06);  // 1/9!
  p = fma(z, p, -1.9841269841269841e-04);  // -1/7!
  p = fma(z, p, 8.3333333333333332e-03);  // 1/5!
  p = fma(z, p, -1.6666666666666666e-01);  // -1/3!
  *s = fma(a * z, p, a);
  double q = -1.5619206968586225e-16;     // -1/18!
  q = fma(z, q, 4.779477332387385e-14);   // 1/16!
  q = fma(z, q, -1.1470745597729725e-11);  // -1/14!
  q = fma(z, q, 2.08767569878681e-09);    // 1/12!
  q = fma(z, q, -2.7557319223985888e-07);  // -1/10!
  q = fma(z, q, 2.4801587301587302e-05);  // 1/8!
  q = fma(z, q, -1.3888888888888889e-03);  // -1/6!
  q = fma(z, q, 4.1666666666666664e-02);  // 1/4!
  q = fma(z, q, -0.5);
  *c = fma(z, q, 1.0);
}

// sin / cos of an RK4 stage offset of a rate-bounded step, |d| <= kRateAngle
// (dt * max commanded rate: 0.03 at the defaults): Taylor polynomials to d^7 /
// d^6, truncation below 8e-20 (sin) and 2.2e-17 (cos, the d^8 / 8! term).
constexpr double kRateAngle = 0.031;

// The two leading coefficients as values: a loop can hold them in vector
// registers (RateCoef::pin), since an fma takes one scalar-register operand
// and the next coefficient already is one.
struct RateCoef {
  double s7 = -1.9841269841269841e-04;  // -1/7!
  double c6 = -1.3888888888888889e-03;  // -1/6!
  double s5 = 8.3333333333333332e-03;   // 1/5! (resid_sincos)
#if defined(__HIP_DEVICE_COMPILE__)
  // opaque to the optimiser: kept in VGPRs across a loop instead of being
  // re-materialised from scalar registers each trip (no instruction emitted)
  __device__ __forceinline__ void pin() { asm("" : "+v"(s7), "+v"(c6), "+v"(s5)); }
#else
  void pin() {}
#endif
};

QT_HD void rate_sincos(double d, double* s, double* c, const RateCoef& k = RateCoef{}) {
  const double z = d * d;
  double p = fma(z, k.s7, 8.3333333333333332e-03);  // 1/5!
  p = fma(z, p, -1.6666666666666666e-01);  // -1/3!
  *s = fma(d * z, p, d);
  double q = fma(z, k.c6, 4.1666666666666664e-02);  // 1/4!
  q = fma(z, q, -0.5);
  *c = fma(z, q, 1.0);
}

// sin d and cos d - 1 of the residual between two nearby RK4 stage offsets
// (the yaw-at-rest step's third stage relative to its second),
// |d| <= kStage3Angle: Taylor polynomials to d^5 / d^4, truncation below
// 3e-21 (sin) and 5.7e-18 (cos - 1, the d^6 / 6! term).  The rotation takes
// cos d - 1 (rotate_cm), so that no digit of the small correction is lost to
// the rounding of cos d near 1.
constexpr double kStage3Angle = 4e-3;

QT_HD void resid_sincos(double d, double* s, double* cm, const RateCoef& k = RateCoef{}) {
  const double z = d * d;
  const double p = fma(z, k.s5, -1.6666666666666666e-01);  // -1/3!
  *s = fma(d * z, p, d);
  const double q = fma(z, 4.1666666666666664e-02, -0.5);  // 1/4!, -1/2!
  *cm = z * q;
}

// sin d and cos d - 1 of a tiny angle, |d| <= kAdvanceAngle: d - d^3 / 6 and
// -d^2 / 2, truncation below 3e-22 (sin) and 4.2e-18 (cos - 1).
constexpr double kAdvanceAngle = 1e-4;

QT_HD void tiny_sincos(double d, double* s, double* cm, const SmallCoef& k = SmallCoef{}) {
  *cm = d * (-0.5 * d);
  *s = fma(d * *cm, k.third, d);  // d + d (-d^2 / 2) / 3
}

// (s, c) rotated by the angle whose sine is sd and cosine 1 + cm:
// s' = s + (s cm + c sd), c' = c + (c cm - s sd)
QT_HD void rotate_cm(double s0, double c0, double sd, double cm, double* s, double* c) {
  *s = fma(c0, sd, fma(s0, cm, s0));
  *c = fma(-s0, sd, fma(c0, cm, c0));
}

#if defined(__HIPCC__)
// sqrt(x) of a non-negative finite x, correctly rounded for x >= 2^-767
// (sqrt_noscale's sequence) and a tiny positive value instead of 0 for
// x < 2^-1000 (the zero test becomes one max: a tracking error below 1e-150 m
// reads as ~1e-150 m, which no metric or comparison can show).
__device__ __forceinline__ double sqrt_pos(double x) {
  x = fmax(x, 0x1p-1000);
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
}

// sqrt_pos without its final correction: within an ulp of sqrt(x) (one
// Goldschmidt step on v_rsq_f64 and one Newton correction), for sums whose
// terms need no correct rounding (the control-effort metric).
__device__ __forceinline__ double sqrt_sum(double x) {
  x = fmax(x, 0x1p-1000);
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  const double d = fma(-g, g, x);
  return fma(d, h, g);
}

// sqrt(x) for the metric accumulators of the fast step: the device library's
// correctly rounded sequence (v_rsq_f64 + two Goldschmidt / Newton
// corrections) without its rescaling of x < 2^-767.  Bit-identical to sqrt
// for x >= 2^-767 and for x == 0; below that (a tracking error under 1e-115 m
// or a command norm under 1e-115) it may differ in the last bits, which no
// metric can show.  x must be finite and >= 0.
__device__ __forceinline__ double sqrt_noscale(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  g = fma(d, h, g);
  return x == 0.0 ? x : g;
}
#endif

// numpy's float remainder: (a % b) with the sign of b, b = 2*pi here
// (quadcopter_env.py:457).  For |a| < 4*pi the single subtraction / addition
// is exact (Sterbenz), so it equals fmod bit for bit; larger |a| use fmod.
QT_HD double py_mod_2pi(double a, double two_pi) {
  double m;
  if (fabs(a) < 2.0 * two_pi) {
    m = a >= two_pi ? a - two_pi : (a <= -two_pi ? a + two_pi : a);
  } else {
    m = fmod(a, two_pi);
  }
  if (m != 0.0) {
    if (m < 0) m += two_pi;
  } else {
    m = 0.0;
  }
  return m;
}

}  // namespace qt
