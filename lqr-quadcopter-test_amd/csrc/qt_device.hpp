// qt_device.hpp — per-episode device math of the closed loop, FP64.
//
// Everything here is a register-resident restatement of one episode's
// arithmetic; the kernels in qt_rollout.hip map one episode to one lane and
// keep state, target, gains and accumulators in VGPRs (shared gains in
// SGPRs) across thousands of steps.  Reference functions are cited as
// file:line relative to src/quadcopter_tracking/ of the reference repo.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/quadtrack.h"
#include "qt_glibc.hpp"
#include "qt_math.hpp"

namespace qt {

constexpr double kPi = 3.141592653589793;
constexpr double kTwoPi = 6.283185307179586;  // 2 * np.pi
constexpr double kMaxTilt = kPi / 3.0;        // math.pi / 3 (quadcopter_env.py:461)

// np.clip == minimum(maximum(v, lo), hi): NaN propagates (a NaN action is
// zeroed later by the env, quadcopter_env.py:266-269).
__device__ __forceinline__ double clipd(double v, double lo, double hi) {
  double r = v < lo ? lo : v;
  return r > hi ? hi : r;
}

// np.linalg.norm of a 1-D 3-vector: sqrt(v.dot(v)), and the image's OpenBLAS
// ddot accumulates with FMA, i.e. sqrt(fma(c, c, fma(b, b, a * a))) (the
// reference's velocity clamp, acceleration clamp, direction normalisation,
// feed-forward magnitudes and LQI error norm; quadcopter_env.py:443,
// target_motion.py:47, 321, 403, riccati_lqr.py:839, 858, 873).  Metrics
// rows (np.linalg.norm(..., axis=1)) are plain sums instead (sq3_ref).
__device__ __forceinline__ double dot3_blas(double a, double b, double c) { return fma(c, c, fma(b, b, a * a)); }
__device__ __forceinline__ double norm3(double a, double b, double c) { return sqrt(dot3_blas(a, b, c)); }

// np.sign equality used by the LQI anti-windup (riccati_lqr.py:881-883):
// sign(NaN) is NaN, which equals nothing.
__device__ __forceinline__ bool same_sign(double a, double b) {
  if (a != a || b != b) return false;
  int sa = (a > 0) - (a < 0), sb = (b > 0) - (b < 0);
  return sa == sb;
}

// A rare per-lane case handled in a wave-uniform branch: the common case is
// computed branch-free for every lane, and only a wavefront holding a lane
// that needs the rare path enters it (one ballot and a not-taken scalar
// branch otherwise).  Each lane's result depends on its own inputs only.
__device__ __forceinline__ bool any_lane(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// ---------------------------------------------------------------- target

// Per-episode constants of a motion pattern, precomputed once per launch.
struct Pattern {
  double c0, c1, c2;  // linear: velocity xyz | circular: theta0, omega | sinusoidal: phases
  double o0, o1, o2;  // sinusoidal: omegas | figure8: omega | circular: pow(omega, 2)
};

// TargetMotion._create_pattern + pattern constructors (target_motion.py:306-369,
// 32-49, 62-82, 121-140, 156-172): raw draw -> per-episode constants.
__device__ __forceinline__ Pattern make_pattern(const qt_env_params& e, int motion, double r0, double r1,
                                                double r2) {
  Pattern p{0, 0, 0, 0, 0, 0};
  if (motion == QT_MOTION_LINEAR) {
    // direction /= norm (321), then direction / norm(direction) (47), * speed (49)
    double n1 = norm3(r0, r1, r2);
    double d0 = r0 / n1, d1 = r1 / n1, d2 = r2 / n1;
    double n2 = norm3(d0, d1, d2);
    p.c0 = (d0 / n2) * e.speed;
    p.c1 = (d1 / n2) * e.speed;
    p.c2 = (d2 / n2) * e.speed;
  } else if (motion == QT_MOTION_CIRCULAR) {
    p.c0 = r0;
    p.c1 = e.speed / e.radius;
    p.o0 = glibc::pow2(p.c1);  // omega**2 of a Python float: libm pow (target_motion.py:107)
  } else if (motion == QT_MOTION_SINUSOIDAL) {
    p.c0 = r0;
    p.c1 = r1;
    p.c2 = r2;
    p.o0 = 2.0 * kPi * e.frequency;
    p.o1 = 2.0 * kPi * (e.frequency * 1.3);
    p.o2 = 2.0 * kPi * (e.frequency * 0.7);
  } else if (motion == QT_MOTION_FIGURE8) {
    p.o0 = e.speed / e.amplitude;
  }
  return p;
}

struct Target {
  double p[3], v[3], a[3];
};

// Position / velocity / acceleration of a periodic pattern from the sin / cos
// of its angles (circular target_motion.py:84-100, sinusoidal 142-153).
// Every branch forms all nine components as values and o is written once at
// the end: stores of different fields in the two branches would otherwise be
// sunk into one store through a pointer phi, which keeps the Target in
// scratch memory.
template <bool WANT_ACC>
__device__ __forceinline__ void periodic_state(const qt_env_params& e, int motion, const Pattern& pt,
                                               const double* s, const double* c, Target& o) {
  double p[3], v[3], a[3];
  if (motion == QT_MOTION_CIRCULAR) {
    const double r = e.radius, om = pt.c1;
    p[0] = e.center[0] + r * c[0];
    p[1] = e.center[1] + r * s[0];
    p[2] = e.center[2];
    v[0] = -r * om * s[0];
    v[1] = r * om * c[0];
    v[2] = 0.0;
    a[0] = WANT_ACC ? -r * pt.o0 * c[0] : 0.0;
    a[1] = WANT_ACC ? -r * pt.o0 * s[0] : 0.0;
    a[2] = 0.0;
  } else {
    const double amp[3] = {e.amplitude, e.amplitude * 0.5, e.amplitude * 0.25};
    const double om[3] = {pt.o0, pt.o1, pt.o2};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      p[i] = e.center[i] + amp[i] * s[i];
      v[i] = amp[i] * om[i] * c[i];
      a[i] = WANT_ACC ? -amp[i] * (om[i] * om[i]) * s[i] : 0.0;
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) o.p[i] = p[i], o.v[i] = v[i], o.a[i] = a[i];
}

// TargetMotion.get_state's acceleration clamp (target_motion.py:403-405).
__device__ __forceinline__ void clamp_acceleration(const qt_env_params& e, Target& o) {
  double am = norm3(o.a[0], o.a[1], o.a[2]);
  if (am > e.max_acceleration) {
#pragma unroll
    for (int i = 0; i < 3; ++i) o.a[i] = o.a[i] / am * e.max_acceleration;
  }
}

// The periodic patterns' angles at time t: circular theta0 + omega t
// (target_motion.py:84-86), sinusoidal 2 pi f_i t + phase_i (142-147).
// Returns the number of angles (1 or 3).
__device__ __forceinline__ int periodic_angles(int motion, const Pattern& pt, double t, double* th) {
  if (motion == QT_MOTION_CIRCULAR) {
    th[0] = pt.c0 + pt.c1 * t;
    return 1;
  }
  th[0] = pt.o0 * t + pt.c0;
  th[1] = pt.o1 * t + pt.c1;
  th[2] = pt.o2 * t + pt.c2;
  return 3;
}

// Figure-8 position / velocity (target_motion.py:173-204) from sin / cos of
// theta = omega t, without the acceleration: the four divisions by den and
// den^2 as one reciprocal (within an ulp) and products (<= 3 ulp per
// component; without feed-forward no forward difference reads them).
__device__ __forceinline__ void figure8_recip(const qt_env_params& e, double om, double st, double ct, Target& o) {
  const double sc = e.amplitude;
  const double den = 1.0 + st * st;
  const double dcos = -st * om, dsin = ct * om;
  const double dden = 2.0 * st * dsin;
  // 1 / den for den in [1, 2]: v_rcp_f64's estimate and two Newton steps
  // (within an ulp; the division's scale / fixup steps are not needed there)
  double r = __builtin_amdgcn_rcp(den);
  r = fma(r, fma(-den, r, 1.0), r);
  r = fma(r, fma(-den, r, 1.0), r);
  const double r2 = r * r;
  o.p[0] = e.center[0] + sc * ct * r;
  o.p[1] = e.center[1] + sc * st * ct * r;
  o.p[2] = e.center[2];
  o.v[0] = sc * ((dcos * den - ct * dden) * r2);
  o.v[1] = sc * (((dsin * ct + st * dcos) * den - st * ct * dden) * r2);
  o.v[2] = 0.0;
  o.a[0] = o.a[1] = o.a[2] = 0.0;
}

// pattern.get_state(t) (target_motion.py:51-248) + TargetMotion.get_state's
// acceleration clamp (403-405).  WANT_ACC = false skips the acceleration,
// which only the feed-forward path reads (riccati_lqr.py:853-861).
// RECIP (fast step, no acceleration wanted): the figure-8's four divisions
// by den and den^2 become one reciprocal (within an ulp) and products
// (<= 3 ulp per component; without feed-forward no forward difference reads
// them).
template <bool WANT_ACC, bool RECIP = false>
__device__ __forceinline__ void target_state(const qt_env_params& e, int motion, const Pattern& pt, double t,
                                             Target& o) {
  if (motion == QT_MOTION_LINEAR) {
    o.p[0] = e.center[0] + pt.c0 * t;
    o.p[1] = e.center[1] + pt.c1 * t;
    o.p[2] = e.center[2] + pt.c2 * t;
    o.v[0] = pt.c0;
    o.v[1] = pt.c1;
    o.v[2] = pt.c2;
    o.a[0] = o.a[1] = o.a[2] = 0.0;
  } else if (motion == QT_MOTION_CIRCULAR || motion == QT_MOTION_SINUSOIDAL) {
    double th[3], s[3], c[3];
    const int na = periodic_angles(motion, pt, t, th);
#pragma unroll
    for (int i = 0; i < 3; ++i)  // compile-time indices: the arrays stay in registers
      if (i < na) fast_sincos(th[i], &s[i], &c[i]);
    periodic_state<WANT_ACC>(e, motion, pt, s, c, o);
  } else if (motion == QT_MOTION_FIGURE8 && RECIP && !WANT_ACC) {
    double st, ct;
    fast_sincos(pt.o0 * t, &st, &ct);
    figure8_recip(e, pt.o0, st, ct, o);
  } else if (motion == QT_MOTION_FIGURE8) {
    // With the acceleration wanted (feed-forward) the forward difference
    // below multiplies the positions' last bit by ~1e12, so they are formed
    // exactly as numpy forms them: glibc's sin / cos and pow(x, 2)
    // (qt_glibc.hpp, bitwise the host libm) and no FMA contraction.
#pragma clang fp contract(off)
    const double sc = e.amplitude, om = pt.o0;
    double st, ct;
    if (WANT_ACC) {
      ct = glibc::cos(om * t);
      st = glibc::sin(om * t);
    } else {
      fast_sincos(om * t, &st, &ct);
    }
    const double den = 1.0 + (WANT_ACC ? glibc::pow2(st) : st * st);
    const double dcos = -st * om, dsin = ct * om;
    const double dden = 2.0 * st * dsin;
    const double den2 = WANT_ACC ? glibc::pow2(den) : den * den;
    const double p0 = e.center[0] + sc * ct / den;
    const double p1 = e.center[1] + sc * st * ct / den;
    const double v0 = sc * ((dcos * den - ct * dden) / den2);
    const double v1 = sc * (((dsin * ct + st * dcos) * den - st * ct * dden) / den2);
    double a0 = 0.0, a1 = 0.0;
    if (WANT_ACC) {
      // the reference's 1e-6 forward difference (target_motion.py:215-229)
      const double h = 1e-6;
      const double thp = om * (t + h);
      const double ctp = glibc::cos(thp), stp = glibc::sin(thp);
      const double denp = 1.0 + glibc::pow2(stp);
      const double pp0 = e.center[0] + sc * ctp / denp;
      const double pp1 = e.center[1] + sc * stp * ctp / denp;
      a0 = ((pp0 - p0) / h - v0) / h;
      a1 = ((pp1 - p1) / h - v1) / h;
    }
    o.p[0] = p0, o.p[1] = p1, o.p[2] = e.center[2];
    o.v[0] = v0, o.v[1] = v1, o.v[2] = 0.0;
    o.a[0] = a0, o.a[1] = a1, o.a[2] = 0.0;
  } else {  // stationary
    o.p[0] = e.center[0], o.p[1] = e.center[1], o.p[2] = e.center[2];
    o.v[0] = o.v[1] = o.v[2] = 0.0;
    o.a[0] = o.a[1] = o.a[2] = 0.0;
  }
  if (WANT_ACC) clamp_acceleration(e, o);
}

// Fast-step target of a periodic pattern (MOTION circular: one angle,
// sinusoidal: three) with the sin / cos of its angles carried across steps.
// Each step forms the angles exactly as target_state does (same expression,
// same rounding) and rotates the carried sin / cos by the increment
// d = theta_k - theta_{k-1} (~ omega dt: 0.041 rad for the default
// sinusoid; small_sincos, |d| <= kSmallAngle) by angle addition, so they
// follow sin / cos of the rounded angle the reference evaluates, with a drift
// of a few ulp per step and none from t's accumulated rounding.  A wave with
// an increment outside small_sincos's range takes fast_sincos for that step
// (a uniform branch).
template <int MOTION>
struct PeriodicTrig {
  static constexpr int NA = MOTION == QT_MOTION_SINUSOIDAL ? 3 : 1;
  double th[NA], s[NA], c[NA];
};

template <int MOTION>
__device__ __forceinline__ void periodic_trig_init(const Pattern& pt, double t, PeriodicTrig<MOTION>& r) {
  double th[3];
  periodic_angles(MOTION, pt, t, th);
#pragma unroll
  for (int i = 0; i < PeriodicTrig<MOTION>::NA; ++i) {
    r.th[i] = th[i];
    fast_sincos(th[i], &r.s[i], &r.c[i]);
  }
}

template <bool WANT_ACC, int MOTION>
__device__ __forceinline__ void target_state_carried(const qt_env_params& e, const Pattern& pt, double t,
                                                     PeriodicTrig<MOTION>& r, Target& o) {
  constexpr int NA = PeriodicTrig<MOTION>::NA;
  double th[3], d[NA], dm = 0.0;
  periodic_angles(MOTION, pt, t, th);
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    d[i] = th[i] - r.th[i];
    dm = fmax(dm, fabs(d[i]));
    r.th[i] = th[i];
  }
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(dm <= kSmallAngle)) == 0, 1)) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      double sd, cd;
      small_sincos(d[i], &sd, &cd);
      const double s0 = r.s[i], c0 = r.c[i];
      r.s[i] = fma(s0, cd, c0 * sd);
      r.c[i] = fma(c0, cd, -(s0 * sd));
    }
  } else {
#pragma unroll
    for (int i = 0; i < NA; ++i) fast_sincos(th[i], &r.s[i], &r.c[i]);
  }
  periodic_state<WANT_ACC>(e, MOTION, pt, r.s, r.c, o);
  if (WANT_ACC) clamp_acceleration(e, o);
}

// ----------------------------------------------------------------- plant

// Per-lane plant constants: 1/mass and the gravity force (quadcopter_env.py:396).
struct Plant {
  double inv_mass, gz;
};

QT_HD Plant make_plant(const qt_env_params& e, double mass) {
  return Plant{1.0 / mass, -mass * e.gravity};
}

// _compute_derivatives (quadcopter_env.py:329-426).  Only the third column of
// the ZYX rotation matrix multiplies the body thrust [0,0,T] (393).  Divisions
// by mass and by the 0.1 s rate time constant are taken as multiplications by
// reciprocals (<= 1 ulp per term; the closed loop is not chaotic).
// sin / cos of the three attitude angles of a stage state
struct Trig {
  double s[3], c[3];
};

// YAW0: the yaw angle and yaw rate are exactly zero for the whole launch (a
// structured gain never commands yaw, u[3] = 0, so a yaw that starts at zero
// stays zero: quadcopter_env.py:412-421 with u = 0, omega = 0).  Its sin / cos
// are then exactly 0 / 1 and every yaw term drops out of the arithmetic.
// The YAW0 flavour is also tilt-bounded: roll and pitch start every step
// inside the +-pi/3 clamp (quadcopter_env.py:460-463; checked at kernel entry,
// kept by every constrained step), so their sin / cos need no argument
// reduction (sincos_tilt).
template <bool YAW0 = false>
__device__ __forceinline__ void trig_of(const double* ang, Trig& t) {
#pragma unroll
  for (int i = 0; i < (YAW0 ? 2 : 3); ++i) {
    if (YAW0)
      sincos_tilt(ang[i], &t.s[i], &t.c[i]);
    else
      fast_sincos(ang[i], &t.s[i], &t.c[i]);
  }
  if (YAW0) t.s[2] = 0.0, t.c[2] = 1.0;
}

// Trig of the RK4 stage angles  ang_i + delta_i  from the trig of ang_i:
// sin(a + d) = sin a cos d + cos a sin d,  cos(a + d) = cos a cos d - sin a sin d,
// with sin d / cos d from small_sincos.  The stage offsets are h * (body rate)
// <= dt * ~12 rad/s; an offset beyond the polynomial's range takes fast_sincos.
// SMALL: the caller has proven |delta| <= kSmallAngle (small_angle_bound).
// YAW0 (the yaw-at-rest flavour, which is also rate-bounded: rate_bounded_ok)
// has |delta| <= kRateAngle and takes the shorter rate_sincos.
template <bool SMALL = false, bool YAW0 = false>
__device__ __forceinline__ void trig_shift(const double* ang, const Trig& t0, const double* delta, Trig& t,
                                           const RateCoef& rk = RateCoef{}, const SmallCoef& sk = SmallCoef{}) {
  constexpr int NA = YAW0 ? 2 : 3;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    double sd, cd;
    if (YAW0)
      rate_sincos(delta[i], &sd, &cd, rk);
    else
      small_sincos(delta[i], &sd, &cd, sk);
    t.s[i] = fma(t0.s[i], cd, t0.c[i] * sd);
    t.c[i] = fma(t0.c[i], cd, -(t0.s[i] * sd));
  }
  if (!SMALL) {
    // a lane with an offset beyond small_sincos' range evaluates the stage
    // angles directly (a wave-uniform branch; per lane the same choice as
    // `dm <= kSmallAngle ? rotated : direct`)
    const double dm = fmax(fabs(delta[0]), fmax(fabs(delta[1]), fabs(delta[2])));
    const bool big = !(dm <= kSmallAngle);
    if (any_lane(big)) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        double sv, cv;
        fast_sincos(ang[i] + delta[i], &sv, &cv);
        t.s[i] = big ? sv : t.s[i];
        t.c[i] = big ? cv : t.c[i];
      }
    }
  }
  if (YAW0) t.s[2] = 0.0, t.c[2] = 1.0;
}

// _compute_derivatives (quadcopter_env.py:329-426).  Only the third column of
// the ZYX rotation matrix multiplies the body thrust [0,0,T] (393).  Divisions
// by mass and by the 0.1 s rate time constant are taken as multiplications by
// reciprocals (<= 1 ulp per term; the closed loop is not chaotic).
template <bool YAW0 = false>
__device__ __forceinline__ void derivatives(const qt_env_params& e, const Plant& pl, const double* s,
                                            const double* u, const Trig& tr, double* d) {
  const double sphi = tr.s[0], cphi = tr.c[0], sth = tr.s[1], cth = tr.c[1], spsi = tr.s[2], cpsi = tr.c[2];
  const double T = u[0];
  // with psi = 0: cpsi * a + spsi * b = a and spsi * a - cpsi * b = -b, exactly
  // (up to the sign of a zero, which no later operation distinguishes)
  const double tw0 = (YAW0 ? sth * cphi : cpsi * sth * cphi + spsi * sphi) * T;
  const double tw1 = (YAW0 ? -sphi : spsi * sth * cphi - cpsi * sphi) * T;
  const double tw2 = (cth * cphi) * T;
  d[0] = s[3];
  d[1] = s[4];
  d[2] = s[5];
  d[3] = (tw0 + (-e.drag_linear * s[3])) * pl.inv_mass;
  d[4] = (tw1 + (-e.drag_linear * s[4])) * pl.inv_mass;
  d[5] = ((tw2 + pl.gz) + (-e.drag_linear * s[5])) * pl.inv_mass;
  d[6] = s[9];
  d[7] = s[10];
  d[8] = YAW0 ? 0.0 : s[11];
#pragma unroll
  for (int i = 0; i < (YAW0 ? 2 : 3); ++i) d[9 + i] = (u[1 + i] - s[9 + i]) * 10.0 - e.drag_angular * s[9 + i];
  if (YAW0) d[11] = 0.0;
}

// RK4 of the yaw-at-rest fast step in closed form.  With yaw at rest the
// step's only nonlinearity is the thrust direction at the four stage
// attitudes; the rest is linear with constant coefficients:
//   body rates  w' = 10 u - lambda w, lambda = 10 + drag_angular (quadcopter_env.py:417-424)
//   attitudes   a' = w                                          (413)
//   velocities  v' = acc_i - delta v, delta = drag_linear / m   (377-405)
//   positions   p' = v
// with acc_i = T R3(a_i) / m + g the stage's thrust + gravity acceleration.
// The classic RK4 combination (_rk4_step, 295-317) of each linear part is
// therefore a fixed linear map of (w, u) and of (v, acc_1..acc_4), whose
// coefficients are the staged recurrences evaluated on unit inputs
// (rk4_linear): once per launch on the host for the rates / attitudes
// (make_rate_lin, a kernel argument) and once per lane for the velocities /
// positions (make_vel_lin; per-episode mass).  A step then costs about two operations per linear term
// instead of the stage-by-stage updates; the result equals the staged RK4 up
// to the rounding of the reassociation (~1e-16 relative per step).
// Rates / attitudes (uniform: launch constants, computed on the host and
// passed as a kernel argument, so they live in SGPRs):
// w_new = wy w + wu u, a_new = a + ay w + au u, stage attitude offsets
// d2 = h2 w, d3 = d3y w + d3u u, d4 = d4y w + d4u u, and the third stage's
// offset relative to the second, e3 = d3 - d2 = e3y w + d3u u (|e3| is
// O(dt^2): the stage rates differ by h/2 times the rate derivative).
struct RateLin {
  double wy, wu, ay, au, h2, d3y, d3u, d4y, d4u, e3y;
};

// Velocities / positions (per lane: delta depends on the episode's mass):
// v_new = cv v + sum_i wv_i acc_i, p_new = p + pv v + sum_i pa_i acc_i
// (acc_4 does not reach the positions); gravity: gv = g sum wv, gp = g sum pa.
struct VelLin {
  double cv, wv[4], pv, pa[3], gv, gp;
};

// Stage values of y' = f_i - lam y over one RK4 step of length h:
// o = {y2, y3, y4, y_new, h/6 (y1 + 2 y2 + 2 y3 + y4)} (the last is the
// step's integral of y, i.e. the update of a state whose derivative is y).
QT_HD void rk4_linear(double lam, double h, double y, const double* f, double* o) {
  const double k1 = f[0] - lam * y, y2 = y + 0.5 * h * k1;
  const double k2 = f[1] - lam * y2, y3 = y + 0.5 * h * k2;
  const double k3 = f[2] - lam * y3, y4 = y + h * k3;
  const double k4 = f[3] - lam * y4;
  o[0] = y2, o[1] = y3, o[2] = y4;
  o[3] = y + h / 6.0 * (k1 + 2.0 * k2 + 2.0 * k3 + k4);
  o[4] = h / 6.0 * (y + 2.0 * y2 + 2.0 * y3 + y4);
}

// The Euler step (_euler_step, quadcopter_env.py:319-327: x + dt f(x, u)) in
// the same closed form: one stage at the step-start attitude, so
// w_new = (1 - h lam) w + 10 h u, a_new = a + h w, v_new = (1 - h delta) v
// + h acc_1, p_new = p + h v; no stage offsets (d2 = d3 = e3 = 0) and the
// fourth "stage" offset d4 = h w is the whole attitude step, so that
// attitude_trig_resid rotates the carried trig by the step's rounding only.
QT_HD RateLin make_rate_lin(const qt_env_params& e) {
  RateLin L;
  const double h = e.dt, lam = 10.0 + e.drag_angular;
  if (e.integrator == 1) {
    L.wy = 1.0 - h * lam, L.wu = 10.0 * h, L.ay = h, L.au = 0.0;
    L.h2 = 0.0, L.d3y = 0.0, L.d3u = 0.0, L.e3y = 0.0, L.d4y = h, L.d4u = 0.0;
    return L;
  }
  const double zero[4] = {0.0, 0.0, 0.0, 0.0}, ten[4] = {10.0, 10.0, 10.0, 10.0};
  double o[5];
  rk4_linear(lam, h, 1.0, zero, o);
  L.wy = o[3], L.ay = o[4], L.d3y = 0.5 * h * o[0], L.d4y = h * o[1];
  L.e3y = 0.5 * h * (o[0] - 1.0);  // o[0] = 1 - h lam / 2 in [1/2, 1]: the difference is exact
  rk4_linear(lam, h, 0.0, ten, o);
  L.wu = o[3], L.au = o[4], L.d3u = 0.5 * h * o[0], L.d4u = h * o[1];
  L.h2 = 0.5 * h;
  return L;
}

QT_HD VelLin make_vel_lin(const qt_env_params& e, const Plant& pl) {
  VelLin L;
  const double h = e.dt, delta = e.drag_linear * pl.inv_mass;
  if (e.integrator == 1) {  // Euler (make_rate_lin)
    L.cv = 1.0 - h * delta, L.pv = h;
    L.wv[0] = h, L.wv[1] = L.wv[2] = L.wv[3] = 0.0;
    L.pa[0] = L.pa[1] = L.pa[2] = 0.0;
    L.gv = pl.gz * pl.inv_mass * h, L.gp = 0.0;
    return L;
  }
  const double zero[4] = {0.0, 0.0, 0.0, 0.0};
  double o[5];
  rk4_linear(delta, h, 1.0, zero, o);
  L.cv = o[3], L.pv = o[4];
  double sw = 0.0, sp = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double f[4] = {0.0, 0.0, 0.0, 0.0};
    f[i] = 1.0;
    rk4_linear(delta, h, 0.0, f, o);
    L.wv[i] = o[3];
    sw += o[3];
    if (i < 3) L.pa[i] = o[4], sp += o[4];
  }
  const double g = pl.gz * pl.inv_mass;  // gravity force / m (quadcopter_env.py:396, 405)
  L.gv = g * sw;
  L.gp = g * sp;
  return L;
}

// Launch-level constants of the yaw-at-rest fast loop (run_yaw0), computed on
// the host and passed as a kernel argument, so that they live in SGPRs:
// the rate / attitude closed form, the velocity / position closed form and
// plant constants at env.mass (launches whose plant is uniform), and the
// rotors of the periodic target patterns: a carried sin / cos pair of an
// angle theta_i = omega_i t + phase_i advances by the fixed rotation
// (cos, sin)(fl(omega_i dt)) and omega_i times the time step's rounding each
// step (qt_kernels.hpp, Rotor).
// Safe horizon of the yaw-at-rest loop (run_yaw0, yaw0_horizon): uniform
// bounds on how far one step can move the quantities the loop's stop vote
// tests, so that a wave can run the steps no lane can stop at without the
// vote.  Per step, with |T| <= tmax (the controller's thrust clip) and every
// stage thrust direction a unit vector (integrate_yaw0):
//   speed     |v'| <= cv |v| + |T| / m sum_i |wv_i| + |gv|   (0 <= cv <= 1)
//   position  |p'_j - p_j| <= |pv| vmax + |T| / m sum_i |pa_i| + |gp|
//   tilt      |a' - a| <= (|ay| + |au|) max_rate   (rate-bounded: |w|, |u| <= max_rate)
//   time      t' - t <= dt + the rounding of t + dt
// each widened by `slack` (relative) and an absolute term for the rounding of
// the step's few operations.  on == 0 (a non-finite or non-positive limit):
// no horizon, the loop votes every step.
struct Horizon {
  int on;
  double tmax;       // max(|min_thrust|, |max_thrust|) of the controller
  double vmax;       // max_velocity (1 - 1e-12): the speed bound kept below the vote's
  double vmax2;      // vmax^2
  double inv_2vmax;  // 1 / (2 vmax): (vmax^2 - |v|^2) / (2 vmax) <= vmax - |v|
  double vabs;       // absolute slack per step on the speed bound
  double pmax;       // max_position
  double pabs;       // absolute slack per step on a position
  double inv_dang;   // 1 / per-step tilt bound
  double inv_tstep;  // 1 / per-step time bound
  double slack;      // relative widening of the per-lane step bounds
  // The one binade of t in which t + dt rounds to a tie (dt's lowest set bit
  // is half an ulp of t there: round-half-even then alternates the step),
  // as the biased-exponent bits of t; elsewhere fl(t + dt) - t is the same
  // for every t of a binade (t is a multiple of its ulp).
  long long tie_exp_bits;
  // run_yaw0's DUAL: a tilt-bounded horizon shorter than this tries the
  // clamping no-vote body (kDualBelow; 0 never does, for the bitwise test)
  int dual_below;
};

QT_HD Horizon make_horizon(const qt_env_params& e, const qt_ctrl_params& c, const RateLin& rl) {
  Horizon h{};
  const double tm = fmax(fabs(c.min_thrust), fabs(c.max_thrust));
  // (limits bounded away from 0 and infinity, so every per-step bound and its
  // reciprocal in yaw0_horizon is a finite positive number)
  const bool ok = e.max_velocity > 1e-100 && e.max_velocity < 1e150 && e.max_position > 1e-100 &&
                  e.max_position < 1e150 && e.dt > 1e-100 && e.dt < 1e3 && fabs(e.max_episode_time) < 1e150 &&
                  tm < 1e150 && c.max_rate >= 0.0 && c.max_rate < 1e150;
  if (!ok) return h;
  h.on = 1;
  h.tmax = tm;
  h.vmax = e.max_velocity * (1.0 - 1e-12);
  h.vmax2 = h.vmax * h.vmax;
  h.inv_2vmax = 1.0 / (2.0 * h.vmax);
  h.vabs = e.max_velocity * 1e-14;
  h.pmax = e.max_position;
  h.pabs = e.max_position * 1e-15 + 1e-300;
  h.inv_dang = 1.0 / ((fabs(rl.ay) + fabs(rl.au)) * c.max_rate * (1.0 + 1e-9) + 2e-15);
  h.inv_tstep = 1.0 / ((e.dt + (fabs(e.max_episode_time) + e.dt) * 4.5e-16) * (1.0 + 1e-9));
  h.slack = 1.0 + 1e-9;
  {
    // dt = m 2^q with m odd: the lowest set bit 2^q is half an ulp of t
    // for t in [2^(q + 53), 2^(q + 54))
    int q = 0;
    double m = frexp(e.dt, &q) * 9007199254740992.0;  // 53-bit integer mantissa, dt = m 2^(q - 53)
    q -= 53;
    while (fmod(m, 2.0) == 0.0) m *= 0.5, ++q;
    const long long be = (long long)(q + 53) + 1023;
    h.tie_exp_bits = (be > 0 && be < 2047) ? (be << 52) : -1;
  }
  return h;
}

struct LaunchConst {
  RateLin rl;
  VelLin vl;
  Plant pl;
  Horizon hz;
  double rc[5][3], rs[5][3];  // per motion type: cos / sin of fl(omega_i dt)
  double om[5][3];            // per motion type: omega_i
  // deferred-wave flag of this launch set (per stream, qt_rollout.hip): a
  // fast-flavour wave that leaves its episodes to the exact pass writes
  // `epoch` there; the exact pass returns at once unless it reads its epoch
  unsigned long long* defer_flag;
  unsigned long long epoch;
  // qt_rollout_rewards (exact step only): [2][n] reward sum and last
  // post-step tracking error, accumulated across launches; null otherwise
  double* reward;
  // qt_rollout_fresh: the reset offsets[3][n] (the kernel forms the reset
  // state instead of loading one; null: load) and the metrics rows
  // met[QT_MET_ROWS][n] written at the end (null: none)
  const double* fresh_off;
  double* met;
};

// omega of the periodic patterns' angles (make_pattern; target_motion.py:78, 135, 171)
QT_HD int pattern_omegas(const qt_env_params& e, int motion, double* om) {
  if (motion == QT_MOTION_CIRCULAR) {
    om[0] = e.speed / e.radius;
    return 1;
  }
  if (motion == QT_MOTION_SINUSOIDAL) {
    om[0] = 2.0 * kPi * e.frequency;
    om[1] = 2.0 * kPi * (e.frequency * 1.3);
    om[2] = 2.0 * kPi * (e.frequency * 0.7);
    return 3;
  }
  if (motion == QT_MOTION_FIGURE8) {
    om[0] = e.speed / e.amplitude;
    return 1;
  }
  return 0;
}

inline LaunchConst make_launch_const(const qt_env_params& e) {
  LaunchConst k{};
  k.rl = make_rate_lin(e);
  k.pl = make_plant(e, e.mass);
  k.vl = make_vel_lin(e, k.pl);
  for (int m = 0; m < 5; ++m) {
    double om[3] = {0.0, 0.0, 0.0};
    const int na = pattern_omegas(e, m, om);
    for (int i = 0; i < na; ++i) {
      const double a = om[i] * e.dt;
      k.rc[m][i] = cos(a);
      k.rs[m][i] = sin(a);
      k.om[m][i] = om[i];
    }
  }
  return k;
}

// Roll / pitch sin / cos carried across yaw-at-rest fast steps.  The new
// attitude differs from the fourth RK4 stage's by a residual of O(dt^3)
// (attitude_residual_bound), so the carried values are the stage-4 trig
// (integrate_yaw0's t4) rotated by r = (a_new - a0) - d4, the exact
// difference of the rounded angles less the stage-4 offset, with tiny_sincos:
// they follow sin / cos of the angles the reference evaluates with a drift of
// a few ulp per step.  Taken before the tilt clamp (the bound holds for the
// unclamped update), which run_yaw0 then applies to the trig as well.
__device__ __forceinline__ void attitude_trig_resid(const double* a_new, const double* a0, const double* d4,
                                                    const Trig& t4, Trig& ta) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    double sd, cm;
    tiny_sincos((a_new[i] - a0[i]) - d4[i], &sd, &cm);
    rotate_cm(t4.s[i], t4.c[i], sd, cm, &ta.s[i], &ta.c[i]);
  }
}

// One yaw-at-rest RK4 step in closed form (RateLin, VelLin); x[8], x[11] untouched.
// ta: sin / cos of roll and pitch at the step start (carried by the caller).
// Out: the stage-4 attitude offsets d4 and their trig t4 (attitude_trig_resid).
__device__ __forceinline__ void integrate_yaw0(const RateLin& R, const VelLin& L, const Plant& pl, const Trig& ta,
                                               double* x, const double* u, const RateCoef& rk, double* d4,
                                               Trig& t4) {
  const double w0 = x[9], w1 = x[10];
  Trig t[4];
  t[0] = ta;
  const double d2[3] = {R.h2 * w0, R.h2 * w1, 0.0};
  d4[0] = fma(R.d4y, w0, R.d4u * u[1]);
  d4[1] = fma(R.d4y, w1, R.d4u * u[2]);
  const double d4v[3] = {d4[0], d4[1], 0.0};
  trig_shift<true, true>(x + 6, t[0], d2, t[1], rk);
  // stage 3 from stage 2 by e3 = d3 - d2, |e3| <= kStage3Angle (rate_bounded_ok)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double e3 = fma(R.e3y, x[9 + i], R.d3u * u[1 + i]);
    double sd, cm;
    resid_sincos(e3, &sd, &cm, rk);
    rotate_cm(t[1].s[i], t[1].c[i], sd, cm, &t[2].s[i], &t[2].c[i]);
  }
  trig_shift<true, true>(x + 6, t[0], d4v, t[3], rk);
  t4 = t[3];
  // thrust direction R3 at each stage (derivatives<true>): (sin th cos phi, -sin phi, cos th cos phi)
  double sv[3] = {0.0, 0.0, 0.0}, sp[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double r0 = t[i].s[1] * t[i].c[0], r1 = -t[i].s[0], r2 = t[i].c[1] * t[i].c[0];
    sv[0] = fma(L.wv[i], r0, sv[0]);
    sv[1] = fma(L.wv[i], r1, sv[1]);
    sv[2] = fma(L.wv[i], r2, sv[2]);
    sp[0] = fma(L.pa[i], r0, sp[0]);
    sp[1] = fma(L.pa[i], r1, sp[1]);
    sp[2] = fma(L.pa[i], r2, sp[2]);
  }
  {  // stage 4 reaches the velocities only: its weight folded into cos phi
    const double wc = L.wv[3] * t[3].c[0];
    sv[0] = fma(wc, t[3].s[1], sv[0]);
    sv[1] = fma(L.wv[3], -t[3].s[0], sv[1]);
    sv[2] = fma(wc, t[3].c[1], sv[2]);
  }
  const double tm = u[0] * pl.inv_mass;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double v = x[3 + j];
    x[j] = fma(tm, sp[j], fma(L.pv, v, j == 2 ? x[j] + L.gp : x[j]));
    x[3 + j] = fma(tm, sv[j], j == 2 ? fma(L.cv, v, L.gv) : L.cv * v);
  }
  x[6] = fma(R.ay, w0, fma(R.au, u[1], x[6]));
  x[7] = fma(R.ay, w1, fma(R.au, u[2], x[7]));
  x[9] = fma(R.wy, w0, R.wu * u[1]);
  x[10] = fma(R.wy, w1, R.wu * u[2]);
}

// One RK4 / Euler step of the exact flavour in closed form, for any attitude
// and body rates (yaw included): integrate_yaw0's linear maps (RateLin:
// rates / attitudes, VelLin: velocities / positions; they hold for any w and
// u, the rate dynamics being linear) with the thrust direction R3 at the
// four stage attitudes (derivatives: cpsi sth cphi + spsi sphi,
// spsi sth cphi - cpsi sphi, cth cphi).  The stage trig is the step-start
// trig `ta` shifted by each stage's offset (trig_shift: small_sincos, or the
// direct evaluation for an offset beyond its range).  Equal to the staged
// RK4 up to the rounding of the reassociation (~1e-16 relative per step), as
// the yaw-at-rest step.  Out: the fourth stage's offsets d4 and trig t4
// (carry_attitude_trig).  Euler (make_rate_lin / make_vel_lin's one-stage
// coefficients): stages 2 and 3 carry zero weight and are skipped.  INTEG:
// the integrator when the caller knows it at compile time (0 "rk4", 1
// "euler": no uniform branch on it per step), -1 read from e.
template <int INTEG = -1>
__device__ __forceinline__ void integrate_closed(const qt_env_params& e, const RateLin& R, const VelLin& L,
                                                 const Plant& pl, const Trig& ta, double* x, const double* u,
                                                 double* d4, Trig& t4, const SmallCoef& sk = SmallCoef{}) {
  const double w[3] = {x[9], x[10], x[11]};
  double d2[3], d3[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    d2[i] = R.h2 * w[i];
    d3[i] = fma(R.d3y, w[i], R.d3u * u[1 + i]);
    d4[i] = fma(R.d4y, w[i], R.d4u * u[1 + i]);
  }
  Trig t[4];
  t[0] = ta;
  trig_shift<true>(x + 6, ta, d4, t[3], RateCoef{}, sk);
  double em = 0.0;
  if (INTEG == 0 || (INTEG < 0 && e.integrator != 1)) {
    trig_shift<true>(x + 6, ta, d2, t[1], RateCoef{}, sk);
    // the third stage from the second by e3 = d3 - d2 = O(dt^2) (resid_sincos)
    RateCoef rk;
    rk.s5 = sk.s5;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double e3 = fma(R.e3y, w[i], R.d3u * u[1 + i]);
      em = fmax(em, fabs(e3));
      double sd, cm;
      resid_sincos(e3, &sd, &cm, rk);
      rotate_cm(t[1].s[i], t[1].c[i], sd, cm, &t[2].s[i], &t[2].c[i]);
    }
  }
  // an offset beyond small_sincos' range, or a third-stage residual beyond
  // resid_sincos': that lane's stage angles are evaluated directly (one
  // wave-uniform branch for the three stages)
  double dm = 0.0;
#pragma unroll
  for (int i = 0; i < 3; ++i) dm = fmax(dm, fmax(fabs(d2[i]), fmax(fabs(d3[i]), fabs(d4[i]))));
  const bool big = !(dm <= kSmallAngle) || !(em <= kStage3Angle);
  if (any_lane(big)) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double sv, cv;
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const double* d = k == 1 ? d2 : (k == 2 ? d3 : d4);
        fast_sincos(x[6 + i] + d[i], &sv, &cv);
        t[k].s[i] = big ? sv : t[k].s[i];
        t[k].c[i] = big ? cv : t[k].c[i];
      }
    }
  }
  t4 = t[3];
  double sv[3] = {0.0, 0.0, 0.0}, sp[3] = {0.0, 0.0, 0.0};
  auto add_stage = [&](const Trig& q, double wv, double pa, bool pos) {
    const double sphi = q.s[0], cphi = q.c[0], sth = q.s[1], cth = q.c[1], spsi = q.s[2], cpsi = q.c[2];
    const double sc = sth * cphi;
    const double r0 = fma(cpsi, sc, spsi * sphi), r1 = fma(spsi, sc, -(cpsi * sphi)), r2 = cth * cphi;
    sv[0] = fma(wv, r0, sv[0]);
    sv[1] = fma(wv, r1, sv[1]);
    sv[2] = fma(wv, r2, sv[2]);
    if (pos) {
      sp[0] = fma(pa, r0, sp[0]);
      sp[1] = fma(pa, r1, sp[1]);
      sp[2] = fma(pa, r2, sp[2]);
    }
  };
  add_stage(t[0], L.wv[0], L.pa[0], true);
  if (INTEG == 0 || (INTEG < 0 && e.integrator != 1)) {  // RK4: stages 2 and 3 (uniform)
    add_stage(t[1], L.wv[1], L.pa[1], true);
    add_stage(t[2], L.wv[2], L.pa[2], true);
  }
  add_stage(t[3], L.wv[3], 0.0, false);  // the fourth stage reaches the velocities only (0 for Euler)
  const double tm = u[0] * pl.inv_mass;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double v = x[3 + j];
    x[j] = fma(tm, sp[j], fma(L.pv, v, j == 2 ? x[j] + L.gp : x[j]));
    x[3 + j] = fma(tm, sv[j], j == 2 ? fma(L.cv, v, L.gv) : L.cv * v);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    x[6 + i] = fma(R.ay, w[i], fma(R.au, u[1 + i], x[6 + i]));
    x[9 + i] = fma(R.wy, w[i], R.wu * u[1 + i]);
  }
}

// _integrate / _rk4_step / _euler_step (quadcopter_env.py:295-327), stage by
// stage as the reference evaluates it; u is held constant across the four
// stages.  The per-step API's env.step (any caller-supplied state, overflow
// and NaN propagation as numpy's); the rollout's steps use integrate_closed.
__device__ __forceinline__ void integrate(const qt_env_params& e, const Plant& pl, double* x, const double* u) {
  const double dt = e.dt;
  double k[12];
  Trig t0, ts;
  trig_of(x + 6, t0);
  derivatives(e, pl, x, u, t0, k);
  if (e.integrator == 1) {
#pragma unroll
    for (int i = 0; i < 12; ++i) x[i] = x[i] + k[i] * dt;
    return;
  }
  // Stage states.  Their angles only enter through sin/cos (derivatives of
  // the angles are the body rates), so stage trig is the step-start trig
  // shifted by the stage offset h * k[6..8].
  double acc[12], tmp[12], del[3];
  const double h2 = 0.5 * dt;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    acc[i] = k[i];
    tmp[i] = x[i] + h2 * k[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) del[i] = h2 * k[6 + i];
  trig_shift(x + 6, t0, del, ts);
  derivatives(e, pl, tmp, u, ts, k);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    acc[i] = acc[i] + 2.0 * k[i];
    tmp[i] = x[i] + h2 * k[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) del[i] = h2 * k[6 + i];
  trig_shift(x + 6, t0, del, ts);
  derivatives(e, pl, tmp, u, ts, k);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    acc[i] = acc[i] + 2.0 * k[i];
    tmp[i] = x[i] + dt * k[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) del[i] = dt * k[6 + i];
  trig_shift(x + 6, t0, del, ts);
  derivatives(e, pl, tmp, u, ts, k);
  const double h6 = dt / 6.0;
#pragma unroll
  for (int i = 0; i < 12; ++i) x[i] = x[i] + h6 * (acc[i] + k[i]);
}

// The exact step's carried attitude trig: sin / cos of the constrained new
// attitude a1 from those of the last RK4 stage's (t4, offset d4 from the
// step-start a0), rotated by the exact difference of the rounded angles,
// r = (a1 - a0) - d4 (O(dt^3) for an RK4 step, the rounding alone for
// Euler), with tiny_sincos.  An angle that the wrap or the tilt clamp moved,
// or whose r exceeds kAdvanceAngle, is evaluated directly (a wave-uniform
// branch).  The carried values follow sin / cos of the angles the reference
// evaluates with a drift of a few ulp per step (as the fast step's,
// attitude_trig_resid); a launch starts from the direct evaluation.
__device__ __forceinline__ void carry_attitude_trig(const double* a0, const double* a1, const double* d4,
                                                    const Trig& t4, Trig& ta, const SmallCoef& sk = SmallCoef{}) {
  bool far[3], any = false;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double r = (a1[i] - a0[i]) - d4[i];
    far[i] = !(fabs(r) <= kAdvanceAngle);
    any = any | far[i];
    double sd, cm;
    tiny_sincos(r, &sd, &cm, sk);
    rotate_cm(t4.s[i], t4.c[i], sd, cm, &ta.s[i], &ta.c[i]);
  }
  if (any_lane(any)) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double sv, cv;
      fast_sincos(a1[i], &sv, &cv);
      ta.s[i] = far[i] ? sv : ta.s[i];
      ta.c[i] = far[i] ? cv : ta.c[i];
    }
  }
}

// Clip of a value known to be a number: one v_max + one v_min.  (IEEE maxNum
// would turn a NaN into a bound, which np.clip does not; callers use it only
// where NaN cannot reach or check for it separately.)
__device__ __forceinline__ double clip_num(double v, double lo, double hi) { return fmin(fmax(v, lo), hi); }

// `sqrt(s) > r` for s = a sum of squares and r >= 0, without the square root
// unless s lies within 1e-14 of r^2 (sqrt is correctly rounded and monotone,
// so outside that band the squared comparison decides it identically).
__device__ __forceinline__ bool norm_gt(double s, double r) {
  const double r2 = r * r;
  if (s > r2 * (1.0 + 1e-14)) return true;
  if (!(s >= r2 * (1.0 - 1e-14))) return false;  // also NaN -> false, like NaN > r
  return sqrt(s) > r;
}

// `sqrt(s) <= r` likewise (NaN -> false), branch-free outside the band.
__device__ __forceinline__ bool norm_le(double s, double r) {
  const double r2 = r * r;
  bool le = s < r2 * (1.0 - 1e-14);
  const bool band = !le && !(s > r2 * (1.0 + 1e-14));  // in the band, or NaN
  if (any_lane(band)) le = band ? sqrt(s) <= r : le;
  return le;
}

// numpy's (a + pi) % (2 pi) - pi of the three attitude angles
// (quadcopter_env.py:457, _normalize_angle 468-470): for |a + pi| < 4 pi
// (every angle a constrained step produces) the remainder takes at most one
// exact correction (Sterbenz), computed by selects as py_mod_2pi does; larger
// magnitudes and infinities take py_mod_2pi's fmod in a wave-uniform branch.
__device__ __forceinline__ void wrap_angles(double* ang) {
  double b[3], m[3];
  bool big[3], any = false;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    b[i] = ang[i] + kPi;
    big[i] = !(fabs(b[i]) < 2.0 * kTwoPi) && b[i] == b[i];
    any = any | big[i];
    double m1 = b[i] >= kTwoPi ? b[i] - kTwoPi : b[i];
    m1 = b[i] <= -kTwoPi ? b[i] + kTwoPi : m1;
    const double m2 = m1 < 0.0 ? m1 + kTwoPi : m1;
    m[i] = m1 == 0.0 ? 0.0 : m2;  // numpy returns +0.0 for a zero remainder
  }
  if (any_lane(any)) {
#pragma unroll
    for (int i = 0; i < 3; ++i) m[i] = big[i] ? py_mod_2pi(b[i], kTwoPi) : m[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) ang[i] = m[i] - kPi;
}

// _apply_state_constraints (quadcopter_env.py:428-465).  EXACT_NAN keeps
// np.clip's NaN propagation for the rate / tilt clips (open-loop step on
// caller-supplied states); inside the fused rollout the state is finite by
// construction (finite reset, finite clipped actions, bounded updates).
// The speed clamp acts on a lane whose squared speed reaches within 1e-14 of
// the limit (norm_gt decides it exactly): a wave-uniform branch.
template <bool EXACT_NAN = true>
__device__ __forceinline__ void constrain(const qt_env_params& e, double* x) {
  const double s = dot3_blas(x[3], x[4], x[5]);
  const bool near = !(s < e.max_velocity * e.max_velocity * (1.0 - 1e-14));  // or NaN
  if (any_lane(near)) {
    const bool clamp = near && norm_gt(s, e.max_velocity);
    const double vm = sqrt(s);
#pragma unroll
    for (int i = 3; i < 6; ++i) x[i] = clamp ? x[i] / vm * e.max_velocity : x[i];
  }
#pragma unroll
  for (int i = 9; i < 12; ++i)
    x[i] = EXACT_NAN ? clipd(x[i], -e.max_angular_velocity, e.max_angular_velocity)
                     : clip_num(x[i], -e.max_angular_velocity, e.max_angular_velocity);
  wrap_angles(x + 6);
  x[6] = EXACT_NAN ? clipd(x[6], -kMaxTilt, kMaxTilt) : clip_num(x[6], -kMaxTilt, kMaxTilt);
  x[7] = EXACT_NAN ? clipd(x[7], -kMaxTilt, kMaxTilt) : clip_num(x[7], -kMaxTilt, kMaxTilt);
}

// _apply_state_constraints (quadcopter_env.py:428-465) followed by
// _check_termination (513-535) at the new time t, with ONE wave-uniform
// branch for every rare case, its predicates taken on the unconstrained
// state: the speed clamp (squared speed within 1e-14 of the limit or above;
// norm_gt decides it), an angle with (a + pi) outside (-2 pi, 4 pi) (numpy's
// floor-mod by fmod, py_mod_2pi; also NaN), and a non-finite component (the
// element test, on the constrained state: a clipped infinite rate is finite
// again).  Otherwise: the rate clip, one exact wrap correction and the tilt
// clip as selects.  EXACT_NAN: np.clip's NaN propagation in the clips (the
// per-step API's caller-supplied states); the fused rollout's state is finite.
template <bool EXACT_NAN = true>
__device__ __forceinline__ int constrain_terminate(const qt_env_params& e, double* x, double t) {
  const double s = dot3_blas(x[3], x[4], x[5]);
  const bool near = !(s < e.max_velocity * e.max_velocity * (1.0 - 1e-14));  // or NaN
  double sum = 0.0;
#pragma unroll
  for (int i = 0; i < 12; ++i) sum += x[i];
  const bool nf = !isfinite(sum);
  double b[3];
  bool big[3], rare = near | nf;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    b[i] = x[6 + i] + kPi;
    big[i] = !(b[i] > -kTwoPi && b[i] < 2.0 * kTwoPi);  // or NaN
    rare = rare | big[i];
    // (b % 2 pi) for b in (-2 pi, 4 pi): one exact correction, numpy's rounding
    const double adj = b[i] < 0.0 ? kTwoPi : (b[i] >= kTwoPi ? -kTwoPi : 0.0);
    x[6 + i] = (b[i] + adj) - kPi;
  }
#pragma unroll
  for (int i = 9; i < 12; ++i)
    x[i] = EXACT_NAN ? clipd(x[i], -e.max_angular_velocity, e.max_angular_velocity)
                     : clip_num(x[i], -e.max_angular_velocity, e.max_angular_velocity);
  auto tilt_clip = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const double a = x[6 + i];
      x[6 + i] = EXACT_NAN ? clipd(a, -kMaxTilt, kMaxTilt) : clip_num(a, -kMaxTilt, kMaxTilt);
    }
  };
  tilt_clip();
  bool fin = true;
  if (any_lane(rare)) {
    const bool clamp = near && norm_gt(s, e.max_velocity);
    const double vm = sqrt(s);
#pragma unroll
    for (int i = 3; i < 6; ++i) x[i] = clamp ? x[i] / vm * e.max_velocity : x[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) x[6 + i] = big[i] ? py_mod_2pi(b[i], kTwoPi) - kPi : x[6 + i];
    tilt_clip();  // again for the angles the fmod wrap set (a no-op for the others)
    bool f = true;
#pragma unroll
    for (int i = 0; i < 12; ++i) f = f & isfinite(x[i]);
    fin = !nf || f;
  }
  const bool tl = t >= e.max_episode_time;
  const bool pb = fmax(fabs(x[0]), fmax(fabs(x[1]), fabs(x[2]))) > e.max_position;
  return tl ? QT_TERM_TIME_LIMIT : (pb ? QT_TERM_POSITION_BOUNDS : (fin ? QT_TERM_RUNNING : QT_TERM_NUMERICAL_INSTABILITY));
}

// _parse_and_validate_action (quadcopter_env.py:234-293) on an array action;
// returns true when any violation was recorded.  A finite 4-sum proves every
// component finite; otherwise (a wave-uniform branch) the per-component
// NaN/Inf zeroing runs.
__device__ __forceinline__ bool parse_action(const qt_env_params& e, const double* in, double* a) {
  bool viol = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = in[i];
  const bool nf = !isfinite((in[0] + in[1]) + (in[2] + in[3]));
  if (any_lane(nf)) {  // for a lane with finite components these are no-ops
    const bool finite = isfinite(in[0]) && isfinite(in[1]) && isfinite(in[2]) && isfinite(in[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = isfinite(in[i]) ? in[i] : 0.0;
    viol = !finite;
  }
  // thrust: min if below, else max if above; rates: clip when |r| > max
  const double t = a[0] < e.min_thrust ? e.min_thrust : fmin(a[0], e.max_thrust);
  viol = viol || (t != a[0]);
  a[0] = t;
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    const double r = clip_num(a[i], -e.max_angular_rate, e.max_angular_rate);
    viol = viol || (r != a[i]);
    a[i] = r;
  }
  return viol;
}

// ------------------------------------------------- fast-path preconditions
//
// The fused rollout has a branch-light variant of the step (the "fast path")
// that takes the same decisions as the exact one and computes the same
// expressions (up to the compiler's FMA contraction) whenever these hold:
//  * RK4 integration;
//  * the controller's clamps lie inside the env's action clamps, so
//    _parse_and_validate_action never clips or flags a finite command;
//  * every RK4 stage attitude offset is within small_sincos' range: the body
//    rates start a step within +-max_angular_velocity (constrained every step)
//    and the commanded rates within +-max_angular_rate, which bounds the stage
//    rates through the first-order rate dynamics (quadcopter_env.py:412-421);
//  * per lane: finite gains, hover thrust and state (checked at kernel entry).
__host__ __device__ inline double small_angle_bound(const qt_env_params& e) {
  const double h2 = 0.5 * e.dt, w = e.max_angular_velocity, r = e.max_angular_rate, cd = fabs(e.drag_angular);
  const double k1 = (r + w) * 10.0 + cd * w;     // |d omega / dt| at stage 1
  const double w2 = w + h2 * k1;                  // |omega| at stages 2, 3
  const double k2 = (r + w2) * 10.0 + cd * w2;
  const double w3 = w + h2 * k2;                  // |omega| at stage 3 (offset of stage 4)
  return fmax(h2 * w2, e.dt * w3) * (1.0 + 1e-12);
}

__host__ __device__ inline bool fast_path_ok(const qt_env_params& e, const qt_ctrl_params& c) {
  return e.integrator == 0 && c.min_thrust >= e.min_thrust && c.max_thrust <= e.max_thrust &&
         c.min_thrust <= c.max_thrust && c.max_rate <= e.max_angular_rate && c.max_rate >= 0.0 &&
         e.max_angular_velocity >= 0.0 && small_angle_bound(e) <= kSmallAngle;
}

// Rate-bounded steps (the yaw-at-rest flavour's third precondition).  The
// body-rate dynamics are linear, w' = 10 (u - w) - c w with the command u
// constant over the step and |u| <= max_rate (the controller's clip).  With
// c >= 0 and dt (10 + c) <= 1 every RK4 stage rate is a combination of w and u
// with non-negative weights summing to at most 1 (stage 2: (1 - a) w + b u,
// a = dt / 2 (10 + c), b = 5 dt; stages 3, 4 and the update likewise), so a
// lane whose |w| starts within max_rate keeps every stage rate, and the next
// step's rate, within max_rate (the rate clamp only shrinks it).  A stage
// attitude offset h * w (h <= dt) is then at most dt * max_rate <= kRateAngle,
// and with max_rate below max_angular_velocity the env's angular-velocity
// clamp (quadcopter_env.py:446-450) never acts (constrain_fast_apply<true>).
// The residuals of the yaw-at-rest step's trig (integrate_yaw0,
// attitude_trig_resid) follow from the same linear rate dynamics: with
// k1 = 10 u - lam w (lam = 10 + c, |k1| <= (10 + lam) max_rate) the third
// stage's offset exceeds the second's by e3 = (h/2)(h/2) k1, and the step's
// attitude update h/6 (y1 + 2 y2 + 2 y3 + y4) exceeds the fourth stage's
// offset h y3 by h/6 (y1 + 2 y2 - 4 y3 + y4) = h^3 lam (1 + lam h / 2) k1 / 12.
// At the defaults (dt 0.01, max_rate 3): 1.5e-3 and 5.3e-5.
__host__ __device__ inline double stage3_residual_bound(const qt_env_params& e, const qt_ctrl_params& c) {
  const double lam = 10.0 + e.drag_angular, k1 = (10.0 + lam) * c.max_rate;
  return 0.25 * e.dt * e.dt * k1 * (1.0 + 1e-6);
}
__host__ __device__ inline double attitude_residual_bound(const qt_env_params& e, const qt_ctrl_params& c) {
  const double lam = 10.0 + e.drag_angular, h = e.dt, k1 = (10.0 + lam) * c.max_rate;
  return h * h * h * lam * (1.0 + 0.5 * lam * h) / 12.0 * k1 * (1.0 + 1e-6) + 1e-15;  // + the wrap's rounding
}

// The yaw-at-rest flavour for the Euler integrator (make_rate_lin): the
// controller clamps inside the env's (parsing is the identity) and the rate
// bound below; the RK4 stage-offset bound does not apply (no stages).
__host__ __device__ inline bool rate_bounded_ok(const qt_env_params& e, const qt_ctrl_params& c);
__host__ __device__ inline bool euler_yaw0_ok(const qt_env_params& e, const qt_ctrl_params& c) {
  return e.integrator == 1 && c.min_thrust >= e.min_thrust && c.max_thrust <= e.max_thrust &&
         c.min_thrust <= c.max_thrust && c.max_rate <= e.max_angular_rate && c.max_rate >= 0.0 &&
         e.max_angular_velocity >= 0.0 && rate_bounded_ok(e, c);
}

__host__ __device__ inline bool rate_bounded_ok(const qt_env_params& e, const qt_ctrl_params& c) {
  return c.max_rate >= 0.0 && e.drag_angular >= 0.0 && e.dt > 0.0 && e.dt * (10.0 + e.drag_angular) <= 1.0 &&
         e.dt * c.max_rate * (1.0 + 1e-9) <= kRateAngle && c.max_rate * (1.0 + 1e-9) <= e.max_angular_velocity &&
         stage3_residual_bound(e, c) <= kStage3Angle && attitude_residual_bound(e, c) <= kAdvanceAngle;
}

// Fast-path state constraints: the common case of _apply_state_constraints
// without branches.  constrain_fast_ok is false when the exact path is
// needed: speed within 1e-14 of the clamp or above it, or an attitude angle
// with (a + pi) outside (-2 pi, 4 pi), where numpy's floor-mod takes more
// than one correction (or the state is not finite).
// YAW0 (tilt-bounded, see trig_of): after an RK4 step from inside the tilt
// clamp, |roll|, |pitch| <= pi/3 + small_angle_bound < pi, so a + pi lies in
// (0, 2 pi) and numpy's floor-mod makes no correction: only the speed test
// remains.
template <bool YAW0 = false>
__device__ __forceinline__ bool constrain_fast_ok(const qt_env_params& e, const double* x) {
  const double sv = x[3] * x[3] + x[4] * x[4] + x[5] * x[5];
  const double vm2 = e.max_velocity * e.max_velocity * (1.0 - 1e-14);
  bool ok = sv < vm2;
  if (YAW0) return ok;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double b = x[6 + i] + kPi;
    ok = ok & (b > -kTwoPi) & (b < 2.0 * kTwoPi);
  }
  return ok;
}

template <bool YAW0 = false>
__device__ __forceinline__ void constrain_fast_apply(const qt_env_params& e, double* x) {
  // YAW0 (rate-bounded, rate_bounded_ok): |w| <= max_rate < max_angular_velocity, the clip is inactive
  if (!YAW0)
#pragma unroll
    for (int i = 9; i < 12; ++i) x[i] = clip_num(x[i], -e.max_angular_velocity, e.max_angular_velocity);
#pragma unroll
  for (int i = 0; i < (YAW0 ? 2 : 3); ++i) {
    // (b % 2 pi) for b in (-2 pi, 4 pi): one correction, the same rounding as
    // numpy's (b < 0: b + 2 pi; b >= 2 pi: b - 2 pi, exact by Sterbenz);
    // YAW0: b in (0, 2 pi), none (constrain_fast_ok)
    const double b = x[6 + i] + kPi;
    const double adj = YAW0 ? 0.0 : (b < 0.0 ? kTwoPi : (b >= kTwoPi ? -kTwoPi : 0.0));
    x[6 + i] = YAW0 ? b - kPi : (b + adj) - kPi;
  }
  // YAW0: the tilt clamp is the caller's (run_yaw0's tilt_clamp, after the carried trig)
  if (!YAW0) {
    x[6] = clip_num(x[6], -kMaxTilt, kMaxTilt);
    x[7] = clip_num(x[7], -kMaxTilt, kMaxTilt);
  }
}

// _check_termination without branches, for the fast step.  Its state stays
// finite by construction: the lanes start finite (state, gains, hover thrust,
// target, |t| < 1e300: checked at kernel entry), the commands are clipped to
// finite bounds, velocities and rates are clamped, angles wrapped, and a step
// moves a position by a bounded amount; so the non-finite test (531-533)
// cannot fire and is not evaluated.
__device__ __forceinline__ int termination_fast(const qt_env_params& e, double t, const double* x) {
  const bool tl = t >= e.max_episode_time;
  const bool pb = fmax(fabs(x[0]), fmax(fabs(x[1]), fabs(x[2]))) > e.max_position;
  return tl ? QT_TERM_TIME_LIMIT : (pb ? QT_TERM_POSITION_BOUNDS : QT_TERM_RUNNING);
}

// ------------------------------------------------------------ controller

// Gains as seen by one lane, loaded once per launch.  Dense: the full 4 x KC
// matrix.  Structured (KS): only the per-axis entries — K[0][2], K[0][5],
// K[1][1], K[1][4], K[2][0], K[2][3] (+ K[0][8], K[1][7], K[2][6] for LQI) —
// for gains whose every other entry is exactly zero (the per-axis DARE with
// diagonal Q/R, riccati_lqr.py:602-700).  With finite errors (a running
// episode) adding those exact zeros changes nothing, so both forms agree bit
// for bit.
//
// KC == 3 is the PID controller: k = kp[3], ki[3], kd[3] (PIDController,
// controllers/__init__.py:196-203); KS only marks that it never commands yaw.
template <int KC, bool KS>
struct Gains {
  static constexpr int kCount = KC == 3 ? 9 : (KS ? (KC == 9 ? 9 : 6) : 4 * KC);
  double k[kCount];
};

// element index (row-major r*KC + c) of structured slot j
template <int KC>
__host__ __device__ constexpr int structured_index(int j) {
  // (row, col): (0,2) (0,5) (1,1) (1,4) (2,0) (2,3) [(0,8) (1,7) (2,6)]
  constexpr int rows[9] = {0, 0, 1, 1, 2, 2, 0, 1, 2};
  constexpr int cols[9] = {2, 5, 1, 4, 0, 3, 8, 7, 6};
  return rows[j] * KC + cols[j];
}

// Feed-forward parameters of one episode (riccati_lqr.py:836-861,
// controllers/__init__.py:286-330): velocity / acceleration gains and the
// velocity clamp.  Feed-forward off is the identity with these parameters:
// zero gains and no clamp give the reference's plain v_T - v and zero
// acceleration terms (up to the sign of a zero, which no later operation
// distinguishes), so one code path serves lanes with and without it — the
// per-episode form of qt_batch.ff (the tuner's feed-forward gain ranges; the
// heuristic fallback of a failed DARE, which runs without feed-forward,
// riccati_lqr.py:764-776).
struct FFLane {
  double vg[3], ag[3], vmax;
};

__host__ __device__ inline FFLane ff_uniform(const qt_ctrl_params& c) {
  if (!c.feedforward_enabled) return FFLane{{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, INFINITY};
  return FFLane{{c.ff_velocity_gain[0], c.ff_velocity_gain[1], c.ff_velocity_gain[2]},
                {c.ff_acceleration_gain[0], c.ff_acceleration_gain[1], c.ff_acceleration_gain[2]},
                c.ff_max_velocity};
}

// a + b * c rounded twice, as numpy evaluates it (no FMA contraction)
__device__ __forceinline__ double add_product_rn(double a, double b, double c) {
#pragma clang fp contract(off)
  return a + b * c;
}

// RiccatiLQRController.compute_action (riccati_lqr.py:779-967) given the
// observation the env returned (quad p, v; target p, v, a).  LQI integral
// update 869-900, output clamps 907-921.  Returns true when saturated.
// FAST: gains, hover thrust and observation are known finite, so the raw
// command is finite and np.clip's NaN pass-through cannot arise.
// FF: the feed-forward arithmetic is compiled in (some lane may have it on);
// its parameters are the lane's, `f` (ff_uniform / qt_batch.ff).
template <int KC, bool FF, bool KS, bool FAST = false>
__device__ __forceinline__ bool compute_action(const qt_ctrl_params& c, const Gains<KC, KS>& G, double hover,
                                               const double* qp, const double* qv, const Target& tg,
                                               const FFLane& f, double* integ, double* u, double* diag = nullptr,
                                               double em_fast = 0.0) {
  double ep[3], ev[3], tv[3] = {tg.v[0], tg.v[1], tg.v[2]}, ffa[3] = {0, 0, 0}, ffv[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 3; ++i) ep[i] = tg.p[i] - qp[i];
  if (FF) {
    double vm = norm3(tv[0], tv[1], tv[2]);
    if (vm > f.vmax) {
      double scl = f.vmax / vm;
#pragma unroll
      for (int i = 0; i < 3; ++i) tv[i] = tv[i] * scl;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ffv[i] = f.vg[i] * tv[i];  // diagnostics term (riccati_lqr.py:851)
      tv[i] = (1.0 + f.vg[i]) * tv[i];
    }
    double ac[3] = {tg.a[0], tg.a[1], tg.a[2]};
    double am = norm3(ac[0], ac[1], ac[2]);
    if (am > c.ff_max_acceleration && am > 0) {
#pragma unroll
      for (int i = 0; i < 3; ++i) ac[i] = ac[i] / am * c.ff_max_acceleration;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) ffa[i] = f.ag[i] * ac[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) ev[i] = tv[i] - qv[i];
  const double s[6] = {ep[0], ep[1], ep[2], ev[0], ev[1], ev[2]};
  double uf[4];
  if (KC == 9) {
    // FAST: the caller passes ||e_p|| (the metric's pre-step error, the same
    // correctly rounded square root of the same sum of squares), and the
    // integral and errors are finite.  The anti-windup block then needs no
    // test: it holds only when lim > 0, |I| >= lim and e has I's sign, and
    // then |I + dt e| >= |I| >= lim (rounding is monotone), so the clip below
    // returns sign(I) lim — which is I when |I| == lim, and what the
    // reference's clip makes of a blocked |I| > lim.  np.clip is fmin / fmax.
    const double em = FAST ? em_fast : norm3(ep[0], ep[1], ep[2]);
    const double lim = c.integral_limit;
    if (FAST) {
      // the threshold gate as a step size: I + 0 e == I (up to the sign of a
      // zero integral, which no later operation distinguishes); I + dt * e
      // rounded as the reference rounds it (no contraction)
      const double g = em > c.integral_zero_threshold ? c.dt : 0.0;
#pragma unroll
      for (int i = 0; i < 3; ++i) integ[i] = add_product_rn(integ[i], g, ep[i]);
    } else {
      // the threshold gate and the anti-windup block (riccati_lqr.py:873-895)
      // as selects; I += dt * e rounded as numpy rounds it
      const bool gate = em > c.integral_zero_threshold;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const bool block = fabs(integ[i]) >= lim && lim > 0 && same_sign(integ[i], ep[i]);
        integ[i] = (gate && !block) ? add_product_rn(integ[i], c.dt, ep[i]) : integ[i];
      }
    }
    if (FAST) {
      // the clip to +-lim when lim > 0, else none: a clip to +-inf (the
      // integral is finite), so no branch in the step loop
      const double lc = lim > 0 ? lim : INFINITY;
#pragma unroll
      for (int i = 0; i < 3; ++i) integ[i] = clip_num(integ[i], -lc, lc);
    } else if (lim > 0) {
#pragma unroll
      for (int i = 0; i < 3; ++i) integ[i] = clipd(integ[i], -lim, lim);
    }
    if (KS) {
      uf[0] = (G.k[0] * s[2] + G.k[1] * s[5]) + G.k[6] * integ[2];
      uf[1] = (G.k[2] * s[1] + G.k[3] * s[4]) + G.k[7] * integ[1];
      uf[2] = (G.k[4] * s[0] + G.k[5] * s[3]) + G.k[8] * integ[0];
      uf[3] = 0.0;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) a += G.k[r * KC + j] * s[j];
#pragma unroll
        for (int j = 0; j < 3; ++j) b += G.k[r * KC + 6 + j] * integ[j];
        uf[r] = a + b;
      }
    }
  } else if (KS) {
    uf[0] = G.k[0] * s[2] + G.k[1] * s[5];
    uf[1] = G.k[2] * s[1] + G.k[3] * s[4];
    uf[2] = G.k[4] * s[0] + G.k[5] * s[3];
    uf[3] = 0.0;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) a += G.k[r * KC + j] * s[j];
      uf[r] = a;
    }
  }
  // Without feed-forward the reference adds ff terms that are exactly 0.0;
  // x + 0.0 differs from x only for x = -0.0, which no later operation
  // distinguishes (clips, products and sums all treat the zeros alike).
  const double raw0 = FF ? hover + uf[0] + ffa[2] : hover + uf[0];
  const double raw1 = FF ? uf[1] + -ffa[1] : uf[1];
  const double raw2 = FF ? uf[2] + ffa[0] : uf[2];
  const double raw3 = uf[3];
  u[0] = clip_num(raw0, c.min_thrust, c.max_thrust);
  u[1] = clip_num(raw1, -c.max_rate, c.max_rate);
  u[2] = clip_num(raw2, -c.max_rate, c.max_rate);
  // structured gains have no yaw row: clip(0, -max_rate, max_rate) = 0 for
  // the max_rate >= 0 that fast_path_ok requires
  u[3] = (KS && FAST) ? 0.0 : clip_num(raw3, -c.max_rate, c.max_rate);
  if (!FAST && any_lane(!isfinite((raw0 + raw1) + (raw2 + raw3)))) {  // np.clip keeps NaN (e.g. NaN fallback gains)
    u[0] = raw0 != raw0 ? raw0 : u[0];
    u[1] = raw1 != raw1 ? raw1 : u[1];
    u[2] = raw2 != raw2 ? raw2 : u[2];
    u[3] = raw3 != raw3 ? raw3 : u[3];
  }
  if (diag) {  // get_control_components (riccati_lqr.py:946-954)
#pragma unroll
    for (int i = 0; i < 6; ++i) diag[i] = s[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) diag[6 + i] = uf[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) diag[10 + i] = ffv[i], diag[13 + i] = ffa[i];
  }
  return (u[0] != raw0) || (u[1] != raw1) || (u[2] != raw2) || (u[3] != raw3);
}

// PIDController.compute_action (controllers/__init__.py:243-379) given the
// observation (quad p, v; target p, v, a) and its time `now`.  integ[4]:
// integral error xyz and the last observation time (NaN = None, 263-265).
// The integral advances by pos_error * dt only when dt > 0 and is clipped to
// +-integral_limit (266-271); yaw rate is always 0 (373).  diag (optional, 18):
// p, i, d, ff_velocity, ff_acceleration terms and the total correction
// (get_control_components, 346-353).
// FAST: gains, hover thrust, state and integral are known finite.
template <bool FF, bool FAST = false>
__device__ __forceinline__ void compute_action_pid(const qt_ctrl_params& c, const double* g, double hover,
                                                   const double* qp, const double* qv, const Target& tg, double now,
                                                   const FFLane& f, double* integ, double* u,
                                                   double* diag = nullptr) {
  const double *kp = g, *ki = g + 3, *kd = g + 6;
  double ep[3], tv[3] = {tg.v[0], tg.v[1], tg.v[2]}, ffa[3] = {0, 0, 0}, ffv[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 3; ++i) ep[i] = tg.p[i] - qp[i];
  const double last = integ[3];
  // NaN = None (the first observation); a bit test, since the fast kernels are
  // built with relaxed NaN handling (qt_rollout_fast.hip)
  const bool none = (__double_as_longlong(last) & 0x7fffffffffffffffLL) > 0x7ff0000000000000LL;
  const double dt = none ? 0.0 : now - last;
  integ[3] = now;
  const double lim = c.integral_limit;
  if (FAST) {  // select, not branch: the update is a handful of FMAs
    const bool upd = dt > 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double v = clipd(integ[i] + ep[i] * dt, -lim, lim);
      integ[i] = upd ? v : integ[i];
    }
  } else if (dt > 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) integ[i] = clipd(integ[i] + ep[i] * dt, -lim, lim);
  }
  if (FF) {
    const double vm = norm3(tv[0], tv[1], tv[2]);
    if (vm > f.vmax && vm > 0) {
      const double scl = f.vmax / vm;
#pragma unroll
      for (int i = 0; i < 3; ++i) tv[i] = tv[i] * scl;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      tv[i] = (1.0 + f.vg[i]) * tv[i];
      ffv[i] = kd[i] * f.vg[i] * tv[i] / (1.0 + f.vg[i]);
    }
    double ac[3] = {tg.a[0], tg.a[1], tg.a[2]};
    const double am = norm3(ac[0], ac[1], ac[2]);
    if (am > c.ff_max_acceleration && am > 0) {
#pragma unroll
      for (int i = 0; i < 3; ++i) ac[i] = ac[i] / am * c.ff_max_acceleration;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) ffa[i] = f.ag[i] * ac[i];
  }
  double p[3], it[3], d[3], corr[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    p[i] = kp[i] * ep[i];
    it[i] = ki[i] * integ[i];
    d[i] = kd[i] * (tv[i] - qv[i]);
    corr[i] = ((p[i] + it[i]) + d[i]) + ffa[i];
  }
  const double raw0 = hover + corr[2], raw1 = -corr[1], raw2 = corr[0];
  u[0] = clip_num(raw0, c.min_thrust, c.max_thrust);
  u[1] = clip_num(raw1, -c.max_rate, c.max_rate);
  u[2] = clip_num(raw2, -c.max_rate, c.max_rate);
  u[3] = 0.0;
  if (!FAST && !isfinite((raw0 + raw1) + raw2)) {  // np.clip keeps NaN
    u[0] = raw0 != raw0 ? raw0 : u[0];
    u[1] = raw1 != raw1 ? raw1 : u[1];
    u[2] = raw2 != raw2 ? raw2 : u[2];
  }
  if (diag) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      diag[i] = p[i];
      diag[3 + i] = it[i];
      diag[6 + i] = d[i];
      diag[9 + i] = ffv[i];
      diag[12 + i] = ffa[i];
      diag[15 + i] = corr[i];
    }
  }
}

}  // namespace qt
