/*
 * qt_oracle.c — CPU restatement of the reference hot path.  TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker / CPU baseline, never by the
 * product (lqr-quadcopter-test_amd/quadtrack), which runs on HIP only.
 *
 * Scalar FP64 C, one episode at a time, operation order following the
 * reference's NumPy expressions (AgentFoundryExamples/lqr-quadcopter-test,
 * paths relative to src/quadcopter_tracking/).  Episodes are independent and
 * spread over OpenMP threads.  Parity pinning: tests/test_oracle.py checks this
 * file against the golden fixtures generated from the reference itself
 * (tests/golden/gen_golden.py).
 *
 * Build: oracle/Makefile -> oracle/libqt_oracle.so
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/quadtrack.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#define OQ_PI 3.141592653589793
#define OQ_TWO_PI 6.283185307179586 /* 2 * np.pi */

static double sq(double v) { return v * v; }
/* np.linalg.norm of a 1-D 3-vector is sqrt(x.dot(x)), and this image's
   OpenBLAS ddot accumulates with FMA: sqrt(fma(z, z, fma(y, y, x * x)))
   (identical to numpy on 20,000 random vectors; the plain sum differs in
   ~11%).  norm3_rows: np.linalg.norm(..., axis=1) of the metrics
   (utils/metrics.py:162), a plain left-to-right sum of squares. */
static double norm3(const double* v) { return sqrt(fma(v[2], v[2], fma(v[1], v[1], v[0] * v[0]))); }
static double norm3_rows(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
/* np.clip = minimum(maximum(a, lo), hi), NaN-propagating */
static double clipd(double v, double lo, double hi) {
  double r = v;
  if (r < lo) r = lo;
  if (r > hi) r = hi;
  return r;
}

/* ----------------------------------------------------------- target motion */

/* pattern.get_state(t) for the five patterns (env/target_motion.py:29-248)
   and the acceleration clamp of TargetMotion.get_state (387-411).
   pat: linear raw standard_normal(3) draw | circular theta0 | sinusoidal phases. */
void oq_target_state(const qt_env_params* e, int motion, const double* pat, double t, double* out) {
  double p[3] = {e->center[0], e->center[1], e->center[2]};
  double v[3] = {0, 0, 0}, a[3] = {0, 0, 0};
  if (motion == QT_MOTION_LINEAR) {
    /* target_motion.py:320-321 then LinearMotion.__init__ 47-49 */
    double d[3] = {pat[0], pat[1], pat[2]};
    double n1 = norm3(d);
    for (int i = 0; i < 3; ++i) d[i] /= n1;
    double n2 = norm3(d);
    for (int i = 0; i < 3; ++i) {
      double vel = (d[i] / n2) * e->speed;
      p[i] = e->center[i] + vel * t;
      v[i] = vel;
    }
  } else if (motion == QT_MOTION_CIRCULAR) {
    /* CircularMotion 59-115 */
    double om = e->speed / e->radius;
    double ang = pat[0] + om * t;
    double c = cos(ang), s = sin(ang);
    p[0] = e->center[0] + e->radius * c;
    p[1] = e->center[1] + e->radius * s;
    v[0] = -e->radius * om * s;
    v[1] = e->radius * om * c;
    a[0] = -e->radius * pow(om, 2.0) * c; /* omega**2: Python's float pow (libm), */
    a[1] = -e->radius * pow(om, 2.0) * s; /* not always om * om rounded */
  } else if (motion == QT_MOTION_SINUSOIDAL) {
    /* _create_pattern 337-359, SinusoidalMotion 118-150 */
    double amp[3] = {e->amplitude, e->amplitude * 0.5, e->amplitude * 0.25};
    double fr[3] = {e->frequency, e->frequency * 1.3, e->frequency * 0.7};
    for (int i = 0; i < 3; ++i) {
      double om = 2.0 * OQ_PI * fr[i];
      double th = om * t + pat[i];
      double s = sin(th), c = cos(th);
      p[i] = e->center[i] + amp[i] * s;
      v[i] = amp[i] * om * c;
      a[i] = -amp[i] * (om * om) * s; /* omega is an ndarray: omega**2 is np.square */
    }
  } else if (motion == QT_MOTION_FIGURE8) {
    /* Figure8Motion 153-231 (scale = amplitude) */
    double sc = e->amplitude, om = e->speed / sc;
    double th = om * t;
    double ct = cos(th), st = sin(th);
    /* sin_t**2, denom**2: numpy float64 scalar power = libm pow, which
       rounds x^2 differently from x * x in ~0.2% of arguments */
    double den = 1.0 + pow(st, 2.0);
    p[0] = e->center[0] + sc * ct / den;
    p[1] = e->center[1] + sc * st * ct / den;
    double dcos = -st * om, dsin = ct * om;
    double dden = 2.0 * st * dsin;
    double den2 = pow(den, 2.0);
    double dx = (dcos * den - ct * dden) / den2;
    double dy = ((dsin * ct + st * dcos) * den - st * ct * dden) / den2;
    v[0] = sc * dx;
    v[1] = sc * dy;
    double h = 1e-6;
    double thp = om * (t + h);
    double ctp = cos(thp), stp = sin(thp);
    double denp = 1.0 + pow(stp, 2.0);
    double pp0 = e->center[0] + sc * ctp / denp;
    double pp1 = e->center[1] + sc * stp * ctp / denp;
    a[0] = ((pp0 - p[0]) / h - v[0]) / h;
    a[1] = ((pp1 - p[1]) / h - v[1]) / h;
    a[2] = ((e->center[2] - p[2]) / h - v[2]) / h;
  }
  double am = norm3(a);
  if (am > e->max_acceleration)
    for (int i = 0; i < 3; ++i) a[i] = a[i] / am * e->max_acceleration;
  for (int i = 0; i < 3; ++i) {
    out[i] = p[i];
    out[3 + i] = v[i];
    out[6 + i] = a[i];
  }
}

/* ------------------------------------------------------------------ plant */

/* _compute_derivatives (env/quadcopter_env.py:329-426) */
static void deriv(const qt_env_params* e, double mass, const double* s, const double* u, double* d) {
  double cphi = cos(s[6]), sphi = sin(s[6]);
  double cth = cos(s[7]), sth = sin(s[7]);
  double cpsi = cos(s[8]), spsi = sin(s[8]);
  double T = u[0];
  double tw[3] = {(cpsi * sth * cphi + spsi * sphi) * T, (spsi * sth * cphi - cpsi * sphi) * T,
                  (cth * cphi) * T};
  double g[3] = {0.0, 0.0, -mass * e->gravity};
  for (int i = 0; i < 3; ++i) {
    d[i] = s[3 + i];
    d[3 + i] = ((tw[i] + g[i]) + (-e->drag_linear * s[3 + i])) / mass;
    d[6 + i] = s[9 + i];
    double aa = (u[1 + i] - s[9 + i]) / 0.1;
    d[9 + i] = aa - e->drag_angular * s[9 + i];
  }
}

/* _integrate / _rk4_step / _euler_step (295-327) */
static void integrate(const qt_env_params* e, double mass, const double* s, const double* u, double* out) {
  double dt = e->dt;
  if (e->integrator == 1) {
    double d[12];
    deriv(e, mass, s, u, d);
    for (int i = 0; i < 12; ++i) out[i] = s[i] + d[i] * dt;
    return;
  }
  double k1[12], k2[12], k3[12], k4[12], tmp[12];
  deriv(e, mass, s, u, k1);
  for (int i = 0; i < 12; ++i) tmp[i] = s[i] + (0.5 * dt) * k1[i];
  deriv(e, mass, tmp, u, k2);
  for (int i = 0; i < 12; ++i) tmp[i] = s[i] + (0.5 * dt) * k2[i];
  deriv(e, mass, tmp, u, k3);
  for (int i = 0; i < 12; ++i) tmp[i] = s[i] + dt * k3[i];
  deriv(e, mass, tmp, u, k4);
  double h6 = dt / 6.0;
  for (int i = 0; i < 12; ++i) out[i] = s[i] + h6 * (((k1[i] + 2.0 * k2[i]) + 2.0 * k3[i]) + k4[i]);
}

/* numpy float remainder (floor-mod: result takes the sign of the divisor) */
static double py_mod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}

/* _apply_state_constraints (428-465) */
static void constrain(const qt_env_params* e, double* s) {
  double vm = norm3(s + 3);
  if (vm > e->max_velocity)
    for (int i = 3; i < 6; ++i) s[i] = s[i] / vm * e->max_velocity;
  for (int i = 9; i < 12; ++i) s[i] = clipd(s[i], -e->max_angular_velocity, e->max_angular_velocity);
  for (int i = 6; i < 9; ++i) s[i] = py_mod(s[i] + OQ_PI, OQ_TWO_PI) - OQ_PI;
  double tilt = OQ_PI / 3.0;
  s[6] = clipd(s[6], -tilt, tilt);
  s[7] = clipd(s[7], -tilt, tilt);
}

/* _parse_and_validate_action (234-293); returns 1 if any violation */
static int parse_action(const qt_env_params* e, const double* in, double* a) {
  int viol = 0;
  for (int i = 0; i < 4; ++i) a[i] = in[i];
  if (!(isfinite(a[0]) && isfinite(a[1]) && isfinite(a[2]) && isfinite(a[3]))) {
    viol = 1;
    for (int i = 0; i < 4; ++i)
      if (!isfinite(a[i])) a[i] = 0.0;
  }
  if (a[0] < e->min_thrust) {
    viol = 1;
    a[0] = e->min_thrust;
  } else if (a[0] > e->max_thrust) {
    viol = 1;
    a[0] = e->max_thrust;
  }
  for (int i = 1; i < 4; ++i) {
    if (fabs(a[i]) > e->max_angular_rate) {
      viol = 1;
      a[i] = clipd(a[i], -e->max_angular_rate, e->max_angular_rate);
    }
  }
  return viol;
}

/* _check_termination (513-535) */
static int termination(const qt_env_params* e, double t, const double* s) {
  if (t >= e->max_episode_time) return QT_TERM_TIME_LIMIT;
  for (int i = 0; i < 3; ++i)
    if (fabs(s[i]) > e->max_position) return QT_TERM_POSITION_BOUNDS;
  for (int i = 0; i < 12; ++i)
    if (!isfinite(s[i])) return QT_TERM_NUMERICAL_INSTABILITY;
  return QT_TERM_RUNNING;
}

/* One QuadcopterEnv.step (152-232).  x, t updated in place; tgt receives the
   target at the new time; returns termination code; *err, *viol out. */
int oq_env_step(const qt_env_params* e, int motion, const double* pat, double mass, double* x, double* t,
                const double* action, double* tgt, double* err, int* viol) {
  double a[4], xn[12];
  *viol = parse_action(e, action, a);
  integrate(e, mass, x, a, xn);
  constrain(e, xn);
  memcpy(x, xn, sizeof(xn));
  *t += e->dt;
  oq_target_state(e, motion, pat, *t, tgt);
  double d[3] = {x[0] - tgt[0], x[1] - tgt[1], x[2] - tgt[2]};
  *err = norm3(d);
  return termination(e, *t, x);
}

/* ------------------------------------------------------------- controller */

static double npsign(double v) { return v > 0 ? 1.0 : (v < 0 ? -1.0 : (v == 0 ? 0.0 : NAN)); }

/* RiccatiLQRController.compute_action (controllers/riccati_lqr.py:779-967).
   obs15: quad pos, quad vel, target pos, target vel, target acc.
   K: 4 x kcols row-major.  integ updated in LQI mode.  Returns saturated flag. */
int oq_compute_action(const qt_ctrl_params* c, const double* K, int kcols, double hover, const double* obs15,
                      double* integ, double* u_out) {
  const double* qp = obs15;
  const double* qv = obs15 + 3;
  const double* tp = obs15 + 6;
  const double* tv = obs15 + 9;
  const double* ta = obs15 + 12;
  double ep[3], ev[3], etv[3] = {tv[0], tv[1], tv[2]}, ffa[3] = {0, 0, 0};
  for (int i = 0; i < 3; ++i) ep[i] = tp[i] - qp[i];
  if (c->feedforward_enabled) {
    double vm = norm3(etv);
    if (vm > c->ff_max_velocity) {
      double scl = c->ff_max_velocity / vm;
      for (int i = 0; i < 3; ++i) etv[i] = etv[i] * scl;
    }
    for (int i = 0; i < 3; ++i) etv[i] = (1.0 + c->ff_velocity_gain[i]) * etv[i];
    double acc[3] = {ta[0], ta[1], ta[2]};
    double am = norm3(acc);
    if (am > c->ff_max_acceleration && am > 0)
      for (int i = 0; i < 3; ++i) acc[i] = acc[i] / am * c->ff_max_acceleration;
    for (int i = 0; i < 3; ++i) ffa[i] = c->ff_acceleration_gain[i] * acc[i];
  }
  for (int i = 0; i < 3; ++i) ev[i] = etv[i] - qv[i];
  double s[6] = {ep[0], ep[1], ep[2], ev[0], ev[1], ev[2]};
  double u[4];
  if (c->use_lqi && kcols == 9) {
    double em = norm3(ep);
    if (em > c->integral_zero_threshold) {
      for (int i = 0; i < 3; ++i) {
        int sat = fabs(integ[i]) >= c->integral_limit && c->integral_limit > 0;
        int worse = npsign(integ[i]) == npsign(ep[i]);
        if (!(sat && worse)) integ[i] += c->dt * ep[i];
      }
    }
    if (c->integral_limit > 0)
      for (int i = 0; i < 3; ++i) integ[i] = clipd(integ[i], -c->integral_limit, c->integral_limit);
    for (int r = 0; r < 4; ++r) {
      double a = 0, b = 0;
      for (int j = 0; j < 6; ++j) a += K[r * 9 + j] * s[j];
      for (int j = 0; j < 3; ++j) b += K[r * 9 + 6 + j] * integ[j];
      u[r] = a + b;
    }
  } else {
    for (int r = 0; r < 4; ++r) {
      double a = 0;
      for (int j = 0; j < 6; ++j) a += K[r * kcols + j] * s[j];
      u[r] = a;
    }
  }
  double raw[4] = {hover + u[0] + ffa[2], u[1] + -ffa[1], u[2] + ffa[0], u[3]};
  u_out[0] = clipd(raw[0], c->min_thrust, c->max_thrust);
  for (int i = 1; i < 4; ++i) u_out[i] = clipd(raw[i], -c->max_rate, c->max_rate);
  int sat = 0;
  for (int i = 0; i < 4; ++i) sat |= (u_out[i] != raw[i]);
  return sat;
}

/* PIDController.compute_action (controllers/__init__.py:243-379).
   gains: kp[3], ki[3], kd[3].  obs16: obs15 + observation time.
   state: integral error[3], last observation time (NaN = None).
   diag (optional, 18): p, i, d, ff_velocity, ff_acceleration, total correction. */
void oq_compute_action_pid(const qt_ctrl_params* c, const double* gains, double hover, const double* obs16,
                           double* state, double* u_out, double* diag) {
  const double* kp = gains;
  const double* ki = gains + 3;
  const double* kd = gains + 6;
  const double* qp = obs16;
  const double* qv = obs16 + 3;
  const double* tp = obs16 + 6;
  const double* tv = obs16 + 9;
  const double* ta = obs16 + 12;
  const double now = obs16[15];
  double ep[3];
  for (int i = 0; i < 3; ++i) ep[i] = tp[i] - qp[i];
  const double dt = isnan(state[3]) ? 0.0 : now - state[3]; /* 263-265 */
  state[3] = now;
  if (dt > 0) {
    for (int i = 0; i < 3; ++i) state[i] += ep[i] * dt;
    for (int i = 0; i < 3; ++i) state[i] = clipd(state[i], -c->integral_limit, c->integral_limit);
  }
  double p[3], it[3], etv[3] = {tv[0], tv[1], tv[2]}, ffv[3] = {0, 0, 0}, ffa[3] = {0, 0, 0};
  for (int i = 0; i < 3; ++i) {
    p[i] = kp[i] * ep[i];
    it[i] = ki[i] * state[i];
  }
  if (c->feedforward_enabled) {
    double vm = norm3(etv);
    if (vm > c->ff_max_velocity && vm > 0) {
      double scl = c->ff_max_velocity / vm;
      for (int i = 0; i < 3; ++i) etv[i] = etv[i] * scl;
    }
    for (int i = 0; i < 3; ++i) etv[i] = (1.0 + c->ff_velocity_gain[i]) * etv[i];
    for (int i = 0; i < 3; ++i) ffv[i] = kd[i] * c->ff_velocity_gain[i] * etv[i] / (1.0 + c->ff_velocity_gain[i]);
    double acc[3] = {ta[0], ta[1], ta[2]};
    double am = norm3(acc);
    if (am > c->ff_max_acceleration && am > 0)
      for (int i = 0; i < 3; ++i) acc[i] = acc[i] / am * c->ff_max_acceleration;
    for (int i = 0; i < 3; ++i) ffa[i] = c->ff_acceleration_gain[i] * acc[i];
  }
  double d[3], corr[3];
  for (int i = 0; i < 3; ++i) {
    d[i] = kd[i] * (etv[i] - qv[i]);
    corr[i] = ((p[i] + it[i]) + d[i]) + ffa[i];
  }
  u_out[0] = clipd(hover + corr[2], c->min_thrust, c->max_thrust);
  u_out[1] = clipd(-corr[1], -c->max_rate, c->max_rate);
  u_out[2] = clipd(corr[0], -c->max_rate, c->max_rate);
  u_out[3] = 0.0;
  if (diag)
    for (int i = 0; i < 3; ++i) {
      diag[i] = p[i];
      diag[3 + i] = it[i];
      diag[6 + i] = d[i];
      diag[9 + i] = ffv[i];
      diag[12 + i] = ffa[i];
      diag[15 + i] = corr[i];
    }
}

/* ----------------------------------------------------------- closed loop */

/* Evaluator.run_episode with a fresh controller (eval.py:95-167), per-episode
   metrics as compute_episode_metrics (utils/metrics.py:264-338).
   Inputs (AoS): x0[12], pat[4], K[4*kcols]; met[QT_MET_ROWS] out; xf[12],
   integ_out[3] out; rec (optional) [max_steps][16] states + actions. */
void oq_episode(const qt_env_params* e, const qt_ctrl_params* c, const qt_criteria* cr, int motion,
                const double* pat, double mass, double hover, const double* K, int kcols, const double* x0,
                int max_steps, double* met, double* xf, double* integ_out, double* rec) {
  double x[12], integ[4] = {0, 0, 0, NAN}, tgt[9], t = 0.0; /* PID: integ[3] = last time */
  memcpy(x, x0, sizeof(x));
  oq_target_state(e, motion, pat, 0.0, tgt);
  double sum_e = 0, sum_e2 = 0, max_e = -INFINITY, sum_u = 0;
  long on_pre = 0, on_post = 0, nviol = 0, steps = 0;
  int os_in = 0, os_streak = 0, os_count = 0, prev_on = 0;
  double os_cur = 0, os_max = 0;
  int term = QT_TERM_RUNNING;
  double R = cr->target_radius;
  int W = cr->overshoot_window;
  while (term == QT_TERM_RUNNING && (max_steps < 0 || steps < max_steps)) {
    double obs[15];
    for (int i = 0; i < 3; ++i) {
      obs[i] = x[i];
      obs[3 + i] = x[3 + i];
    }
    for (int i = 0; i < 9; ++i) obs[6 + i] = tgt[i];
    double u[4];
    if (kcols == 3) { /* PID: K holds kp, ki, kd */
      double obs16[16];
      memcpy(obs16, obs, sizeof(obs));
      obs16[15] = t;
      oq_compute_action_pid(c, K, hover, obs16, integ, u, NULL);
    } else {
      oq_compute_action(c, K, kcols, hover, obs, integ, u);
    }
    /* pre-step record (eval.py:142-159) */
    double d[3] = {tgt[0] - x[0], tgt[1] - x[1], tgt[2] - x[2]};
    double ep = norm3_rows(d);
    sum_e += ep;
    sum_e2 += ep * ep;
    if (!(ep <= max_e)) max_e = (isnan(max_e) ? max_e : ep);
    int on = ep <= R;
    on_pre += on;
    sum_u += sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2] + u[3] * u[3]);
    if (steps > 0) { /* detect_overshoots transition (metrics.py:236-254) */
      double ov = ep - R;
      if (prev_on && !on) {
        os_in = 1;
        os_streak = 1;
        os_cur = ov;
      } else if (os_in && !on) {
        os_streak += 1;
        if (ov > os_cur) os_cur = ov;
      } else if (os_in && on) {
        if (os_streak >= W) {
          os_count += 1;
          if (os_cur > os_max) os_max = os_cur;
        }
        os_in = 0;
        os_streak = 0;
        os_cur = 0.0;
      }
    }
    prev_on = on;
    double err;
    int viol;
    term = oq_env_step(e, motion, pat, mass, x, &t, u, tgt, &err, &viol);
    nviol += viol;
    on_post += err <= e->target_radius;
    if (rec) {
      for (int i = 0; i < 12; ++i) rec[steps * 16 + i] = x[i];
      for (int i = 0; i < 4; ++i) rec[steps * 16 + 12 + i] = u[i];
    }
    steps += 1;
  }
  if (os_in && os_streak >= W) {
    os_count += 1;
    if (os_cur > os_max) os_max = os_cur;
  }
  if (steps < W) {
    os_count = 0;
    os_max = 0.0;
  }
  if (steps == 0) { /* compute_episode_metrics on no data (metrics.py:287-291) */
    memset(met, 0, sizeof(double) * QT_MET_ROWS);
    memcpy(xf, x, sizeof(x));
    memcpy(integ_out, integ, 3 * sizeof(double));
    return;
  }
  double ns = (double)steps;
  double ratio = steps ? (double)on_pre / ns : 0.0;
  met[QT_MET_DURATION] = t;
  met[QT_MET_ON_TARGET_RATIO] = ratio;
  met[QT_MET_MEAN_ERR] = sum_e / ns;
  met[QT_MET_MAX_ERR] = max_e;
  met[QT_MET_RMS_ERR] = sqrt(sum_e2 / ns);
  met[QT_MET_TOTAL_EFFORT] = sum_u;
  met[QT_MET_MEAN_EFFORT] = sum_u / ns;
  met[QT_MET_OS_COUNT] = os_count;
  met[QT_MET_OS_MAX] = os_max;
  met[QT_MET_SUCCESS] = (t >= cr->min_episode_duration && ratio >= cr->min_on_target_ratio) ? 1.0 : 0.0;
  met[QT_MET_TERM] = term;
  met[QT_MET_VIOLATIONS] = (double)nviol;
  met[QT_MET_ENV_ON_TARGET_RATIO] = steps ? (double)on_post / ns : 0.0;
  met[QT_MET_STEPS] = ns;
  memcpy(xf, x, sizeof(x));
  memcpy(integ_out, integ, 3 * sizeof(double));
}

/* Many episodes (AoS inputs, stride per episode), OpenMP over episodes.
   k_stride = 0 shares one K.  Returns the number of threads used. */
int oq_rollout(const qt_env_params* e, const qt_ctrl_params* c, const qt_criteria* cr, long n,
               const int8_t* motion, const double* pat, const double* mass, const double* hover,
               const double* K, int kcols, long k_stride, const double* x0, int max_steps, double* met,
               double* xf, double* integ) {
  int nthreads = 1;
#pragma omp parallel
  {
#pragma omp single
    {
#ifdef _OPENMP
      nthreads = omp_get_num_threads();
#endif
    }
#pragma omp for schedule(dynamic, 4)
    for (long i = 0; i < n; ++i) {
      oq_episode(e, c, cr, motion ? motion[i] : e->motion, pat + 4 * i, mass ? mass[i] : e->mass,
                 hover ? hover[i] : c->hover_thrust, K + k_stride * i, kcols, x0 + 12 * i, max_steps,
                 met + QT_MET_ROWS * i, xf + 12 * i, integ + 3 * i, NULL);
    }
  }
  return nthreads;
}

/* ------------------------------------------------------------------- DARE */

/* LU with partial pivoting, in place (n <= 16); returns 0 if singular. */
static int lu(int n, double* a, int* piv) {
  for (int k = 0; k < n; ++k) {
    int p = k;
    double best = fabs(a[k * n + k]);
    for (int i = k + 1; i < n; ++i)
      if (fabs(a[i * n + k]) > best) {
        best = fabs(a[i * n + k]);
        p = i;
      }
    piv[k] = p;
    if (best == 0.0) return 0;
    if (p != k)
      for (int j = 0; j < n; ++j) {
        double tmp = a[k * n + j];
        a[k * n + j] = a[p * n + j];
        a[p * n + j] = tmp;
      }
    for (int i = k + 1; i < n; ++i) {
      double f = a[i * n + k] / a[k * n + k];
      a[i * n + k] = f;
      for (int j = k + 1; j < n; ++j) a[i * n + j] -= f * a[k * n + j];
    }
  }
  return 1;
}

/* solve (LU) X = B for B n x m row-major, in place */
static void lu_solve(int n, const double* a, const int* piv, double* b, int m) {
  for (int k = 0; k < n; ++k)
    if (piv[k] != k)
      for (int j = 0; j < m; ++j) {
        double tmp = b[k * m + j];
        b[k * m + j] = b[piv[k] * m + j];
        b[piv[k] * m + j] = tmp;
      }
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < i; ++k)
      for (int j = 0; j < m; ++j) b[i * m + j] -= a[i * n + k] * b[k * m + j];
  for (int i = n - 1; i >= 0; --i) {
    for (int k = i + 1; k < n; ++k)
      for (int j = 0; j < m; ++j) b[i * m + j] -= a[i * n + k] * b[k * m + j];
    for (int j = 0; j < m; ++j) b[i * m + j] /= a[i * n + i];
  }
}

static void matmul(int n, int k, int m, const double* a, const double* b, double* c) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) {
      double s = 0;
      for (int l = 0; l < k; ++l) s += a[i * k + l] * b[l * m + j];
      c[i * m + j] = s;
    }
}

/* The linearised hover model (build_linearized_system, riccati_lqr.py:187-263;
   build_augmented_lqi_system 266-316). */
void oq_build_system(int n, double dt, double mass, double gravity, double* A, double* B) {
  memset(A, 0, sizeof(double) * n * n);
  memset(B, 0, sizeof(double) * n * 4);
  for (int i = 0; i < n; ++i) A[i * n + i] = 1.0;
  for (int i = 0; i < 3; ++i) A[i * n + 3 + i] = dt;
  B[5 * 4 + 0] = 1.0 / mass * dt;
  B[4 * 4 + 1] = -gravity * dt;
  B[3 * 4 + 2] = gravity * dt;
  if (n == 9)
    for (int i = 0; i < 3; ++i) A[(6 + i) * n + i] = dt;
}

/* Structure-preserving doubling algorithm for the DARE
   A'XA - X - A'XB(R + B'XB)^-1 B'XA + Q = 0 (the equation scipy's
   solve_discrete_are solves, riccati_lqr.py:176), then
   K = (R + B'PB)^-1 B'PA (181-182).  Returns iterations (>0) or a negative
   status (-QT_DARE_*). */
int oq_dare(int n, const double* A, const double* B, const double* Q, const double* R, double* P, double* K,
            int max_iter, double tol) {
  double Ak[81], G[81], H[81], W[81], Y[162], T1[81], T2[81], Rl[16], BtX[36];
  int piv[16];
  /* G = B R^-1 B' */
  memcpy(Rl, R, sizeof(double) * 16);
  if (!lu(4, Rl, piv)) return -QT_DARE_SINGULAR;
  double RiBt[36];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < n; ++j) RiBt[i * n + j] = B[j * 4 + i];
  lu_solve(4, Rl, piv, RiBt, n);
  matmul(n, 4, n, B, RiBt, G);
  memcpy(Ak, A, sizeof(double) * n * n);
  memcpy(H, Q, sizeof(double) * n * n);
  int it;
  for (it = 1; it <= max_iter; ++it) {
    /* W = I + G H */
    matmul(n, n, n, G, H, W);
    for (int i = 0; i < n; ++i) W[i * n + i] += 1.0;
    if (!lu(n, W, piv)) return -QT_DARE_SINGULAR;
    /* Y = W^-1 [Ak | G] */
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        Y[i * 2 * n + j] = Ak[i * n + j];
        Y[i * 2 * n + n + j] = G[i * n + j];
      }
    lu_solve(n, W, piv, Y, 2 * n);
    double Y1[81], Y2[81], AkT[81];
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        Y1[i * n + j] = Y[i * 2 * n + j];
        Y2[i * n + j] = Y[i * 2 * n + n + j];
        AkT[i * n + j] = Ak[j * n + i];
      }
    /* H' = H + Ak' H Y1 */
    matmul(n, n, n, H, Y1, T1);
    matmul(n, n, n, AkT, T1, T2);
    double dn = 0, hn = 0;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double nh = H[i * n + j] + 0.5 * (T2[i * n + j] + T2[j * n + i]);
        T1[i * n + j] = nh;
      }
    for (int i = 0; i < n * n; ++i) {
      dn += sq(T1[i] - H[i]);
      hn += sq(T1[i]);
    }
    memcpy(H, T1, sizeof(double) * n * n);
    /* G' = G + Ak Y2 Ak' */
    matmul(n, n, n, Y2, AkT, T1);
    matmul(n, n, n, Ak, T1, T2);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) G[i * n + j] += 0.5 * (T2[i * n + j] + T2[j * n + i]);
    /* A' = Ak Y1 */
    matmul(n, n, n, Ak, Y1, T1);
    memcpy(Ak, T1, sizeof(double) * n * n);
    if (!isfinite(hn)) return -QT_DARE_NO_CONVERGE;
    if (sqrt(dn) <= tol * sqrt(hn)) break;
  }
  if (it > max_iter) return -QT_DARE_NO_CONVERGE;
  memcpy(P, H, sizeof(double) * n * n);
  /* K = (R + B'PB)^-1 B'PA */
  double Bt[36], M[16], BtPA[36];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < n; ++j) Bt[i * n + j] = B[j * 4 + i];
  matmul(4, n, n, Bt, P, BtX);
  matmul(4, n, 4, BtX, B, M);
  for (int i = 0; i < 16; ++i) M[i] += R[i];
  matmul(4, n, n, BtX, A, BtPA);
  if (!lu(4, M, piv)) return -QT_DARE_SINGULAR;
  lu_solve(4, M, piv, BtPA, n);
  memcpy(K, BtPA, sizeof(double) * 4 * n);
  return it;
}

/* LQRController._compute_gains (controllers/__init__.py:522-574): the
   heuristic fallback gains; K 4x6 row-major. */
void oq_heuristic_gains(const double* qpos, const double* qvel, double r_thrust, double r_rate, double* K) {
  memset(K, 0, sizeof(double) * 24);
  K[0 * 6 + 2] = sqrt(qpos[2] / r_thrust);
  K[0 * 6 + 5] = sqrt(2 * sqrt(qpos[2] / r_thrust) + qvel[2] / r_thrust);
  K[1 * 6 + 1] = -sqrt(qpos[1] / r_rate);
  K[1 * 6 + 4] = -sqrt(2 * sqrt(qpos[1] / r_rate) + qvel[1] / r_rate);
  K[2 * 6 + 0] = sqrt(qpos[0] / r_rate);
  K[2 * 6 + 3] = sqrt(2 * sqrt(qpos[0] / r_rate) + qvel[0] / r_rate);
}

int oq_abi_version(void) { return QT_ABI_VERSION; }

/* thread count for oq_rollout (the cpu_baseline leg states the cores it used) */
void oq_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#endif
}
