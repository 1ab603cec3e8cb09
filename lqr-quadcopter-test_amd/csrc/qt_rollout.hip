// qt_rollout.hip — batched closed-loop kernels and their C ABI (include/quadtrack.h).
//
// One lane = one episode.  A launch walks `nsteps` closed-loop steps with the
// whole episode (12-state plant, target pattern constants, 4x6 / 4x9 gains,
// LQI integral, metric accumulators) resident in registers; HBM is touched
// only to load the state at the start of a chunk and to store it at the end.
// Reference functions: src/quadcopter_tracking/... of the reference repo.
#include <hip/hip_runtime.h>

#include "qt_device.hpp"

using namespace qt;

// Measurement-only ablation switches (scripts/ablate.sh builds timing-only
// variants with -DQT_ABLATE=<bits>; results of such builds are wrong by
// construction).  The product build has QT_ABLATE == 0.
#ifndef QT_ABLATE
#define QT_ABLATE 0
#endif
#define QT_ABL_METRICS 1
#define QT_ABL_CONSTRAIN 2
#define QT_ABL_TERMINATION 4
#define QT_ABL_CONTROLLER 8
#define QT_ABL_TARGET 16

// Diagnostic clock-stamp build (scripts/clock_stamp.py; -DQT_CLOCK_STAMP=1):
// lane 0 of every wave of a fast-flavour launch records s_memtime (shader
// clock) and s_memrealtime (100 MHz) around its step loop into a buffer of
// its own, which no other code reads; qt_debug_stamps copies it out.  The
// product build has QT_CLOCK_STAMP == 0 and executes no stamp.
#ifndef QT_CLOCK_STAMP
#define QT_CLOCK_STAMP 0
#endif
#if QT_CLOCK_STAMP
constexpr int kStampWaves = 1 << 16;
__device__ unsigned long long g_qt_stamps[kStampWaves][4];
#endif

namespace {

constexpr int kBlock = 256;

struct Acc {
  double sum_e, sum_e2, max_e, sum_u, os_max, os_cur;
  int on_pre, on_post, os_count, os_streak, prev_on, steps, viol, term;
};

__device__ __forceinline__ Acc load_acc(const double* acc, int64_t n, int64_t e) {
  Acc a;
  a.sum_e = acc[QT_ACC_SUM_ERR * n + e];
  a.sum_e2 = acc[QT_ACC_SUM_ERR2 * n + e];
  a.max_e = acc[QT_ACC_MAX_ERR * n + e];
  a.on_pre = (int)acc[QT_ACC_ON_PRE * n + e];
  a.on_post = (int)acc[QT_ACC_ON_POST * n + e];
  a.sum_u = acc[QT_ACC_SUM_EFFORT * n + e];
  a.os_count = (int)acc[QT_ACC_OS_COUNT * n + e];
  a.os_max = acc[QT_ACC_OS_MAX * n + e];
  a.os_cur = acc[QT_ACC_OS_CUR * n + e];
  a.os_streak = (int)acc[QT_ACC_OS_STREAK * n + e];
  a.prev_on = (int)acc[QT_ACC_PREV_ON * n + e];
  a.steps = (int)acc[QT_ACC_STEPS * n + e];
  a.viol = (int)acc[QT_ACC_VIOLATIONS * n + e];
  a.term = (int)acc[QT_ACC_TERM * n + e];
  return a;
}

__device__ __forceinline__ void store_acc(double* acc, int64_t n, int64_t e, const Acc& a) {
  acc[QT_ACC_SUM_ERR * n + e] = a.sum_e;
  acc[QT_ACC_SUM_ERR2 * n + e] = a.sum_e2;
  acc[QT_ACC_MAX_ERR * n + e] = a.max_e;
  acc[QT_ACC_ON_PRE * n + e] = a.on_pre;
  acc[QT_ACC_ON_POST * n + e] = a.on_post;
  acc[QT_ACC_SUM_EFFORT * n + e] = a.sum_u;
  acc[QT_ACC_OS_COUNT * n + e] = a.os_count;
  acc[QT_ACC_OS_MAX * n + e] = a.os_max;
  acc[QT_ACC_OS_CUR * n + e] = a.os_cur;
  acc[QT_ACC_OS_STREAK * n + e] = a.os_streak;
  acc[QT_ACC_PREV_ON * n + e] = a.prev_on;
  acc[QT_ACC_STEPS * n + e] = a.steps;
  acc[QT_ACC_VIOLATIONS * n + e] = a.viol;
  acc[QT_ACC_TERM * n + e] = a.term;
}

struct BatchDev {
  int64_t n;
  const int8_t* motion;
  const double* pattern;
  const double* plant_mass;
  const double* hover;
  const double* K;
  int32_t k_cols;
  int32_t k_per_episode;
  const int32_t* order;
  int64_t slot0, slot_end;  // the slot range this launch covers (grouped launches)
};

__device__ __forceinline__ int64_t episode_of(const BatchDev& b, int64_t slot) {
  return b.order ? (int64_t)b.order[slot] : slot;
}

__device__ __forceinline__ int motion_of(const BatchDev& b, const qt_env_params& e, int64_t ep) {
  return b.motion ? (int)b.motion[ep] : e.motion;
}

__device__ __forceinline__ Pattern pattern_of(const BatchDev& b, const qt_env_params& e, int motion, int64_t ep) {
  const int64_t n = b.n;
  double r0 = 0, r1 = 0, r2 = 0;
  if (b.pattern) {
    r0 = b.pattern[0 * n + ep];
    r1 = b.pattern[1 * n + ep];
    r2 = b.pattern[2 * n + ep];
  }
  return make_pattern(e, motion, r0, r1, r2);
}

template <int KC, bool KS>
__device__ __forceinline__ void load_gains(const BatchDev& b, int64_t ep, Gains<KC, KS>& G) {
  const int64_t m = b.k_per_episode ? b.n : 1;
  const int64_t col = b.k_per_episode ? ep : 0;  // shared: uniform address -> scalar loads
#pragma unroll
  for (int j = 0; j < Gains<KC, KS>::kCount; ++j) {
    const int idx = (KS && KC != 3) ? structured_index<KC>(j) : j;
    G.k[j] = b.K[(int64_t)idx * m + col];
  }
}

// Overshoot state machine of detect_overshoots (utils/metrics.py:205-261),
// streamed over the pre-step errors: called for every step k >= 1 with the
// on-target flag of step k (the flag of k-1 is a.prev_on).  os_streak is the
// off-target streak while in an overshoot phase, -1 outside one.
__device__ __forceinline__ void overshoot_step(Acc& a, bool on, double over, int window) {
  // Branch-free form of the three transitions (metrics.py:238-254).  `start`
  // (previous step on target, this one off) and `in_phase` (previous step
  // off target inside a phase) exclude each other.  os_cur is only read
  // inside a phase; outside one it holds -inf after an on-target step (so a
  // phase start takes `over` through the same max) and is otherwise unused.
  const bool in_phase = a.os_streak >= 0;
  const bool start = (a.prev_on > 0) && !on;
  const bool counted = on && in_phase && a.os_streak >= window;
  a.os_count += counted;
  a.os_max = counted ? fmax(a.os_max, a.os_cur) : a.os_max;
  a.os_cur = on ? -INFINITY : fmax(over, a.os_cur);
  a.os_streak = on ? -1 : (start ? 1 : (in_phase ? a.os_streak + 1 : -1));
}

// ------------------------------------------------------------------ reset

__global__ __launch_bounds__(kBlock) void reset_kernel(qt_env_params e, BatchDev b, const double* __restrict__ off,
                                                       qt_state st) {
  const int64_t slot = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (slot >= b.n) return;
  const int64_t n = b.n, ep = episode_of(b, slot);
  const int motion = motion_of(b, e, ep);
  const Pattern pt = pattern_of(b, e, motion, ep);
  Target tg;
  target_state<true>(e, motion, pt, 0.0, tg);  // quadcopter_env.py:133-139
#pragma unroll
  for (int i = 0; i < 3; ++i) st.x[i * n + ep] = tg.p[i] + off[i * n + ep];
#pragma unroll
  for (int i = 3; i < 12; ++i) st.x[i * n + ep] = 0.0;
  if (st.integ) {  // fresh controller (riccati_lqr.py:1073-1086, controllers/__init__.py:389-393)
#pragma unroll
    for (int i = 0; i < 3; ++i) st.integ[i * n + ep] = 0.0;
    if (b.k_cols == 3) st.integ[3 * n + ep] = NAN;  // PID: no previous observation time
  }
  st.t[ep] = 0.0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    st.target[i * n + ep] = tg.p[i];
    st.target[(3 + i) * n + ep] = tg.v[i];
    st.target[(6 + i) * n + ep] = tg.a[i];
  }
  Acc a{0, 0, -INFINITY, 0, 0, 0, 0, 0, 0, -1, -1, 0, 0, QT_TERM_RUNNING};
  store_acc(st.acc, n, ep, a);
}

// ---------------------------------------------------------------- rollout

// The closed-loop steps of one lane.  FAST: the branch-light step of
// qt_device.hpp (fast_path_ok + finite lane inputs, no recording), which
// takes the exact step's decisions; rare lanes/steps (speed at the
// clamp, attitude far outside [-pi, pi), tracking error at the radius within
// 1e-14) fall back to the exact constraint / comparison code inside the step.
template <bool FAST, bool YAW0, int MOTION, int KC, bool FF, bool KS>
__device__ __forceinline__ void run_steps(const qt_env_params& e, const qt_ctrl_params& c, const qt_criteria& cr,
                                          int motion, const Pattern& pt, const Plant& pl, double hover,
                                          const Gains<KC, KS>& G, double* x, double* integ, Target& tg, double& t,
                                          Acc& a, int nsteps, double* __restrict__ rec, int64_t n, int64_t ep,
                                          const RateLin& rl) {
  const double R = cr.target_radius;
  const double er2lo = e.target_radius * e.target_radius * (1.0 - 1e-14);
  const double er2hi = e.target_radius * e.target_radius * (1.0 + 1e-14);
  // squared pre-step tracking error: the previous step's post-step error
  // (same positions, same target: positions are not constrained), carried
  double se_pre;
  {
    const double ep0 = tg.p[0] - x[0], ep1 = tg.p[1] - x[1], ep2 = tg.p[2] - x[2];
    se_pre = ep0 * ep0 + ep1 * ep1 + ep2 * ep2;
  }
  // fast steps of a periodic pattern carry its angles' sin / cos (target_state_carried)
  constexpr bool kCarry = FAST && (MOTION == QT_MOTION_SINUSOIDAL || MOTION == QT_MOTION_CIRCULAR);
  PeriodicTrig<kCarry ? MOTION : QT_MOTION_CIRCULAR> ptrig;
  if constexpr (kCarry) periodic_trig_init(pt, t, ptrig);
  // yaw-at-rest fast steps: RK4 in closed form (integrate_yaw0)
  // and carried roll / pitch sin / cos (attitude_trig_advance)
  VelLin lin;
  Trig ta;
  double aprev[2];
  if constexpr (FAST && YAW0) {
    lin = make_vel_lin(e, pl);
    trig_of<true>(x + 6, ta);
    aprev[0] = x[6], aprev[1] = x[7];
  }
  for (int s = 0; s < nsteps; ++s) {
    if (a.term != QT_TERM_RUNNING) break;
    // ---- compute_action on the current observation (riccati_lqr.py:779-967)
    double u[4];
    // fast step: the pre-step tracking error, also the LQI's ||e_p|| (riccati_lqr.py:873)
    const double err_fast = FAST ? sqrt_noscale(se_pre) : 0.0;
    if (QT_ABLATE & QT_ABL_CONTROLLER) {
      u[0] = hover, u[1] = u[2] = u[3] = 0.0;
    } else {
      if constexpr (KC == 3)
        compute_action_pid<FF, FAST>(c, G.k, hover, x, x + 3, tg, t, integ, u);  // observation time = t
      else
        compute_action<KC, FF, KS, FAST>(c, G, hover, x, x + 3, tg, integ, u, nullptr, err_fast);
    }
    // ---- the Evaluator's pre-step record (eval.py:142-159) -> metrics accumulators
    if (!(QT_ABLATE & QT_ABL_METRICS)) {
      double err, un;
      if (FAST) {
        err = err_fast;
        un = sqrt_noscale(u[0] * u[0] + u[1] * u[1] + u[2] * u[2] + u[3] * u[3]);
      } else {
        const double ep0 = tg.p[0] - x[0], ep1 = tg.p[1] - x[1], ep2 = tg.p[2] - x[2];
        err = sqrt(ep0 * ep0 + ep1 * ep1 + ep2 * ep2);
        un = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2] + u[3] * u[3]);
      }
      a.sum_e += err;
      a.sum_e2 += err * err;
      if (FAST)  // err and max_e are numbers here (finite state): a plain max
        a.max_e = fmax(a.max_e, err);
      else if (!(err <= a.max_e) && !(a.max_e != a.max_e))
        a.max_e = err;  // np.max, NaN-propagating
      const bool on = err <= R;
      a.on_pre += on;
      a.sum_u += un;
      overshoot_step(a, on, err - R, cr.overshoot_window);  // no-op on the first step (prev_on < 0)
      a.prev_on = on;
    }
    // ---- env.step (quadcopter_env.py:152-232)
    if (FAST) {
      // the command is finite and inside the env clamps: parsing is the identity
      if constexpr (YAW0)
        integrate_yaw0(rl, lin, pl, ta, x, u);
      else
        integrate<true, false>(e, pl, x, u);
      t += e.dt;
      if (!(QT_ABLATE & QT_ABL_TARGET)) {
        if constexpr (kCarry)
          target_state_carried<FF, MOTION>(e, pt, t, ptrig, tg);
        else
          target_state<FF, true>(e, motion, pt, t, tg);
      }
      const double q0 = x[0] - tg.p[0], q1 = x[1] - tg.p[1], q2 = x[2] - tg.p[2];
      const double se = q0 * q0 + q1 * q1 + q2 * q2;  // positions are not constrained
      se_pre = se;
      const bool ok = ((se < er2lo) | (se > er2hi)) & ((QT_ABLATE & QT_ABL_CONSTRAIN) || constrain_fast_ok<YAW0>(e, x));
      // Wave-uniform choice: when any lane is off the fast preconditions the
      // whole wave runs the exact code, which takes the fast code's decisions
      // on the lanes that qualify.  A uniform, expected condition is a
      // not-taken scalar branch with the exact code out of line; a divergent
      // if / else cost a taken branch around the else block every step.
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) == 0, 1)) {
        if (!(QT_ABLATE & QT_ABL_CONSTRAIN)) constrain_fast_apply<YAW0>(e, x);
        if constexpr (YAW0) attitude_trig_advance(x + 6, aprev, ta);
        a.on_post += se < er2lo;
      } else {  // rare: exact constraints and comparison
        if (!(QT_ABLATE & QT_ABL_CONSTRAIN)) constrain<false>(e, x);
        if constexpr (YAW0) {  // restart the carried attitude trig (|roll|, |pitch| <= pi/3 again)
          trig_of<true>(x + 6, ta);
          aprev[0] = x[6], aprev[1] = x[7];
        }
        a.on_post += norm_le(se, e.target_radius);
      }
      if (QT_ABLATE & QT_ABL_TERMINATION)
        a.term = t >= e.max_episode_time ? QT_TERM_TIME_LIMIT : QT_TERM_RUNNING;
      else
        a.term = termination_fast(e, t, x);
      a.steps += 1;
    } else {
      double ua[4];
      a.viol += parse_action(e, u, ua);
      integrate(e, pl, x, ua);
      if (!(QT_ABLATE & QT_ABL_CONSTRAIN)) constrain<false>(e, x);
      t += e.dt;
      if (!(QT_ABLATE & QT_ABL_TARGET)) target_state<FF>(e, motion, pt, t, tg);
      const double q0 = x[0] - tg.p[0], q1 = x[1] - tg.p[1], q2 = x[2] - tg.p[2];
      a.on_post += norm_le(q0 * q0 + q1 * q1 + q2 * q2, e.target_radius);
      if (QT_ABLATE & QT_ABL_TERMINATION)
        a.term = t >= e.max_episode_time ? QT_TERM_TIME_LIMIT : QT_TERM_RUNNING;
      else
        a.term = termination(e, t, x);
      a.steps += 1;
      if (rec) {
        double* r = rec + (int64_t)s * 16 * n + ep;
#pragma unroll
        for (int i = 0; i < 12; ++i) r[i * n] = x[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) r[(12 + i) * n] = u[i];
      }
    }
  }
}

__device__ __forceinline__ bool all_finite(const double* v, int k) {
  double s = 0.0;
  for (int i = 0; i < k; ++i) s += v[i] * 0.0;  // NaN iff some v[i] is NaN or infinite
  return s == 0.0;
}

// step flavours: the exact step, the fast step, the fast step with yaw at rest
constexpr int kExact = 0, kFast = 1, kYaw0 = 2;

// MOTION >= 0 specialises the target pattern; -1 reads it per episode.
template <int FLAVOR, int MOTION, int KC, bool FF, bool KS>
__global__ __launch_bounds__(kBlock) void rollout_kernel(qt_env_params e, qt_ctrl_params c, qt_criteria cr,
                                                         BatchDev b, qt_state st, int nsteps,
                                                         double* __restrict__ rec, int deferred, RateLin rl) {
  const int64_t slot = b.slot0 + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (slot >= b.slot_end) return;
  const int64_t n = b.n, ep = episode_of(b, slot);
  const int motion = MOTION >= 0 ? MOTION : motion_of(b, e, ep);
  const Pattern pt = pattern_of(b, e, motion, ep);
  const Plant pl = make_plant(e, b.plant_mass ? b.plant_mass[ep] : e.mass);
  const double hover = b.hover ? b.hover[ep] : c.hover_thrust;
  Gains<KC, KS> G;
  load_gains<KC, KS>(b, ep, G);

  // integ: LQI integral (KC 9) | PID integral error + last observation time (KC 3)
  constexpr int NI = KC == 9 ? 3 : (KC == 3 ? 4 : 0);
  double x[12], integ[4] = {0, 0, 0, NAN};
#pragma unroll
  for (int i = 0; i < 12; ++i) x[i] = st.x[i * n + ep];
#pragma unroll
  for (int i = 0; i < NI; ++i) integ[i] = st.integ[i * n + ep];
  Target tg;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    tg.p[i] = st.target[i * n + ep];
    tg.v[i] = st.target[(3 + i) * n + ep];
    tg.a[i] = st.target[(6 + i) * n + ep];
  }
  double t = st.t[ep];
  Acc a = load_acc(st.acc, n, ep);

  // Which step the wavefront runs (uniform).  A fast flavour is launched only
  // when the launch-level preconditions hold (fast_path_ok, no recording); it
  // takes the waves whose lanes all qualify and leaves the others untouched,
  // and the exact kernel launched after it with `deferred` = that flavour
  // takes exactly those (the same test on the same inputs).
  bool lane_ok = a.term != QT_TERM_RUNNING ||
                 (all_finite(G.k, Gains<KC, KS>::kCount) && all_finite(x, 12) && all_finite(integ, 3) &&
                  all_finite(tg.p, 3) && all_finite(tg.v, 3) && all_finite(tg.a, 3) && isfinite(hover) &&
                  isfinite(pl.inv_mass) && fabs(t) < 1e300);
  for (int i = 9; i < 12; ++i) lane_ok = lane_ok && fabs(x[i]) <= e.max_angular_velocity;
  // structured gains (or any K whose yaw-rate row is zero: qt_batch.k_no_yaw)
  // never command yaw: a yaw at rest stays exactly zero
  // (and, tilt-bounded, roll and pitch inside the tilt clamp: trig_of<YAW0>;
  // rate-bounded, roll and pitch rates within the command clip: rate_bounded_ok)
  if (FLAVOR == kYaw0 || deferred == kYaw0)
    lane_ok = lane_ok && x[8] == 0.0 && x[11] == 0.0 && fabs(x[6]) <= kMaxTilt && fabs(x[7]) <= kMaxTilt &&
              fabs(x[9]) <= c.max_rate && fabs(x[10]) <= c.max_rate;
  const bool wave_ok = __builtin_amdgcn_ballot_w64(!lane_ok) == 0;
  if (FLAVOR != kExact) {
    if (!wave_ok) return;
#if QT_CLOCK_STAMP
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
    run_steps<true, FLAVOR == kYaw0, MOTION, KC, FF, KS>(e, c, cr, motion, pt, pl, hover, G, x, integ, tg, t, a,
                                                         nsteps, rec, n, ep, rl);
#if QT_CLOCK_STAMP
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const int64_t wave = (slot - b.slot0) >> 6;
    if ((threadIdx.x & 63) == 0 && wave < kStampWaves) {
      g_qt_stamps[wave][0] = t0, g_qt_stamps[wave][1] = t1;
      g_qt_stamps[wave][2] = r0, g_qt_stamps[wave][3] = r1;
    }
#endif
  } else {
    if (deferred != kExact && wave_ok) return;
    run_steps<false, false, MOTION, KC, FF, KS>(e, c, cr, motion, pt, pl, hover, G, x, integ, tg, t, a, nsteps, rec,
                                                n, ep, rl);
  }

#pragma unroll
  for (int i = 0; i < 12; ++i) st.x[i * n + ep] = x[i];
#pragma unroll
  for (int i = 0; i < NI; ++i) st.integ[i * n + ep] = integ[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    st.target[i * n + ep] = tg.p[i];
    st.target[(3 + i) * n + ep] = tg.v[i];
    st.target[(6 + i) * n + ep] = tg.a[i];
  }
  st.t[ep] = t;
  store_acc(st.acc, n, ep, a);
}

// ------------------------------------------------------ open-loop env.step

__global__ __launch_bounds__(kBlock) void env_step_kernel(qt_env_params e, BatchDev b,
                                                          const double* __restrict__ action, qt_state st,
                                                          double* err_out, int8_t* on_out, int8_t* done_out,
                                                          int8_t* term_out, int8_t* viol_out) {
  const int64_t slot = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (slot >= b.n) return;
  const int64_t n = b.n, ep = episode_of(b, slot);
  const int motion = motion_of(b, e, ep);
  const Pattern pt = pattern_of(b, e, motion, ep);
  const Plant pl = make_plant(e, b.plant_mass ? b.plant_mass[ep] : e.mass);
  double x[12], u[4], ua[4];
#pragma unroll
  for (int i = 0; i < 12; ++i) x[i] = st.x[i * n + ep];
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = action[i * n + ep];
  const bool viol = parse_action(e, u, ua);
  integrate(e, pl, x, ua);
  constrain(e, x);
  double t = st.t[ep] + e.dt;
  Target tg;
  target_state<true>(e, motion, pt, t, tg);
  const double q0 = x[0] - tg.p[0], q1 = x[1] - tg.p[1], q2 = x[2] - tg.p[2];
  const double err = sqrt(q0 * q0 + q1 * q1 + q2 * q2);
  const bool on = err <= e.target_radius;
  const int term = termination(e, t, x);
#pragma unroll
  for (int i = 0; i < 12; ++i) st.x[i * n + ep] = x[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    st.target[i * n + ep] = tg.p[i];
    st.target[(3 + i) * n + ep] = tg.v[i];
    st.target[(6 + i) * n + ep] = tg.a[i];
  }
  st.t[ep] = t;
  st.acc[QT_ACC_ON_POST * n + ep] += on;
  st.acc[QT_ACC_STEPS * n + ep] += 1.0;
  st.acc[QT_ACC_VIOLATIONS * n + ep] += viol;
  st.acc[QT_ACC_TERM * n + ep] = term;
  if (err_out) err_out[ep] = err;
  if (on_out) on_out[ep] = on;
  if (done_out) done_out[ep] = term != QT_TERM_RUNNING;
  if (term_out) term_out[ep] = (int8_t)term;
  if (viol_out) viol_out[ep] = viol;
}

// ------------------------------------------------------ controller alone

template <int KC>
__global__ __launch_bounds__(kBlock) void action_kernel(qt_ctrl_params c, BatchDev b, const double* __restrict__ obs,
                                                        double* integ, double* action, int8_t* sat_out,
                                                        double* diag) {
  const int64_t slot = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (slot >= b.n) return;
  const int64_t n = b.n, ep = episode_of(b, slot);
  Gains<KC, false> G;
  load_gains<KC, false>(b, ep, G);
  constexpr int NI = KC == 9 ? 3 : (KC == 3 ? 4 : 0);
  constexpr int ND = KC == 3 ? 18 : 16;
  double qp[3], qv[3], in[4] = {0, 0, 0, NAN}, u[4];
  Target tg;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    qp[i] = obs[i * n + ep];
    qv[i] = obs[(3 + i) * n + ep];
    tg.p[i] = obs[(6 + i) * n + ep];
    tg.v[i] = obs[(9 + i) * n + ep];
    tg.a[i] = obs[(12 + i) * n + ep];
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) in[i] = integ[i * n + ep];
  const double hover = b.hover ? b.hover[ep] : c.hover_thrust;
  double dg[ND];
  bool sat = false;
  if constexpr (KC == 3)
    compute_action_pid<true>(c, G.k, hover, qp, qv, tg, obs[15 * n + ep], in, u, dg);  // row 15: time
  else
    sat = compute_action<KC, true, false>(c, G, hover, qp, qv, tg, in, u, dg);
#pragma unroll
  for (int i = 0; i < 4; ++i) action[i * n + ep] = u[i];
  if (diag) {
#pragma unroll
    for (int i = 0; i < ND; ++i) diag[i * n + ep] = dg[i];
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) integ[i * n + ep] = in[i];
  if (sat_out) sat_out[ep] = sat;
}

// ---------------------------------------------------------------- target

__global__ __launch_bounds__(kBlock) void target_kernel(qt_env_params e, BatchDev b, const double* __restrict__ t,
                                                        double* out) {
  const int64_t slot = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (slot >= b.n) return;
  const int64_t n = b.n, ep = episode_of(b, slot);
  const int motion = motion_of(b, e, ep);
  const Pattern pt = pattern_of(b, e, motion, ep);
  Target tg;
  target_state<true>(e, motion, pt, t[ep], tg);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    out[i * n + ep] = tg.p[i];
    out[(3 + i) * n + ep] = tg.v[i];
    out[(6 + i) * n + ep] = tg.a[i];
  }
}

// ---------------------------------------------------------------- metrics

// compute_episode_metrics (utils/metrics.py:264-338) from the fused accumulators.
__global__ __launch_bounds__(kBlock) void metrics_kernel(qt_criteria cr, int64_t n, const double* __restrict__ acc,
                                                         const double* __restrict__ t, double* met) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  Acc a = load_acc(acc, n, e);
  double m[QT_MET_ROWS];
  if (a.steps == 0) {
#pragma unroll
    for (int i = 0; i < QT_MET_ROWS; ++i) m[i] = 0.0;
  } else {
    // an overshoot still open at the end counts if long enough (metrics.py:256-259)
    if (a.os_streak >= cr.overshoot_window) {
      a.os_count += 1;
      if (a.os_cur > a.os_max) a.os_max = a.os_cur;
    }
    if (a.steps < cr.overshoot_window) {  // metrics.py:225-226
      a.os_count = 0;
      a.os_max = 0.0;
    }
    const double ns = a.steps;
    const double ratio = a.on_pre / ns;
    m[QT_MET_DURATION] = t[e];
    m[QT_MET_ON_TARGET_RATIO] = ratio;
    m[QT_MET_MEAN_ERR] = a.sum_e / ns;
    m[QT_MET_MAX_ERR] = a.max_e;
    m[QT_MET_RMS_ERR] = sqrt(a.sum_e2 / ns);
    m[QT_MET_TOTAL_EFFORT] = a.sum_u;
    m[QT_MET_MEAN_EFFORT] = a.sum_u / ns;
    m[QT_MET_OS_COUNT] = a.os_count;
    m[QT_MET_OS_MAX] = a.os_max;
    m[QT_MET_SUCCESS] = (t[e] >= cr.min_episode_duration && ratio >= cr.min_on_target_ratio) ? 1.0 : 0.0;
    m[QT_MET_TERM] = a.term;
    m[QT_MET_VIOLATIONS] = a.viol;
    m[QT_MET_ENV_ON_TARGET_RATIO] = a.on_post / ns;
    m[QT_MET_STEPS] = ns;
  }
#pragma unroll
  for (int i = 0; i < QT_MET_ROWS; ++i) met[i * n + e] = m[i];
}

// compute_episode_metrics over recorded arrays (utils/metrics.py:144-338):
// one lane per episode streams its rows.
__global__ __launch_bounds__(kBlock) void metrics_arrays_kernel(qt_criteria cr, int64_t n, int32_t max_steps,
                                                                const double* __restrict__ qpos,
                                                                const double* __restrict__ tpos,
                                                                const double* __restrict__ act,
                                                                const int32_t* __restrict__ steps,
                                                                const double* __restrict__ last_time,
                                                                double* met) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  Acc a{0, 0, -INFINITY, 0, 0, 0, 0, 0, 0, -1, -1, 0, 0, 0};
  const int S = steps[e] < max_steps ? steps[e] : max_steps;
  const double R = cr.target_radius;
  for (int s = 0; s < S; ++s) {
    const int64_t b3 = (int64_t)s * 3 * n + e, b4 = (int64_t)s * 4 * n + e;
    const double d0 = tpos[b3] - qpos[b3], d1 = tpos[b3 + n] - qpos[b3 + n], d2 = tpos[b3 + 2 * n] - qpos[b3 + 2 * n];
    const double err = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    a.sum_e += err;
    a.sum_e2 += err * err;
    if (!(err <= a.max_e) && !(a.max_e != a.max_e)) a.max_e = err;
    const bool on = err <= R;
    a.on_pre += on;
    const double u0 = act[b4], u1 = act[b4 + n], u2 = act[b4 + 2 * n], u3 = act[b4 + 3 * n];
    a.sum_u += sqrt(u0 * u0 + u1 * u1 + u2 * u2 + u3 * u3);
    if (a.prev_on >= 0) {
      overshoot_step(a, on, err - R, cr.overshoot_window);
    }
    a.prev_on = on;
    a.steps += 1;
  }
  double m[QT_MET_ROWS];
#pragma unroll
  for (int i = 0; i < QT_MET_ROWS; ++i) m[i] = 0.0;
  if (S > 0) {
    if (a.os_streak >= cr.overshoot_window) {
      a.os_count += 1;
      if (a.os_cur > a.os_max) a.os_max = a.os_cur;
    }
    if (S < cr.overshoot_window) {
      a.os_count = 0;
      a.os_max = 0.0;
    }
    const double ns = S, ratio = a.on_pre / ns, dur = last_time[e];
    m[QT_MET_DURATION] = dur;
    m[QT_MET_ON_TARGET_RATIO] = ratio;
    m[QT_MET_MEAN_ERR] = a.sum_e / ns;
    m[QT_MET_MAX_ERR] = a.max_e;
    m[QT_MET_RMS_ERR] = sqrt(a.sum_e2 / ns);
    m[QT_MET_TOTAL_EFFORT] = a.sum_u;
    m[QT_MET_MEAN_EFFORT] = a.sum_u / ns;
    m[QT_MET_OS_COUNT] = a.os_count;
    m[QT_MET_OS_MAX] = a.os_max;
    m[QT_MET_SUCCESS] = (dur >= cr.min_episode_duration && ratio >= cr.min_on_target_ratio) ? 1.0 : 0.0;
    m[QT_MET_STEPS] = ns;
  }
#pragma unroll
  for (int i = 0; i < QT_MET_ROWS; ++i) met[i * n + e] = m[i];
}

// EvaluationSummary partials (utils/metrics.py:341-390): fixed summation
// order (bitwise reproducible for a given n), first-index argmax/argmin.
// Partial vector: [7 sums, max, argmax, min, argmin]; an argmax/argmin < 0
// marks an empty partial.
constexpr int kSumBlock = 256;
constexpr int kSumParts = 11;

struct SumPart {
  double s[7];
  double vmax, vmin;
  int64_t imax, imin;
};

__device__ __forceinline__ void sum_empty(SumPart& p) {
#pragma unroll
  for (int k = 0; k < 7; ++k) p.s[k] = 0.0;
  p.vmax = -INFINITY, p.vmin = INFINITY, p.imax = -1, p.imin = -1;
}

// episodes [lo, hi) of met, strided over the block's threads
__device__ __forceinline__ void sum_accumulate(SumPart& p, int64_t n, const double* __restrict__ met, double mu_r,
                                               double mu_e, int64_t lo, int64_t hi) {
  for (int64_t e = lo + threadIdx.x; e < hi; e += kSumBlock) {
    const double r = met[QT_MET_ON_TARGET_RATIO * n + e], er = met[QT_MET_MEAN_ERR * n + e];
    p.s[0] += r;
    p.s[1] += er;
    p.s[2] += met[QT_MET_MEAN_EFFORT * n + e];
    p.s[3] += met[QT_MET_SUCCESS * n + e];
    p.s[4] += 1.0;
    p.s[5] += (r - mu_r) * (r - mu_r);
    p.s[6] += (er - mu_e) * (er - mu_e);
    if (r > p.vmax || p.imax < 0) p.vmax = r, p.imax = e;
    if (r < p.vmin || p.imin < 0) p.vmin = r, p.imin = e;
  }
}

// tree-combine every thread's partial (fixed pairing); thread 0 writes out[11]
__device__ void sum_block_reduce(const SumPart& p, double* out) {
  __shared__ double sh[7][kSumBlock];
  __shared__ double shx[2][kSumBlock];
  __shared__ int64_t shi[2][kSumBlock];
#pragma unroll
  for (int k = 0; k < 7; ++k) sh[k][threadIdx.x] = p.s[k];
  shx[0][threadIdx.x] = p.vmax;
  shx[1][threadIdx.x] = p.vmin;
  shi[0][threadIdx.x] = p.imax;
  shi[1][threadIdx.x] = p.imin;
  __syncthreads();
  for (int w = kSumBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const int o = threadIdx.x + w;
#pragma unroll
      for (int k = 0; k < 7; ++k) sh[k][threadIdx.x] += sh[k][o];
      // keep the lowest index among equal values (np.argmax/argmin first occurrence)
      const int64_t ia = shi[0][threadIdx.x], ib = shi[0][o];
      if (ib >= 0 && (ia < 0 || shx[0][o] > shx[0][threadIdx.x] ||
                      (shx[0][o] == shx[0][threadIdx.x] && ib < ia)))
        shx[0][threadIdx.x] = shx[0][o], shi[0][threadIdx.x] = ib;
      const int64_t ja = shi[1][threadIdx.x], jb = shi[1][o];
      if (jb >= 0 && (ja < 0 || shx[1][o] < shx[1][threadIdx.x] ||
                      (shx[1][o] == shx[1][threadIdx.x] && jb < ja)))
        shx[1][threadIdx.x] = shx[1][o], shi[1][threadIdx.x] = jb;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 7; ++k) out[k] = sh[k][0];
    out[7] = shx[0][0];
    out[8] = (double)shi[0][0];
    out[9] = shx[1][0];
    out[10] = (double)shi[1][0];
  }
}

// one workgroup over all episodes
__global__ __launch_bounds__(kSumBlock) void summary_kernel(int64_t n, const double* __restrict__ met, double mu_r,
                                                            double mu_e, double* out) {
  SumPart p;
  sum_empty(p);
  sum_accumulate(p, n, met, mu_r, mu_e, 0, n);
  sum_block_reduce(p, out);
}

// stage 1 of the multi-workgroup form: workgroup b reduces episodes
// [b * chunk, (b + 1) * chunk) into part[b][11]
__global__ __launch_bounds__(kSumBlock) void summary_part_kernel(int64_t n, const double* __restrict__ met,
                                                                 double mu_r, double mu_e, int64_t chunk,
                                                                 double* part) {
  SumPart p;
  sum_empty(p);
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  sum_accumulate(p, n, met, mu_r, mu_e, lo, lo + chunk < n ? lo + chunk : n);
  sum_block_reduce(p, part + (int64_t)blockIdx.x * kSumParts);
}

// stage 2: one workgroup combines the nparts partials in a fixed order
__global__ __launch_bounds__(kSumBlock) void summary_final_kernel(int nparts, const double* __restrict__ part,
                                                                  double* out) {
  SumPart p;
  sum_empty(p);
  for (int j = threadIdx.x; j < nparts; j += kSumBlock) {
    const double* q = part + (int64_t)j * kSumParts;
#pragma unroll
    for (int k = 0; k < 7; ++k) p.s[k] += q[k];
    const int64_t ia = (int64_t)q[8], ja = (int64_t)q[10];
    if (ia >= 0 && (p.imax < 0 || q[7] > p.vmax || (q[7] == p.vmax && ia < p.imax))) p.vmax = q[7], p.imax = ia;
    if (ja >= 0 && (p.imin < 0 || q[9] < p.vmin || (q[9] == p.vmin && ja < p.imin))) p.vmin = q[9], p.imin = ja;
  }
  sum_block_reduce(p, out);
}

BatchDev to_dev(const qt_batch* b) {
  return BatchDev{b->n,     b->motion,        b->pattern, b->plant_mass, b->hover_thrust, b->K,
                  b->k_cols, b->k_per_episode, b->order,   0,             b->n};
}

int grid_of(int64_t n) { return (int)((n + kBlock - 1) / kBlock); }

int check_launch() { return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH; }

template <int MOTION, int KC, bool FF, bool KS>
void launch_flavours(bool fast, bool no_yaw, int grid, hipStream_t s, const qt_env_params& e, const qt_ctrl_params& c,
                     const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps, double* rec) {
  const RateLin rl = make_rate_lin(e);  // yaw-at-rest closed-form RK4 (integrate_yaw0)
  if (fast && (KS || no_yaw) && rate_bounded_ok(e, c)) {
    rollout_kernel<kYaw0, MOTION, KC, FF, KS><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, rec, kExact, rl);
    rollout_kernel<kExact, MOTION, KC, FF, KS><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, rec, kYaw0, rl);
  } else if (fast) {
    rollout_kernel<kFast, MOTION, KC, FF, KS><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, rec, kExact, rl);
    rollout_kernel<kExact, MOTION, KC, FF, KS><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, rec, kFast, rl);
  } else {
    rollout_kernel<kExact, MOTION, KC, FF, KS><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, rec, kExact, rl);
  }
}

template <int KC, bool FF, bool KS>
void launch_rollout_motion(int motion, bool fast, bool no_yaw, int grid, hipStream_t s, const qt_env_params& e,
                           const qt_ctrl_params& c, const qt_criteria& cr, const BatchDev& b, const qt_state& st,
                           int nsteps, double* rec) {
  switch (motion) {
    case QT_MOTION_STATIONARY:
      launch_flavours<QT_MOTION_STATIONARY, KC, FF, KS>(fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
      break;
    case QT_MOTION_LINEAR:
      launch_flavours<QT_MOTION_LINEAR, KC, FF, KS>(fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
      break;
    case QT_MOTION_CIRCULAR:
      launch_flavours<QT_MOTION_CIRCULAR, KC, FF, KS>(fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
      break;
    case QT_MOTION_SINUSOIDAL:
      launch_flavours<QT_MOTION_SINUSOIDAL, KC, FF, KS>(fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
      break;
    case QT_MOTION_FIGURE8:
      launch_flavours<QT_MOTION_FIGURE8, KC, FF, KS>(fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
      break;
    default:
      launch_flavours<-1, KC, FF, KS>(fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
  }
}

template <int KC>
void launch_rollout(bool ff, bool ks, bool no_yaw, int motion, int grid, hipStream_t s, const qt_env_params& e,
                    const qt_ctrl_params& c, const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps,
                    double* rec) {
  const bool fast = QT_ABLATE == 0 && rec == nullptr && fast_path_ok(e, c);
  if constexpr (KC == 3) {  // PID never commands yaw (controllers/__init__.py:373): the yaw-at-rest flavour applies
    if (ff)
      launch_rollout_motion<3, true, true>(motion, fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
    else
      launch_rollout_motion<3, false, true>(motion, fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
  } else if (ff) {
    if (ks)
      launch_rollout_motion<KC, true, true>(motion, fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
    else
      launch_rollout_motion<KC, true, false>(motion, fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
  } else {
    if (ks)
      launch_rollout_motion<KC, false, true>(motion, fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
    else
      launch_rollout_motion<KC, false, false>(motion, fast, no_yaw, grid, s, e, c, cr, b, st, nsteps, rec);
  }
}

bool valid_state(const qt_state& st, bool need_integ) {
  return st.x && st.t && st.acc && st.target && (!need_integ || st.integ);
}

}  // namespace

extern "C" {

int qt_abi_version(void) { return QT_ABI_VERSION; }

#if QT_CLOCK_STAMP
// Diagnostic build only: copy the first `waves` stamp records
// {memtime start, end, realtime start, end} to host memory out[waves][4].
int qt_debug_stamps(unsigned long long* out, int64_t waves) {
  if (!out || waves < 0 || waves > kStampWaves) return QT_EINVAL;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qt_stamps), sizeof(unsigned long long) * 4 * waves) == hipSuccess
             ? QT_OK
             : QT_ELAUNCH;
}
#endif

int qt_reset(const qt_env_params* env, const qt_batch* batch, const double* offset, qt_state st, void* stream) {
  if (!env || !batch || batch->n < 0) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;  // empty: no per-episode pointer is read
  if (!offset || !valid_state(st, false)) return QT_EINVAL;
  reset_kernel<<<grid_of(batch->n), kBlock, 0, (hipStream_t)stream>>>(*env, to_dev(batch), offset, st);
  return check_launch();
}

int qt_rollout(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_criteria* crit, const qt_batch* batch,
               qt_state st, int32_t nsteps, double* rec, void* stream) {
  if (!env || !ctrl || !crit || !batch || batch->n < 0 || nsteps < 0 || !batch->K) return QT_EINVAL;
  if (batch->k_cols != 3 && batch->k_cols != 6 && batch->k_cols != 9) return QT_EINVAL;
  if (batch->n == 0 || nsteps == 0) return QT_OK;  // nothing to run: no per-episode pointer is read
  if (!valid_state(st, batch->k_cols != 6)) return QT_EINVAL;
  const BatchDev b = to_dev(batch);
  const int grid = grid_of(batch->n);
  const int motion = batch->motion ? -1 : env->motion;
  hipStream_t s = (hipStream_t)stream;
  const bool ff = ctrl->feedforward_enabled != 0;
  const bool ks = batch->k_structured != 0;
  const bool no_yaw = batch->k_no_yaw != 0;  // yaw-rate gains all zero: yaw stays at rest (dense K too)
  if (batch->k_cols == 9)
    launch_rollout<9>(ff, ks, no_yaw, motion, grid, s, *env, *ctrl, *crit, b, st, nsteps, rec);
  else if (batch->k_cols == 3)
    launch_rollout<3>(ff, ks, no_yaw, motion, grid, s, *env, *ctrl, *crit, b, st, nsteps, rec);
  else
    launch_rollout<6>(ff, ks, no_yaw, motion, grid, s, *env, *ctrl, *crit, b, st, nsteps, rec);
  return check_launch();
}

int qt_rollout_grouped(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_criteria* crit,
                       const qt_batch* batch, qt_state st, int32_t nsteps, double* rec, int32_t nseg,
                       const int32_t* seg_motion, const int64_t* seg_end, void* stream) {
  if (!env || !ctrl || !crit || !batch || batch->n < 0 || nsteps < 0 || !batch->K) return QT_EINVAL;
  if (batch->k_cols != 3 && batch->k_cols != 6 && batch->k_cols != 9) return QT_EINVAL;
  if (batch->n > 0 && nsteps > 0 && !valid_state(st, batch->k_cols != 6)) return QT_EINVAL;
  if (nseg < 0 || (nseg > 0 && (!seg_motion || !seg_end))) return QT_EINVAL;
  int64_t prev = 0;
  for (int32_t i = 0; i < nseg; ++i) {
    if (seg_end[i] < prev || seg_end[i] > batch->n || seg_motion[i] < 0 || seg_motion[i] > 4) return QT_EINVAL;
    prev = seg_end[i];
  }
  if (prev != batch->n) return QT_EINVAL;
  if (batch->n == 0 || nsteps == 0) return QT_OK;
  BatchDev b = to_dev(batch);
  hipStream_t s = (hipStream_t)stream;
  const bool ff = ctrl->feedforward_enabled != 0;
  const bool ks = batch->k_structured != 0;
  const bool no_yaw = batch->k_no_yaw != 0;  // yaw-rate gains all zero: yaw stays at rest (dense K too)
  for (int32_t i = 0; i < nseg; ++i) {
    b.slot0 = i ? seg_end[i - 1] : 0;
    b.slot_end = seg_end[i];
    if (b.slot_end == b.slot0) continue;
    const int grid = grid_of(b.slot_end - b.slot0);
    if (batch->k_cols == 9)
      launch_rollout<9>(ff, ks, no_yaw, seg_motion[i], grid, s, *env, *ctrl, *crit, b, st, nsteps, rec);
    else if (batch->k_cols == 3)
      launch_rollout<3>(ff, ks, no_yaw, seg_motion[i], grid, s, *env, *ctrl, *crit, b, st, nsteps, rec);
    else
      launch_rollout<6>(ff, ks, no_yaw, seg_motion[i], grid, s, *env, *ctrl, *crit, b, st, nsteps, rec);
    if (hipGetLastError() != hipSuccess) return QT_ELAUNCH;
  }
  return QT_OK;
}

int qt_env_step(const qt_env_params* env, const qt_batch* batch, const double* action, qt_state st, double* err,
                int8_t* on_target, int8_t* done, int8_t* term, int8_t* violation, void* stream) {
  if (!env || !batch || batch->n < 0) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;
  if (!action || !valid_state(st, false)) return QT_EINVAL;
  env_step_kernel<<<grid_of(batch->n), kBlock, 0, (hipStream_t)stream>>>(*env, to_dev(batch), action, st, err,
                                                                         on_target, done, term, violation);
  return check_launch();
}

int qt_compute_action(const qt_ctrl_params* ctrl, const qt_batch* batch, const double* obs, double* integ,
                      double* action, int8_t* saturated, double* diag, void* stream) {
  if (!ctrl || !batch || !batch->K || batch->n < 0) return QT_EINVAL;
  if (batch->k_cols != 3 && batch->k_cols != 6 && batch->k_cols != 9) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;
  if (!obs || !action || (batch->k_cols != 6 && !integ)) return QT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (batch->k_cols == 9)
    action_kernel<9><<<grid_of(batch->n), kBlock, 0, s>>>(*ctrl, to_dev(batch), obs, integ, action, saturated, diag);
  else if (batch->k_cols == 3)
    action_kernel<3><<<grid_of(batch->n), kBlock, 0, s>>>(*ctrl, to_dev(batch), obs, integ, action, saturated, diag);
  else
    action_kernel<6><<<grid_of(batch->n), kBlock, 0, s>>>(*ctrl, to_dev(batch), obs, integ, action, saturated, diag);
  return check_launch();
}

int qt_target_state(const qt_env_params* env, const qt_batch* batch, const double* t, double* out, void* stream) {
  if (!env || !batch || batch->n < 0) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;
  if (!t || !out) return QT_EINVAL;
  target_kernel<<<grid_of(batch->n), kBlock, 0, (hipStream_t)stream>>>(*env, to_dev(batch), t, out);
  return check_launch();
}

int qt_episode_metrics(const qt_criteria* crit, int64_t n, const double* acc, const double* t, double* met,
                       void* stream) {
  if (!crit || n < 0) return QT_EINVAL;
  if (n == 0) return QT_OK;
  if (!acc || !t || !met) return QT_EINVAL;
  metrics_kernel<<<grid_of(n), kBlock, 0, (hipStream_t)stream>>>(*crit, n, acc, t, met);
  return check_launch();
}

int qt_metrics_from_arrays(const qt_criteria* crit, int64_t n, int32_t max_steps, const double* qpos,
                           const double* tpos, const double* actions, const int32_t* steps,
                           const double* last_time, double* met, void* stream) {
  if (!crit || n < 0 || max_steps < 0) return QT_EINVAL;
  if (n == 0) return QT_OK;
  if (!steps || !last_time || !met || (max_steps > 0 && (!qpos || !tpos || !actions))) return QT_EINVAL;
  metrics_arrays_kernel<<<grid_of(n), kBlock, 0, (hipStream_t)stream>>>(*crit, n, max_steps, qpos, tpos, actions,
                                                                        steps, last_time, met);
  return check_launch();
}

int qt_summary(int64_t n, const double* met, double mu_ratio, double mu_err, double* out, void* stream) {
  if (!out || n < 0 || (n > 0 && !met)) return QT_EINVAL;  // n == 0: writes the empty partial
  summary_kernel<<<1, kSumBlock, 0, (hipStream_t)stream>>>(n, met, mu_ratio, mu_err, out);
  return check_launch();
}

int qt_summary_parts(int64_t n, const double* met, double mu_ratio, double mu_err, double* out, double* work,
                     int32_t nparts, void* stream) {
  if (!out || !work || n < 0 || (n > 0 && !met) || nparts < 1 || nparts > 4096) return QT_EINVAL;
  const int64_t chunk = (n + nparts - 1) / nparts > 0 ? (n + nparts - 1) / nparts : 1;
  hipStream_t s = (hipStream_t)stream;
  summary_part_kernel<<<nparts, kSumBlock, 0, s>>>(n, met, mu_ratio, mu_err, chunk, work);
  summary_final_kernel<<<1, kSumBlock, 0, s>>>(nparts, work, out);
  return check_launch();
}

}  // extern "C"
