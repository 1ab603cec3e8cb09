// qt_kernels.hpp — the fused closed-loop rollout kernel and the per-episode
// containers shared by qt_rollout.hip (exact step, other kernels, C ABI) and
// qt_rollout_fast.hip (the fast step flavours, built with relaxed NaN
// handling: their state is finite by construction, see rollout_kernel).
//
// One lane = one episode.  A launch walks `nsteps` closed-loop steps with the
// whole episode (12-state plant, target pattern constants, 4x6 / 4x9 gains,
// LQI integral, metric accumulators) resident in registers; HBM is touched
// only to load the state at the start of a chunk and to store it at the end.
// Reference functions: src/quadcopter_tracking/... of the reference repo.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "qt_device.hpp"


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

namespace qtk {

using namespace qt;

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
  const double* ff;         // [7][n] per-episode feed-forward (qt_batch.ff) or NULL
  int64_t slot0, slot_end;  // the slot range this launch covers (grouped launches)
  // Wave-aligned motion groups (one-launch grouped rollout): group i covers
  // slots [seg_end[i-1], seg_end[i]) of motion seg_motion[i] and starts a new
  // wavefront (waves [wave_end[i-1], wave_end[i])), so every wave holds one
  // motion type.  nseg = 0: slots follow launch positions (slot0 + p).
  int32_t nseg;
  int8_t seg_motion[8];
  int64_t seg_end[8], wave_end[8];
  // Stationary riders (one-launch grouped rollout, rollout_batch): the free
  // lanes of a group's last wave take episodes of the stationary group, whose
  // target (a fixed point) the group's loop forms by a per-lane select
  // (ride_target).  Group i's waves run its own slots [seg_lo[i], seg_end[i])
  // and then the riders [ride_lo[i], ride_lo[i] + ride_cnt[i]); the riders come
  // from the front of the stationary group's slot range, whose own waves start
  // after them (its seg_lo).  Slot ranges, and so slot_motion, are unchanged.
  int64_t seg_lo[8], ride_lo[8], ride_cnt[8];
  // A per-segment launch of a grouped batch (qt_rollout_grouped's one launch
  // set per group): the group's motion, which its slots' batch->motion must
  // match (-1: none to check).  A wave holding a slot that does not is left to
  // the exact pass, which then runs with each episode's own motion.
  int32_t seg_check;
};

// The slot a launch position runs, or -1 past the launch's slot range (or in
// the unused tail of a group's last wave); `ride`: the slot is a stationary
// rider in another group's wave (BatchDev::ride_lo).
__device__ __forceinline__ int64_t slot_at(const BatchDev& b, int64_t p, bool& ride) {
  ride = false;
  if (b.nseg == 0) {
    const int64_t slot = b.slot0 + p;
    return slot < b.slot_end ? slot : -1;
  }
  const int64_t w = p >> 6;
  int64_t w0 = 0;
  for (int i = 0; i < b.nseg; ++i) {  // uniform per wave
    if (w < b.wave_end[i]) {
      int64_t q = ((w - w0) << 6) + (p & 63);
      const int64_t own = b.seg_end[i] - b.seg_lo[i];
      if (q < own) return b.seg_lo[i] + q;
      q -= own;
      ride = q < b.ride_cnt[i];
      return ride ? b.ride_lo[i] + q : -1;
    }
    w0 = b.wave_end[i];
  }
  return -1;
}

__device__ __forceinline__ int64_t slot_at(const BatchDev& b, int64_t p) {
  bool ride;
  return slot_at(b, p, ride);
}

// The motion of a wave-aligned group's wave (b.nseg > 0), uniform per wave.
__device__ __forceinline__ int wave_motion(const BatchDev& b, int64_t p) {
  const int64_t w = p >> 6;
  for (int i = 0; i < b.nseg; ++i)
    if (w < b.wave_end[i]) return b.seg_motion[i];
  return -1;
}

// The motion of the wave-aligned group holding `slot` (b.nseg > 0).
__device__ __forceinline__ int slot_motion(const BatchDev& b, int64_t slot) {
  for (int i = 0; i < b.nseg; ++i)
    if (slot < b.seg_end[i]) return b.seg_motion[i];
  return -1;
}

// The lane's feed-forward parameters: per episode (qt_batch.ff rows: velocity
// gain xyz, acceleration gain xyz, velocity clamp) or the controller's.
__device__ __forceinline__ FFLane ff_of(const BatchDev& b, const qt_ctrl_params& c, int64_t ep) {
  if (!b.ff) return ff_uniform(c);
  const int64_t n = b.n;
  return FFLane{{b.ff[0 * n + ep], b.ff[1 * n + ep], b.ff[2 * n + ep]},
                {b.ff[3 * n + ep], b.ff[4 * n + ep], b.ff[5 * n + ep]},
                b.ff[6 * n + ep]};
}

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

// UNI: the launch shares one gain matrix (k_per_episode == 0, checked on the
// host): uniform addresses, scalar loads, gains in SGPRs.
template <int KC, bool KS, bool UNI = false>
__device__ __forceinline__ void load_gains(const BatchDev& b, int64_t ep, Gains<KC, KS>& G) {
  const int64_t m = UNI ? 1 : (b.k_per_episode ? b.n : 1);
  const int64_t col = UNI ? 0 : (b.k_per_episode ? ep : 0);
#pragma unroll
  for (int j = 0; j < Gains<KC, KS>::kCount; ++j) {
    const int idx = (KS && KC != 3) ? structured_index<KC>(j) : j;
    G.k[j] = b.K[(int64_t)idx * m + col];
  }
}

// compute_episode_metrics (utils/metrics.py:264-338) of one episode from its
// accumulators and env time (the Evaluator's record, eval.py:142-159) into
// met[QT_MET_ROWS][n] column e: metrics_kernel, and the rollout epilogue of a
// fresh pass (qt_rollout_fresh).
__device__ __forceinline__ void store_metrics(const qt_criteria& cr, Acc a, double t, double* met, int64_t n,
                                              int64_t e) {
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
    m[QT_MET_DURATION] = t;
    m[QT_MET_ON_TARGET_RATIO] = ratio;
    m[QT_MET_MEAN_ERR] = a.sum_e / ns;
    m[QT_MET_MAX_ERR] = a.max_e;
    m[QT_MET_RMS_ERR] = sqrt(a.sum_e2 / ns);
    m[QT_MET_TOTAL_EFFORT] = a.sum_u;
    m[QT_MET_MEAN_EFFORT] = a.sum_u / ns;
    m[QT_MET_OS_COUNT] = a.os_count;
    m[QT_MET_OS_MAX] = a.os_max;
    m[QT_MET_SUCCESS] = (t >= cr.min_episode_duration && ratio >= cr.min_on_target_ratio) ? 1.0 : 0.0;
    m[QT_MET_TERM] = a.term;
    m[QT_MET_VIOLATIONS] = a.viol;
    m[QT_MET_ENV_ON_TARGET_RATIO] = a.on_post / ns;
    m[QT_MET_STEPS] = ns;
  }
#pragma unroll
  for (int i = 0; i < QT_MET_ROWS; ++i) met[i * n + e] = m[i];
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

// ---------------------------------------------------------------- rollout

// Sum of squares in the reference's order, ((a^2 + b^2) + c^2) without FMA
// contraction (np.linalg.norm / the oracle's norm3): with sqrt_pos's
// correctly rounded root, the fast loop's tracking error equals the exact
// step's bit for bit on the same state, so its on-target and LQI-gate
// decisions need no knife-edge band.
__device__ __forceinline__ double sq3_ref(double a, double b, double c) {
#pragma clang fp contract(off)
  return (a * a + b * b) + c * c;
}

// A loop-invariant uniform value held in a VGPR pair (every lane a copy).
// The inline asm's VGPR result is divergent to the compiler, so the value
// takes no SGPR and is never rematerialised: for a loop whose uniform values
// overflow the wave's 102 SGPRs, which the compiler otherwise spills to VGPR
// lanes and reads back with v_readlane in every step (the exact step).
__device__ __forceinline__ double vpin(double x) {
  double r;
  asm("v_mov_b64 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// QT_EXACT_VPIN bits: 1 the env / controller / plant uniforms, 2 the
// closed-form rate and velocity maps, 4 the Taylor coefficients (SmallCoef),
// 8 the gains
#ifndef QT_EXACT_VPIN
#define QT_EXACT_VPIN 5
#endif
// the same for the full-gain fast step (kFast's run_steps<true>)
#ifndef QT_FAST_VPIN
#define QT_FAST_VPIN 0
#endif

// The closed-loop steps of one lane.  FAST: the branch-light step of
// qt_device.hpp (fast_path_ok + finite lane inputs, no recording), which
// takes the exact step's decisions; rare lanes/steps (speed at the
// clamp, attitude far outside [-pi, pi), tracking error at the radius within
// 1e-14) fall back to the exact constraint / comparison code inside the step.
template <bool FAST, int MOTION, int KC, bool FF, bool KS, int INTEG = -1, bool PIN = true>
__device__ __forceinline__ void run_steps(const qt_env_params& e0, const qt_ctrl_params& c0, const qt_criteria& cr,
                                          int motion, const Pattern& pt, const Plant& pl0, double hover,
                                          const Gains<KC, KS>& G0, const FFLane& fl, double* x, double* integ,
                                          Target& tg, double& t, Acc& a, int nsteps, double* __restrict__ rec,
                                          int64_t n, int64_t ep, double* __restrict__ reward = nullptr) {
  // The exact step holds its loop-invariant uniforms (env limits and centre,
  // controller clamps, plant; QT_EXACT_VPIN) and its Taylor coefficients in
  // VGPRs (vpin, SmallCoef::pin) instead of spilled SGPRs.  PIN (the exact
  // kernel's launch choice, ExactLaunch) turns that off for batches of more
  // than one wave per SIMD, where a second resident wave (unpinned: <= 256
  // VGPRs) hides the FP64 latency that pinning's fewer instructions cannot.
  constexpr int kPinBits = FAST ? QT_FAST_VPIN : (PIN ? QT_EXACT_VPIN : 0);
  constexpr bool kPin = kPinBits & 1;
  constexpr bool kPinLin = kPinBits & 2;
  constexpr bool kPinTaylor = kPinBits & 4;
  qt_env_params e = e0;
  qt_ctrl_params c = c0;
  Plant pl = pl0;
  Gains<KC, KS> G = G0;
  if (kPin) {
    e.min_thrust = vpin(e.min_thrust), e.max_thrust = vpin(e.max_thrust);
    e.max_angular_rate = vpin(e.max_angular_rate), e.dt = vpin(e.dt);
    e.max_episode_time = vpin(e.max_episode_time), e.max_velocity = vpin(e.max_velocity);
    e.max_angular_velocity = vpin(e.max_angular_velocity), e.max_position = vpin(e.max_position);
    e.target_radius = vpin(e.target_radius);
    for (int i = 0; i < 3; ++i) e.center[i] = vpin(e.center[i]);
    c.min_thrust = vpin(c.min_thrust), c.max_thrust = vpin(c.max_thrust), c.max_rate = vpin(c.max_rate);
    pl.inv_mass = vpin(pl.inv_mass), pl.gz = vpin(pl.gz);
  }
  if (kPinBits & 8) {
    for (int j = 0; j < Gains<KC, KS>::kCount; ++j) G.k[j] = vpin(G.k[j]);
  }
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
  // exact step: the pre-step tracking error, carried from the previous step's
  // post-step error (positions are not constrained, so they are the same
  // number), ||p - p_T|| in np.linalg.norm(axis=1)'s order (sq3_ref)
  double err_pre = 0.0;
  // (sqrt, not sqrt_noscale: a caller's state may hold an infinite position
  // still marked running, whose error numpy's norm gives as inf; once per launch)
  if (!FAST) err_pre = sqrt(sq3_ref(tg.p[0] - x[0], tg.p[1] - x[1], tg.p[2] - x[2]));
  // fast steps of a periodic pattern carry its angles' sin / cos (target_state_carried)
  constexpr bool kCarry = FAST && (MOTION == QT_MOTION_SINUSOIDAL || MOTION == QT_MOTION_CIRCULAR);
  PeriodicTrig<kCarry ? MOTION : QT_MOTION_CIRCULAR> ptrig;
  if constexpr (kCarry) periodic_trig_init(pt, t, ptrig);
  // env.step's reward = -(post-step tracking error) (quadcopter_env.py:198-199,
  // 498-511), summed in step order as the trainer does (train.py:627), and the
  // last step's tracking error (info["tracking_error"], train.py:630)
  double rew_sum = 0.0, rew_last = 0.0;
  if (!FAST && reward) rew_sum = reward[ep], rew_last = reward[n + ep];
  // closed-form RK4 / Euler (integrate_closed) with sin / cos of the attitude
  // carried across steps (carry_attitude_trig): the exact step, and the
  // full-gain fast step (kFast, whose launch knows the integrator is RK4)
  Trig ta;
  trig_of(x + 6, ta);
  RateLin rl = make_rate_lin(e);
  VelLin vl = make_vel_lin(e, pl);
  if (kPinLin) {
    rl.wy = vpin(rl.wy), rl.wu = vpin(rl.wu), rl.ay = vpin(rl.ay), rl.au = vpin(rl.au), rl.h2 = vpin(rl.h2);
    rl.d3y = vpin(rl.d3y), rl.d3u = vpin(rl.d3u), rl.d4y = vpin(rl.d4y), rl.d4u = vpin(rl.d4u);
    rl.e3y = vpin(rl.e3y);
    vl.cv = vpin(vl.cv), vl.pv = vpin(vl.pv), vl.gv = vpin(vl.gv), vl.gp = vpin(vl.gp);
    for (int i = 0; i < 4; ++i) vl.wv[i] = vpin(vl.wv[i]);
    for (int i = 0; i < 3; ++i) vl.pa[i] = vpin(vl.pa[i]);
  }
  SmallCoef sk;  // the stage / carry Taylor coefficients (pinned in VGPRs in the exact step)
  if (kPinTaylor) sk.pin();
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
        compute_action_pid<FF, FAST>(c, G.k, hover, x, x + 3, tg, t, fl, integ, u);  // observation time = t
      else
        compute_action<KC, FF, KS, FAST>(c, G, hover, x, x + 3, tg, fl, integ, u, nullptr, err_fast);
    }
    // ---- the Evaluator's pre-step record (eval.py:142-159) -> metrics accumulators
    if (!(QT_ABLATE & QT_ABL_METRICS)) {
      double err, un;
      if (FAST) {
        err = err_fast;
        un = sqrt_noscale(u[0] * u[0] + u[1] * u[1] + u[2] * u[2] + u[3] * u[3]);
      } else {
        // sqrt_noscale: correctly rounded (x >= 2^-767), NaN kept; the command is
        // finite or NaN (clipped), an infinite position has terminated the episode
        err = err_pre;
        un = sqrt_noscale(u[0] * u[0] + u[1] * u[1] + u[2] * u[2] + u[3] * u[3]);
      }
      a.sum_e += err;
      a.sum_e2 += err * err;
      if (FAST)  // err and max_e are numbers here (finite state): a plain max
        a.max_e = fmax(a.max_e, err);
      else  // np.max, NaN-propagating
        a.max_e = (!(err <= a.max_e) && !(a.max_e != a.max_e)) ? err : a.max_e;
      const bool on = err <= R;
      a.on_pre += on;
      a.sum_u += un;
      overshoot_step(a, on, err - R, cr.overshoot_window);  // no-op on the first step (prev_on < 0)
      a.prev_on = on;
    }
    // ---- env.step (quadcopter_env.py:152-232)
    if (FAST) {
      // the command is finite and inside the env clamps: parsing is the identity
      double a0[3] = {x[6], x[7], x[8]}, d4[3];
      Trig t4;
      integrate_closed<0>(e, rl, vl, pl, ta, x, u, d4, t4, sk);
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
      const bool ok = ((se < er2lo) | (se > er2hi)) & ((QT_ABLATE & QT_ABL_CONSTRAIN) || constrain_fast_ok<false>(e, x));
      // Wave-uniform choice: when any lane is off the fast preconditions the
      // whole wave runs the exact code, which takes the fast code's decisions
      // on the lanes that qualify.  A uniform, expected condition is a
      // not-taken scalar branch with the exact code out of line; a divergent
      // if / else cost a taken branch around the else block every step.
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) == 0, 1)) {
        if (!(QT_ABLATE & QT_ABL_CONSTRAIN)) constrain_fast_apply<false>(e, x);
        a.on_post += se < er2lo;
      } else {  // rare: exact constraints and comparison
        if (!(QT_ABLATE & QT_ABL_CONSTRAIN)) constrain<false>(e, x);
        a.on_post += norm_le(se, e.target_radius);
      }
      carry_attitude_trig(a0, x + 6, d4, t4, ta, sk);
      if (QT_ABLATE & QT_ABL_TERMINATION)
        a.term = t >= e.max_episode_time ? QT_TERM_TIME_LIMIT : QT_TERM_RUNNING;
      else
        a.term = termination_fast(e, t, x);
      a.steps += 1;
    } else {
      double ua[4], a0[3] = {x[6], x[7], x[8]}, d4[3];
      a.viol += parse_action(e, u, ua);
      Trig t4;
      integrate_closed<INTEG>(e, rl, vl, pl, ta, x, ua, d4, t4, sk);
      t += e.dt;
      const int term = constrain_terminate<false>(e, x, t);
      carry_attitude_trig(a0, x + 6, d4, t4, ta, sk);
      if (!(QT_ABLATE & QT_ABL_TARGET)) target_state<FF>(e, motion, pt, t, tg);
      const double q0 = x[0] - tg.p[0], q1 = x[1] - tg.p[1], q2 = x[2] - tg.p[2];
      err_pre = sqrt_noscale(sq3_ref(q0, q1, q2));  // this step's post-step error, the next one's pre-step
      a.on_post += err_pre <= e.target_radius;
      if (reward) {
        const double pe = sqrt(dot3_blas(q0, q1, q2));  // float(np.linalg.norm(quad_pos - target_pos))
        rew_sum += -pe;
        rew_last = pe;
      }
      a.term = term;
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
  if (!FAST && reward) reward[ep] = rew_sum, reward[n + ep] = rew_last;
}

// Finiteness by the exponent bits: the same answer under IEEE and under the
// fast translation unit's relaxed NaN handling (which may fold a floating
// point isfinite or x != x), so the fast and the exact kernel take the same
// wave decision.
__device__ __forceinline__ bool finite_bits(double v) {
  return (__double_as_longlong(v) & 0x7ff0000000000000LL) != 0x7ff0000000000000LL;
}

__device__ __forceinline__ bool all_finite(const double* v, int k) {
  bool ok = true;
  for (int i = 0; i < k; ++i) ok = ok & finite_bits(v[i]);
  return ok;
}

// step flavours: the exact step, the fast step, the fast step with yaw at rest
constexpr int kExact = 0, kFast = 1, kYaw0 = 2;

// ------------------------------------------------- yaw-at-rest fast loop


// Carried sin / cos of a periodic target's angles (circular: 1, sinusoidal:
// 3, figure-8: theta = omega t).  Each step rotates them by the launch's
// fixed rotor (cos, sin)(fl(omega dt)) and then to first order by
// omega ((t_new - t) - dt), the rounding of the env's time step (t += dt,
// quadcopter_env.py:191; exact by Sterbenz, <= ulp(t)): 7 operations per
// angle where a sin / cos costs ~30.  They so follow sin / cos of
// omega t_k + phase for the accumulated t_k, which the reference evaluates
// rounded (target_motion.py:86, 144, 179), up to the rotor's own rounding
// (k (omega dt - fl(omega dt)) < 1e-14 rad over 3,000 steps) and a few ulp
// of drift.
template <int MOTION>
struct Rotor {
  static constexpr int NA = MOTION == QT_MOTION_SINUSOIDAL ? 3 : 1;
  double s[3], c[3];  // the first NA used
};

template <int MOTION>
__device__ __forceinline__ void rotor_init(const Pattern& pt, double t, double* rs, double* rc) {
  double th[3];
  if (MOTION == QT_MOTION_FIGURE8)
    th[0] = pt.o0 * t;
  else
    periodic_angles(MOTION, pt, t, th);
#pragma unroll
  for (int i = 0; i < Rotor<MOTION>::NA; ++i) fast_sincos(th[i], &rs[i], &rc[i]);
}

template <int MOTION>
__device__ __forceinline__ void rotor_advance(const LaunchConst& k, double dtt, double* rs, double* rc) {
#pragma unroll
  for (int i = 0; i < Rotor<MOTION>::NA; ++i) {
    const double s0 = rs[i], c0 = rc[i];
    const double s1 = fma(s0, k.rc[MOTION][i], c0 * k.rs[MOTION][i]);
    const double c1 = fma(c0, k.rc[MOTION][i], -(s0 * k.rs[MOTION][i]));
    const double d = k.om[MOTION][i] * dtt;
    rs[i] = fma(c1, d, s1);
    rc[i] = fma(-s1, d, c1);
  }
}

// The rotor of one step inside a safe horizon (run_yaw0): t's binade, and
// with it the step's rounding dtt = (fl(t + dt) - t) - dt, is the same for
// every step of the horizon, so the rotation by fl(omega dt) and the
// first-order turn by omega dtt are folded once per horizon into one
// rotation (fc, fs): 4 operations per angle instead of 7.
template <int MOTION>
__device__ __forceinline__ void rotor_fold(const LaunchConst& k, double dtt, double* fc, double* fs) {
#pragma unroll
  for (int i = 0; i < Rotor<MOTION>::NA; ++i) {
    const double d = k.om[MOTION][i] * dtt;
    fc[i] = fma(-k.rs[MOTION][i], d, k.rc[MOTION][i]);
    fs[i] = fma(k.rc[MOTION][i], d, k.rs[MOTION][i]);
  }
}

template <int MOTION>
__device__ __forceinline__ void rotor_turn(const double* fc, const double* fs, double* rs, double* rc) {
#pragma unroll
  for (int i = 0; i < Rotor<MOTION>::NA; ++i) {
    const double s0 = rs[i], c0 = rc[i];
    rs[i] = fma(s0, fc[i], c0 * fs[i]);
    rc[i] = fma(c0, fc[i], -(s0 * fs[i]));
  }
}

template <bool WANT_ACC, int MOTION>
__device__ __forceinline__ void target_from_rotor(const qt_env_params& e, const Pattern& pt, const double* rs,
                                                  const double* rc, Target& o) {
  if constexpr (MOTION == QT_MOTION_FIGURE8) {
    figure8_recip(e, pt.o0, rs[0], rc[0], o);  // no feed-forward: no acceleration
  } else {
    periodic_state<WANT_ACC>(e, MOTION, pt, rs, rc, o);
    if (WANT_ACC) clamp_acceleration(e, o);
  }
}

// Runtime-motion form (a wave whose lanes have different motion types): the
// same per-motion rotor arithmetic as the specialised loops, chosen per lane,
// so that an episode's results do not depend on the wave it lands in.
template <bool FF>
__device__ __forceinline__ void rotor_init_rt(int motion, const Pattern& pt, double t, double* rs, double* rc) {
  if (motion == QT_MOTION_SINUSOIDAL)
    rotor_init<QT_MOTION_SINUSOIDAL>(pt, t, rs, rc);
  else if (motion == QT_MOTION_CIRCULAR)
    rotor_init<QT_MOTION_CIRCULAR>(pt, t, rs, rc);
  else if (motion == QT_MOTION_FIGURE8 && !FF)
    rotor_init<QT_MOTION_FIGURE8>(pt, t, rs, rc);
}

// ADVANCE: rotate by one step first (dtt: the time step's rounding)
template <bool FF, bool ADVANCE>
__device__ __forceinline__ void rotor_target_rt(const qt_env_params& e, const LaunchConst& k, int motion,
                                                const Pattern& pt, double t, double dtt, double* rs, double* rc,
                                                Target& tg) {
  if (motion == QT_MOTION_SINUSOIDAL) {
    if (ADVANCE) rotor_advance<QT_MOTION_SINUSOIDAL>(k, dtt, rs, rc);
    target_from_rotor<FF, QT_MOTION_SINUSOIDAL>(e, pt, rs, rc, tg);
  } else if (motion == QT_MOTION_CIRCULAR) {
    if (ADVANCE) rotor_advance<QT_MOTION_CIRCULAR>(k, dtt, rs, rc);
    target_from_rotor<FF, QT_MOTION_CIRCULAR>(e, pt, rs, rc, tg);
  } else if (motion == QT_MOTION_FIGURE8 && !FF) {
    if (ADVANCE) rotor_advance<QT_MOTION_FIGURE8>(k, dtt, rs, rc);
    target_from_rotor<false, QT_MOTION_FIGURE8>(e, pt, rs, rc, tg);
  } else {
    target_state<FF, true>(e, motion, pt, t, tg);
  }
}

// The env's velocity clamp (quadcopter_env.py:442-445) alone: the only part
// of _apply_state_constraints that a yaw-at-rest fast step can need beyond
// constrain_fast_apply (rates stay inside their clamp, angles inside the
// wrap's range: rate_bounded_ok, trig_of<true>).
__device__ __forceinline__ void clamp_velocity(const qt_env_params& e, double* x) {
  const double s = dot3_blas(x[3], x[4], x[5]);
  if (norm_gt(s, e.max_velocity)) {
    const double vm = sqrt(s);
#pragma unroll
    for (int i = 3; i < 6; ++i) x[i] = x[i] / vm * e.max_velocity;
  }
}

// The tilt clamp (quadcopter_env.py:460-463) on roll / pitch and on their
// carried sin / cos: sin is increasing and cos decreasing in |a| on the fast
// step's range (|a| <= pi/3 + kRateAngle < pi/2), so
// sin(clip(a)) = clip(sin a, -sin(pi/3), sin(pi/3)) and
// cos(clip(a)) = max(cos a, cos(pi/3)), with the bounds as sincos_tilt gives
// them (trig_of of a clamped angle).  Near the clamp a rounding of sin a or
// cos a to the bound moves it by <= 1 ulp.
__device__ __forceinline__ void tilt_clamp(double* x, Trig& ta) {
  double sm, cm;
  sincos_tilt(kMaxTilt, &sm, &cm);  // folded at compile time
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    x[6 + i] = clip_num(x[6 + i], -kMaxTilt, kMaxTilt);
    ta.s[i] = clip_num(ta.s[i], -sm, sm);
    ta.c[i] = fmax(ta.c[i], cm);
  }
}

// Safe horizon of the yaw-at-rest loop: an even number H of steps (wave-
// uniform, 0 <= H <= kMaxHorizon, H <= rem - 1) that no active lane of the
// wave can stop at, so the wave runs them without the stop vote.  Each lane
// bounds its distance to every stop condition the vote tests by the per-step
// bounds of Horizon (LaunchConst::hz): speed from the velocity clamp's guard,
// the position bound, (TILT) roll / pitch from the tilt clamp, the time limit;
// the wave takes the minimum over its active lanes by ballots (inactive lanes
// cast no vote).  The bounds hold for the state the loop is in at every
// step start (finite, |v| below the clamp, |w| and |u| within max_rate:
// rate_bounded_ok), so a no-vote step is exactly a voted step that did not
// stop.  H = 0 (one voted step) when the wave is near a stop or hz.on == 0.
constexpr int kMaxHorizon = 62;
constexpr int kVotedBurst = 4;

template <bool TILT, bool BINADE>
__device__ __forceinline__ int yaw0_horizon(const qt_env_params& e, const Horizon& hz, const VelLin& lin,
                                            const Plant& pl, const double* x, double t, int rem) {
  const double tmi = hz.tmax * pl.inv_mass;
  const double sw = (fabs(lin.wv[0]) + fabs(lin.wv[1])) + (fabs(lin.wv[2]) + fabs(lin.wv[3]));
  const double spa = (fabs(lin.pa[0]) + fabs(lin.pa[1])) + fabs(lin.pa[2]);
  const double dv = fma(fma(tmi, sw, fabs(lin.gv)), hz.slack, hz.vabs);                        // speed per step
  const double dp = fma(fma(fabs(lin.pv), hz.vmax, fma(tmi, spa, fabs(lin.gp))), hz.slack, hz.pabs);  // position
  // speed: (vmax^2 - |v|^2) / (2 vmax) <= vmax - |v| (no square root)
  const double s = fma(x[5], x[5], fma(x[4], x[4], x[3] * x[3]));
  double h = (hz.vmax2 - s) * hz.inv_2vmax * __builtin_amdgcn_rcp(dv);
  h = fmin(h, (hz.pmax - fmax(fabs(x[0]), fmax(fabs(x[1]), fabs(x[2])))) * __builtin_amdgcn_rcp(dp));
  if (TILT) h = fmin(h, (kMaxTilt - fmax(fabs(x[6]), fabs(x[7]))) * hz.inv_dang);
  h = fmin(h, (e.max_episode_time - t) * hz.inv_tstep);
  bool bin_ok = true;
  if (BINADE) {
    // t stays inside its binade [2^E, 2^(E+1)) and the binade has no tie, so
    // every step of the horizon advances t by the same fl(t + dt) - t
    const long long eb = __double_as_longlong(t) & 0x7ff0000000000000LL;
    h = fmin(h, (__longlong_as_double(eb + (1LL << 52)) - t) * hz.inv_tstep);
    bin_ok = t > 0.0 && eb != hz.tie_exp_bits;
  }
  // rcp's error (well below 1e-6) and the step about to be voted on
  h = fma(h, 1.0 - 1e-6, -1.0);
  const bool lane_ok = h >= 2.0 && lin.cv >= 0.0 && lin.cv <= 1.0 && bin_ok;
  const int hl = lane_ok ? (int)fmin(h, (double)kMaxHorizon) : 0;
  int H = 0;
#pragma unroll
  for (int bit = 32; bit >= 2; bit >>= 1)
    if (__builtin_amdgcn_ballot_w64(hl < H + bit) == 0) H += bit;
  const int rcap = (rem - 1) & ~1;
  return hz.on ? (H < rcap ? H : rcap) : 0;
}

// The yaw-at-rest fast loop (flavour kYaw0).  One wave-uniform loop: every
// step runs branch-free (closed-form RK4, carried roll / pitch and target
// trig, fused metrics) and ends with ONE wave vote; the loop leaves only when
// some lane needs the exact velocity clamp, terminates (time limit, position
// bounds) or the chunk ends.  Such a step is then finished exactly (the
// velocity clamp, per-lane termination) and the loop restarts for the lanes
// still running, so a wave pays no per-lane exec-mask bookkeeping and one
// taken branch (the back edge) per step.
// Overshoot state machine (detect_overshoots, utils/metrics.py:205-261) as
// one counter z: 1 after an on-target step, k + 1 in an off-target phase of
// length k that began on->off, <= 0 off target outside a phase; a phase's
// running maximum `cur` restarts at the on-target step's err - R <= 0, which
// any off-target excess > 0 replaces.
// DUAL: a second no-vote body that applies the tilt clamp, for waves whose
// tilt-bounded horizon is short because some lane sits at (or near) the tilt
// clamp (config 4's tuner candidates: 46% of a wave's steps were voted).  Such
// a wave bounds its horizon without the tilt (speed, position, time only) and
// runs it with the clamp in every step — exactly the voted step without the
// vote, so results are bitwise those of the voted loop.
constexpr int kDualBelow = 8;  // tilt-bounded horizons shorter than this try the clamping body (Horizon::dual_below)
#ifndef QT_GROUPED_DUAL
#define QT_GROUPED_DUAL 0  // the grouped kernel (two waves per SIMD, 256 VGPRs) too
#endif

// A stationary rider (BatchDev::ride_lo) in another group's wave: the
// stationary pattern's observation (target_motion.py:233-246, 387-411: the
// fixed point, zero velocity and acceleration) in place of what the group's
// loop formed, by a per-lane select.  The values are the stationary loop's
// bit for bit, and so is every step built on them (-ffp-contract=on: the
// same source expressions round alike in every specialised loop).
template <bool RIDE>
__device__ __forceinline__ void ride_target(const qt_env_params& e, bool still, Target& tg) {
  if constexpr (RIDE) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      tg.p[i] = still ? e.center[i] : tg.p[i];
      tg.v[i] = still ? 0.0 : tg.v[i];
      tg.a[i] = still ? 0.0 : tg.a[i];
    }
  }
}

template <int MOTION, int KC, bool FF, bool KS, bool UNI, bool DUAL = false, bool RIDE = false>
__device__ __forceinline__ void run_yaw0(const qt_env_params& e, const qt_ctrl_params& c, const qt_criteria& cr,
                                         int motion, const Pattern& pt, const Plant& pl_lane, double hover,
                                         const Gains<KC, KS>& G, const FFLane& fl, double* x, double* integ,
                                         Target& tg, double& t, Acc& a, int nsteps, const LaunchConst& k,
                                         bool still = false) {
  constexpr bool kRotor = MOTION == QT_MOTION_CIRCULAR || MOTION == QT_MOTION_SINUSOIDAL ||
                          (MOTION == QT_MOTION_FIGURE8 && !FF);
  constexpr int kNeg = -(1 << 30);
  const Plant pl = UNI ? k.pl : pl_lane;
  const VelLin lin = UNI ? k.vl : make_vel_lin(e, pl_lane);
  const double R = cr.target_radius, eR = e.target_radius;
  const double vm2 = e.max_velocity * e.max_velocity * (1.0 - 1e-14);
  // position bounds |p|_inf > max_position as a >= test (the vote's one compare)
  const double pos_up = nextafter(e.max_position, INFINITY);
  const int W = cr.overshoot_window;
  // Launch start: the pre-step tracking error of the current observation,
  // roll / pitch trig, target rotor, overshoot counter.  The observation is
  // re-derived from t (the stored one is the same function of t), so that
  // loop-invariant target rows (a linear target's velocity) stay invariant in
  // registers.  Nothing is re-derived after a vote stops the loop (the exact
  // finish changes only velocities and termination codes), so a lane's
  // results do not depend on the other lanes of its wave.
  double rs[3] = {0.0, 0.0, 0.0}, rc[3] = {1.0, 1.0, 1.0};  // carried target rotor (Rotor)
  if constexpr (kRotor) {
    rotor_init<MOTION>(pt, t, rs, rc);
    target_from_rotor<FF, MOTION>(e, pt, rs, rc, tg);
  } else if constexpr (MOTION < 0) {
    rotor_init_rt<FF>(motion, pt, t, rs, rc);
    rotor_target_rt<FF, false>(e, k, motion, pt, t, 0.0, rs, rc, tg);
  } else {
    target_state<FF, true>(e, motion, pt, t, tg);
  }
  ride_target<RIDE>(e, still, tg);
  double err = sqrt_pos(sq3_ref(tg.p[0] - x[0], tg.p[1] - x[1], tg.p[2] - x[2]));
  Trig ta;
  trig_of<true>(x + 6, ta);
  int z = a.prev_on == 1 ? 1 : (a.os_streak >= 0 ? a.os_streak + 1 : kNeg);
  double cur = a.os_cur;
  int on_pre = a.on_pre, on_post = a.on_post, os_count = a.os_count;
  bool stepped = false;
  // Where the tilt clamp goes (the same arithmetic either way): every voted
  // step applies it; the horizon's steps skip it where the horizon also bounds
  // the tilt (kTiltHorizon), which spares them its ~10 operations.  LQI runs
  // can diverge and hold their tilt at the clamp, so a tilt bound
  // would keep their horizon at zero: their horizon leaves the tilt out and
  // every step applies the clamp.
  constexpr bool kTiltHorizon = KC != 9;
  // The horizon's folded target rotor (rotor_fold; its horizon also ends at
  // t's binade edge): 3 operations per angle fewer in every no-vote step, but
  // two more live doubles per angle.  Taken where it pays in the gfx950 build:
  // the LQI loops (LQI sinusoidal 281.5 -> 270.5 VALU per step); the 6-column
  // loops sit at 256 architectural VGPRs and answer it with ~17 register
  // copies per step (circular 237 -> 243), so they keep the per-step rotor.
  constexpr bool kFold = kRotor && KC == 9;
  int s = 0;
  while (a.term == QT_TERM_RUNNING && s < nsteps) {
    const int s0 = s;
    int rem = nsteps - s0 > (1 << 29) ? (1 << 29) : nsteps - s0;  // steps left in this run (z stays < 1 off phase)
    RateCoef rk;
    // one closed-loop step; VOTE: end it with the stop vote (true: stop here)
    auto step = [&](auto vote, auto clamp, const double* fc, const double* fs) -> bool {
      constexpr bool VOTE = decltype(vote)::value, CLAMP = decltype(clamp)::value;
      rk.pin();
      const double a0[2] = {x[6], x[7]};  // step-start roll / pitch (attitude_trig_resid)
      // ---- compute_action on the current observation (riccati_lqr.py:779-967)
      double u[4];
      if (QT_ABLATE & QT_ABL_CONTROLLER) {
        u[0] = hover, u[1] = u[2] = u[3] = 0.0;
      } else {
        if constexpr (KC == 3)
          compute_action_pid<FF, true>(c, G.k, hover, x, x + 3, tg, t, fl, integ, u);  // observation time = t
        else
          compute_action<KC, FF, KS, true>(c, G, hover, x, x + 3, tg, fl, integ, u, nullptr, err);
      }
      // ---- the Evaluator's pre-step record (eval.py:142-159) -> metrics
      if (!(QT_ABLATE & QT_ABL_METRICS)) {
        a.sum_e += err;
        a.sum_e2 = fma(err, err, a.sum_e2);
        a.max_e = fmax(a.max_e, err);
        const bool on = err <= R;
        on_pre += on;
        a.sum_u += sqrt_sum(fma(u[2], u[2], fma(u[1], u[1], u[0] * u[0])));  // u[3] = 0: no yaw command
        const bool counted = on & (z > W);
        os_count += counted;
        a.os_max = counted ? fmax(a.os_max, cur) : a.os_max;
        cur = on ? err - R : fmax(cur, err - R);
        z = on ? 1 : z + 1;
      }
      // ---- env.step (quadcopter_env.py:152-232): the command is finite and
      // inside the env clamps, so parsing is the identity
      double d4[2];
      Trig t4;
      integrate_yaw0(k.rl, lin, pl, ta, x, u, rk, d4, t4);
      const double t0 = t;
      t += e.dt;
      if (!(QT_ABLATE & QT_ABL_TARGET)) {
        if constexpr (kRotor) {
          if (VOTE || !kFold)
            rotor_advance<MOTION>(k, (t - t0) - e.dt, rs, rc);
          else
            rotor_turn<MOTION>(fc, fs, rs, rc);  // the horizon's folded rotor
          target_from_rotor<FF, MOTION>(e, pt, rs, rc, tg);
        } else if constexpr (MOTION < 0) {
          rotor_target_rt<FF, true>(e, k, motion, pt, t, (t - t0) - e.dt, rs, rc, tg);
        } else {
          target_state<FF, true>(e, motion, pt, t, tg);
        }
        ride_target<RIDE>(e, still, tg);
      }
      // post-step tracking error: the env's on-target count now, the next
      // step's pre-step error (positions are not constrained)
      err = sqrt_pos(sq3_ref(x[0] - tg.p[0], x[1] - tg.p[1], x[2] - tg.p[2]));
      on_post += err <= eR;
      // angle wrap (no correction: tilt-bounded), carried roll / pitch trig of
      // the wrapped angles (attitude_trig_resid's bound holds for them), then
      // the tilt clamp on both the angles and their trig (tilt_clamp): here,
      // in every voted step and (!kTiltHorizon) in the horizon's steps too
      if (!(QT_ABLATE & QT_ABL_CONSTRAIN)) constrain_fast_apply<true>(e, x);
      attitude_trig_resid(x + 6, a0, d4, t4, ta);
      if ((VOTE || CLAMP || !kTiltHorizon) && !(QT_ABLATE & QT_ABL_CONSTRAIN)) tilt_clamp(x, ta);
      // the stop conditions as one maximum >= 0 (the state is finite): speed
      // at the clamp's guard band, position bounds, time limit, end of the run
      // (rem, uniform) — one compare and one
      // ballot straight into the branch, no serial scalar chain at the end of
      // the step
      if constexpr (!VOTE) return false;
      --rem;
      double stop_m =
          fmax(fmax(fmax(fabs(x[0]), fmax(fabs(x[1]), fabs(x[2]))) - pos_up, (x[3] * x[3] + x[4] * x[4] + x[5] * x[5]) - vm2),
               fmax(t - e.max_episode_time, -(double)rem));
      return __builtin_amdgcn_ballot_w64(stop_m >= 0.0) != 0;
    };
    // The safe horizon's steps without the vote (four per back edge, then
    // the horizon's last two); voted steps only where no horizon is left.
    do {
      int H = yaw0_horizon<kTiltHorizon, kFold>(e, k.hz, lin, pl, x, t, rem);
      bool clamp_body = false;  // wave-uniform (H comes from ballots)
      if constexpr (DUAL) {
        if (H < k.hz.dual_below) {
          const int H2 = yaw0_horizon<false, kFold>(e, k.hz, lin, pl, x, t, rem);
          if (H2 > H) H = H2, clamp_body = true;
        }
      }
      using F = std::false_type;
      using T = std::true_type;
      if constexpr (kFold) {
        double fc[3], fs[3];  // the horizon's folded target rotor
        rotor_fold<MOTION>(k, ((t + e.dt) - t) - e.dt, fc, fs);
        for (int j = 4; j <= H; j += 4) {
          step(F{}, F{}, fc, fs);
          step(F{}, F{}, fc, fs);
          step(F{}, F{}, fc, fs);
          step(F{}, F{}, fc, fs);
        }
        if (H & 2) {
          step(F{}, F{}, fc, fs);
          step(F{}, F{}, fc, fs);
        }
      } else if (DUAL && clamp_body) {
        for (int j = 4; j <= H; j += 4) {
          step(F{}, T{}, nullptr, nullptr);
          step(F{}, T{}, nullptr, nullptr);
          step(F{}, T{}, nullptr, nullptr);
          step(F{}, T{}, nullptr, nullptr);
        }
        if (H & 2) {
          step(F{}, T{}, nullptr, nullptr);
          step(F{}, T{}, nullptr, nullptr);
        }
      } else {
        // four steps per back edge, then the horizon's last two (H is even)
        for (int j = 4; j <= H; j += 4) {
          step(F{}, F{}, nullptr, nullptr);
          step(F{}, F{}, nullptr, nullptr);
          step(F{}, F{}, nullptr, nullptr);
          step(F{}, F{}, nullptr, nullptr);
        }
        if (H & 2) {
          step(F{}, F{}, nullptr, nullptr);
          step(F{}, F{}, nullptr, nullptr);
        }
      }
      rem -= H;
      // Horizons chain: the state after a horizon's steps is one no lane
      // stopped at, so the next horizon is bounded from it directly.  Only a
      // wave with a lane near a stop (H = 0) takes voted steps, a few before
      // it bounds again; without a horizon (hz.on == 0: a non-finite limit)
      // every step is voted.
      const int nv = H > 0 ? 0 : (k.hz.on ? kVotedBurst : (1 << 30));
      bool stop = false;
      for (int j = 0; j < nv && !stop; ++j) stop = step(std::true_type{}, std::false_type{}, nullptr, nullptr);
      if (stop) break;
    } while (true);
    const int ran = (nsteps - s0 > (1 << 29) ? (1 << 29) : nsteps - s0) - rem;
    s += ran;
    a.steps += ran;
    stepped = true;
    z = z <= 0 ? kNeg : z;  // off phase: keep z far below 1 for the next run
    // finish the last step exactly: the velocity clamp where it acts and
    // per-lane termination (no-ops for a lane the vote did not stop)
    if (!(QT_ABLATE & QT_ABL_CONSTRAIN)) clamp_velocity(e, x);
    a.term = (QT_ABLATE & QT_ABL_TERMINATION) ? (t >= e.max_episode_time ? QT_TERM_TIME_LIMIT : QT_TERM_RUNNING)
                                               : termination_fast(e, t, x);
  }
  if (stepped) {
    a.on_pre = on_pre, a.on_post = on_post, a.os_count = os_count;
    a.prev_on = z == 1 ? 1 : 0;
    a.os_streak = z >= 2 ? z - 1 : -1;
    a.os_cur = cur;
  }
}

// MOTION >= 0 specialises the target pattern; -1 reads it per episode.
// UNI (fast flavours): no per-episode mass, hover thrust or gains — the
// plant constants come from the launch (LaunchConst) and the gains from
// uniform addresses, all in SGPRs (checked on the host, launch_rollout).
// FRESH: the fresh-pass prologue / epilogue (LaunchConst::fresh_off, met) is
// compiled in (the grouped kernel leaves it out: its two-waves-per-SIMD
// register budget has no room, and its fresh passes take qt_reset and
// metrics_kernel around the launch).
// REC (the exact flavour): the launch may record steps (rec) or keep rewards
// (lc.reward); without them the exact loop carries neither pointer.  INTEG
// (the exact flavour): the integrator, known at launch (integrate_closed).
template <int FLAVOR, int MOTION, int KC, bool FF, bool KS, bool UNI = false, bool FRESH = true, bool REC = true,
          int INTEG = -1, bool RIDE = false, bool PIN = true>
__device__ __forceinline__ void rollout_lane(const qt_env_params& e, const qt_ctrl_params& c, const qt_criteria& cr,
                                             const BatchDev& b, const qt_state& st, int nsteps,
                                             double* __restrict__ rec, int deferred, const LaunchConst& lc,
                                             int64_t slot) {
  const int64_t n = b.n, ep = episode_of(b, slot);
  const int motion = MOTION >= 0 ? MOTION : motion_of(b, e, ep);
  // RIDE (the grouped kernel's waves with stationary riders): a rider lane
  // runs the group's loop with the stationary target (ride_target); its
  // pattern constants are zeroed so the group's target arithmetic, whose
  // result the select replaces, stays on finite numbers
  const bool still = RIDE && slot_motion(b, slot) == QT_MOTION_STATIONARY;
  Pattern pt = pattern_of(b, e, motion, ep);
  if (RIDE) pt.c0 = still ? 0.0 : pt.c0, pt.c1 = still ? 0.0 : pt.c1, pt.c2 = still ? 0.0 : pt.c2;
  const Plant pl = UNI ? lc.pl : make_plant(e, b.plant_mass ? b.plant_mass[ep] : e.mass);
  const double hover = UNI ? c.hover_thrust : (b.hover ? b.hover[ep] : c.hover_thrust);
  Gains<KC, KS> G;
  load_gains<KC, KS, UNI>(b, ep, G);
  const FFLane fl = FF ? ff_of(b, c, ep) : FFLane{};

  // integ: LQI integral (KC 9) | PID integral error + last observation time (KC 3)
  constexpr int NI = KC == 9 ? 3 : (KC == 3 ? 4 : 0);
  double x[12], integ[4] = {0, 0, 0, 0};  // PID: row 3 (last observation time) is loaded
  Target tg;
  double t;
  Acc a;
  if (FRESH && lc.fresh_off) {
    // a fresh pass (qt_rollout_fresh): the state qt_reset would store
    // (reset_kernel, quadcopter_env.py:111-150; fresh controller,
    // riccati_lqr.py:1073-1086), formed here instead of loaded
    target_state<true>(e, motion, pt, 0.0, tg);
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = tg.p[i] + lc.fresh_off[i * n + ep];
#pragma unroll
    for (int i = 3; i < 12; ++i) x[i] = 0.0;
    if (KC == 3) integ[3] = __longlong_as_double(0x7ff8000000000000LL);  // PID: no previous observation time (NaN)
    t = 0.0;
    a = Acc{0, 0, -INFINITY, 0, 0, 0, 0, 0, 0, -1, -1, 0, 0, QT_TERM_RUNNING};
  } else {
#pragma unroll
    for (int i = 0; i < 12; ++i) x[i] = st.x[i * n + ep];
#pragma unroll
    for (int i = 0; i < NI; ++i) integ[i] = st.integ[i * n + ep];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      tg.p[i] = st.target[i * n + ep];
      tg.v[i] = st.target[(3 + i) * n + ep];
      tg.a[i] = st.target[(6 + i) * n + ep];
    }
    t = st.t[ep];
    a = load_acc(st.acc, n, ep);
  }
  auto store_state = [&]() {
#pragma unroll
    for (int i = 0; i < 12; ++i) st.x[i * n + ep] = x[i];
#pragma unroll
    for (int i = 0; i < NI; ++i) st.integ[i * n + ep] = integ[i];
    // a fresh pass without integral rows (KC 6) stores the zeros qt_reset would
    if (FRESH && NI == 0 && lc.fresh_off && st.integ) {
#pragma unroll
      for (int i = 0; i < 3; ++i) st.integ[i * n + ep] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      st.target[i * n + ep] = tg.p[i];
      st.target[(3 + i) * n + ep] = tg.v[i];
      st.target[(6 + i) * n + ep] = tg.a[i];
    }
    st.t[ep] = t;
    store_acc(st.acc, n, ep, a);
  };

  // Which step the wavefront runs (uniform).  A fast flavour is launched only
  // when the launch-level preconditions hold (fast_path_ok, no recording); it
  // takes the waves whose lanes all qualify and leaves the others untouched,
  // and the exact kernel launched after it with `deferred` = that flavour
  // takes exactly those (the same test on the same inputs).
  // (every comparison below is taken on values the bit tests proved finite)
  bool lane_ok = a.term != QT_TERM_RUNNING ||
                 (all_finite(G.k, Gains<KC, KS>::kCount) && all_finite(x, 12) && all_finite(integ, 3) &&
                  all_finite(tg.p, 3) && all_finite(tg.v, 3) && all_finite(tg.a, 3) && finite_bits(hover) &&
                  (!FF || (all_finite(fl.vg, 3) && all_finite(fl.ag, 3) && !(fl.vmax < 0.0))) &&
                  finite_bits(pl.inv_mass) && finite_bits(t) && fabs(t) < 1e300);
  for (int i = 9; i < 12; ++i) lane_ok = lane_ok && fabs(x[i]) <= e.max_angular_velocity;
  // the grouped launch runs each wave's loop for its group's seg_motion and
  // leaves a wave holding a lane whose own motion differs (a caller's
  // inconsistent seg_motion, rollout_grouped_kernel) to this exact pass, which
  // reads the motion per lane
  if (FLAVOR == kExact && b.nseg && b.motion) lane_ok = lane_ok && (int)b.motion[ep] == slot_motion(b, slot);
  // a per-segment launch (BatchDev::seg_check): a slot whose own motion is not
  // the segment's fails the wave test in both kernels, so the exact pass (which
  // then runs with runtime motion, rollout_batch) takes the wave
  if (b.seg_check >= 0 && b.motion) lane_ok = lane_ok && (int)b.motion[ep] == b.seg_check;
  // structured gains (or any K whose yaw-rate row is zero: qt_batch.k_no_yaw)
  // never command yaw: a yaw at rest stays exactly zero
  // (and, tilt-bounded, roll and pitch inside the tilt clamp: trig_of<YAW0>;
  // rate-bounded, roll and pitch rates within the command clip: rate_bounded_ok)
  if (FLAVOR == kYaw0 || deferred == kYaw0)
    lane_ok = lane_ok && x[8] == 0.0 && x[11] == 0.0 && fabs(x[6]) <= kMaxTilt && fabs(x[7]) <= kMaxTilt &&
              fabs(x[9]) <= c.max_rate && fabs(x[10]) <= c.max_rate;
  const bool wave_ok = __builtin_amdgcn_ballot_w64(!lane_ok) == 0;
  if (FLAVOR != kExact) {
    if (!wave_ok) {
      if (lc.defer_flag) *lc.defer_flag = lc.epoch;  // the exact pass has work (every lane stores the same value)
      if (FRESH && lc.fresh_off) store_state();  // the reset state, for the exact pass (launched without fresh_off)
      return;
    }
    // qt_rollout_rewards on a fast flavour: the loop's pre-step tracking errors
    // telescope into the env's post-step ones (post_k = pre_(k+1): positions
    // are not constrained), so this launch's reward sum is
    // -(dsum_e - pre_first + post_last).  The launch-start terms go to memory
    // at once (nothing stays live across the loop).
    const bool rw = FRESH && lc.reward && a.term == QT_TERM_RUNNING;
    if (rw) lc.reward[ep] += a.sum_e + sqrt_pos(sq3_ref(tg.p[0] - x[0], tg.p[1] - x[1], tg.p[2] - x[2]));
#if QT_CLOCK_STAMP && defined(QT_FAST_TU)
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
    if constexpr (FLAVOR == kYaw0)
      run_yaw0<MOTION, KC, FF, KS, UNI,
               (FRESH || QT_GROUPED_DUAL) && KC != 9 &&
                   (MOTION == QT_MOTION_CIRCULAR || MOTION == QT_MOTION_SINUSOIDAL || MOTION == QT_MOTION_FIGURE8),
               RIDE>(e, c, cr, motion, pt, pl, hover, G, fl, x, integ, tg, t, a, nsteps, lc, still);
    else
      run_steps<true, MOTION, KC, FF, KS>(e, c, cr, motion, pt, pl, hover, G, fl, x, integ, tg, t, a, nsteps, rec,
                                          n, ep);
#if QT_CLOCK_STAMP && defined(QT_FAST_TU)
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0 && wave < kStampWaves) {
      g_qt_stamps[wave][0] = t0, g_qt_stamps[wave][1] = t1;
      g_qt_stamps[wave][2] = r0, g_qt_stamps[wave][3] = r1;
      // where the wave ran: HW_ID (wave, SIMD, CU, SH, SE fields) and the XCD
      g_qt_stamps[wave][4] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
      g_qt_stamps[wave][5] = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);
    }
#endif
    if (rw) {
      const double q0 = x[0] - tg.p[0], q1 = x[1] - tg.p[1], q2 = x[2] - tg.p[2];
      lc.reward[ep] -= a.sum_e + sqrt_pos(sq3_ref(q0, q1, q2));
      lc.reward[n + ep] = sqrt(dot3_blas(q0, q1, q2));  // float(np.linalg.norm(...)), as the exact step
    }
  } else {
    if (deferred != kExact && wave_ok) return;
    run_steps<false, MOTION, KC, FF, KS, INTEG, PIN>(e, c, cr, motion, pt, pl, hover, G, fl, x, integ, tg, t, a, nsteps,
                                         REC ? rec : nullptr, n, ep, REC ? lc.reward : nullptr);
  }
  // Without feed-forward the loop leaves the acceleration rows at zero (only
  // feed-forward reads them); the stored observation carries the reference's
  // acceleration (target_motion.py:387-411) for later chunks and callers.
  if (!FF && (motion == QT_MOTION_CIRCULAR || motion == QT_MOTION_SINUSOIDAL || motion == QT_MOTION_FIGURE8)) {
    Target full;
    target_state<true>(e, motion, pt, t, full);
#pragma unroll
    for (int i = 0; i < 3; ++i) tg.a[i] = still ? 0.0 : full.a[i];  // a rider's: the stationary target's zero
  }

  store_state();
  if (FRESH && lc.met) store_metrics(cr, a, t, lc.met, n, ep);  // a fresh pass: the metrics rows (metrics_kernel)
}

template <int FLAVOR, int MOTION, int KC, bool FF, bool KS, bool UNI = false, bool REC = true, int INTEG = -1,
          bool PIN = true>
__global__ __launch_bounds__(kBlock) void rollout_kernel(qt_env_params e, qt_ctrl_params c, qt_criteria cr,
                                                         BatchDev b, qt_state st, int nsteps,
                                                         double* __restrict__ rec, int deferred, LaunchConst lc) {
  // the exact pass after a fast flavour that deferred no wave: nothing to do
  // (one uniform load per wave instead of the wave test's ~40 per lane)
  if (FLAVOR == kExact && deferred != kExact && lc.defer_flag && *lc.defer_flag != lc.epoch) return;
  const int64_t slot = slot_at(b, (int64_t)blockIdx.x * kBlock + threadIdx.x);
  if (slot < 0) return;
  rollout_lane<FLAVOR, MOTION, KC, FF, KS, UNI, true, REC, INTEG, false, PIN>(e, c, cr, b, st, nsteps, rec, deferred, lc,
                                                                             slot);
}

// The yaw-at-rest fast flavour over a batch grouped by motion type
// (qt_rollout_grouped: `order` lists the episodes motion by motion) in ONE
// launch: the groups start at wavefront boundaries (BatchDev's wave-aligned
// segments), so each wave runs the loop specialised for its motion and no
// wave needs a runtime-motion loop; the last wave of a group may be partly
// empty (at most one per group).  One launch keeps every SIMD busy where one
// launch per group would run each group's waves alone (65,536 episodes of five
// groups: ~205 waves per launch on 1,024 SIMDs).
// Two waves per SIMD: mixed batches are large (config 5: 1,048,576 episodes,
// 16 waves per SIMD on one GPU, 2 on each of 8), and a second resident wave
// issues in the first one's stall and encoding slots.
#ifndef QT_GROUPED_WAVES
#define QT_GROUPED_WAVES 2
#endif
#ifndef QT_GROUPED_RIDERS
#define QT_GROUPED_RIDERS 1  // the rider loops (rollout_batch sets up riders only when this is 1)
#endif
template <int KC, bool FF, bool KS>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(QT_GROUPED_WAVES))) void rollout_grouped_kernel(qt_env_params e, qt_ctrl_params c, qt_criteria cr,
                                                                 BatchDev b, qt_state st, int nsteps, LaunchConst lc) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  bool ride;
  const int64_t slot = slot_at(b, p, ride);
  if (slot < 0) return;
  const int wm = wave_motion(b, p);
  // the motion a lane's slot belongs to (a rider's: stationary), which the
  // exact pass's wave test compares too (rollout_lane)
  if (b.motion && __builtin_amdgcn_ballot_w64((int)b.motion[episode_of(b, slot)] != slot_motion(b, slot)) != 0) {
    // a lane's own motion is not its group's: the exact pass runs the wave
    if (lc.defer_flag) *lc.defer_flag = lc.epoch;
    return;
  }
  // one switch over (motion, riders): a wave with stationary riders (uniform)
  // takes its group's loop with the rider select (rollout_lane's RIDE)
  const int key = wm + ((QT_GROUPED_RIDERS && __builtin_amdgcn_ballot_w64(ride) != 0) ? 8 : 0);
  switch (key) {
    case QT_MOTION_STATIONARY:
      rollout_lane<kYaw0, QT_MOTION_STATIONARY, KC, FF, KS, false, false>(e, c, cr, b, st, nsteps, nullptr, kExact, lc, slot);
      break;
    case QT_MOTION_LINEAR:
      rollout_lane<kYaw0, QT_MOTION_LINEAR, KC, FF, KS, false, false>(e, c, cr, b, st, nsteps, nullptr, kExact, lc, slot);
      break;
    case QT_MOTION_CIRCULAR:
      rollout_lane<kYaw0, QT_MOTION_CIRCULAR, KC, FF, KS, false, false>(e, c, cr, b, st, nsteps, nullptr, kExact, lc, slot);
      break;
    case QT_MOTION_SINUSOIDAL:
      rollout_lane<kYaw0, QT_MOTION_SINUSOIDAL, KC, FF, KS, false, false>(e, c, cr, b, st, nsteps, nullptr, kExact, lc, slot);
      break;
    case QT_MOTION_FIGURE8:
      rollout_lane<kYaw0, QT_MOTION_FIGURE8, KC, FF, KS, false, false>(e, c, cr, b, st, nsteps, nullptr, kExact, lc, slot);
      break;
#if QT_GROUPED_RIDERS
    case 8 + QT_MOTION_LINEAR:
      rollout_lane<kYaw0, QT_MOTION_LINEAR, KC, FF, KS, false, false, true, -1, true>(e, c, cr, b, st, nsteps, nullptr,
                                                                                   kExact, lc, slot);
      break;
    case 8 + QT_MOTION_CIRCULAR:
      rollout_lane<kYaw0, QT_MOTION_CIRCULAR, KC, FF, KS, false, false, true, -1, true>(e, c, cr, b, st, nsteps, nullptr,
                                                                                     kExact, lc, slot);
      break;
    case 8 + QT_MOTION_SINUSOIDAL:
      rollout_lane<kYaw0, QT_MOTION_SINUSOIDAL, KC, FF, KS, false, false, true, -1, true>(e, c, cr, b, st, nsteps,
                                                                                       nullptr, kExact, lc, slot);
      break;
    case 8 + QT_MOTION_FIGURE8:
      rollout_lane<kYaw0, QT_MOTION_FIGURE8, KC, FF, KS, false, false, true, -1, true>(e, c, cr, b, st, nsteps, nullptr,
                                                                                    kExact, lc, slot);
      break;
#endif
    default:  // (no other key: rollout_batch gives a stationary group no riders)
      break;
  }
}

inline BatchDev to_dev(const qt_batch* b) {
  BatchDev d{};
  d.n = b->n, d.motion = b->motion, d.pattern = b->pattern, d.plant_mass = b->plant_mass;
  d.hover = b->hover_thrust, d.K = b->K, d.k_cols = b->k_cols, d.k_per_episode = b->k_per_episode;
  d.order = b->order, d.ff = b->ff, d.slot0 = 0, d.slot_end = b->n;
  d.nseg = 0;
  d.seg_check = -1;
  return d;
}

inline int grid_of(int64_t n) { return (int)((n + kBlock - 1) / kBlock); }

inline int check_launch() { return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH; }

inline bool valid_state(const qt_state& st, bool need_integ) {
  return st.x && st.t && st.acc && st.target && (!need_integ || st.integ);
}

// Fast step flavours (qt_rollout_fast.hip): launches rollout_kernel<flavor>
// (kFast or kYaw0) for the runtime controller / target choice.
// uni: no per-episode mass, hover thrust or gains (rollout_kernel's UNI).
// grouped: the yaw-at-rest flavour of a motion-grouped batch in one launch
// (rollout_grouped_kernel; `motion` is ignored).
void launch_fast(int flavor, bool uni, bool grouped, int kc, bool ff, bool ks, int motion, int grid, hipStream_t s,
                 const qt_env_params& e, const qt_ctrl_params& c, const qt_criteria& cr, const BatchDev& b,
                 const qt_state& st, int nsteps, const LaunchConst& lc);

// The pair-lane yaw-at-rest flavour (qt_pair.hpp; qt_rollout_fast.hip): one
// episode on two lanes, for a batch of at most one wave per SIMD in pairs;
// motion QT_MOTION_LINEAR or QT_MOTION_STATIONARY, grid of 2 n lanes.
void launch_pair(int motion, int grid, hipStream_t s, const qt_env_params& e, const qt_ctrl_params& c,
                 const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps, const LaunchConst& lc);

// Calls L::template run<MOTION, KC, FF, KS>(args...) for a runtime (kc, ff, ks, motion);
// PID (kc 3) never commands yaw and always takes the structured form.
template <class L, int KC, bool FF, bool KS, class... A>
void dispatch_motion(int motion, A&&... args) {
  switch (motion) {
    case QT_MOTION_STATIONARY: L::template run<QT_MOTION_STATIONARY, KC, FF, KS>(args...); break;
    case QT_MOTION_LINEAR: L::template run<QT_MOTION_LINEAR, KC, FF, KS>(args...); break;
    case QT_MOTION_CIRCULAR: L::template run<QT_MOTION_CIRCULAR, KC, FF, KS>(args...); break;
    case QT_MOTION_SINUSOIDAL: L::template run<QT_MOTION_SINUSOIDAL, KC, FF, KS>(args...); break;
    case QT_MOTION_FIGURE8: L::template run<QT_MOTION_FIGURE8, KC, FF, KS>(args...); break;
    default: L::template run<-1, KC, FF, KS>(args...);
  }
}

template <class L, int KC, class... A>
void dispatch_ffks(bool ff, bool ks, int motion, A&&... args) {
  if constexpr (KC == 3) {
    if (ff) dispatch_motion<L, 3, true, true>(motion, args...);
    else dispatch_motion<L, 3, false, true>(motion, args...);
  } else if (ff) {
    if (ks) dispatch_motion<L, KC, true, true>(motion, args...);
    else dispatch_motion<L, KC, true, false>(motion, args...);
  } else {
    if (ks) dispatch_motion<L, KC, false, true>(motion, args...);
    else dispatch_motion<L, KC, false, false>(motion, args...);
  }
}

template <class L, class... A>
void dispatch_rollout(int kc, bool ff, bool ks, int motion, A&&... args) {
  if (kc == 9) dispatch_ffks<L, 9>(ff, ks, motion, args...);
  else if (kc == 3) dispatch_ffks<L, 3>(ff, ks, motion, args...);
  else dispatch_ffks<L, 6>(ff, ks, motion, args...);
}

}  // namespace qtk

