// qt_step.hip — the per-step API (include/quadtrack.h, ABI 9): one batched
// env.step, compute_action or closed-loop step per launch.
//
// The fused rollout (qt_kernels.hpp) keeps an episode in registers for a
// whole launch.  Callers that drive the loop themselves — the reference's
// `obs, r, done, info = env.step(ctrl.compute_action(obs))` (eval.py:119-165)
// on a batch — need every step's observation in HBM instead.  Here the state
// round-trips HBM once per step in "frames" (quadtrack.h qt_frame_row): one
// contiguous block per step holding the observation and the info the
// reference's step returns, SoA, one column per episode.  A step reads the
// previous frame and writes a new one, so the observation a caller keeps is
// never overwritten (the reference's arrays are fresh copies,
// quadcopter_env.py:481-486) and no copy is made for it.
//
// Bound: HBM.  One lane per episode, every load and store a coalesced
// 512-byte wave access.  The exact step's arithmetic (staged RK4, the
// reference's control flow: ~1,000 VALU per episode-step) keeps the SIMDs
// ~25% busy at 160 VGPRs, three waves per SIMD (DESIGN §3 "Per-step API":
// 0.57 of HBM at 1,048,576 episodes; fewer registers spill, a lighter step
// needs more of them).
// Reference functions: src/quadcopter_tracking/... of the reference repo.
#include "qt_kernels.hpp"

using namespace qtk;

namespace {

struct FrameDev {
  double* f;
  int64_t* c;
  int8_t* b;
};

__device__ __forceinline__ FrameDev frame_of(const void* base, int64_t n) {
  double* f = static_cast<double*>(const_cast<void*>(base));
  return FrameDev{f, reinterpret_cast<int64_t*>(f + QT_FR_ROWS * n),
                  reinterpret_cast<int8_t*>(f + (QT_FR_ROWS + QT_FC_ROWS) * n)};
}

__device__ __forceinline__ double view_at(const qt_view& v, int r, int64_t e) { return v.p[r * v.rs + e * v.es]; }

// An episode that is done and frozen carries its frame over unchanged.
__device__ __forceinline__ void copy_column(const FrameDev& I, const FrameDev& O, int64_t n, int64_t ep) {
#pragma unroll
  for (int r = 0; r < QT_FR_ROWS; ++r) O.f[r * n + ep] = I.f[r * n + ep];
#pragma unroll
  for (int r = 0; r < QT_FC_ROWS; ++r) O.c[r * n + ep] = I.c[r * n + ep];
#pragma unroll
  for (int r = 0; r < QT_FB_ROWS; ++r) O.b[r * n + ep] = I.b[r * n + ep];
}

__device__ __forceinline__ void store_target(const FrameDev& O, int64_t n, int64_t ep, const Target& tg) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    O.f[(QT_FR_TARGET + i) * n + ep] = tg.p[i];
    O.f[(QT_FR_TARGET + 3 + i) * n + ep] = tg.v[i];
    O.f[(QT_FR_TARGET + 6 + i) * n + ep] = tg.a[i];
  }
}

// Counters carried from frame to frame (info["step"], info["action_violations"],
// the env's on-target count).
struct Counts {
  int64_t step, viol, on;
};

// An episode's per-launch inputs outside the frame: motion type, target
// pattern, plant.  Loaded with everything else before any data-dependent
// branch, so that a step waits for memory once (DESIGN §3 "Per-step API").
struct EpisodeIn {
  int motion;
  Pattern pt;
  Plant pl;
};

__device__ __forceinline__ EpisodeIn episode_in(const qt_env_params& e, const BatchDev& b, int64_t ep) {
  const int motion = motion_of(b, e, ep);
  return EpisodeIn{motion, pattern_of(b, e, motion, ep), make_plant(e, b.plant_mass ? b.plant_mass[ep] : e.mass)};
}

// QuadcopterEnv.step (quadcopter_env.py:152-232) of episode ep from state x
// at time t with the raw action u, into frame O: _parse_and_validate_action
// (234-293), _integrate (295-327), _apply_state_constraints (428-465),
// t += dt (191), observation (472-496), reward (504-511), termination
// (513-535), on-target count (204-207), info (209-226), success (537-553).
__device__ __forceinline__ void env_step_into(const qt_env_params& e, const EpisodeIn& in, int64_t n, int64_t ep,
                                              double* x, double t, Counts k, const double* u, const FrameDev& O) {
  const int motion = in.motion;
  const Pattern& pt = in.pt;
  const Plant& pl = in.pl;
  double ua[4];
  // The rows that depend on time only (the target observation, time, step
  // count) first: their stores drain while the step computes, which shortens
  // a small batch's launch (one wave per SIMD: load, compute, store in
  // series; 65,536 episodes 9.0 -> 8.0-8.7 us, profiles/r06/step_kernel_ab_r06_early.jsonl).
  // Every load of the step precedes this (in == out steps in place).
  t += e.dt;
  Target tg;
  target_state<true>(e, motion, pt, t, tg);
  store_target(O, n, ep, tg);
  O.f[QT_FR_TIME * n + ep] = t;
  O.c[QT_FC_STEP * n + ep] = k.step + 1;
  const bool viol = parse_action(e, u, ua);
  integrate(e, pl, x, ua);
  // np.clip's NaN propagation kept: a caller's action may drive the state anywhere
  const int term = constrain_terminate<true>(e, x, t);
  const double q0 = x[0] - tg.p[0], q1 = x[1] - tg.p[1], q2 = x[2] - tg.p[2];
  const double err = sqrt(dot3_blas(q0, q1, q2));  // float(np.linalg.norm(quad_pos - target_pos))
  const bool on = err <= e.target_radius;
  k.step += 1;
  k.viol += viol;
  k.on += on;
  const double ratio = (double)k.on / (double)k.step;
  const bool success = !(t < e.min_episode_duration) && ratio >= e.min_on_target_ratio;
#pragma unroll
  for (int i = 0; i < 12; ++i) O.f[(QT_FR_X + i) * n + ep] = x[i];
  O.f[QT_FR_ERR * n + ep] = err;
  O.f[QT_FR_REWARD * n + ep] = -err;
  O.f[QT_FR_RATIO * n + ep] = ratio;
  O.c[QT_FC_VIOLATIONS * n + ep] = k.viol;
  O.c[QT_FC_ON_TARGET * n + ep] = k.on;
  O.b[QT_FB_DONE * n + ep] = term != QT_TERM_RUNNING;
  O.b[QT_FB_ON_TARGET * n + ep] = on;
  O.b[QT_FB_VIOLATION * n + ep] = viol;
  O.b[QT_FB_SUCCESS * n + ep] = success;
  O.b[QT_FB_TERM * n + ep] = (int8_t)term;
}

// The controller of one episode: RiccatiLQRController / LQRController
// (compute_action) or PIDController (compute_action_pid, observation time
// `now`).  KS (the caller asserts the structured gain pattern): the six
// (nine) per-axis gains are read, which equals K s exactly for a finite s;
// a non-finite observation or integral takes the dense product, whose
// 0 * NaN terms the reference's K @ s has (riccati_lqr.py:864-900).
template <int KC, bool KS>
using CtlGains = Gains<KC, KC == 3 || KS>;

template <int KC, bool FF, bool KS>
__device__ __forceinline__ bool control(const qt_ctrl_params& c, const BatchDev& b, int64_t ep,
                                        const CtlGains<KC, KS>& G, double hover, const double* qp, const double* qv,
                                        const Target& tg, double now, const FFLane& fl, double* in, double* u) {
  if constexpr (KC == 3) {
    compute_action_pid<FF>(c, G.k, hover, qp, qv, tg, now, fl, in, u);
    return false;
  } else if constexpr (KS) {
    double s = ((qp[0] + qp[1]) + (qp[2] + qv[0])) + ((qv[1] + qv[2]) + (tg.p[0] + tg.p[1])) +
               ((tg.p[2] + tg.v[0]) + (tg.v[1] + tg.v[2]));
    if (KC == 9) s += (in[0] + in[1]) + in[2];
    if (__builtin_expect(isfinite(s), 1)) return compute_action<KC, FF, true>(c, G, hover, qp, qv, tg, fl, in, u);
    Gains<KC, false> D;
    load_gains<KC, false>(b, ep, D);
    return compute_action<KC, FF, false>(c, D, hover, qp, qv, tg, fl, in, u);
  } else {
    return compute_action<KC, FF, false>(c, G, hover, qp, qv, tg, fl, in, u);
  }
}

// integral / controller-state rows: LQI 3, PID 4 (integral error + last time)
template <int KC>
constexpr int integ_rows() {
  return KC == 9 ? 3 : (KC == 3 ? 4 : 0);
}

// ------------------------------------------------------------------ reset

__global__ __launch_bounds__(kBlock) void frame_reset_kernel(qt_env_params e, BatchDev b,
                                                             const double* __restrict__ off, void* out) {
  const int64_t ep = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t n = b.n;
  if (ep >= n) return;
  const FrameDev O = frame_of(out, n);
  const int motion = motion_of(b, e, ep);
  const Pattern pt = pattern_of(b, e, motion, ep);
  Target tg;
  target_state<true>(e, motion, pt, 0.0, tg);  // quadcopter_env.py:133-139
  double p[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    p[i] = tg.p[i] + off[i * n + ep];
    O.f[(QT_FR_X + i) * n + ep] = p[i];
  }
#pragma unroll
  for (int i = 3; i < 12; ++i) O.f[(QT_FR_X + i) * n + ep] = 0.0;
  store_target(O, n, ep, tg);
  const double err = sqrt(dot3_blas(p[0] - tg.p[0], p[1] - tg.p[1], p[2] - tg.p[2]));
  O.f[QT_FR_TIME * n + ep] = 0.0;
  O.f[QT_FR_ERR * n + ep] = err;
  O.f[QT_FR_REWARD * n + ep] = -err;
  O.f[QT_FR_RATIO * n + ep] = 0.0;
#pragma unroll
  for (int r = 0; r < QT_FC_ROWS; ++r) O.c[r * n + ep] = 0;
#pragma unroll
  for (int r = 0; r < QT_FB_ROWS; ++r) O.b[r * n + ep] = 0;
}

// ----------------------------------------------------------- open-loop step

template <bool FREEZE>
__global__ __launch_bounds__(kBlock) void frame_step_kernel(qt_env_params e, BatchDev b, const void* in,
                                                            qt_view a, void* out, int inplace) {
  const int64_t ep = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t n = b.n;
  if (ep >= n) return;
  const FrameDev I = frame_of(in, n), O = frame_of(out, n);
  // every load before the first data-dependent branch (one memory latency)
  const bool done = FREEZE && I.b[QT_FB_DONE * n + ep];
  double x[12], u[4];
#pragma unroll
  for (int i = 0; i < 12; ++i) x[i] = I.f[(QT_FR_X + i) * n + ep];
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = view_at(a, i, ep);
  const double t = I.f[QT_FR_TIME * n + ep];
  const Counts k{I.c[QT_FC_STEP * n + ep], I.c[QT_FC_VIOLATIONS * n + ep], I.c[QT_FC_ON_TARGET * n + ep]};
  const EpisodeIn ei = episode_in(e, b, ep);
  if (done) {
    if (!inplace) copy_column(I, O, n, ep);
    return;
  }
  env_step_into(e, ei, n, ep, x, t, k, u, O);
}

// --------------------------------------------------- controller on a view

template <int KC, bool FF, bool KS>
__global__ __launch_bounds__(kBlock) void action_obs_kernel(qt_ctrl_params c, BatchDev b, qt_obs_view o,
                                                            double* integ, double* action, int8_t* sat_out) {
  const int64_t ep = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t n = b.n;
  if (ep >= n) return;
  constexpr int NI = integ_rows<KC>();
  double qp[3], qv[3], in[4] = {0.0, 0.0, 0.0, NAN}, u[4];
  Target tg;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    qp[i] = view_at(o.pos, i, ep);
    qv[i] = view_at(o.vel, i, ep);
    tg.p[i] = view_at(o.tpos, i, ep);
    tg.v[i] = view_at(o.tvel, i, ep);
    tg.a[i] = (FF && o.tacc.p) ? view_at(o.tacc, i, ep) : 0.0;  // read only by feed-forward
  }
  const double now = (KC == 3 && o.time.p) ? view_at(o.time, 0, ep) : 0.0;
#pragma unroll
  for (int i = 0; i < NI; ++i) in[i] = integ[i * n + ep];
  const double hover = b.hover ? b.hover[ep] : c.hover_thrust;
  CtlGains<KC, KS> G;
  load_gains<KC, KC == 3 || KS>(b, ep, G);
  const bool sat = control<KC, FF, KS>(c, b, ep, G, hover, qp, qv, tg, now, ff_of(b, c, ep), in, u);
#pragma unroll
  for (int i = 0; i < 4; ++i) action[i * n + ep] = u[i];
#pragma unroll
  for (int i = 0; i < NI; ++i) integ[i * n + ep] = in[i];
  if (sat_out) sat_out[ep] = sat;
}

// ---------------------------------------------------- closed-loop step

// compute_action on frame I's observation, then env.step into frame O: the
// reference's `env.step(ctrl.compute_action(obs))` for every episode in one
// launch.  Reads 22 doubles (25 with feed-forward), 3 counters and the
// pattern per episode, writes the frame (229 B) and the action.
template <int KC, bool FF, bool KS, bool FREEZE>
__global__ __launch_bounds__(kBlock) void closed_step_kernel(qt_env_params e, qt_ctrl_params c, BatchDev b,
                                                             const void* in, double* integ, void* out,
                                                             double* action, int inplace) {
  const int64_t ep = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t n = b.n;
  if (ep >= n) return;
  const FrameDev I = frame_of(in, n), O = frame_of(out, n);
  // every load before the first data-dependent branch (the done test, the
  // controller's finiteness test): one memory latency per step, not three
  const bool done = FREEZE && I.b[QT_FB_DONE * n + ep];
  constexpr int NI = integ_rows<KC>();
  double x[12], in4[4] = {0.0, 0.0, 0.0, NAN}, u[4];
  Target tg;
#pragma unroll
  for (int i = 0; i < 12; ++i) x[i] = I.f[(QT_FR_X + i) * n + ep];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    tg.p[i] = I.f[(QT_FR_TARGET + i) * n + ep];
    tg.v[i] = I.f[(QT_FR_TARGET + 3 + i) * n + ep];
    tg.a[i] = FF ? I.f[(QT_FR_TARGET + 6 + i) * n + ep] : 0.0;
  }
  const double t = I.f[QT_FR_TIME * n + ep];
  const Counts k{I.c[QT_FC_STEP * n + ep], I.c[QT_FC_VIOLATIONS * n + ep], I.c[QT_FC_ON_TARGET * n + ep]};
#pragma unroll
  for (int i = 0; i < NI; ++i) in4[i] = integ[i * n + ep];
  const double hover = b.hover ? b.hover[ep] : c.hover_thrust;
  CtlGains<KC, KS> G;
  load_gains<KC, KC == 3 || KS>(b, ep, G);
  const FFLane fl = ff_of(b, c, ep);
  const EpisodeIn ei = episode_in(e, b, ep);
  if (done) {
    if (!inplace) copy_column(I, O, n, ep);
    if (action) {
#pragma unroll
      for (int i = 0; i < 4; ++i) action[i * n + ep] = 0.0;
    }
    return;
  }
  // the observation time is the env time (quadcopter_env.py:495)
  control<KC, FF, KS>(c, b, ep, G, hover, x, x + 3, tg, t, fl, in4, u);
#pragma unroll
  for (int i = 0; i < NI; ++i) integ[i * n + ep] = in4[i];
  if (action) {
#pragma unroll
    for (int i = 0; i < 4; ++i) action[i * n + ep] = u[i];
  }
  env_step_into(e, ei, n, ep, x, t, k, u, O);
}

// ------------------------------------------------------------- dispatch

// Calls L::template run<KC, FF, KS>() for a runtime (kc, ff, ks); PID (kc 3)
// is per-axis by construction.
template <class L>
int dispatch_ctl(int kc, bool ff, bool ks, L& l) {
  if (kc == 3) return ff ? l.template run<3, true, true>() : l.template run<3, false, true>();
  if (kc == 9) {
    if (ff) return ks ? l.template run<9, true, true>() : l.template run<9, true, false>();
    return ks ? l.template run<9, false, true>() : l.template run<9, false, false>();
  }
  if (ff) return ks ? l.template run<6, true, true>() : l.template run<6, true, false>();
  return ks ? l.template run<6, false, true>() : l.template run<6, false, false>();
}

struct ActionObsLaunch {
  hipStream_t s;
  const qt_ctrl_params& c;
  const BatchDev& b;
  const qt_obs_view& o;
  double* integ;
  double* action;
  int8_t* sat;
  template <int KC, bool FF, bool KS>
  int run() {
    action_obs_kernel<KC, FF, KS><<<grid_of(b.n), kBlock, 0, s>>>(c, b, o, integ, action, sat);
    return check_launch();
  }
};

struct ClosedLaunch {
  hipStream_t s;
  const qt_env_params& e;
  const qt_ctrl_params& c;
  const BatchDev& b;
  const void* in;
  double* integ;
  void* out;
  double* action;
  bool freeze;
  template <int KC, bool FF, bool KS>
  int run() {
    const int inplace = in == out;
    if (freeze)
      closed_step_kernel<KC, FF, KS, true><<<grid_of(b.n), kBlock, 0, s>>>(e, c, b, in, integ, out, action, inplace);
    else
      closed_step_kernel<KC, FF, KS, false><<<grid_of(b.n), kBlock, 0, s>>>(e, c, b, in, integ, out, action, inplace);
    return check_launch();
  }
};

bool valid_view(const qt_view& v) { return v.p != nullptr; }

}  // namespace

extern "C" {

int qt_frame_reset(const qt_env_params* env, const qt_batch* batch, const double* offset, void* frame,
                   void* stream) {
  if (!env || !batch || batch->n < 0 || batch->order) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;
  if (!offset || !frame) return QT_EINVAL;
  frame_reset_kernel<<<grid_of(batch->n), kBlock, 0, (hipStream_t)stream>>>(*env, to_dev(batch), offset, frame);
  return check_launch();
}

int qt_frame_step(const qt_env_params* env, const qt_batch* batch, const void* in, qt_view action, void* out,
                  int32_t freeze_done, void* stream) {
  if (!env || !batch || batch->n < 0 || batch->order) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;
  if (!in || !out || !valid_view(action)) return QT_EINVAL;
  const BatchDev b = to_dev(batch);
  hipStream_t s = (hipStream_t)stream;
  const int inplace = in == out;
  if (freeze_done)
    frame_step_kernel<true><<<grid_of(b.n), kBlock, 0, s>>>(*env, b, in, action, out, inplace);
  else
    frame_step_kernel<false><<<grid_of(b.n), kBlock, 0, s>>>(*env, b, in, action, out, inplace);
  return check_launch();
}

int qt_compute_action_obs(const qt_ctrl_params* ctrl, const qt_batch* batch, const qt_obs_view* obs,
                          double* integ, double* action, int8_t* saturated, void* stream) {
  if (!ctrl || !batch || !obs || !batch->K || batch->n < 0 || batch->order) return QT_EINVAL;
  if (batch->k_cols != 3 && batch->k_cols != 6 && batch->k_cols != 9) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;
  if (!action || (batch->k_cols != 6 && !integ)) return QT_EINVAL;
  if (!valid_view(obs->pos) || !valid_view(obs->vel) || !valid_view(obs->tpos) || !valid_view(obs->tvel))
    return QT_EINVAL;
  if (batch->k_cols == 3 && !valid_view(obs->time)) return QT_EINVAL;
  const BatchDev b = to_dev(batch);
  const bool ff = ctrl->feedforward_enabled != 0 || batch->ff != nullptr;
  ActionObsLaunch l{(hipStream_t)stream, *ctrl, b, *obs, integ, action, saturated};
  return dispatch_ctl(batch->k_cols, ff, batch->k_structured != 0, l);
}

int qt_frame_closed_step(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_batch* batch,
                         const void* in, double* integ, void* out, double* action, int32_t freeze_done,
                         void* stream) {
  if (!env || !ctrl || !batch || !batch->K || batch->n < 0 || batch->order) return QT_EINVAL;
  if (batch->k_cols != 3 && batch->k_cols != 6 && batch->k_cols != 9) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;
  if (!in || !out || (batch->k_cols != 6 && !integ)) return QT_EINVAL;
  const BatchDev b = to_dev(batch);
  const bool ff = ctrl->feedforward_enabled != 0 || batch->ff != nullptr;
  ClosedLaunch l{(hipStream_t)stream, *env, *ctrl, b, in, integ, out, action, freeze_done != 0};
  return dispatch_ctl(batch->k_cols, ff, batch->k_structured != 0, l);
}

}  // extern "C"
