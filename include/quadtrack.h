/*
 * quadtrack.h — C ABI of the MI355X batched quadcopter-tracking hot path.
 *
 * This is the drop-in boundary for the reference's closed-loop
 * `RiccatiLQRController.compute_action` -> `QuadcopterEnv.step` loop
 * (AgentFoundryExamples/lqr-quadcopter-test, src/quadcopter_tracking/...).
 * Every entry point takes plain pointers and sizes; every array pointer is a
 * DEVICE pointer (HBM, e.g. the data_ptr() of a torch tensor on cuda:N) and
 * every call is asynchronous on the given HIP stream (`stream` is a
 * hipStream_t passed as void*; NULL = the legacy default stream).
 * The library keeps no global state.  Return value: 0 on success, a negative
 * QT_E* code on an invalid argument or a HIP launch error.
 *
 * Layout conventions (HBM, FP64, structure-of-arrays):
 *   state  x[12][n]   rows: px py pz vx vy vz roll pitch yaw p q r
 *                     (quadcopter_env.py:63-70)
 *   aux    integ[4][n] controller state: LQI integral (rows 0-2, riccati_lqr.py:484-486) or
 *                     PID integral error (rows 0-2) + last observation time (row 3, NaN = None;
 *                     controllers/__init__.py:229-230, 262-271); LQR-only callers may pass NULL,
 *                     LQI-only callers a [3][n] array
 *   time   t[n]       per-episode accumulated time (t += dt, quadcopter_env.py:191)
 *   gains  K[kcols*4][m] SoA: element (row r, col c) of episode e at
 *                     K[(r*kcols + c)*m + e], with m = n (per-episode gains)
 *                     or m = 1 (one shared gain matrix, k_per_episode = 0).
 *                     k_cols = 6: RiccatiLQRController / LQRController (4x6),
 *                     9: LQI (4x9), 3: PIDController — K[9][m] = kp[3], ki[3], kd[3]
 *                     (controllers/__init__.py:196-203).
 */
#ifndef QUADTRACK_H
#define QUADTRACK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QT_ABI_VERSION 9

/* error codes */
#define QT_OK 0
#define QT_EINVAL (-1)
#define QT_ELAUNCH (-2)

/* TargetMotion.VALID_MOTION_TYPES (target_motion.py:264-270) */
enum qt_motion {
  QT_MOTION_STATIONARY = 0,
  QT_MOTION_LINEAR = 1,
  QT_MOTION_CIRCULAR = 2,
  QT_MOTION_SINUSOIDAL = 3,
  QT_MOTION_FIGURE8 = 4
};

/* QuadcopterEnv._check_termination reasons (quadcopter_env.py:513-535) */
enum qt_term {
  QT_TERM_RUNNING = 0,
  QT_TERM_TIME_LIMIT = 1,
  QT_TERM_POSITION_BOUNDS = 2,
  QT_TERM_NUMERICAL_INSTABILITY = 3
};

/* solve_dare outcome per episode (riccati_lqr.py:153-178) */
enum qt_dare_status {
  QT_DARE_OK = 0,
  QT_DARE_Q_NOT_PSD = 1,      /* "Q matrix must be positive semi-definite" */
  QT_DARE_R_NOT_PD = 2,       /* "R matrix must be positive definite" */
  QT_DARE_NO_CONVERGE = 3,    /* "DARE solver failed" */
  QT_DARE_SINGULAR = 4        /* singular (R + B'PB) / doubling matrix */
};

/* Plant + target + success parameters: EnvConfig (env/config.py:11-95). */
typedef struct qt_env_params {
  /* QuadcopterParams (config.py:12-38); Ixx/Iyy/Izz/arm_length/k_* are never
     read by the dynamics and are not carried. */
  double mass, gravity, drag_linear, drag_angular;
  double min_thrust, max_thrust, max_angular_rate;
  /* SimulationParams (config.py:41-51) */
  double dt, max_episode_time, max_velocity, max_angular_velocity, max_position;
  int32_t integrator;   /* 0 = "rk4", 1 = "euler" (quadcopter_env.py:309-312) */
  int32_t motion;       /* enum qt_motion, used when no per-episode motion array */
  /* TargetParams (config.py:55-65) */
  double speed, amplitude, frequency, radius, center[3], max_acceleration;
  /* SuccessCriteria of the ENV (config.py:69-74): post-step on-target and
     info["success"] (quadcopter_env.py:204-226, 537-553) */
  double target_radius, min_on_target_ratio, min_episode_duration;
} qt_env_params;

/* RiccatiLQRController options that shape compute_action
   (riccati_lqr.py:418-535, 779-967). */
typedef struct qt_ctrl_params {
  double dt;                                 /* integral step */
  double hover_thrust;                       /* mass * gravity (riccati_lqr.py:471) */
  double min_thrust, max_thrust, max_rate;   /* output clamps (907-921) */
  int32_t use_lqi;                           /* K has 9 columns when set */
  int32_t feedforward_enabled;
  double integral_limit, integral_zero_threshold;
  double ff_velocity_gain[3], ff_acceleration_gain[3];
  double ff_max_velocity, ff_max_acceleration;
} qt_ctrl_params;

/* Evaluator criteria for the per-episode metrics (utils/metrics.py:26-39);
   these are the Evaluator's own, distinct from qt_env_params' criteria. */
typedef struct qt_criteria {
  double min_on_target_ratio, min_episode_duration, target_radius;
  int32_t overshoot_window;                  /* detect_overshoots window_size */
  int32_t pad_;
} qt_criteria;

/* Per-episode running accumulators kept in HBM between rollout chunks.
   Row index into acc[QT_ACC_ROWS][n] (doubles). */
enum qt_acc_row {
  QT_ACC_SUM_ERR = 0,      /* sum of pre-step tracking errors (metrics.py:300) */
  QT_ACC_SUM_ERR2,         /* sum of squares (rms, metrics.py:330) */
  QT_ACC_MAX_ERR,          /* max pre-step error (NaN-propagating like np.max) */
  QT_ACC_ON_PRE,           /* count err_pre <= criteria.target_radius */
  QT_ACC_ON_POST,          /* env post-step on-target count (quadcopter_env.py:205-207) */
  QT_ACC_SUM_EFFORT,       /* sum |u|_2 (metrics.py:182-202) */
  QT_ACC_OS_COUNT,         /* overshoot count (metrics.py:205-261) */
  QT_ACC_OS_MAX,           /* max overshoot */
  QT_ACC_OS_CUR,           /* overshoot state machine: current phase max */
  QT_ACC_OS_STREAK,        /* off-target streak (-1 = not in an overshoot phase) */
  QT_ACC_PREV_ON,          /* on-target flag of the previous pre-step error (-1 = none) */
  QT_ACC_STEPS,            /* executed steps */
  QT_ACC_VIOLATIONS,       /* steps with an action violation (quadcopter_env.py:174-181) */
  QT_ACC_TERM,             /* enum qt_term */
  QT_ACC_ROWS
};

/* Final per-episode metrics, row index into met[QT_MET_ROWS][n] (doubles),
   EpisodeMetrics field order (utils/metrics.py:42-73). */
enum qt_met_row {
  QT_MET_DURATION = 0, QT_MET_ON_TARGET_RATIO, QT_MET_MEAN_ERR, QT_MET_MAX_ERR,
  QT_MET_RMS_ERR, QT_MET_TOTAL_EFFORT, QT_MET_MEAN_EFFORT, QT_MET_OS_COUNT,
  QT_MET_OS_MAX, QT_MET_SUCCESS, QT_MET_TERM, QT_MET_VIOLATIONS,
  QT_MET_ENV_ON_TARGET_RATIO, QT_MET_STEPS, QT_MET_ROWS
};

/* Per-episode inputs of a batch.  NULL optional arrays fall back to the
   scalar in the params structs.  `order` (optional) maps work slot -> episode
   so that a launch can walk episodes grouped by motion type. */
typedef struct qt_batch {
  int64_t n;                    /* episodes */
  const int8_t* motion;         /* [n] enum qt_motion, or NULL */
  const double* pattern;        /* [4][n]: linear raw normal draw xyz (normalised twice in
                                   kernel, target_motion.py:320-321,47) | circular theta0 |
                                   sinusoidal phase xyz (target_motion.py:306-369) */
  const double* plant_mass;     /* [n] or NULL -> env.mass */
  const double* hover_thrust;   /* [n] or NULL -> ctrl.hover_thrust */
  const double* K;              /* gains, layout above */
  int32_t k_cols;               /* 6 (LQR, heuristic LQR), 9 (LQI) or 3 (PID) */
  int32_t k_per_episode;        /* 0: one shared K (m = 1), 1: m = n */
  int32_t k_structured;         /* 1: the caller asserts every K entry outside the per-axis
                                   pattern (z->thrust, y->roll, x->pitch) is exactly 0, as the
                                   diagonal-weight DARE produces; the kernel then skips them */
  int32_t k_no_yaw;             /* 1: the caller asserts the yaw-rate row of K is exactly 0 (B has
                                   no yaw column, riccati_lqr.py:215-232, so any DARE gain has
                                   it): yaw never moves from rest and the yaw-at-rest fast
                                   flavour applies to dense gains too */
  const int32_t* order;         /* [n] or NULL */
  const double* ff;             /* ABI 3: [7][n] per-episode feed-forward, or NULL (then the qt_ctrl_params
                                   feed-forward applies to every episode): rows velocity gain xyz,
                                   acceleration gain xyz, target-velocity clamp (riccati_lqr.py:836-861,
                                   controllers/__init__.py:286-330).  An episode without feed-forward has
                                   gains 0 and clamp +inf: the tuner's per-candidate feed-forward gain
                                   ranges (controllers/tuning.py:689-735) and the heuristic fallback of a
                                   failed DARE, which runs without it (riccati_lqr.py:764-776).  The
                                   acceleration clamp stays qt_ctrl_params.ff_max_acceleration. */
} qt_batch;

/* Mutable per-episode rollout state, all [.][n] SoA device arrays. */
typedef struct qt_state {
  double* x;          /* [12][n] */
  double* integ;      /* [3][n] LQI integral | [4][n] PID integral + last time (NULL for LQR) */
  double* t;          /* [n] */
  double* acc;        /* [QT_ACC_ROWS][n] */
  double* target;     /* [9][n] target p,v,a at t (the observation the controller sees next) */
} qt_state;

/* ABI 9.  A strided [rows][n] view of FP64 device memory: element (row r,
   episode e) at p[r * rs + e * es].  A torch tensor of shape [n, k] is the view
   {data_ptr, stride(1), stride(0)}: a contiguous [n, k] array (es = k, rs = 1)
   and the [n, k] transpose of a [k][n] SoA array (es = 1, rs = n) both pass
   without a copy. */
typedef struct qt_view {
  double* p;
  int64_t rs, es;
} qt_view;

/* ABI 9.  The observation the controller reads (QuadcopterEnv._get_observation,
   quadcopter_env.py:472-496): quadcopter position / velocity and target
   position / velocity / acceleration, [3][n] each, and the observation time
   (row 0 of `time`; PIDController only, controllers/__init__.py:262-265).
   tacc.p and time.p may be NULL (zeros / unused). */
typedef struct qt_obs_view {
  qt_view pos, vel, tpos, tvel, tacc, time;
} qt_obs_view;

/* ABI 9.  Observation frame: what one batched env.step returns
   (quadcopter_env.py:152-232) for every episode, in ONE contiguous device
   block of QT_FRAME_BYTES(n) bytes (8-byte aligned):
     double  f[QT_FR_ROWS][n]   rows below (state, target observation, info floats)
     int64_t c[QT_FC_ROWS][n]   info counters
     int8_t  b[QT_FB_ROWS][n]   done / info flags (0 or 1) and the termination code
   A frame is written once by the launch that produces it and only read after:
   the per-step entry points read the previous step's frame and write a new
   one, so a frame the caller keeps (the observation of step k) never changes
   (the reference's observation arrays are fresh copies, 481-486). */
enum qt_frame_row {
  QT_FR_X = 0,            /* 12 rows: px py pz vx vy vz roll pitch yaw p q r (quadcopter_env.py:63-70) */
  QT_FR_TARGET = 12,      /* 9 rows: target position, velocity, clamped acceleration at `time` */
  QT_FR_TIME = 21,        /* env time, t += dt (quadcopter_env.py:191) */
  QT_FR_ERR = 22,         /* info["tracking_error"], post-step ||p - p_T|| (498-502) */
  QT_FR_REWARD = 23,      /* reward = -tracking error (504-511) */
  QT_FR_RATIO = 24,       /* info["on_target_ratio"] (215-219) */
  QT_FR_ROWS = 25
};
enum qt_frame_count {
  QT_FC_STEP = 0,         /* info["step"] */
  QT_FC_VIOLATIONS,       /* info["action_violations"]: steps with a violation record (174-181) */
  QT_FC_ON_TARGET,        /* env on-target count (205-207) */
  QT_FC_ROWS
};
enum qt_frame_flag {
  QT_FB_DONE = 0,         /* done (513-535) */
  QT_FB_ON_TARGET,        /* info["on_target"] */
  QT_FB_VIOLATION,        /* this step's action had a violation */
  QT_FB_SUCCESS,          /* info["success"] (_evaluate_success, 537-553; the reference reports it when done) */
  QT_FB_TERM,             /* enum qt_term: info["termination_reason"] */
  QT_FB_ROWS
};
#define QT_FRAME_BYTES(n) ((int64_t)(n) * (QT_FR_ROWS * 8 + QT_FC_ROWS * 8 + QT_FB_ROWS))

/* ---------------------------------------------------------------- entry points */

/* ABI version of the loaded library. */
int qt_abi_version(void);

/* Page-locked host memory mapped into the devices' address space (zero copy):
   *host and *dev address the same zeroed bytes.  The batch-1 drop-in objects
   (QuadcopterEnv, the one-episode controllers) keep their per-episode arrays
   here and pass *dev pointers to the entry points below, so a reference-style
   step is one launch and one qt_stream_sync with no copies.  Kernel writes are
   visible to the host after qt_stream_sync.  Not a replacement of any
   reference interface: the reference's env and controller hold numpy arrays
   (quadcopter_env.py:99-109, riccati_lqr.py:779-967). */
int qt_host_alloc(int64_t bytes, void** host, void** dev);
int qt_host_free(void* host);

/* hipStreamSynchronize(stream): waits for the stream's launches. */
int qt_stream_sync(void* stream);

/* QuadcopterEnv.reset(seed) from pre-drawn randoms (quadcopter_env.py:111-150):
   x = [p_target(0) + offset, 0...], t = 0, accumulators cleared, target row
   filled with the t = 0 observation, LQI integral zeroed (fresh controller,
   riccati_lqr.py:1073-1086).  offset[3][n] = uniform(-0.5, 0.5, 3) draws. */
int qt_reset(const qt_env_params* env, const qt_batch* batch, const double* offset,
             qt_state st, void* stream);

/* The per-episode draws of QuadcopterEnv.reset(seed) (quadcopter_env.py:122-137,
   target_motion.py:318-366), reproducing numpy.random.default_rng(seed) on the
   device (SeedSequence + PCG64 + numpy's ziggurat): pattern[4][n] in qt_batch
   form and the start offset[3][n] of qt_reset.  seeds[n] >= 0; motion[n] or
   NULL (then motion_default for all). */
int qt_seed_draws(int64_t n, const int64_t* seeds, const int8_t* motion, int32_t motion_default,
                  double* pattern, double* offset, void* stream);

/* The first k draws of numpy.random.default_rng(seeds[e]).uniform(lo[j], hi[j])
   for every episode e (per-episode parameters drawn from per-episode streams,
   e.g. SURVEY §8d config 5's masses from default_rng(1e9 + i)).  lo, hi: [k]
   DEVICE arrays; out[k][n]; k <= 64. */
int qt_seed_uniform(int64_t n, const int64_t* seeds, int32_t k, const double* lo, const double* hi,
                    double* out, void* stream);

/* ABI 6.  Draw vectors first .. first+n-1 of ONE stream
   numpy.random.default_rng(seed).uniform(lo, hi, size=(first + n, k)): lane i
   jumps the PCG64 state k * (first + i) outputs ahead (PCG64.advance) and draws
   its k uniforms, so a shard of a long candidate stream needs none of the draws
   before it (controllers/tuning.py:683-735's random candidates, SURVEY §8d
   config 4).  lo, hi: [k] DEVICE arrays; out[k][n]; k <= 64. */
int qt_stream_uniform(uint64_t seed, int64_t first, int64_t n, int32_t k, const double* lo, const double* hi,
                      double* out, void* stream);

/* The fused closed loop: `nsteps` iterations of
   compute_action (riccati_lqr.py:779-967; k_cols 3: PIDController.compute_action,
   controllers/__init__.py:243-379, with the observation time = the env time)
   -> env.step (quadcopter_env.py:152-232)
   per episode, register-resident, with the Evaluator's per-episode metric
   accumulation fused (eval.py:119-159, utils/metrics.py:264-338).  Episodes that
   are done stay frozen.  May be called repeatedly (chunks).  If rec != NULL it
   receives, for every step s of this call, x after the step at
   rec[((s*16 + j) * n) + e] for j < 12 and the applied controller action at j = 12..15.
   A batch of at most one wave per SIMD in lane pairs (n <= 32,768 on MI355X) with
   one target motion and structured LQR gains (shared or per episode) runs each
   episode on two lanes (the pair flavour, csrc/qt_pair.hpp), with the same
   results bit for bit; QT_PAIR=0 in the environment turns it off. */
int qt_rollout(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_criteria* crit,
               const qt_batch* batch, qt_state st, int32_t nsteps, double* rec, void* stream);

/* ABI 7.  qt_rollout with the env's per-step rewards kept, for the trainer's
   classical evaluation epoch (train.py:578-652, which the reference runs one
   env.step at a time): reward[0][e] += env.step's reward, -(post-step tracking
   error) (quadcopter_env.py:198-199, 498-511), in step order (the trainer's
   sum(), train.py:627); reward[1][e] = the last step's post-step tracking
   error (info["tracking_error"], train.py:630).  Its on-target ratio
   (info["on_target_ratio"]) is acc[QT_ACC_ON_POST] / acc[QT_ACC_STEPS].
   reward[2][n] is read and written (zero it before the first chunk).  Runs the
   exact step; `motion` / `order` batches as qt_rollout. */
int qt_rollout_rewards(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_criteria* crit,
                       const qt_batch* batch, qt_state st, int32_t nsteps, double* reward, void* stream);

/* qt_rollout for a batch of mixed motion types without per-step motion
   dispatch.  batch->order must list the episodes grouped by motion: slots
   [seg_end[i-1], seg_end[i]) (seg_end[-1] = 0) all have motion seg_motion[i];
   seg_end[nseg-1] == n.  seg_motion and seg_end are HOST arrays.  The
   yaw-at-rest fast flavour runs every group in ONE launch: each group starts
   at a 64-lane wave boundary, so every wave takes the loop specialised for its
   motion (<= 8 non-empty groups; more fall back to one launch per group);
   other flavours launch once per group.  seg_motion[i] == -1 marks a mixed
   segment whose slots take each episode's motion from batch->motion (the
   per-lane-motion loop); a batch with one takes one launch set per segment.
   Results are qt_rollout's: bit for bit with 6-column gains; with 9-column
   (LQI) gains within ~1e-10, where the specialised loops fold a periodic
   target's carried rotor once per horizon.  seg_motion must agree with
   batch->motion (when given) for every slot; a wave holding a slot whose
   batch->motion differs is run by the exact pass, which takes each episode's
   motion from batch->motion — in the one-launch grouped flavour and in the
   per-segment launch sets alike.  Stationary riders (one-launch flavour, with
   batch->motion given; QT_RIDERS=0 in the environment turns them off): the
   first episodes of the stationary group fill the free lanes of every other
   group's last wave (the group's loop with the stationary target selected per
   lane, the same numbers bit for bit), so N episodes take ceil(N / 64) waves
   when the stationary group can fill the other groups' gaps (round 6:
   config 5's 8-GPU shard, 2,050 -> 2,048 waves). */
int qt_rollout_grouped(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_criteria* crit,
                       const qt_batch* batch, qt_state st, int32_t nsteps, double* rec, int32_t nseg,
                       const int32_t* seg_motion, const int64_t* seg_end, void* stream);

/* ABI 8.  One evaluation pass from reset to per-episode metrics: qt_reset
   (offset[3][n]), then qt_rollout (nsteps, no recording), then
   qt_episode_metrics into met[QT_MET_ROWS][n], with the same results bit for
   bit, in one launch set: the rollout kernel forms the reset state in its
   prologue instead of loading it and writes the metrics rows in its epilogue.
   st receives the state qt_rollout leaves.  nseg > 0: a motion-grouped batch
   as qt_rollout_grouped (seg_motion, seg_end HOST arrays); nseg == 0: as
   qt_rollout. */
int qt_rollout_fresh(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_criteria* crit,
                     const qt_batch* batch, const double* offset, qt_state st, int32_t nsteps, double* met,
                     int32_t nseg, const int32_t* seg_motion, const int64_t* seg_end, void* stream);

/* Open-loop QuadcopterEnv.step(action) for a batch (quadcopter_env.py:152-293):
   action[4][n] (NaN/Inf zeroed, thrust and rate clipping), RK4/Euler, state
   constraints, t += dt, post-step error and termination.  Outputs:
   err[n] (info["tracking_error"]), on_target[n] (0/1), done[n] (0/1),
   term[n] (enum qt_term), violation[n] (0/1 for this step).  Counters in
   acc (ON_POST, STEPS, VIOLATIONS, TERM) are updated.  Episodes already done are
   stepped anyway (the reference does not refuse a step after done). */
int qt_env_step(const qt_env_params* env, const qt_batch* batch, const double* action,
                qt_state st, double* err, int8_t* on_target, int8_t* done, int8_t* term,
                int8_t* violation, void* stream);

/* RiccatiLQRController.compute_action for a batch of observations
   (riccati_lqr.py:779-967).  obs[15][n]: quad pos(3), quad vel(3), target
   pos(3), target vel(3), target acc(3).  integ[3][n] is updated in LQI mode.
   action[4][n] out; saturated[n] (0/1) out (may be NULL); diag[16][n] (may be
   NULL) receives get_control_components() (969-978): state_error(6),
   feedback_u(4), ff_velocity_term(3), ff_acceleration_term(3).
   k_cols = 6 with heuristic gains is LQRController.compute_action
   (controllers/__init__.py:576-690).  k_cols = 3 is PIDController.compute_action
   (controllers/__init__.py:243-379): obs[16][n] (row 15 = observation["time"]),
   integ[4][n] (integral error, last time; NaN = None) updated, saturated = 0,
   diag[18][n]: p, i, d, ff_velocity, ff_acceleration terms, total correction. */
int qt_compute_action(const qt_ctrl_params* ctrl, const qt_batch* batch, const double* obs,
                      double* integ, double* action, int8_t* saturated, double* diag, void* stream);

/* ---- ABI 9: the per-step API (one launch per step) ------------------------
   The batched counterparts of the reference's step-at-a-time plugin calls,
   for callers that drive the loop themselves (BatchedQuadcopterEnv.step,
   Batched*.compute_action).  Episodes are in index order (batch->order must
   be NULL).  Frames: QT_FRAME_BYTES(n) device blocks (qt_frame_row above). */

/* QuadcopterEnv.reset(seed) (quadcopter_env.py:111-150) into a frame:
   x = [p_target(0) + offset, 0...], target observation at t = 0, counters
   and flags 0, tracking error / reward of the reset state. */
int qt_frame_reset(const qt_env_params* env, const qt_batch* batch, const double* offset, void* frame,
                   void* stream);

/* QuadcopterEnv.step(action) (quadcopter_env.py:152-293) for every episode:
   reads the state, time and counters of frame `in`, the action view ([4][n]:
   thrust, roll, pitch, yaw rate; NaN / Inf zeroed and clipped as
   _parse_and_validate_action), and writes frame `out` (in == out allowed).
   freeze_done != 0: an episode whose `in` frame is done is not stepped (its
   frame is carried over), as the Evaluator stops at done (eval.py:119-165);
   0: it is stepped, as the reference's env does after done. */
int qt_frame_step(const qt_env_params* env, const qt_batch* batch, const void* in, qt_view action, void* out,
                  int32_t freeze_done, void* stream);

/* compute_action on an observation view (RiccatiLQRController.compute_action,
   riccati_lqr.py:779-967; k_cols 6 with heuristic gains: LQRController,
   controllers/__init__.py:576-690; k_cols 3: PIDController, 243-379, with
   obs->time).  integ as qt_compute_action (LQI [3][n], PID [4][n]) is read and
   updated; action[4][n] and saturated[n] (may be NULL) are written. */
int qt_compute_action_obs(const qt_ctrl_params* ctrl, const qt_batch* batch, const qt_obs_view* obs,
                          double* integ, double* action, int8_t* saturated, void* stream);

/* One closed-loop step in one launch: compute_action on frame `in`'s
   observation (integ updated), then env.step with that action into frame
   `out` (in == out allowed).  action[4][n] (may be NULL) receives the
   controller's command.  freeze_done as qt_frame_step; a frozen episode's
   controller state is not advanced either and its action row is 0. */
int qt_frame_closed_step(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_batch* batch,
                         const void* in, double* integ, void* out, double* action, int32_t freeze_done,
                         void* stream);

/* TargetMotion.get_state(t) (target_motion.py:387-411) for every episode at
   per-episode times t[n]: out[9][n] = position, velocity, clamped acceleration. */
int qt_target_state(const qt_env_params* env, const qt_batch* batch, const double* t,
                    double* out, void* stream);

/* Finalise accumulators into EpisodeMetrics rows (utils/metrics.py:264-338). */
int qt_episode_metrics(const qt_criteria* crit, int64_t n, const double* acc, const double* t,
                       double* met, void* stream);

/* compute_episode_metrics over recorded per-step arrays (utils/metrics.py:144-338):
   qpos/tpos [steps][3][n], actions [steps][4][n], last_time[n]; steps[n] valid
   rows per episode.  Writes met[QT_MET_ROWS][n] (TERM/VIOLATIONS rows are 0). */
int qt_metrics_from_arrays(const qt_criteria* crit, int64_t n, int32_t max_steps,
                           const double* qpos, const double* tpos, const double* actions,
                           const int32_t* steps, const double* last_time, double* met,
                           void* stream);

/* Batched DARE + gain (solve_dare, riccati_lqr.py:119-184) for the linearised
   hover model (build_linearized_system / build_augmented_lqi_system,
   riccati_lqr.py:187-316) with per-episode mass and cost matrices.
   n_state = 6 (LQR) or 9 (LQI).  q[n_state*n_state][m], r[16][m]: full matrices,
   SoA per element (row-major element index), m = number of problems.
   Validation follows _is_positive_semidefinite / _is_positive_definite
   (riccati_lqr.py:57-116).  Outputs: K[4*n_state][m] (SoA), P[n_state^2][m]
   (may be NULL), status[m] (enum qt_dare_status), iters[m] (may be NULL).
   structured != 0 asserts Q, R are diagonal (the per-axis decoupled fast
   path: one lane per (problem, axis)); 0 runs the dense one-wavefront solver. */
int qt_dare_batched(int32_t n_state, int64_t m, double dt, double gravity,
                    const double* mass, const double* q, const double* r,
                    int32_t structured, double* K, double* P, int8_t* status,
                    int32_t* iters, void* stream);

/* General dense DARE + gain (solve_dare, riccati_lqr.py:119-184) for arbitrary
   systems: n <= 16 states, p <= 8 inputs, m problems.  A[n*n][m'] and B[n*p][m']
   SoA with m' = m (ab_per_problem = 1) or 1 (shared); q[n*n][m], r[p*p][m].
   Outputs K[p*n][m], P[n*n][m] (may be NULL), status[m], iters[m] (may be NULL).
   No heuristic fallback: failed problems get K = 0 and a nonzero status. */
int qt_dare_dense(int32_t n, int32_t p, int64_t m, const double* A, const double* B,
                  int32_t ab_per_problem, const double* q, const double* r, double* K, double* P,
                  int8_t* status, int32_t* iters, void* stream);

/* EvaluationSummary reductions (utils/metrics.py:341-390) over met[QT_MET_ROWS][n],
   one workgroup, fixed order (bitwise reproducible).  out[11] (device):
   [sum ratio, sum mean_err, sum mean_effort, sum success, count,
    sum (ratio - mu_ratio)^2, sum (mean_err - mu_err)^2,
    max ratio, first argmax, min ratio, first argmin].  A second call with the
   means of the first gives the population std (np.std) without cancellation. */
int qt_summary(int64_t n, const double* met, double mu_ratio, double mu_err, double* out, void* stream);

/* qt_summary over `nparts` workgroups (1..4096): workgroup b reduces the
   contiguous episodes [b*c, (b+1)*c), c = ceil(n / nparts), into work[b][11],
   then one workgroup combines the parts in index order.  Same out[11];
   bitwise reproducible for a given (n, nparts).  work: DEVICE [nparts * 11]. */
int qt_summary_parts(int64_t n, const double* met, double mu_ratio, double mu_err, double* out, double* work,
                     int32_t nparts, void* stream);

/* ABI 5.  The EvaluationSummary sums in numpy's own order, so that means and
   stds equal np.mean / np.std (utils/metrics.py:380-384) bit for bit.
   numpy reduces a contiguous float64 vector in blocks of 8192 elements,
   adding each block's pairwise sum to a running total in block order; this
   writes the blocks' pairwise sums, out[rows][ceil(n / 8192)] (device); the
   caller adds them in order starting from 0.0.
   pass 0: rows = on_target_ratio, mean_err, mean_effort (np.mean);
   pass 1: rows = (on_target_ratio - mu_ratio)^2, (mean_err - mu_err)^2 as np.std
   forms them (subtract, then multiply; no fused multiply-add), with mu the
   pass-0 means. */
int qt_summary_numpy(int64_t n, const double* met, int32_t pass, double mu_ratio, double mu_err, double* out,
                     void* stream);

#ifdef __cplusplus
}
#endif

#endif /* QUADTRACK_H */
