// qt_rollout.hip — batched closed-loop kernels and their C ABI (include/quadtrack.h).
//
// One lane = one episode.  A launch walks `nsteps` closed-loop steps with the
// whole episode (12-state plant, target pattern constants, 4x6 / 4x9 gains,
// LQI integral, metric accumulators) resident in registers; HBM is touched
// only to load the state at the start of a chunk and to store it at the end.
// The rollout kernel itself lives in qt_kernels.hpp; its fast flavours are
// instantiated in qt_rollout_fast.hip.
// Reference functions: src/quadcopter_tracking/... of the reference repo.
#include "qt_kernels.hpp"
#include <atomic>
#include <cstring>
#include <map>
#include <mutex>

using namespace qtk;

namespace {

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
  double t = st.t[ep] + e.dt;
  const int term = constrain_terminate<true>(e, x, t);
  Target tg;
  target_state<true>(e, motion, pt, t, tg);
  const double q0 = x[0] - tg.p[0], q1 = x[1] - tg.p[1], q2 = x[2] - tg.p[2];
  const double err = sqrt(q0 * q0 + q1 * q1 + q2 * q2);
  const bool on = err <= e.target_radius;
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
    compute_action_pid<true>(c, G.k, hover, qp, qv, tg, obs[15 * n + ep], ff_of(b, c, ep), in, u, dg);  // row 15: time
  else
    sat = compute_action<KC, true, false>(c, G, hover, qp, qv, tg, ff_of(b, c, ep), in, u, dg);
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
  store_metrics(cr, load_acc(acc, n, e), t[e], met, n, e);
}

// numpy's summation order (np.add.reduce of a contiguous float64 vector; see
// np_block_sum_kernel below for the rules) restated for ONE thread summing K
// sequences at once over the same index range, values from val(i, v[K]).
constexpr int kNpBlock = 8192, kNpLeaf = 128, kNpMaxLeaves = 2 * kNpBlock / kNpLeaf;

__device__ __forceinline__ int np_half(int m) { return m / 2 - (m / 2) % 8; }

template <int K, class F>
__device__ void np_leaf_seq(const F& val, int lo, int len, double* res) {
#pragma clang fp contract(off)
  double v[K];
  if (len < 8) {
#pragma unroll
    for (int k = 0; k < K; ++k) res[k] = 0.0;
    for (int i = 0; i < len; ++i) {
      val(lo + i, v);
#pragma unroll
      for (int k = 0; k < K; ++k) res[k] += v[k];
    }
    return;
  }
  double r[8][K];
#pragma unroll
  for (int j = 0; j < 8; ++j) val(lo + j, r[j]);
  int i = 8;
  for (; i < len - len % 8; i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      val(lo + i + j, v);
#pragma unroll
      for (int k = 0; k < K; ++k) r[j][k] += v[k];
    }
#pragma unroll
  for (int k = 0; k < K; ++k) res[k] = ((r[0][k] + r[1][k]) + (r[2][k] + r[3][k])) + ((r[4][k] + r[5][k]) + (r[6][k] + r[7][k]));
  for (; i < len; ++i) {
    val(lo + i, v);
#pragma unroll
    for (int k = 0; k < K; ++k) res[k] += v[k];
  }
}

// pairwise sum of [lo0, lo0 + len), len <= kNpBlock: depth-first over the
// halves, each node = left + right
template <int K, class F>
__device__ void np_pairwise_seq(const F& val, int lo0, int len, double* out) {
  int fn[16], flo[16], fs[16], sp = 1;
  double fv[16][K], ret[K];
  bool have = false;  // a child of the top frame returned `ret`
  fn[0] = len, flo[0] = lo0, fs[0] = 0;
  while (sp > 0) {
    const int f = sp - 1;
    if (have) {
      if (fs[f] == 1) {
#pragma unroll
        for (int k = 0; k < K; ++k) fv[f][k] = ret[k];
        fs[f] = 2, have = false;
        const int h = np_half(fn[f]);
        flo[sp] = flo[f] + h, fn[sp] = fn[f] - h, fs[sp] = 0, ++sp;
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) ret[k] = fv[f][k] + ret[k];
        --sp;
      }
      continue;
    }
    if (fn[f] <= kNpLeaf) {
      np_leaf_seq<K>(val, flo[f], fn[f], ret);
      have = true, --sp;
      continue;
    }
    fs[f] = 1;
    flo[sp] = flo[f], fn[sp] = np_half(fn[f]), fs[sp] = 0, ++sp;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = ret[k];
}

// np.add.reduce of [0, len): blocks of kNpBlock, folded in order from 0.0
template <int K, class F>
__device__ void np_sum_seq(const F& val, int len, double* out) {
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = 0.0;
  for (int lo = 0; lo < len; lo += kNpBlock) {
    double b[K];
    np_pairwise_seq<K>(val, lo, len - lo < kNpBlock ? len - lo : kNpBlock, b);
#pragma unroll
    for (int k = 0; k < K; ++k) out[k] += b[k];
  }
}

// compute_episode_metrics over recorded arrays (utils/metrics.py:144-338):
// one lane per episode streams its rows for the max, on-target count and
// overshoot machine; the means and sums (np.mean / np.sum of the row norms,
// metrics.py:198-202, 330-332) are formed in numpy's order (np_sum_seq), with
// the norms as np.linalg.norm(axis=1) forms them (squares added in order, no
// fused multiply-add), so they equal the reference's bit for bit.
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
  // step s -> (err, err * err, |u|)
  auto vals = [&](int s, double* v) {
#pragma clang fp contract(off)
    const int64_t b3 = (int64_t)s * 3 * n + e, b4 = (int64_t)s * 4 * n + e;
    const double d0 = tpos[b3] - qpos[b3], d1 = tpos[b3 + n] - qpos[b3 + n], d2 = tpos[b3 + 2 * n] - qpos[b3 + 2 * n];
    const double err = sqrt((d0 * d0 + d1 * d1) + d2 * d2);
    const double u0 = act[b4], u1 = act[b4 + n], u2 = act[b4 + 2 * n], u3 = act[b4 + 3 * n];
    v[0] = err;
    v[1] = err * err;
    v[2] = sqrt(((u0 * u0 + u1 * u1) + u2 * u2) + u3 * u3);
  };
  double sums[3];
  np_sum_seq<3>(vals, S, sums);
  a.sum_e = sums[0], a.sum_e2 = sums[1], a.sum_u = sums[2];
  for (int s = 0; s < S; ++s) {
    double v[3];
    vals(s, v);
    const double err = v[0];
    if (!(err <= a.max_e) && !(a.max_e != a.max_e)) a.max_e = err;
    const bool on = err <= R;
    a.on_pre += on;
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

// ------------------------------------------- numpy-order sums (np.add.reduce)
// compute_evaluation_summary's np.mean / np.std (utils/metrics.py:382-384)
// reduce a contiguous float64 vector.  numpy (2.2, the reference's pinned
// dependency) walks it in buffer-sized blocks of kNpBlock elements and adds
// each block's pairwise sum to the running total in order; pairwise_sum
// (numpy/_core/src/umath/loops_utils.h.src): < 8 elements summed in order
// from 0.0; <= 128 elements as 8 strided accumulators, combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail in order; larger halves
// split at n/2 rounded down to a multiple of 8.  np.std sums (x - mean)^2
// formed as a subtraction and a product (no fused multiply-add).  One
// wavefront per block: lane 0 lists the leaves (<= 128 elements each, in
// order), the lanes sum them, lane 0 combines them along the same tree.  The
// blocks' running total is the host's (a few per million episodes).
struct NpRows {
  int row[3];
  double mu[3];
  int nrows, squares;
};

__device__ double np_leaf(const double* __restrict__ x, int lo, int len, bool sq, double mu) {
#pragma clang fp contract(off)
  auto val = [&](int i) {
    const double v = x[lo + i];
    if (!sq) return v;
    const double d = v - mu;
    return d * d;
  };
  if (len < 8) {
    double r = 0.0;
    for (int i = 0; i < len; ++i) r += val(i);
    return r;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = val(j);
  int i = 8;
  for (; i < len - len % 8; i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += val(i + j);
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < len; ++i) res += val(i);
  return res;
}

// grid (blocks, rows): out[row][block] = pairwise sum of that block
__global__ __launch_bounds__(64) void np_block_sum_kernel(int64_t n, const double* __restrict__ met, NpRows rs,
                                                          double* __restrict__ out) {
  __shared__ int leaf_lo[kNpMaxLeaves], leaf_len[kNpMaxLeaves];
  __shared__ double leaf_sum[kNpMaxLeaves];
  __shared__ int nleaves;
  const int64_t lo = (int64_t)blockIdx.x * kNpBlock;
  const int len = (int)(n - lo < kNpBlock ? n - lo : kNpBlock);
  const double* x = met + (int64_t)rs.row[blockIdx.y] * n + lo;
  if (threadIdx.x == 0) {  // leaves in order: depth-first, left half first
    int st_lo[16], st_len[16], sp = 1, k = 0;
    st_lo[0] = 0, st_len[0] = len;
    while (sp > 0) {
      --sp;
      const int a = st_lo[sp], m = st_len[sp];
      if (m <= kNpLeaf) {
        leaf_lo[k] = a, leaf_len[k] = m, ++k;
      } else {
        const int m2 = np_half(m);
        st_lo[sp] = a + m2, st_len[sp] = m - m2, ++sp;
        st_lo[sp] = a, st_len[sp] = m2, ++sp;
      }
    }
    nleaves = k;
  }
  __syncthreads();
  const bool sq = rs.squares != 0;
  const double mu = rs.mu[blockIdx.y];
  for (int k = threadIdx.x; k < nleaves; k += 64) leaf_sum[k] = np_leaf(x, leaf_lo[k], leaf_len[k], sq, mu);
  __syncthreads();
  if (threadIdx.x == 0) {  // the same tree, each node = left + right
    int fn[16], fs[16], sp = 1, k = 0;
    double fv[16], ret = 0.0;
    bool have = false;  // a child of the top frame returned `ret`
    fn[0] = len, fs[0] = 0;
    while (sp > 0) {
      const int f = sp - 1;
      if (have) {
        if (fs[f] == 1) {  // left done: keep it, descend right
          fv[f] = ret, fs[f] = 2, have = false;
          fn[sp] = fn[f] - np_half(fn[f]), fs[sp] = 0, ++sp;
        } else {
          ret = fv[f] + ret, --sp;
        }
        continue;
      }
      if (fn[f] <= kNpLeaf) {
        ret = leaf_sum[k++], have = true, --sp;
        continue;
      }
      fs[f] = 1;
      fn[sp] = np_half(fn[f]), fs[sp] = 0, ++sp;
    }
    out[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = ret;
  }
}

// The exact step (also the deferred pass after a fast flavour: it takes the
// waves the fast kernel left, see rollout_kernel).
struct ExactLaunch {
  template <int MOTION, int KC, bool FF, bool KS>
  static void run(int deferred, int grid, hipStream_t s, const qt_env_params& e, const qt_ctrl_params& c,
                  const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps, double* rec,
                  const LaunchConst& lc) {
    // the integrator known at compile time: no per-step branch on it (any
    // value but "euler" steps RK4, as integrate_closed reads it at run time)
    if (e.integrator == 1)
      launch<MOTION, KC, FF, KS, 1>(deferred, grid, s, e, c, cr, b, st, nsteps, rec, lc);
    else
      launch<MOTION, KC, FF, KS, 0>(deferred, grid, s, e, c, cr, b, st, nsteps, rec, lc);
  }
  template <int MOTION, int KC, bool FF, bool KS, int INTEG>
  static void launch(int deferred, int grid, hipStream_t s, const qt_env_params& e, const qt_ctrl_params& c,
                     const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps, double* rec,
                     const LaunchConst& lc) {
    // uniforms pinned in VGPRs (run_steps' PIN) while the launch holds at
    // most one wave per SIMD; a bigger one keeps two waves per SIMD resident
    const bool pin = (int64_t)grid * kBlock <= pin_lanes();
    if (rec || lc.reward) {
      if (pin)
        rollout_kernel<kExact, MOTION, KC, FF, KS, false, true, INTEG, true><<<grid, kBlock, 0, s>>>(
            e, c, cr, b, st, nsteps, rec, deferred, lc);
      else
        rollout_kernel<kExact, MOTION, KC, FF, KS, false, true, INTEG, false><<<grid, kBlock, 0, s>>>(
            e, c, cr, b, st, nsteps, rec, deferred, lc);
    } else if (pin) {  // no recording, no rewards: the loop without either pointer
      rollout_kernel<kExact, MOTION, KC, FF, KS, false, false, INTEG, true><<<grid, kBlock, 0, s>>>(
          e, c, cr, b, st, nsteps, nullptr, deferred, lc);
    } else {
      rollout_kernel<kExact, MOTION, KC, FF, KS, false, false, INTEG, false><<<grid, kBlock, 0, s>>>(
          e, c, cr, b, st, nsteps, nullptr, deferred, lc);
    }
  }
  // lanes of one wave per SIMD on the current device (compute units x 4
  // SIMDs x 64), queried once per device
  static int64_t pin_lanes() {
    static std::atomic<int> cache[64];  // compute units + 1 (0: not yet queried)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 65536;
    int v = dev >= 0 && dev < 64 ? cache[dev].load(std::memory_order_relaxed) : 0;
    if (v == 0) {
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 65536;
      v = cus + 1;
      if (dev >= 0 && dev < 64) cache[dev].store(v, std::memory_order_relaxed);
    }
    return (int64_t)(v - 1) * 4 * 64;
  }
};

// Deferred-wave flags, one device word per (device, stream): launches on one
// stream run in order, so a launch set's exact pass reads the word its own
// fast kernel wrote (or an older epoch: no deferred wave).  Epochs are unique
// per process, so a stale word never matches.  Allocated once per stream and
// kept for the process lifetime (8 bytes each).
std::atomic<unsigned long long> g_defer_epoch{0};

unsigned long long* defer_flag_for(hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, unsigned long long*> flags;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto it = flags.find({dev, s});
  if (it != flags.end()) return it->second;
  unsigned long long* f = nullptr;
  if (hipMalloc(&f, sizeof(*f)) != hipSuccess) return nullptr;
  // zeroed on `s` itself: ordered before the first fast launch that writes it
  // there (a null-stream memset is not ordered with non-blocking streams)
  if (hipMemsetAsync(f, 0, sizeof(*f), s) != hipSuccess) {  // epoch 0 is never issued
    (void)hipFree(f);
    return nullptr;
  }
  flags[{dev, s}] = f;
  return f;
}

// run_yaw0's DUAL threshold: kDualBelow, or QT_DUAL_BELOW from the environment
// (a test knob: 0 turns the clamping no-vote body off, so a test can compare
// the two loops' results bit for bit; read at each launch so that a test can
// switch it).  A value that is not a whole number in 0..62 is ignored (the
// default applies) and reported once on stderr, so a typo cannot silently
// switch the body off.
int dual_below() {
  const char* s = getenv("QT_DUAL_BELOW");
  if (!s || !*s) return kDualBelow;
  char* end = nullptr;
  const long x = strtol(s, &end, 10);
  if (*end != '\0' || x < 0 || x > 62) {
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true))
      fprintf(stderr, "quadtrack: ignoring QT_DUAL_BELOW=%s (not a whole number in 0..62)\n", s);
    return kDualBelow;
  }
  return (int)x;
}

// The pair-lane yaw-at-rest flavour (qt_pair.hpp): on unless QT_PAIR=0 (an
// A/B and test knob, read at each launch).
bool pair_on() {
  const char* s = getenv("QT_PAIR");
  return !(s && s[0] == '0' && s[1] == '\0');
}

// A yaw-at-rest launch the pair flavour covers: structured 6-column gains
// (shared or per episode), no feed-forward, no per-episode plant or hover
// thrust, one motion type for every episode, no rewards, the slots in episode
// order, and at most one wave per SIMD in pairs (2 n lanes; beyond that the
// pairs' ~170 instructions per step on two waves per SIMD lose to one wave of
// ~230: profiles/r06/split_step.jsonl).
bool pair_fits(int kc, bool ff, bool ks, bool grouped, int motion, const BatchDev& b, const LaunchConst& lc) {
  return pair_on() && !grouped && kc == 6 && ks && !ff && !b.plant_mass && !b.hover && !lc.reward &&
         motion >= QT_MOTION_STATIONARY && motion <= QT_MOTION_FIGURE8 && b.nseg == 0 && !b.order &&
         b.seg_check < 0 && b.slot0 == 0 && b.slot_end == b.n && b.n > 0 && 2 * b.n <= ExactLaunch::pin_lanes();
}

// The step flavour a launch can take (launch-level preconditions).
int flavor_for(int kc, bool ks, bool no_yaw, const qt_env_params& e, const qt_ctrl_params& c, const double* rec) {
  const bool fast = QT_ABLATE == 0 && rec == nullptr && fast_path_ok(e, c);
  if (fast && (ks || kc == 3 || no_yaw) && rate_bounded_ok(e, c)) return kYaw0;
  // Euler: the yaw-at-rest closed form only (make_rate_lin), no staged fast step
  if (QT_ABLATE == 0 && rec == nullptr && (ks || kc == 3 || no_yaw) && euler_yaw0_ok(e, c)) return kYaw0;
  return fast ? kFast : kExact;
}

// Stationary riders (BatchDev::ride_lo) in the one-launch grouped rollout:
// on unless QT_RIDERS=0 (an A/B and test knob, read at each launch).
bool riders_on() {
  const char* s = getenv("QT_RIDERS");
  return !(s && s[0] == '0' && s[1] == '\0');
}

// The waves of a one-launch grouped rollout (bg's segments: seg_motion,
// seg_lo = previous seg_end, seg_end) and their wave_end.  With riders, the
// first episodes of the stationary group fill the free lanes of every other
// group's last wave, in group order, and the stationary group's own waves
// start after them: a batch of N episodes then needs ceil(N / 64) waves
// whenever the stationary group can fill the other groups' gaps (config 5's
// 131,072-episode 8-GPU shard: 2,048 waves, the resident set at two waves per
// SIMD, instead of 2,050).  Riders need per-episode motions (batch->motion):
// the exact pass takes a deferred rider's motion from there.
int64_t grouped_waves(BatchDev& bg, bool riders) {
  int stat = -1;
  for (int i = 0; i < bg.nseg; ++i)
    if (bg.seg_motion[i] == QT_MOTION_STATIONARY && stat < 0) stat = i;
  if (riders && stat >= 0) {
    int64_t next = bg.seg_lo[stat], avail = bg.seg_end[stat] - bg.seg_lo[stat];
    for (int i = 0; i < bg.nseg; ++i) {
      if (i == stat) continue;
      const int64_t gap = (64 - (bg.seg_end[i] - bg.seg_lo[i]) % 64) % 64;
      const int64_t take = gap < avail ? gap : avail;
      bg.ride_lo[i] = next, bg.ride_cnt[i] = take;
      next += take, avail -= take;
    }
    bg.seg_lo[stat] = next;
  }
  int64_t waves = 0;
  for (int i = 0; i < bg.nseg; ++i) {
    waves += (bg.seg_end[i] - bg.seg_lo[i] + bg.ride_cnt[i] + 63) / 64;
    bg.wave_end[i] = waves;
  }
  return waves;
}

// One rollout launch set: the fast flavour the launch-level preconditions
// allow, then the exact kernel for the waves it left (or for everything).
// grouped: b covers a motion-grouped batch in wave-aligned segments and the
// yaw-at-rest flavour runs it in one launch (rollout_grouped_kernel), the exact
// pass with runtime motion over the same slot mapping.
// exact_motion: the exact pass's motion (default `motion`; -1 for a
// per-segment launch that checks batch->motion, BatchDev::seg_check).
int launch_rollout(int kc, bool ff, bool ks, bool no_yaw, int motion, int grid, hipStream_t s, const qt_env_params& e,
                   const qt_ctrl_params& c, const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps,
                   double* rec, bool grouped = false, double* reward = nullptr, const double* fresh_off = nullptr,
                   double* met = nullptr, int exact_motion = -2) {
  if (exact_motion == -2) exact_motion = motion;
  LaunchConst lc = make_launch_const(e);  // yaw-at-rest closed forms, target rotors
  lc.hz = make_horizon(e, c, lc.rl);       // the yaw-at-rest loop's safe horizon
  lc.hz.dual_below = dual_below();
  lc.reward = reward;
  lc.fresh_off = fresh_off, lc.met = met;  // qt_rollout_fresh: reset in the prologue, metrics in the epilogue
  const bool ks_eff = ks || kc == 3;
  const bool uni = !b.plant_mass && !b.hover && !b.k_per_episode;
  // rewards: the exact step accumulates them per step, a fast flavour from its
  // tracking-error sums (rollout_lane)
  const int flavor = flavor_for(kc, ks, no_yaw, e, c, rec);
  if (flavor != kExact) {
    lc.defer_flag = defer_flag_for(s);  // null (no flag: the exact pass tests every wave) if unavailable
    lc.epoch = g_defer_epoch.fetch_add(1, std::memory_order_relaxed) + 1;
    if (flavor == kYaw0 && pair_fits(kc, ff, ks, grouped, motion, b, lc))
      launch_pair(motion, (int)((2 * b.n + kBlock - 1) / kBlock), s, e, c, cr, b, st, nsteps, lc);
    else
      launch_fast(flavor, uni, grouped, kc, ff, ks_eff, motion, grid, s, e, c, cr, b, st, nsteps, lc);
    if (hipGetLastError() != hipSuccess) return QT_ELAUNCH;
    lc.fresh_off = nullptr;  // the fast kernel stored the reset state of the waves it left
  }
  dispatch_rollout<ExactLaunch>(kc, ff, ks_eff, grouped ? -1 : exact_motion, flavor, grid, s, e, c, cr, b, st, nsteps,
                                rec, lc);
  return check_launch();
}

// qt_rollout / qt_rollout_grouped / qt_rollout_fresh after validation:
// nseg == 0, one launch set over the batch; else motion groups (wave-aligned
// segments in one yaw-at-rest launch, or one launch set per group).
// fresh_off / met: a fresh pass (reset in the prologue, metrics rows in the
// epilogue).
int rollout_batch(const qt_env_params& e, const qt_ctrl_params& c, const qt_criteria& cr, const qt_batch* batch,
                  qt_state st, int nsteps, double* rec, int32_t nseg, const int32_t* seg_motion,
                  const int64_t* seg_end, hipStream_t s, const double* fresh_off = nullptr, double* met = nullptr) {
  BatchDev b = to_dev(batch);
  const bool ff = c.feedforward_enabled != 0 || batch->ff != nullptr;  // per-episode feed-forward: the FF kernels
  const bool ks = batch->k_structured != 0;
  const bool no_yaw = batch->k_no_yaw != 0;  // yaw-rate gains all zero: yaw stays at rest (dense K too)
  if (nseg == 0)
    return launch_rollout(batch->k_cols, ff, ks, no_yaw, batch->motion ? -1 : e.motion, grid_of(batch->n), s, e, c,
                          cr, b, st, nsteps, rec, false, nullptr, fresh_off, met);
  // a mixed segment (seg_motion -1: per-lane motion) has no loop in the grouped
  // kernel: such a batch takes one launch set per segment, the mixed ones with
  // the runtime-motion loop
  bool mixed = false;
  for (int32_t i = 0; i < nseg; ++i) mixed = mixed || seg_motion[i] < 0;
  if (!mixed && flavor_for(batch->k_cols, ks, no_yaw, e, c, rec) == kYaw0) {
    // every group in one launch, each starting at a wavefront boundary (BatchDev's
    // wave-aligned segments; both the fast kernel and its exact pass map slots so)
    BatchDev bg = b;
    int64_t prev_end = 0;
    bool fits = true;
    for (int32_t i = 0; i < nseg && fits; ++i) {
      const int64_t cnt = seg_end[i] - prev_end;
      if (cnt > 0) {
        if (bg.nseg == 8) {
          fits = false;
          break;
        }
        bg.seg_motion[bg.nseg] = (int8_t)seg_motion[i];
        bg.seg_lo[bg.nseg] = prev_end;
        bg.seg_end[bg.nseg] = seg_end[i];
        bg.ride_lo[bg.nseg] = bg.ride_cnt[bg.nseg] = 0;
        ++bg.nseg;
      }
      prev_end = seg_end[i];
    }
    const int64_t waves = fits ? grouped_waves(bg, QT_GROUPED_RIDERS && batch->motion != nullptr && riders_on()) : 0;
    if (fits) {
      // the grouped kernel has no fresh prologue / epilogue (rollout_lane's FRESH)
      if (fresh_off) reset_kernel<<<grid_of(batch->n), kBlock, 0, s>>>(e, b, fresh_off, st);
      const int rc = launch_rollout(batch->k_cols, ff, ks, no_yaw, -1, (int)((waves * 64 + kBlock - 1) / kBlock), s,
                                    e, c, cr, bg, st, nsteps, rec, true);
      if (rc != QT_OK || !met) return rc;
      metrics_kernel<<<grid_of(batch->n), kBlock, 0, s>>>(cr, batch->n, st.acc, st.t, met);
      return check_launch();
    }
  }
  // Per-episode motions given: the reset runs on its own with each episode's
  // motion (a per-segment launch's fresh prologue would form the reset state
  // of a mislabelled episode with its segment's motion before deferring it),
  // and the metrics after the last segment.
  const bool own_reset = fresh_off && batch->motion;
  if (own_reset) reset_kernel<<<grid_of(batch->n), kBlock, 0, s>>>(e, b, fresh_off, st);
  for (int32_t i = 0; i < nseg; ++i) {
    b.slot0 = i ? seg_end[i - 1] : 0;
    b.slot_end = seg_end[i];
    if (b.slot_end == b.slot0) continue;
    const int grid = grid_of(b.slot_end - b.slot0);
    // with per-episode motions given, a slot labelled with another motion than
    // its segment's goes to the exact pass, which takes each episode's own
    // motion (seg_check; the same guarantee as the one-launch grouped path)
    b.seg_check = batch->motion && seg_motion[i] >= 0 ? seg_motion[i] : -1;
    if (launch_rollout(batch->k_cols, ff, ks, no_yaw, seg_motion[i], grid, s, e, c, cr, b, st, nsteps, rec,
                       false, nullptr, own_reset ? nullptr : fresh_off, own_reset ? nullptr : met,
                       batch->motion ? -1 : seg_motion[i]) != QT_OK)
      return QT_ELAUNCH;
  }
  if (own_reset) {
    metrics_kernel<<<grid_of(batch->n), kBlock, 0, s>>>(cr, batch->n, st.acc, st.t, met);
    return check_launch();
  }
  return QT_OK;
}

}  // namespace

extern "C" {

int qt_abi_version(void) { return QT_ABI_VERSION; }

int qt_host_alloc(int64_t bytes, void** host, void** dev) {
  if (bytes <= 0 || !host || !dev) return QT_EINVAL;
  void* h = nullptr;
  // fine-grained (coherent) and mapped into every device's address space
  if (hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) !=
      hipSuccess)
    return QT_ELAUNCH;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return QT_ELAUNCH;
  }
  memset(h, 0, (size_t)bytes);
  *host = h, *dev = d;
  return 0;
}

int qt_host_free(void* host) { return host && hipHostFree(host) == hipSuccess ? 0 : QT_EINVAL; }

int qt_stream_sync(void* stream) {
  return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? 0 : QT_ELAUNCH;
}


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
  return rollout_batch(*env, *ctrl, *crit, batch, st, nsteps, rec, 0, nullptr, nullptr, (hipStream_t)stream);
}

int qt_rollout_rewards(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_criteria* crit,
                       const qt_batch* batch, qt_state st, int32_t nsteps, double* reward, void* stream) {
  if (!env || !ctrl || !crit || !batch || batch->n < 0 || nsteps < 0 || !batch->K) return QT_EINVAL;
  if (batch->k_cols != 3 && batch->k_cols != 6 && batch->k_cols != 9) return QT_EINVAL;
  if (batch->n == 0 || nsteps == 0) return QT_OK;
  if (!reward || !valid_state(st, batch->k_cols != 6)) return QT_EINVAL;
  const BatchDev b = to_dev(batch);
  const int motion = batch->motion ? -1 : env->motion;
  const bool ff = ctrl->feedforward_enabled != 0 || batch->ff != nullptr;
  return launch_rollout(batch->k_cols, ff, batch->k_structured != 0, batch->k_no_yaw != 0, motion, grid_of(batch->n),
                        (hipStream_t)stream, *env, *ctrl, *crit, b, st, nsteps, nullptr, false, reward);
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
    if (seg_end[i] < prev || seg_end[i] > batch->n || seg_motion[i] < -1 || seg_motion[i] > 4) return QT_EINVAL;
    prev = seg_end[i];
  }
  if (prev != batch->n) return QT_EINVAL;
  if (batch->n == 0 || nsteps == 0) return QT_OK;
  return rollout_batch(*env, *ctrl, *crit, batch, st, nsteps, rec, nseg, seg_motion, seg_end, (hipStream_t)stream);
}

int qt_rollout_fresh(const qt_env_params* env, const qt_ctrl_params* ctrl, const qt_criteria* crit,
                     const qt_batch* batch, const double* offset, qt_state st, int32_t nsteps, double* met, int32_t nseg,
                     const int32_t* seg_motion, const int64_t* seg_end, void* stream) {
  if (!env || !ctrl || !crit || !batch || batch->n < 0 || nsteps < 0 || !batch->K) return QT_EINVAL;
  if (batch->k_cols != 3 && batch->k_cols != 6 && batch->k_cols != 9) return QT_EINVAL;
  if (batch->n == 0) return QT_OK;  // empty: no per-episode pointer is read
  if (!offset || !met || !valid_state(st, batch->k_cols != 6)) return QT_EINVAL;
  if (nseg < 0 || (nseg > 0 && (!seg_motion || !seg_end))) return QT_EINVAL;
  int64_t prev = 0;
  for (int32_t i = 0; i < nseg; ++i) {
    if (seg_end[i] < prev || seg_end[i] > batch->n || seg_motion[i] < -1 || seg_motion[i] > 4) return QT_EINVAL;
    prev = seg_end[i];
  }
  if (nseg > 0 && prev != batch->n) return QT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (nsteps == 0) {  // nothing to run: the reset and the metrics of the reset state
    reset_kernel<<<grid_of(batch->n), kBlock, 0, s>>>(*env, to_dev(batch), offset, st);
    metrics_kernel<<<grid_of(batch->n), kBlock, 0, s>>>(*crit, batch->n, st.acc, st.t, met);
    return check_launch();
  }
  return rollout_batch(*env, *ctrl, *crit, batch, st, nsteps, nullptr, nseg, seg_motion, seg_end, s, offset, met);
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

int qt_summary_numpy(int64_t n, const double* met, int32_t pass, double mu_ratio, double mu_err, double* out,
                     void* stream) {
  if (n < 0 || (pass != 0 && pass != 1) || (n > 0 && (!met || !out))) return QT_EINVAL;
  if (n == 0) return QT_OK;
  const int64_t nb = (n + kNpBlock - 1) / kNpBlock;
  if (nb > (1ll << 30)) return QT_EINVAL;
  NpRows rs{};
  if (pass == 0) {
    rs.row[0] = QT_MET_ON_TARGET_RATIO, rs.row[1] = QT_MET_MEAN_ERR, rs.row[2] = QT_MET_MEAN_EFFORT;
    rs.nrows = 3, rs.squares = 0;
  } else {
    rs.row[0] = QT_MET_ON_TARGET_RATIO, rs.row[1] = QT_MET_MEAN_ERR;
    rs.mu[0] = mu_ratio, rs.mu[1] = mu_err;
    rs.nrows = 2, rs.squares = 1;
  }
  np_block_sum_kernel<<<dim3((unsigned)nb, rs.nrows), 64, 0, (hipStream_t)stream>>>(n, met, rs, out);
  return check_launch();
}

}  // extern "C"
