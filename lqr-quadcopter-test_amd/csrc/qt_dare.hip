// qt_dare.hip — batched discrete algebraic Riccati solves for the hover model.
//
// Reference: solve_dare (riccati_lqr.py:119-184) calls
// scipy.linalg.solve_discrete_are (QZ / Schur) once per controller.  Here the
// same equation  A'XA - X - A'XB (R + B'XB)^-1 B'XA + Q = 0  is solved for
// many independent problems with the structure-preserving doubling algorithm
// (SDA): quadratic convergence, 13-20 doublings for this model,
// followed by K = (R + B'PB)^-1 B'PA (riccati_lqr.py:181-182).
//
// Two kernels:
//  * dare_axis_kernel — Q and R diagonal (the q_pos / q_vel / q_int /
//    r_controls form, riccati_lqr.py:602-700, and every tuner candidate).  With
//    diagonal weights the linearised model (build_linearized_system 187-263,
//    build_augmented_lqi_system 266-316) splits into three independent
//    single-input axes (x <- pitch rate, y <- roll rate, z <- thrust) and a
//    yaw row that is identically zero.  One lane per (problem, axis): the
//    2x2 / 3x3 axis DARE lives entirely in registers.
//  * dare_row_kernel — arbitrary symmetric Q and R and general A, B (n <= 16,
//    p <= 8): one problem per 16-lane DPP row, row r of every matrix in lane
//    r's registers, products by DPP-broadcast FMAs (below).
// Both validate Q (PSD) and R (PD) like _is_positive_semidefinite /
// _is_positive_definite (riccati_lqr.py:57-116) and fall back to the
// heuristic gains of LQRController._compute_gains (controllers/__init__.py:
// 522-574) when invalid, as _create_fallback_controller does (747-777).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/quadtrack.h"

namespace {

constexpr int kMaxIter = 64;
constexpr double kTol = 1e-14;
// largest |W (W^-1 1) - 1| the row kernel's inverse without row exchanges may leave
constexpr double kInvCheck = 1e-10;

// heuristic (double-integrator) gains, K row for one axis
__device__ __forceinline__ void heuristic_axis(double qp, double qv, double r, double& kp, double& kv) {
  kp = sqrt(qp / r);
  kv = sqrt(2.0 * sqrt(qp / r) + qv / r);
}

// A failed problem's gain row r (r < p): zeros, or with `heuristic` the
// fallback gains (riccati_lqr.py:756-774, controllers/__init__.py:537-572) —
// row 0 (thrust) from the z axis, row 1 (roll) from -y, row 2 (pitch) from x.
// Each lane writes its own row, whole: one writer per K entry.
template <int N>
__device__ __forceinline__ void store_failed_gain_row(int r, int n, int p, int64_t m, int64_t pb, const double* q,
                                                      const double* rin, bool heuristic, double* K) {
  int c0 = -1;
  double kp = 0.0, kv = 0.0;
  if (heuristic && r < 3) {
    auto qd = [&](int i) { return q[(int64_t)(i * n + i) * m + pb]; };
    auto rd = [&](int i) { return rin[(int64_t)(i * p + i) * m + pb]; };
    const double rrate = (rd(1) + rd(2) + rd(3)) / 3.0;
    const int ax = 2 - r;
    heuristic_axis(qd(ax), qd(3 + ax), r == 0 ? rd(0) : rrate, kp, kv);
    if (r == 1) kp = -kp, kv = -kv;
    c0 = ax;
  }
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (j < n) K[(int64_t)(r * n + j) * m + pb] = j == c0 ? kp : (c0 >= 0 && j == c0 + 3 ? kv : 0.0);
}

// ------------------------------------------------------------ axis kernel

// N = 2 (LQR axis: pos, vel) or 3 (LQI axis: pos, vel, integral).
template <int N>
__device__ bool sda_axis(double dt, double b, double qp, double qv, double qi, double r, double* P, double* Krow,
                         int& iters) {
  // A = [[1, dt, 0], [0, 1, 0], [dt, 0, 1]] ; B = [0, b, 0]' ; G = B R^-1 B'
  double A[N][N], G[N][N], H[N][N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) A[i][j] = (i == j) ? 1.0 : 0.0, G[i][j] = 0.0, H[i][j] = 0.0;
  A[0][1] = dt;
  if (N == 3) A[2][0] = dt;
  G[1][1] = b * b / r;
  H[0][0] = qp;
  H[1][1] = qv;
  if (N == 3) H[2][2] = qi;
  int it = 0;
  bool conv = false;
  for (it = 1; it <= kMaxIter; ++it) {
    // W = I + G H ; solve W [Y1 | Y2] = [A | G] by Gauss-Jordan with partial pivoting
    double W[N][N], Y1[N][N], Y2[N][N];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        double s = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) s += G[i][k] * H[k][j];
        W[i][j] = s;
        Y1[i][j] = A[i][j];
        Y2[i][j] = G[i][j];
      }
#pragma unroll
    for (int k = 0; k < N; ++k) {
      int p = k;
      double best = fabs(W[k][k]);
#pragma unroll
      for (int i = k + 1; i < N; ++i)
        if (fabs(W[i][k]) > best) best = fabs(W[i][k]), p = i;
      if (best == 0.0) return false;
      if (p != k) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
          double t0 = W[k][j];
          W[k][j] = W[p][j];
          W[p][j] = t0;
          t0 = Y1[k][j];
          Y1[k][j] = Y1[p][j];
          Y1[p][j] = t0;
          t0 = Y2[k][j];
          Y2[k][j] = Y2[p][j];
          Y2[p][j] = t0;
        }
      }
      const double inv = 1.0 / W[k][k];
#pragma unroll
      for (int j = 0; j < N; ++j) W[k][j] *= inv, Y1[k][j] *= inv, Y2[k][j] *= inv;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        if (i == k) continue;
        const double f = W[i][k];
#pragma unroll
        for (int j = 0; j < N; ++j) W[i][j] -= f * W[k][j], Y1[i][j] -= f * Y1[k][j], Y2[i][j] -= f * Y2[k][j];
      }
    }
    // H' = H + A' H Y1 ; G' = G + A Y2 A' ; A' = A Y1   (symmetrised)
    double HY[N][N], T[N][N], nH[N][N], nG[N][N], nA[N][N];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        double s = 0.0, s2 = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) s += H[i][k] * Y1[k][j], s2 += Y2[i][k] * A[j][k];
        HY[i][j] = s;
        T[i][j] = s2;  // Y2 A'
      }
    double dn = 0.0, hn = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        double s = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) s += A[k][i] * HY[k][j], s2 += A[i][k] * T[k][j], s3 += A[i][k] * Y1[k][j];
        nH[i][j] = s;
        nG[i][j] = s2;
        nA[i][j] = s3;
      }
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const double h = H[i][j] + 0.5 * (nH[i][j] + nH[j][i]);
        dn += (h - H[i][j]) * (h - H[i][j]);
        hn += h * h;
        T[i][j] = h;
      }
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int j = 0; j < N; ++j) {
        G[i][j] = G[i][j] + 0.5 * (nG[i][j] + nG[j][i]);
        H[i][j] = T[i][j];
        A[i][j] = nA[i][j];
      }
    if (!isfinite(hn)) return false;
    if (sqrt(dn) <= kTol * sqrt(hn)) {
      conv = true;
      break;
    }
  }
  iters = it;
  if (!conv) return false;
  // K = (r + b^2 P11)^-1 b (P A)[1, :]   (B has its only entry on the velocity row)
  const double den = r + b * b * H[1][1];
  if (!(den != 0.0)) return false;
  // A is the ORIGINAL system matrix here
  double A0[N][N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) A0[i][j] = (i == j) ? 1.0 : 0.0;
  A0[0][1] = dt;
  if (N == 3) A0[2][0] = dt;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) s += H[1][k] * A0[k][j];
    Krow[j] = b * s / den;
  }
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) P[i * N + j] = H[i][j];
  return true;
}

// Lane layout: 4 lanes per problem; lane a = 0, 1, 2 solves axis x, y, z, lane
// 3 writes the zero yaw row and the status.
template <int NS>
__global__ __launch_bounds__(256) void dare_axis_kernel(int64_t m, double dt, double gravity,
                                                        const double* __restrict__ mass,
                                                        const double* __restrict__ q,
                                                        const double* __restrict__ r, double* K, double* P,
                                                        int8_t* status, int32_t* iters) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pb = gid >> 2;
  const int axis = (int)(gid & 3);
  if (pb >= m) return;  // m is whole problems: all 4 lanes of a problem leave together
  constexpr int NA = NS == 9 ? 3 : 2;
  auto qd = [&](int i) { return q[(int64_t)(i * NS + i) * m + pb]; };
  auto rd = [&](int i) { return r[(int64_t)(i * 4 + i) * m + pb]; };
  // _is_positive_semidefinite / _is_positive_definite on diagonal matrices:
  // the eigenvalues are the diagonal entries.
  bool qok = true, rok = true;
#pragma unroll
  for (int i = 0; i < NS; ++i) qok = qok && !(qd(i) < -1e-10);
#pragma unroll
  for (int i = 0; i < 4; ++i) rok = rok && !(rd(i) <= 1e-10);
  const int st = !qok ? QT_DARE_Q_NOT_PSD : (!rok ? QT_DARE_R_NOT_PD : QT_DARE_OK);
  const double mss = mass ? mass[pb] : 1.0;
  // axis -> input row of K (thrust 0, roll 1, pitch 2) and B entry (riccati_lqr.py:248-261)
  const int urow = axis == 0 ? 2 : (axis == 1 ? 1 : 0);
  const double b = axis == 0 ? gravity * dt : (axis == 1 ? -gravity * dt : (1.0 / mss) * dt);
  const int ax = axis < 3 ? axis : 0;
  auto kout = [&](int row, int col, double v) { K[(int64_t)(row * NS + col) * m + pb] = v; };
  const int idx[3] = {axis, 3 + axis, 6 + axis};
  int it = 0;
  int stat = st;
  double Pa[NA * NA], Kr[NA];
  if (axis < 3 && st == QT_DARE_OK) {
    if (!sda_axis<NA>(dt, b, qd(ax), qd(3 + ax), NS == 9 ? qd(6 + ax) : 0.0, rd(urow), Pa, Kr, it))
      stat = QT_DARE_NO_CONVERGE;
  }
  // One status per problem: the 4 lanes of a problem are adjacent in one
  // wavefront; any failing axis sends the whole problem to the fallback.
  const int base = (threadIdx.x & 63) & ~3;
  int s_all = stat, it_all = it;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int o = __shfl(stat, base + k, 64);
    const int oi = __shfl(it, base + k, 64);
    s_all = o > s_all ? o : s_all;
    it_all = oi > it_all ? oi : it_all;
  }
  if (axis == 3) {  // yaw rate has no column in B: zero row (riccati_lqr.py:255)
#pragma unroll
    for (int c = 0; c < NS; ++c) kout(3, c, 0.0);
    status[pb] = (int8_t)s_all;
    if (iters) iters[pb] = it_all;
    return;
  }
#pragma unroll
  for (int c = 0; c < NS; ++c) kout(urow, c, 0.0);  // cross-axis columns are structurally zero
  if (P) {
#pragma unroll
    for (int c = 0; c < NS; ++c) {
      P[(int64_t)(axis * NS + c) * m + pb] = 0.0;
      P[(int64_t)((3 + axis) * NS + c) * m + pb] = 0.0;
      if (NS == 9) P[(int64_t)((6 + axis) * NS + c) * m + pb] = 0.0;
    }
  }
  if (s_all == QT_DARE_OK) {
#pragma unroll
    for (int j = 0; j < NA; ++j) kout(urow, idx[j], Kr[j]);
    if (P) {
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NA; ++j) P[(int64_t)(idx[i] * NS + idx[j]) * m + pb] = Pa[i * NA + j];
    }
  } else {
    // heuristic fallback (controllers/__init__.py:537-572); r_rate = mean of the rate costs
    const double rrate = (rd(1) + rd(2) + rd(3)) / 3.0;
    double kp, kv;
    if (axis == 2) {
      heuristic_axis(qd(2), qd(5), rd(0), kp, kv);
      kout(0, 2, kp);
      kout(0, 5, kv);
    } else if (axis == 1) {
      heuristic_axis(qd(1), qd(4), rrate, kp, kv);
      kout(1, 1, -kp);
      kout(1, 4, -kv);
    } else {
      heuristic_axis(qd(0), qd(3), rrate, kp, kv);
      kout(2, 0, kp);
      kout(2, 3, kv);
    }
  }
}

constexpr int kMaxN = 16, kMaxP = 8;

#ifndef QT_DARE_ROWS_IN_FLIGHT
#define QT_DARE_ROWS_IN_FLIGHT 3  // rows of a product's right factor loaded ahead of their use
#endif

// ------------------------------------------------- dense-kernel helpers
//
// Group-level pieces of the dense SDA (dare_row_kernel): a group of GS lanes
// holds one problem, lane r row r of every n x n matrix; a product X Y reads
// X from the lane's own row and (row_times) Y's rows from LDS, the group's
// lanes reading the same addresses: broadcasts; Gauss-Jordan solves
// broadcast the pivot row through LDS; reductions (pivot search, norms) are
// DPP butterflies inside the group.  Every group lives in one wavefront, so
// its LDS hand-offs need only wave-level ordering (wave_sync): no workgroup
// barrier, no single-lane serial sections.  Sizes are compile-time (N, PP):
// 6 / 4 (hover LQR), 9 / 4 (hover LQI) and 16 / 8 (anything else), the
// runtime n x n / p x p problem zero-padded to them — padded rows and columns
// of A, B, Q, G, H are zero and R's padding is the identity, which decouples
// them exactly (every padded term is an exact +0 in each sum, pivots stay
// inside the real block).

// Wave-level ordering of LDS accesses: a wavefront's LDS operations complete
// in issue order, so a compiler barrier is all a hand-off inside one
// wavefront needs.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  asm volatile("" ::: "memory");
}

// A compiler-only memory barrier between two passes over the same LDS rows:
// without it the loads of the second pass are merged with the first's and
// every loaded row stays live in registers in between.
__device__ __forceinline__ void pass_break() { asm volatile("" ::: "memory"); }

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// DPP controls: quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror, row_mirror
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

// Butterfly over a group (GS = 8: a half row, 16: a row); every lane of the
// group ends with the same value (each step combines commutatively).
template <int GS, typename Op>
__device__ __forceinline__ double group_reduce(double v, Op op) {
  v = op(v, dpp_f64<kDppXor1>(v));
  v = op(v, dpp_f64<kDppXor2>(v));
  v = op(v, dpp_f64<kDppHalfMirror>(v));
  if (GS == 16) v = op(v, dpp_f64<kDppMirror>(v));
  return v;
}

template <int GS>
__device__ __forceinline__ double group_sum(double v) {
  return group_reduce<GS>(v, [](double a, double b) { return a + b; });
}

template <int GS>
__device__ __forceinline__ double group_max(double v) {
  return group_reduce<GS>(v, [](double a, double b) { return fmax(a, b); });
}

// This lane's group's bits of a wave ballot, at bit 0.
template <int GS>
__device__ __forceinline__ unsigned group_bits(uint64_t ballot) {
  const int base = (threadIdx.x & 63) & ~(GS - 1);
  return (unsigned)((ballot >> base) & ((1ull << GS) - 1));
}

template <int GS>
__device__ __forceinline__ bool group_all(bool v) {
  return group_bits<GS>(__ballot(!v)) == 0;
}

// In-LDS row-major matrix with row stride S (even: rows 16-byte aligned).
template <int S>
__device__ __forceinline__ double2 ld2(const double* m, int row, int col2) {
  return *reinterpret_cast<const double2*>(m + row * S + col2);
}

// Store this lane's row (NCOL entries) as row `row` of an LDS matrix.
template <int NCOL, int S>
__device__ __forceinline__ void st_row(double* m, int row, const double* v) {
#pragma unroll
  for (int j = 0; j + 1 < NCOL; j += 2) *reinterpret_cast<double2*>(m + row * S + j) = make_double2(v[j], v[j + 1]);
  if (NCOL & 1) m[row * S + NCOL - 1] = v[NCOL - 1];
}

// out[j] = sum_l x[l] Y[l][j] for j < NCOL: this lane's row x (K entries) times
// the LDS matrix Y (K x NCOL), in the order of the sum index.
template <int K, int NCOL, int S>
__device__ __forceinline__ void row_times(const double* x, const double* Y, double* out) {
#pragma unroll
  for (int j = 0; j < NCOL; ++j) out[j] = 0.0;
#pragma unroll
  for (int l = 0; l < K; ++l) {
#pragma unroll
    for (int j = 0; j + 1 < NCOL; j += 2) {
      const double2 y = ld2<S>(Y, l, j);
      out[j] += x[l] * y.x;
      out[j + 1] += x[l] * y.y;
    }
    if (NCOL & 1) out[NCOL - 1] += x[l] * Y[l * S + NCOL - 1];
    // keep the scheduler from hoisting every row's loads to the top (it would
    // hold all K rows in registers and halve the waves per SIMD)
    if ((l % QT_DARE_ROWS_IN_FLIGHT) == QT_DARE_ROWS_IN_FLIGHT - 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// Gauss-Jordan with partial pivoting on the group's NR x NC augmented system,
// row r of it in this lane's w (lanes r >= NR hold no row).  Rows are not
// swapped: the row chosen for pivot column k stays in its lane, which records
// k in *col.  The pivot row is normalised (multiplied by the reciprocal of
// its pivot) and broadcast through `piv` (LDS, NC doubles); every other row
// subtracts its multiple.  Ties take the lowest row.  Returns false (uniform
// over the group) when a pivot column is all zero.
template <int NR, int NC, int GS>
__device__ __forceinline__ bool group_gauss_jordan(double (&w)[NC], int r, double* piv, int* col) {
  bool used = r >= NR;
  *col = -1;
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const double cand = used ? -1.0 : fabs(w[k]);
    const double mx = group_max<GS>(cand);
    if (!(mx > 0.0)) return false;
    const int p = __builtin_ctz(group_bits<GS>(__ballot(!used && cand == mx)));
    if (r == p) {
      const double inv = 1.0 / w[k];
#pragma unroll
      for (int j = k; j < NC; ++j) w[j] *= inv;
      // columns < k of a pivot row are already zero: only k+1.. go out
#pragma unroll
      for (int j = (k + 1) & ~1; j + 1 < NC; j += 2) *reinterpret_cast<double2*>(piv + j) = make_double2(w[j], w[j + 1]);
      if (NC & 1) piv[NC - 1] = w[NC - 1];
      used = true;
      *col = k;
    }
    wave_sync();
    if (r != p) {  // lanes r >= NR eliminate too: their values are never used
      const double f = w[k];
#pragma unroll
      for (int j = (k + 1) & ~1; j + 1 < NC; j += 2) {
        const double2 v = *reinterpret_cast<const double2*>(piv + j);
        if (j > k) w[j] -= f * v.x;
        w[j + 1] -= f * v.y;
      }
      if (NC & 1) w[NC - 1] -= f * piv[NC - 1];
      w[k] = 0.0;
    }
    wave_sync();
  }
  return true;
}

// Row-per-lane Cholesky test of the group's N x N matrix c (row r in this
// lane): true iff every pivot is > 0, i.e. c is positive definite.  The
// column of each step goes through `colbuf` (LDS, N doubles).
template <int N, int GS>
__device__ __forceinline__ bool group_cholesky_pd(double (&c)[N], int r, double* colbuf) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (r < N) colbuf[r] = c[k];
    wave_sync();
    const double d = colbuf[k];
    ok = ok && d > 0.0;
    const double isd = 1.0 / sqrt(d);  // a definiteness test: the reciprocal's rounding is immaterial
    const double lr = c[k] * isd;
#pragma unroll
    for (int j = k + 1; j < N; ++j) c[j] -= lr * (colbuf[j] * isd);
    wave_sync();
  }
  return ok;
}

// np.allclose(M, M.T, atol=1e-8) (riccati_lqr.py:70-84, 100-116) for the
// group's N x N matrix, row r in this lane, via `buf` (LDS, N x S).
template <int N, int S, int GS>
__device__ __forceinline__ bool group_symmetric(const double (&row)[N], int r, double* buf) {
  if (r < N) st_row<N, S>(buf, r, row);
  wave_sync();
  bool ok = true;
  if (r < N) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double b = buf[j * S + r];
      ok = ok && fabs(row[j] - b) <= 1e-8 + 1e-5 * fabs(b);
    }
  }
  wave_sync();
  return group_all<GS>(ok);
}

// ------------------------------------------------------- row kernel
//
// The same dense SDA with its products in registers.  One problem per DPP
// row (16 lanes, 4 problems per wavefront), lane r holding row r of H, A and
// G for the whole solve.  A product X Y (row r: sum_l X[r][l] Y[l][:]) reads
// Y's row l from lane l of the row by DPP row_newbcast — the one DPP control
// gfx950 applies to 64-bit operands — so the doubling's eight products are
// register-to-register (no LDS traffic, no LDS latency); X Y' (row r, entry j:
// sum_l X[r][l] Y[j][l]) broadcasts lane j instead.  LDS is left with what
// moves data between lanes by a data-dependent or transposed pattern: the
// inversion's pivot rows (the pivot lane is chosen at run time), the
// inverse's row / column permutation (the pivoted fallback), and the
// transposes (A' for A' H Y1; the symmetrisations with QT_DARE_SYM).
// Validation, G = B R^-1 B' and the final gain are once per problem.

// v_fmac_f64 with its first source broadcast from lane l of each DPP row
// (row_newbcast: the DPP control gfx950 applies to 64-bit operands), N per
// block.  Written as inline asm because the compiler does not fold a 64-bit
// DPP move into the FMA (it would issue a v_mov_b64_dpp per product term).
// Hazards: a DPP source VGPR written by the VALU needs 2 wait states before
// the DPP read, an EXEC write 5, and the compiler's hazard recognizer does not
// look inside inline asm.  The first block of a product (NOP) opens with
// s_nop 4; the blocks after it follow the previous block's FMAs, which write
// only accumulators.  tests/test_dare_asm.py checks the built kernels: no DPP
// source written by a VALU instruction within 2 wait states and no EXEC write
// within 5 before any v_fmac_f64_dpp, and no block entered from a branch
// inside that window.
#define QT_FR(i) "v_fmac_f64_dpp %[a" #i "], %[y" #i "], %[x] row_newbcast:%[l] row_mask:0xf bank_mask:0xf\n\t"
#define QT_FC(i) "v_fmac_f64_dpp %[a" #i "], %[y], %[x] row_newbcast:" #i " row_mask:0xf bank_mask:0xf\n\t"
#define QT_A(i) [a##i] "+v"(a[i])
#define QT_Y(i) [y##i] "v"(y[i])
#define QT_FR6 QT_FR(0) QT_FR(1) QT_FR(2) QT_FR(3) QT_FR(4) QT_FR(5)
#define QT_FC6 QT_FC(0) QT_FC(1) QT_FC(2) QT_FC(3) QT_FC(4) QT_FC(5)
#define QT_A6 QT_A(0), QT_A(1), QT_A(2), QT_A(3), QT_A(4), QT_A(5)
#define QT_Y6 QT_Y(0), QT_Y(1), QT_Y(2), QT_Y(3), QT_Y(4), QT_Y(5)
#define QT_FR9 QT_FR6 QT_FR(6) QT_FR(7) QT_FR(8)
#define QT_FC9 QT_FC6 QT_FC(6) QT_FC(7) QT_FC(8)
#define QT_A9 QT_A6, QT_A(6), QT_A(7), QT_A(8)
#define QT_Y9 QT_Y6, QT_Y(6), QT_Y(7), QT_Y(8)
#define QT_FR16 QT_FR9 QT_FR(9) QT_FR(10) QT_FR(11) QT_FR(12) QT_FR(13) QT_FR(14) QT_FR(15)
#define QT_FC16 QT_FC9 QT_FC(9) QT_FC(10) QT_FC(11) QT_FC(12) QT_FC(13) QT_FC(14) QT_FC(15)
#define QT_A16 QT_A9, QT_A(9), QT_A(10), QT_A(11), QT_A(12), QT_A(13), QT_A(14), QT_A(15)
#define QT_Y16 QT_Y9, QT_Y(9), QT_Y(10), QT_Y(11), QT_Y(12), QT_Y(13), QT_Y(14), QT_Y(15)

// one asm block, with or without the s_nop 4 in front (NOP)
#define QT_BLOCK(NOP, BODY, OUTS, INS) \
  do {                                  \
    if constexpr (NOP)                  \
      asm("s_nop 4\n\t" BODY : OUTS : INS); \
    else                                \
      asm(BODY : OUTS : INS);           \
  } while (0)
#define QT_COMMA ,

// a[j] += Y[L][j] x for j < N, row L of Y in lane L's y
template <int N, int L, bool NOP>
__device__ __forceinline__ void fmac_row(double* a, const double* y, double x) {
  static_assert(N == 6 || N == 9 || N == 16, "row block sizes");
  if constexpr (N == 6)
    QT_BLOCK(NOP, QT_FR6, QT_A6, QT_Y6 QT_COMMA[x] "v"(x) QT_COMMA[l] "n"(L));
  else if constexpr (N == 9)
    QT_BLOCK(NOP, QT_FR9, QT_A9, QT_Y9 QT_COMMA[x] "v"(x) QT_COMMA[l] "n"(L));
  else
    QT_BLOCK(NOP, QT_FR16, QT_A16, QT_Y16 QT_COMMA[x] "v"(x) QT_COMMA[l] "n"(L));
}

// a[l] += Y[l][j] x for l < N, entry j of row l of Y in lane l's yj
template <int N, bool NOP>
__device__ __forceinline__ void fmac_col(double* a, double yj, double x) {
  static_assert(N == 6 || N == 9 || N == 16, "column block sizes");
  if constexpr (N == 6)
    QT_BLOCK(NOP, QT_FC6, QT_A6, [y] "v"(yj) QT_COMMA[x] "v"(x));
  else if constexpr (N == 9)
    QT_BLOCK(NOP, QT_FC9, QT_A9, [y] "v"(yj) QT_COMMA[x] "v"(x));
  else
    QT_BLOCK(NOP, QT_FC16, QT_A16, [y] "v"(yj) QT_COMMA[x] "v"(x));
}

// acc[j] += sum_l x[l] Y[l][j] (l, j < N), row l of Y in lane l's y
template <int N, int L = 0>
__device__ __forceinline__ void bmul_acc(const double* x, const double* y, double* acc) {
  if constexpr (L < N) {
    fmac_row<N, L, L == 0>(acc, y, x[L]);
    bmul_acc<N, L + 1>(x, y, acc);
  }
}

// out = x Y (row r of the product)
template <int N>
__device__ __forceinline__ void bmul(const double* x, const double* y, double* out) {
#pragma unroll
  for (int j = 0; j < N; ++j) out[j] = 0.0;
  bmul_acc<N>(x, y, out);
}

// out = x Y' (out[l] = sum_j x[j] Y[l][j]), row l of Y in lane l's y
template <int N, int J = 0>
__device__ __forceinline__ void bmul_t_acc(const double* x, const double* y, double* out) {
  if constexpr (J < N) {
    fmac_col<N, J == 0>(out, y[J], x[J]);
    bmul_t_acc<N, J + 1>(x, y, out);
  }
}

template <int N>
__device__ __forceinline__ void bmul_t(const double* x, const double* y, double* out) {
#pragma unroll
  for (int j = 0; j < N; ++j) out[j] = 0.0;
  bmul_t_acc<N>(x, y, out);
}

// 1 / x to within an ulp or so (v_rcp_f64 and two Newton steps): x finite, nonzero
__device__ __forceinline__ double recip_newton(double x) {
  double y = __builtin_amdgcn_rcp(x);
  y = fma(y, fma(-x, y, 1.0), y);
  return fma(y, fma(-x, y, 1.0), y);
}

// Lane L's value of each DPP row (row_newbcast), as inline asm with its own
// s_nop 4 (the source was written by inline-asm FMAs just before, which the
// compiler's hazard recognizer does not see)
template <int L>
__device__ __forceinline__ double row_bcast_asm(double v) {
  double o;
  asm("s_nop 4\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(o) : "v"(v), "n"(L));
  return o;
}

// a[j] += A[K][j] x for j < N, row K of A in lane K's a: the elimination of
// row K from every row in place (the DPP reads lane K's register before the
// FMA writes the lane's own), one asm block so that nothing comes between its
// FMAs
#define QT_FS(i) "v_fmac_f64_dpp %[a" #i "], %[a" #i "], %[x] row_newbcast:%[l] row_mask:0xf bank_mask:0xf\n\t"
#define QT_FS6 QT_FS(0) QT_FS(1) QT_FS(2) QT_FS(3) QT_FS(4) QT_FS(5)
#define QT_FS9 QT_FS6 QT_FS(6) QT_FS(7) QT_FS(8)
#define QT_FS16 QT_FS9 QT_FS(9) QT_FS(10) QT_FS(11) QT_FS(12) QT_FS(13) QT_FS(14) QT_FS(15)
template <int N, int K>
__device__ __forceinline__ void elim_row(double* a, double x) {
  static_assert(N == 6 || N == 9 || N == 16, "row block sizes");
  if constexpr (N == 6)
    asm("s_nop 4\n\t" QT_FS6 : QT_A6 : [x] "v"(x), [l] "n"(K));
  else if constexpr (N == 9)
    asm("s_nop 4\n\t" QT_FS9 : QT_A9 : [x] "v"(x), [l] "n"(K));
  else
    asm("s_nop 4\n\t" QT_FS16 : QT_A16 : [x] "v"(x), [l] "n"(K));
}

// acc += sum_l Y[l] x[l] (l < N), Y[l] lane l's y: a dot product whose
// right factor is spread over the row's lanes
template <int N, int L = 0>
__device__ __forceinline__ void dot_lanes(double& acc, double y, const double* x) {
  if constexpr (L < N) {
    if constexpr (L == 0)
      asm("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
          : "+v"(acc) : "v"(y), "v"(x[L]), "n"(L));
    else
      asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
          : "+v"(acc) : "v"(y), "v"(x[L]), "n"(L));
    dot_lanes<N, L + 1>(acc, y, x);
  }
}

// In-place Gauss-Jordan inversion of the group's N x N matrix W (row r in
// this lane's w; lanes r >= N hold zero rows) WITHOUT pivoting: step k
// eliminates with row k itself, broadcast from lane k by DPP (no LDS, no
// branch).  Normalisation is deferred: row k stays scaled by its pivot p_k
// through the later steps (every update is linear in it) and each lane
// divides its row by its own pivot at the end.  Rows come out in natural
// order.  The caller checks the result (W^-1 without pivoting can lose
// accuracy on a matrix that needs row exchanges) and falls back to
// row_gj_invert.
template <int N, int K = 0>
__device__ __forceinline__ void row_gj_nopiv(double (&w)[N], int r, double& myinv) {
  if constexpr (K < N) {
    const double inv = recip_newton(row_bcast_asm<K>(w[K]));
    const double nf = r == K ? 0.0 : -(w[K] * inv);  // minus the multiple of row K in this row
    if (r == K) myinv = inv;
    elim_row<N, K>(w, nf);     // (column K: w[K] - p_K w[K] / p_K, replaced below)
    w[K] = r == K ? 1.0 : nf;  // the inverse's column K (row K: p_K / p_K, scaled at the end)
    row_gj_nopiv<N, K + 1>(w, r, myinv);
  }
}

// Group maximum of a 32-bit unsigned key over the 16 lanes of a DPP row
// (each step's DPP move fuses into v_max_u32).
__device__ __forceinline__ unsigned row_max_u32(unsigned v) {
  v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, kDppXor1, 0xf, 0xf, false));
  v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, kDppXor2, 0xf, 0xf, false));
  v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, kDppHalfMirror, 0xf, 0xf, false));
  v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, kDppMirror, 0xf, 0xf, false));
  return v;
}

// In-place Gauss-Jordan inversion with partial pivoting of the group's
// NR x NR matrix W (one problem per 16-lane DPP row), row r in this lane's w
// (lanes r >= NR hold no row).  Rows are not swapped: pk[k] records the lane
// whose row became pivot k (the same in every lane of the group) and *col the
// pivot this lane's row became; on return the lanes hold S with
// W^-1[a][pk[k]] = S[pk[a]][k].  The pivot is the row whose |w[k]| has the
// largest high word (exponent and the top 20 mantissa bits: partial pivoting
// to 2^-20, ties to the lowest row), found by a 32-bit DPP maximum; the pivot
// row is scaled by a Newton reciprocal and broadcast through `piv` (LDS).
// Returns false (uniform over the group) when a pivot column is all zero.
template <int NR>
__device__ __forceinline__ bool row_gj_invert(double (&w)[NR], int r, double* piv, int (&pk)[NR], int* col) {
  bool used = r >= NR;
  *col = -1;
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const unsigned key = used ? 0u : ((unsigned)__double2hiint(w[k]) & 0x7fffffffu);
    const unsigned mx = row_max_u32(key);
    if (mx == 0u) return false;
    const int p = __builtin_ctz(group_bits<16>(__ballot(!used && key == mx)));
    pk[k] = p;
    if (r == p) {
      const double inv = recip_newton(w[k]);
#pragma unroll
      for (int j = 0; j < NR; ++j) w[j] = j == k ? inv : w[j] * inv;
      st_row<NR, NR + (NR & 1)>(piv, 0, w);
      used = true;
      *col = k;
    }
    wave_sync();
    if (r != p) {
      const double f = w[k];
#pragma unroll
      for (int j = 0; j + 1 < NR; j += 2) {
        const double2 v = *reinterpret_cast<const double2*>(piv + j);
        w[j] = j == k ? -f * v.x : w[j] - f * v.x;
        w[j + 1] = j + 1 == k ? -f * v.y : w[j + 1] - f * v.y;
      }
      if (NR & 1) w[NR - 1] = NR - 1 == k ? -f * piv[NR - 1] : w[NR - 1] - f * piv[NR - 1];
    }
    wave_sync();
  }
  return true;
}

// Column r of the group's N x N matrix whose row r is this lane's `row`,
// through the LDS matrix `buf` (stride S).
template <int N, int S>
__device__ __forceinline__ void lds_transpose(double* buf, const double (&row)[N], int r, int rc, double (&col)[N]) {
  if (r < N) st_row<N, S>(buf, r, row);
  wave_sync();
#pragma unroll
  for (int l = 0; l < N; ++l) col[l] = buf[l * S + rc];
  wave_sync();
}

// 1: symmetrise H and G after every doubling, (M + M') / 2, as round 3's LDS
// kernel did; 0: add M as computed (A' (H W^-1) A and A (W^-1 G) A' are symmetric in
// exact arithmetic: H W^-1 = (I + H G)^-1 H), which spares two LDS transposes
#ifndef QT_DARE_SYM
#define QT_DARE_SYM 0
#endif

// the pivoted inversion behind the row kernel's residual check (0 only for
// instruction counts of the common path)
#ifndef QT_DARE_FALLBACK
#define QT_DARE_FALLBACK 1
#endif

#ifndef QT_DARE_ROW_WAVES
#define QT_DARE_ROW_WAVES 2  // minimum waves per SIMD the row kernel's register allocation must allow
#endif

template <int N, int PP>
struct RowDims {
  static constexpr int GS = 16;
  static constexpr int kProblemsPerWave = 4;
  static constexpr int S = (N + 1) & ~1;
  static constexpr int MAT = N * S;
  static constexpr int RAW = 4 * MAT;  // H (the gain phase's P), A, Y, T
  static constexpr int PROB = RAW + ((8 - RAW % 32) + 32) % 32;
  static_assert(PP + N <= MAT && N <= GS && PP <= GS, "row layout");
};

template <int N, int PP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(QT_DARE_ROW_WAVES, 8))) void dare_row_kernel(
    int n, int p, int64_t m, const double* __restrict__ Ain, const double* __restrict__ Bin, int ab_per_problem,
    double dt, double gravity, const double* __restrict__ mass, const double* __restrict__ q,
    const double* __restrict__ rin, int fallback, double* K, double* P, int8_t* status, int32_t* iters) {
  using D = RowDims<N, PP>;
  constexpr int GS = D::GS, S = D::S;
  __shared__ __attribute__((aligned(16))) double lds[D::kProblemsPerWave * D::PROB];
  const int lane = threadIdx.x & 63, g = lane / GS, r = lane % GS;
  const int rc = r < N ? r : N - 1, rp = r < PP ? r : PP - 1;
  const int64_t pb = (int64_t)blockIdx.x * D::kProblemsPerWave + g;
  const bool valid = pb < m;  // uniform over the group
  double* Hl = lds + g * D::PROB;
  double* Al = Hl + D::MAT;
  double* Yl = Al + D::MAT;
  double* Tl = Yl + D::MAT;
  const bool hover = Ain == nullptr;
  const double mss = (valid && mass) ? mass[pb] : 1.0;
  const int64_t abm = ab_per_problem ? m : 1, abj = ab_per_problem ? pb : 0;
  const bool real = valid && r < n;

  auto a_in = [&](int j) -> double {
    if (!(real && j < n)) return 0.0;
    if (!hover) return Ain[(int64_t)(r * n + j) * abm + abj];
    double a = (r == j) ? 1.0 : 0.0;
    if (r < 3 && j == r + 3) a = dt;             // A_d = I + A_c dt (riccati_lqr.py:260)
    if (n == 9 && r >= 6 && j == r - 6) a = dt;  // integral rows (308)
    return a;
  };
  auto b_in = [&](int c) -> double {
    if (!(real && c < p)) return 0.0;
    if (!hover) return Bin[(int64_t)(r * p + c) * abm + abj];
    if (r == 5 && c == 0) return 1.0 / mss * dt;  // riccati_lqr.py:250,261
    if (r == 4 && c == 1) return -gravity * dt;   // 252
    if (r == 3 && c == 2) return gravity * dt;    // 254
    return 0.0;
  };
  auto r_in = [&](int c) -> double {
    return (valid && r < p && c < p) ? rin[(int64_t)(r * p + c) * m + pb] : (r == c ? 1.0 : 0.0);
  };

  // ---- validation (_is_positive_semidefinite / _is_positive_definite,
  // riccati_lqr.py:57-116): symmetric within np.allclose, then the
  // eigenvalue bounds as Cholesky tests: min eig(Q) >= -1e-10 <=> Q + 1e-10 I
  // positive definite, min eig(R) > 1e-10 <=> R - 1e-10 I positive definite
  // (the same decisions but on the boundary itself, to rounding)
  double hr[N];  // H = Q to start
#pragma unroll
  for (int j = 0; j < N; ++j) hr[j] = (real && j < n) ? q[(int64_t)(r * n + j) * m + pb] : 0.0;
  int st = QT_DARE_OK;
  {
    bool qok = group_symmetric<N, S, GS>(hr, r, Tl);
    double c[N];
#pragma unroll
    for (int j = 0; j < N; ++j) c[j] = hr[j] + ((r == j) ? 1e-10 : 0.0);
    qok = group_cholesky_pd<N, GS>(c, r, Tl) && qok;
    double rr[PP];
#pragma unroll
    for (int j = 0; j < PP; ++j) rr[j] = r_in(j);
    bool rok = group_symmetric<PP, S, GS>(rr, r, Tl);
#pragma unroll
    for (int j = 0; j < PP; ++j) rr[j] -= (r == j) ? 1e-10 : 0.0;
    rok = group_cholesky_pd<PP, GS>(rr, r, Tl) && rok;
    st = !qok ? QT_DARE_Q_NOT_PSD : (!rok ? QT_DARE_R_NOT_PD : QT_DARE_OK);
  }

  // ---- G = B R^-1 B': X = R^-1 B' by Gauss-Jordan on [R | B'] (lanes r < PP), G = B X
  double gr[N];
  int it = 0;
  bool conv = false;
  {
    double br[PP];
#pragma unroll
    for (int c = 0; c < PP; ++c) br[c] = b_in(c);
    if (r < N) st_row<PP, S>(Yl, r, br);
    wave_sync();
    double w[PP + N];
#pragma unroll
    for (int c = 0; c < PP; ++c) w[c] = r_in(c);
#pragma unroll
    for (int j = 0; j < N; ++j) w[PP + j] = r < PP ? Yl[j * S + rp] : 0.0;
    wave_sync();
    int col;
    const bool ok = group_gauss_jordan<PP, PP + N, GS>(w, r, Tl, &col);
    if (st == QT_DARE_OK && !ok) st = QT_DARE_SINGULAR;
    if (col >= 0) st_row<N, S>(Yl, col, w + PP);
    wave_sync();
    row_times<PP, N, S>(br, Yl, gr);
    wave_sync();
  }
  double ar[N];
#pragma unroll
  for (int j = 0; j < N; ++j) ar[j] = a_in(j);
  // the last doubling's |dH|_F^2 / |H|_F^2; NaN before the first doubling, so
  // the quadratic test below always compares two measured changes (a first
  // change that happens to be small proves nothing about the convergence rate)
  double rel_prev = __builtin_nan("");

  // ---- doublings: W = I + G H ; Winv = W^-1 ; Y1 = Winv A ; Y2 = Winv G ;
  // H += sym(A' H Y1) ; G += sym(A Y2 A') ; A = A Y1, until |dH|_F <= tol |H|_F
  while (true) {
    const bool act = valid && st == QT_DARE_OK && !conv && it < kMaxIter;  // uniform over the group
    if (__ballot(act) == 0) break;
    if (!act) continue;
    ++it;
    double wi[N];
    {
      double w[N], w0[N];
#pragma unroll
      for (int j = 0; j < N; ++j) w[j] = j == r ? 1.0 : 0.0;
      bmul_acc<N>(gr, hr, w);  // W = I + G H
#pragma unroll
      for (int j = 0; j < N; ++j) w0[j] = w[j];
      // W^-1 without row exchanges (row_gj_nopiv), checked by the residuals of
      // W (W^-1 v) = v for two probes, v = 1 and the alternating v = (1, -1,
      // 1, ...) (an error of W^-1 that cancels across a row against one probe
      // shows against the other); a problem that misses either takes
      // row_gj_invert's
      double myinv = 1.0, srow = 0.0, salt = 0.0;
      row_gj_nopiv<N>(w, r, myinv);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        w[j] *= myinv;
        srow += w[j];
        salt += (j & 1) ? -w[j] : w[j];
      }
      double res = -1.0, res2 = (r & 1) ? 1.0 : -1.0;  // minus the probes' entry r
      dot_lanes<N>(res, srow, w0);
      dot_lanes<N>(res2, salt, w0);
      const bool gbad = !group_all<GS>(!(r < N) || (fabs(res) <= kInvCheck && fabs(res2) <= kInvCheck));
      if (QT_DARE_FALLBACK && __ballot(gbad) != 0) {
        int col, pk[N];
        double w2[N];
#pragma unroll
        for (int j = 0; j < N; ++j) w2[j] = w0[j];
        const bool ok = row_gj_invert<N>(w2, r, Tl, pk, &col);
        if (ok) {
          // W^-1[a][pk[k]] = S[pk[a]][k]: lane pk[a] (col = a) scatters its row to row a
          if (col >= 0) {
#pragma unroll
            for (int k = 0; k < N; ++k) Tl[col * S + pk[k]] = w2[k];
          }
          wave_sync();
#pragma unroll
          for (int j = 0; j < N; ++j) w2[j] = Tl[rc * S + j];
          wave_sync();
        }
        if (gbad) {
          if (!ok) st = QT_DARE_SINGULAR;
#pragma unroll
          for (int j = 0; j < N; ++j) w[j] = w2[j];
        }
      }
      if (st != QT_DARE_OK) continue;
#pragma unroll
      for (int j = 0; j < N; ++j) wi[j] = w[j];
    }
    // Y2 = Winv G ; Y1 = Winv A ; T2 = Y2 A' ; T = H Y1 ; A_next = A Y1
    double y1[N], y2[N], t[N], t2[N], an[N], u[N];
    bmul<N>(wi, gr, y2);
    bmul<N>(wi, ar, y1);
    bmul_t<N>(y2, ar, t2);
    bmul<N>(hr, y1, t);
    bmul<N>(ar, y1, an);
    // M = A' T ; H' = H + M (QT_DARE_SYM: + (M + M') / 2)
    lds_transpose<N, S>(Al, ar, r, rc, u);  // column r of A
    double mm[N];
    bmul<N>(u, t, mm);
    double dn = 0.0, hn = 0.0;
    if (QT_DARE_SYM) {
      lds_transpose<N, S>(Tl, mm, r, rc, u);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const double hnew = hr[j] + 0.5 * (mm[j] + u[j]);
        dn += (hnew - hr[j]) * (hnew - hr[j]);
        hn += hnew * hnew;
        hr[j] = hnew;
      }
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        hr[j] += mm[j];
        dn = fma(mm[j], mm[j], dn);
        hn = fma(hr[j], hr[j], hn);
      }
    }
    dn = group_sum<GS>(r < N ? dn : 0.0);
    hn = group_sum<GS>(r < N ? hn : 0.0);
    // |dH|_F <= tol |H|_F, squared (tol^2 = 1e-28: no square roots); or, in
    // the doubling's quadratic regime (this change at most 4x the square of
    // the last one, relative to |H|), a change below 1e-8 |H|: the next
    // change, the error left in H, is then below ~1e-16 |H| (one doubling
    // saved; a linearly converging problem, marginal modes with q_int = 0,
    // never passes the quadratic test and runs to tol)
    const double rel = dn / hn;
    const bool quad = rel <= 1e-16 && rel <= 16.0 * rel_prev * rel_prev;
    rel_prev = rel;
    const int flag = !isfinite(hn) ? -1 : ((dn <= kTol * kTol * hn || quad) ? 1 : 0);
    // M = A T2 ; G' = G + M (QT_DARE_SYM: + (M + M') / 2)
    if (QT_DARE_SYM) {
      bmul<N>(ar, t2, mm);
      lds_transpose<N, S>(Yl, mm, r, rc, u);
#pragma unroll
      for (int j = 0; j < N; ++j) gr[j] += 0.5 * (mm[j] + u[j]);
    } else {
      bmul_acc<N>(ar, t2, gr);
    }
#pragma unroll
    for (int j = 0; j < N; ++j) ar[j] = an[j];
    if (flag < 0) st = QT_DARE_NO_CONVERGE;
    if (flag == 1) conv = true;
  }
  if (valid && st == QT_DARE_OK && !conv) st = QT_DARE_NO_CONVERGE;
  if (r < N) st_row<N, S>(Hl, r, hr);  // P for the gain phase and the output
  wave_sync();

  // ---- K = (R + B'PB)^-1 B'PA (riccati_lqr.py:181-182): T = B'P (lanes r < PP),
  // W = R + T B, Y = T A0, solve W K = Y
  if (valid && st == QT_DARE_OK) {
    if (r < N) {
      double br[PP], a0[N];
#pragma unroll
      for (int c = 0; c < PP; ++c) br[c] = b_in(c);
#pragma unroll
      for (int j = 0; j < N; ++j) a0[j] = a_in(j);
      st_row<PP, S>(Yl, r, br);
      st_row<N, S>(Al, r, a0);
    }
    wave_sync();
    double bc[N], tr[N];
#pragma unroll
    for (int l = 0; l < N; ++l) bc[l] = Yl[l * S + rp];
    row_times<N, N, S>(bc, Hl, tr);
    double w[PP + N];
#pragma unroll
    for (int c = 0; c < PP; ++c) {
      double s = r_in(c);
#pragma unroll
      for (int l = 0; l < N; ++l) s += tr[l] * Yl[l * S + c];
      w[c] = s;
    }
    row_times<N, N, S>(tr, Al, w + PP);
    wave_sync();
    int col;
    if (!group_gauss_jordan<PP, PP + N, GS>(w, r, Tl, &col)) st = QT_DARE_SINGULAR;
    if (st == QT_DARE_OK && col >= 0 && col < p) {
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (j < n) K[(int64_t)(col * n + j) * m + pb] = w[PP + j];
    }
  }
  if (!valid) return;
  const bool ok = st == QT_DARE_OK;
  if (P && r < n) {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (j < n) P[(int64_t)(r * n + j) * m + pb] = ok ? Hl[r * S + j] : 0.0;
  }
  if (!ok && r < p) store_failed_gain_row<N>(r, n, p, m, pb, q, rin, fallback && hover, K);
  if (r == 0) {
    status[pb] = (int8_t)st;
    if (iters) iters[pb] = it;
  }
}

// Launch the dense kernel sized for (n, p): 6 / 4, 9 / 4, else 16 / 8.
inline void launch_dare_dense(int n, int p, int64_t m, const double* A, const double* B, int ab_per_problem,
                              double dt, double gravity, const double* mass, const double* q, const double* r,
                              int fallback, double* K, double* P, int8_t* status, int32_t* iters, hipStream_t s) {
  const int grid = (int)((m + 3) / 4);
  if (n <= 6 && p <= 4)
    dare_row_kernel<6, 4><<<grid, 64, 0, s>>>(n, p, m, A, B, ab_per_problem, dt, gravity, mass, q, r, fallback, K, P,
                                              status, iters);
  else if (n <= 9 && p <= 4)
    dare_row_kernel<9, 4><<<grid, 64, 0, s>>>(n, p, m, A, B, ab_per_problem, dt, gravity, mass, q, r, fallback, K, P,
                                              status, iters);
  else
    dare_row_kernel<16, 8><<<grid, 64, 0, s>>>(n, p, m, A, B, ab_per_problem, dt, gravity, mass, q, r, fallback, K,
                                               P, status, iters);
}

}  // namespace

extern "C" int qt_dare_batched(int32_t n_state, int64_t m, double dt, double gravity, const double* mass,
                               const double* q, const double* r, int32_t structured, double* K, double* P,
                               int8_t* status, int32_t* iters, void* stream) {
  if ((n_state != 6 && n_state != 9) || m < 0) return QT_EINVAL;
  if (m == 0) return QT_OK;  // empty: no pointer is read
  if (!q || !r || !K || !status) return QT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (structured) {
    const int64_t lanes = 4 * m;
    const int grid = (int)((lanes + 255) / 256);
    if (n_state == 9)
      dare_axis_kernel<9><<<grid, 256, 0, s>>>(m, dt, gravity, mass, q, r, K, P, status, iters);
    else
      dare_axis_kernel<6><<<grid, 256, 0, s>>>(m, dt, gravity, mass, q, r, K, P, status, iters);
  } else {
    if (m > ((int64_t)0x7fffffff) * 4) return QT_EINVAL;
    launch_dare_dense(n_state, 4, m, nullptr, nullptr, 0, dt, gravity, mass, q, r, 1, K, P, status, iters, s);
  }
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH;
}

extern "C" int qt_dare_dense(int32_t n, int32_t p, int64_t m, const double* A, const double* B,
                             int32_t ab_per_problem, const double* q, const double* r, double* K, double* P,
                             int8_t* status, int32_t* iters, void* stream) {
  if (n < 1 || n > kMaxN || p < 1 || p > kMaxP || m < 0 || m > ((int64_t)0x7fffffff) * 4) return QT_EINVAL;
  if (m == 0) return QT_OK;  // empty: no pointer is read
  if (!A || !B || !q || !r || !K || !status) return QT_EINVAL;
  launch_dare_dense(n, p, m, A, B, ab_per_problem, 0.0, 0.0, nullptr, q, r, 0, K, P, status, iters,
                    (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH;
}
