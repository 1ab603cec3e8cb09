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
//  * dare_dense_kernel — arbitrary symmetric Q (6x6 / 9x9) and R (4x4): one
//    wavefront per problem, matrices in LDS, cooperative LU + products.
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

// heuristic (double-integrator) gains, K row for one axis
__device__ __forceinline__ void heuristic_axis(double qp, double qv, double r, double& kp, double& kv) {
  kp = sqrt(qp / r);
  kv = sqrt(2.0 * sqrt(qp / r) + qv / r);
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

// ----------------------------------------------------------- dense kernel

constexpr int kDenseThreads = 64;

// In-LDS helpers for one wavefront.  Matrices are row-major n x n (ld = n).
__device__ __forceinline__ void mm(int n, int k, int mcols, const double* a, const double* b, double* c, bool transA = false) {
  for (int idx = threadIdx.x; idx < n * mcols; idx += kDenseThreads) {
    const int i = idx / mcols, j = idx % mcols;
    double s = 0.0;
    for (int l = 0; l < k; ++l) s += (transA ? a[l * n + i] : a[i * k + l]) * b[l * mcols + j];
    c[idx] = s;
  }
  __syncthreads();
}

// Gauss-Jordan: W (n x n) is reduced in place, Y (n x ny) receives W^-1 Y.
__device__ __forceinline__ bool gauss_jordan(int n, double* W, double* Y, int ny, int* piv_sh) {
  for (int k = 0; k < n; ++k) {
    if (threadIdx.x == 0) {
      int p = k;
      double best = fabs(W[k * n + k]);
      for (int i = k + 1; i < n; ++i)
        if (fabs(W[i * n + k]) > best) best = fabs(W[i * n + k]), p = i;
      piv_sh[0] = best == 0.0 ? -1 : p;
    }
    __syncthreads();
    const int p = piv_sh[0];
    if (p < 0) return false;
    if (p != k) {
      for (int j = threadIdx.x; j < n + ny; j += kDenseThreads) {
        double* r1 = j < n ? &W[k * n + j] : &Y[k * ny + j - n];
        double* r2 = j < n ? &W[p * n + j] : &Y[p * ny + j - n];
        double t = *r1;
        *r1 = *r2;
        *r2 = t;
      }
    }
    __syncthreads();
    const double inv = 1.0 / W[k * n + k];
    __syncthreads();
    for (int j = threadIdx.x; j < n + ny; j += kDenseThreads) {
      if (j < n)
        W[k * n + j] *= inv;
      else
        Y[k * ny + j - n] *= inv;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < n * (n + ny); idx += kDenseThreads) {
      const int i = idx / (n + ny), j = idx % (n + ny);
      if (i == k) continue;
      const double f = W[i * n + k];
      if (j < n) {
        if (j != k) W[i * n + j] -= f * W[k * n + j];
      } else {
        Y[i * ny + j - n] -= f * Y[k * ny + j - n];
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kDenseThreads)
      if (i != k) W[i * n + k] = 0.0;
    __syncthreads();
  }
  return true;
}

// eigenvalues of a small symmetric matrix by cyclic Jacobi (one thread)
__device__ void jacobi_eigs(int n, double* a, double* ev) {
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) off += a[i * n + j] * a[i * n + j];
    if (off < 1e-300) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = a[p * n + q];
        if (apq == 0.0) continue;
        const double app = a[p * n + p], aqq = a[q * n + q];
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {
          const double akp = a[k * n + p], akq = a[k * n + q];
          a[k * n + p] = c * akp - s * akq;
          a[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = a[p * n + k], aqk = a[q * n + k];
          a[p * n + k] = c * apk - s * aqk;
          a[q * n + k] = s * apk + c * aqk;
        }
      }
  }
  for (int i = 0; i < n; ++i) ev[i] = a[i * n + i];
}

// np.allclose(M, M.T, atol=1e-8) and the eigenvalue test (riccati_lqr.py:70-84, 100-116)
__device__ bool check_sym_eigs(int n, const double* M, double* scratch, bool strict) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      const double a = M[i * n + j], b = M[j * n + i];
      if (!(fabs(a - b) <= 1e-8 + 1e-5 * fabs(b))) return false;
    }
  for (int i = 0; i < n * n; ++i) scratch[i] = M[i];
  double ev[16];
  jacobi_eigs(n, scratch, ev);
  for (int i = 0; i < n; ++i) {
    if (strict ? !(ev[i] > 1e-10) : (ev[i] < -1e-10)) return false;
  }
  return true;
}

constexpr int kMaxN = 16, kMaxP = 8;

// Dynamic LDS layout of dare_dense_kernel (doubles): sA, sA0, sG, sH, sT2,
// sQ (n x n); sW (n x n | p x p systems); sY (n x 2n | p x n right-hand
// sides); sT (n x n | p x n products | the p x p eigen scratch); sB (n x p);
// sR (p x p).
struct DenseLds {
  int nn, w, y, t;
  __host__ __device__ DenseLds(int n, int p) {
    nn = n * n;
    w = nn > p * p ? nn : p * p;
    y = 2 * nn > p * n ? 2 * nn : p * n;
    t = nn > p * n ? nn : p * n;
    t = t > p * p ? t : p * p;
  }
  __host__ __device__ int doubles(int n, int p) const { return 6 * nn + w + y + t + n * p + p * p; }
};

inline size_t dense_lds_bytes(int n, int p) { return sizeof(double) * (size_t)DenseLds(n, p).doubles(n, p); }

// General dense SDA, one wavefront per problem.  Hover model (A, B == NULL):
// A, B built from (dt, mass, gravity) exactly as build_linearized_system /
// build_augmented_lqi_system; otherwise A [n*n] and B [n*p] are read (shared
// when ab_per_problem == 0).  With `fallback`, invalid or failed hover-model
// problems get the heuristic gains (riccati_lqr.py:747-777).
// NT, PT: compile-time n, p (the 6-state hover model, 4 inputs): the LDS
// index arithmetic (idx / n, idx % n) becomes multiplications and the short
// loops unroll (2.5 -> 2.2 ms per 65,536 problems); 0 = sizes at run time.
template <int NT, int PT>
__global__ __launch_bounds__(kDenseThreads) void dare_dense_kernel(int n_rt, int p_rt, int64_t m,
                                                                   const double* __restrict__ Ain,
                                                                   const double* __restrict__ Bin,
                                                                   int ab_per_problem, double dt, double gravity,
                                                                   const double* __restrict__ mass,
                                                                   const double* __restrict__ q,
                                                                   const double* __restrict__ r, int fallback,
                                                                   double* K, double* P, int8_t* status,
                                                                   int32_t* iters) {
  const int n = NT ? NT : n_rt, p = PT ? PT : p_rt;
  const int64_t pb = blockIdx.x;
  if (pb >= m) return;
  // LDS sized to the problem (dense_lds_bytes): ~7 KB at n = 9, p = 4, so
  // ~20 problems share a CU instead of the 6 that fixed 16 x 16 arrays allowed
  extern __shared__ double smem[];
  const DenseLds L(n, p);
  double* sA = smem;
  double* sA0 = sA + L.nn;
  double* sB = sA0 + L.nn;
  double* sG = sB + n * p;
  double* sH = sG + L.nn;
  double* sW = sH + L.nn;
  double* sY = sW + L.w;
  double* sT = sY + L.y;
  double* sT2 = sT + L.t;
  double* sR = sT2 + L.nn;
  double* sQ = sR + p * p;
  __shared__ int sh_i[2];
  const int tid = threadIdx.x;
  const bool hover = Ain == nullptr;
  const double mss = mass ? mass[pb] : 1.0;
  const int64_t abm = ab_per_problem ? m : 1, abj = ab_per_problem ? pb : 0;
  for (int i = tid; i < n * n; i += kDenseThreads) {
    sQ[i] = q[(int64_t)i * m + pb];
    double v;
    if (hover) {
      const int a = i / n, b = i % n;
      v = (a == b) ? 1.0 : 0.0;
      if (a < 3 && b == a + 3) v = dt;             // A_d = I + A_c dt (riccati_lqr.py:260)
      if (n == 9 && a >= 6 && b == a - 6) v = dt;  // integral rows (308)
    } else {
      v = Ain[(int64_t)i * abm + abj];
    }
    sA[i] = v;
    sA0[i] = v;
  }
  for (int i = tid; i < p * p; i += kDenseThreads) sR[i] = r[(int64_t)i * m + pb];
  for (int i = tid; i < n * p; i += kDenseThreads) {
    double v = 0.0;
    if (hover) {
      const int a = i / p, c = i % p;
      if (a == 5 && c == 0) v = 1.0 / mss * dt;  // riccati_lqr.py:250,261
      if (a == 4 && c == 1) v = -gravity * dt;   // 252
      if (a == 3 && c == 2) v = gravity * dt;    // 254
    } else {
      v = Bin[(int64_t)i * abm + abj];
    }
    sB[i] = v;
  }
  __syncthreads();
  if (tid == 0) {
    int st = QT_DARE_OK;
    if (!check_sym_eigs(n, sQ, sT, false))
      st = QT_DARE_Q_NOT_PSD;
    else if (!check_sym_eigs(p, sR, sT, true))
      st = QT_DARE_R_NOT_PD;
    sh_i[1] = st;
  }
  __syncthreads();
  int st = sh_i[1];
  int it = 0;
  if (st == QT_DARE_OK) {
    // G = B R^-1 B' : solve R X = B' (p x n), then G = B X
    for (int i = tid; i < p * p; i += kDenseThreads) sW[i] = sR[i];
    for (int i = tid; i < p * n; i += kDenseThreads) sY[i] = sB[(i % n) * p + i / n];
    __syncthreads();
    if (!gauss_jordan(p, sW, sY, n, sh_i)) st = QT_DARE_SINGULAR;
    if (st == QT_DARE_OK) {
      mm(n, p, n, sB, sY, sG);
      for (int i = tid; i < n * n; i += kDenseThreads) sH[i] = sQ[i];
      __syncthreads();
      bool conv = false;
      for (it = 1; it <= kMaxIter; ++it) {
        mm(n, n, n, sG, sH, sW);
        for (int i = tid; i < n; i += kDenseThreads) sW[i * n + i] += 1.0;
        for (int i = tid; i < n * n; i += kDenseThreads) {
          const int a = i / n, b = i % n;
          sY[a * 2 * n + b] = sA[i];
          sY[a * 2 * n + n + b] = sG[i];
        }
        __syncthreads();
        if (!gauss_jordan(n, sW, sY, 2 * n, sh_i)) {
          st = QT_DARE_SINGULAR;
          break;
        }
        // Y1 = sY[:, :n], Y2 = sY[:, n:] (ld 2n).  T = H Y1 ; T2 = A' T
        for (int idx = tid; idx < n * n; idx += kDenseThreads) {
          const int i = idx / n, j = idx % n;
          double s = 0.0;
          for (int l = 0; l < n; ++l) s += sH[i * n + l] * sY[l * 2 * n + j];
          sT[idx] = s;
        }
        __syncthreads();
        mm(n, n, n, sA, sT, sT2, true);
        for (int idx = tid; idx < n * n; idx += kDenseThreads) {
          const int i = idx / n, j = idx % n;
          sW[idx] = sH[idx] + 0.5 * (sT2[i * n + j] + sT2[j * n + i]);
        }
        __syncthreads();
        if (tid == 0) {
          double dn = 0.0, hn = 0.0;
          for (int i = 0; i < n * n; ++i) {
            dn += (sW[i] - sH[i]) * (sW[i] - sH[i]);
            hn += sW[i] * sW[i];
          }
          sh_i[0] = !isfinite(hn) ? -1 : (sqrt(dn) <= kTol * sqrt(hn) ? 1 : 0);
        }
        __syncthreads();
        const int flag = sh_i[0];
        for (int i = tid; i < n * n; i += kDenseThreads) sH[i] = sW[i];
        // T = Y2 A' ; T2 = A T ; G += sym(T2)
        for (int idx = tid; idx < n * n; idx += kDenseThreads) {
          const int i = idx / n, j = idx % n;
          double s = 0.0;
          for (int l = 0; l < n; ++l) s += sY[i * 2 * n + n + l] * sA[j * n + l];
          sT[idx] = s;
        }
        __syncthreads();
        mm(n, n, n, sA, sT, sT2);
        for (int idx = tid; idx < n * n; idx += kDenseThreads) {
          const int i = idx / n, j = idx % n;
          sG[idx] += 0.5 * (sT2[i * n + j] + sT2[j * n + i]);
        }
        // A = A Y1
        for (int idx = tid; idx < n * n; idx += kDenseThreads) {
          const int i = idx / n, j = idx % n;
          double s = 0.0;
          for (int l = 0; l < n; ++l) s += sA[i * n + l] * sY[l * 2 * n + j];
          sT[idx] = s;
        }
        __syncthreads();
        for (int i = tid; i < n * n; i += kDenseThreads) sA[i] = sT[i];
        __syncthreads();
        if (flag < 0) {
          st = QT_DARE_NO_CONVERGE;
          break;
        }
        if (flag == 1) {
          conv = true;
          break;
        }
      }
      if (st == QT_DARE_OK && !conv) st = QT_DARE_NO_CONVERGE;
    }
  }
  if (st == QT_DARE_OK) {
    // K = (R + B'PB)^-1 B'PA : T = B'P (p x n), W = R + T B (p x p), Y = T A0 (p x n)
    mm(p, n, n, sB, sH, sT, true);
    for (int idx = tid; idx < p * p; idx += kDenseThreads) {
      const int i = idx / p, j = idx % p;
      double s = sR[idx];
      for (int l = 0; l < n; ++l) s += sT[i * n + l] * sB[l * p + j];
      sW[idx] = s;
    }
    for (int idx = tid; idx < p * n; idx += kDenseThreads) {
      const int i = idx / n, j = idx % n;
      double s = 0.0;
      for (int l = 0; l < n; ++l) s += sT[i * n + l] * sA0[l * n + j];
      sY[idx] = s;
    }
    __syncthreads();
    if (!gauss_jordan(p, sW, sY, n, sh_i)) st = QT_DARE_SINGULAR;
  }
  if (st == QT_DARE_OK) {
    for (int i = tid; i < p * n; i += kDenseThreads) K[(int64_t)i * m + pb] = sY[i];
    if (P)
      for (int i = tid; i < n * n; i += kDenseThreads) P[(int64_t)i * m + pb] = sH[i];
  } else {
    for (int i = tid; i < p * n; i += kDenseThreads) K[(int64_t)i * m + pb] = 0.0;
    if (P)
      for (int i = tid; i < n * n; i += kDenseThreads) P[(int64_t)i * m + pb] = 0.0;
    __syncthreads();
    if (fallback && hover && tid == 0) {
      // heuristic gains from the diagonals (riccati_lqr.py:756-774)
      const double rrate = (sR[5] + sR[10] + sR[15]) / 3.0;
      double kp, kv;
      heuristic_axis(sQ[2 * n + 2], sQ[5 * n + 5], sR[0], kp, kv);
      K[(int64_t)(0 * n + 2) * m + pb] = kp;
      K[(int64_t)(0 * n + 5) * m + pb] = kv;
      heuristic_axis(sQ[1 * n + 1], sQ[4 * n + 4], rrate, kp, kv);
      K[(int64_t)(1 * n + 1) * m + pb] = -kp;
      K[(int64_t)(1 * n + 4) * m + pb] = -kv;
      heuristic_axis(sQ[0], sQ[3 * n + 3], rrate, kp, kv);
      K[(int64_t)(2 * n + 0) * m + pb] = kp;
      K[(int64_t)(2 * n + 3) * m + pb] = kv;
    }
  }
  if (tid == 0) {
    status[pb] = (int8_t)st;
    if (iters) iters[pb] = it;
  }
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
    if (m > 0x7fffffff) return QT_EINVAL;
    if (n_state == 9)  // runtime sizes: the unrolled 9-state form needs 169 VGPRs and ran 1.8x slower
      dare_dense_kernel<0, 0><<<(int)m, kDenseThreads, dense_lds_bytes(9, 4), s>>>(n_state, 4, m, nullptr, nullptr, 0, dt, gravity, mass, q, r,
                                                       1, K, P, status, iters);
    else
      dare_dense_kernel<6, 4><<<(int)m, kDenseThreads, dense_lds_bytes(6, 4), s>>>(n_state, 4, m, nullptr, nullptr, 0, dt, gravity, mass, q, r,
                                                       1, K, P, status, iters);
  }
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH;
}

extern "C" int qt_dare_dense(int32_t n, int32_t p, int64_t m, const double* A, const double* B,
                             int32_t ab_per_problem, const double* q, const double* r, double* K, double* P,
                             int8_t* status, int32_t* iters, void* stream) {
  if (n < 1 || n > kMaxN || p < 1 || p > kMaxP || m < 0 || m > 0x7fffffff) return QT_EINVAL;
  if (m == 0) return QT_OK;  // empty: no pointer is read
  if (!A || !B || !q || !r || !K || !status) return QT_EINVAL;
  hipStream_t hs = (hipStream_t)stream;
  const size_t lds = dense_lds_bytes(n, p);
  if (n == 6 && p == 4)
    dare_dense_kernel<6, 4><<<(int)m, kDenseThreads, lds, hs>>>(n, p, m, A, B, ab_per_problem, 0.0, 0.0,
                                                                       nullptr, q, r, 0, K, P, status, iters);
  else
    dare_dense_kernel<0, 0><<<(int)m, kDenseThreads, lds, hs>>>(n, p, m, A, B, ab_per_problem, 0.0, 0.0,
                                                                       nullptr, q, r, 0, K, P, status, iters);
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH;
}
