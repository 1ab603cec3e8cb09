// Split-episode prototype: does spreading one episode's
// yaw-at-rest step over a PAIR of lanes pay when a GPU holds too few episodes
// to give every SIMD a wave ("Small per-GPU batches")?
//
// Two kernels run the same 3,000 no-vote steps of the config-2 loop (linear
// target, structured LQR, RK4 closed form, carried roll / pitch trig,
// Evaluator metrics), i.e. run_yaw0's horizon body without the horizon
// bound, the vote and the termination finish (qt_kernels.hpp:797-868):
//   one   one episode per lane, the product's own device functions
//         (integrate_yaw0, attitude_trig_resid, sqrt_pos / sqrt_sum, ...);
//   pair  one episode per lane pair: lane a = 0 takes roll and the y axis,
//         lane a = 1 pitch and the x axis (the structured gains couple
//         roll to y and pitch to x only); z and the thrust are computed by
//         both lanes; the partner's stage cosine, command and squared
//         horizontal error cross by a DPP quad_perm swap (two 32-bit moves per
//         double); lane 0's square root is the tracking error, lane 1's the
//         command norm (one shared sequence, sqrt_sum's result kept by a zero
//         correction).
// Every operation of `pair` rounds as the one it replaces (products and sums
// that commute, -s == s * -1, (-w) s == w (-s) inside an fma), so both kernels
// must end bit for bit on the same state and metrics; main() checks that
// before it prints a time.  A wave issues one instruction per ~4.4 cycles
// whatever its lanes do, so `pair` is faster only if its per-lane step has
// fewer instructions than `one`'s: the swaps, selects and the per-episode
// work both lanes repeat (z, thrust, metrics, target) decide it.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=on -I../../include \
//          -I../../lqr-quadcopter-test_amd/csrc split_step.hip -o split_step
// Run:   ./split_step [steps]   (prints one JSON line per batch size)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "qt_device.hpp"

using namespace qt;

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int kBlk = 256;
constexpr int kOut = 20;  // per episode: p[3] v[3] roll pitch wr wp | sum_e sum_e2 max_e sum_u os_max cur | on_pre on_post os_count z

struct Consts {
  RateLin R;
  VelLin L;
  Plant pl;
  double K[6];  // K[0][2], K[0][5], K[1][1], K[1][4], K[2][0], K[2][3] (structured_index)
  double hover, tmin, tmax, mr, dt, rad, erad;
  int window;
};

struct Ep {  // per-episode inputs, [n] rows
  const double *p0, *v0, *tp0, *tv;  // [3][n] each
};

// partner lane's double (lanes 2k <-> 2k+1): DPP quad_perm [1,0,3,2]
__device__ __forceinline__ double swap_pair(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double lin_target(double p0, double v, double t) {
#pragma clang fp contract(off)
  return p0 + v * t;
}

__device__ __forceinline__ double add_sq(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}

// sq3_ref (qt_kernels.hpp): ((a^2 + b^2) + c^2), no contraction
__device__ __forceinline__ double sq3_ref(double a, double b, double c) {
#pragma clang fp contract(off)
  return (a * a + b * b) + c * c;
}

__device__ __forceinline__ double sq(double a) {
#pragma clang fp contract(off)
  return a * a;
}

// ------------------------------------------------------------------ one
__global__ __launch_bounds__(kBlk) void k_one(Consts k, Ep in, int64_t n, int nsteps, double* out) {
  const int64_t e = (int64_t)blockIdx.x * kBlk + threadIdx.x;
  if (e >= n) return;
  double x[12] = {};
  double tp0[3], tv[3], tp[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    x[j] = in.p0[j * n + e], x[3 + j] = in.v0[j * n + e];
    tp0[j] = in.tp0[j * n + e], tv[j] = in.tv[j * n + e], tp[j] = tp0[j];
  }
  double t = 0.0;
  double err = sqrt_pos(sq3_ref(tp[0] - x[0], tp[1] - x[1], tp[2] - x[2]));
  Trig ta;
  trig_of<true>(x + 6, ta);
  double sum_e = 0, sum_e2 = 0, max_e = 0, sum_u = 0, os_max = 0, cur = 0;
  int on_pre = 0, on_post = 0, os_count = 0, z = -(1 << 30);
  const double R = k.rad, eR = k.erad;
  const int W = k.window;
  auto step = [&]() {
    RateCoef rk;
    rk.pin();
    const double a0[2] = {x[6], x[7]};
    double ep[3], ev[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) ep[i] = tp[i] - x[i], ev[i] = tv[i] - x[3 + i];
    double u[4];
    u[0] = clip_num(k.hover + (k.K[0] * ep[2] + k.K[1] * ev[2]), k.tmin, k.tmax);
    u[1] = clip_num(k.K[2] * ep[1] + k.K[3] * ev[1], -k.mr, k.mr);
    u[2] = clip_num(k.K[4] * ep[0] + k.K[5] * ev[0], -k.mr, k.mr);
    u[3] = 0.0;
    sum_e += err;
    sum_e2 = fma(err, err, sum_e2);
    max_e = fmax(max_e, err);
    const bool on = err <= R;
    on_pre += on;
    sum_u += sqrt_sum(fma(u[2], u[2], fma(u[1], u[1], u[0] * u[0])));
    const bool counted = on & (z > W);
    os_count += counted;
    os_max = counted ? fmax(os_max, cur) : os_max;
    cur = on ? err - R : fmax(cur, err - R);
    z = on ? 1 : z + 1;
    double d4[2];
    Trig t4;
    integrate_yaw0(k.R, k.L, k.pl, ta, x, u, rk, d4, t4);
    t += k.dt;
#pragma unroll
    for (int j = 0; j < 3; ++j) tp[j] = lin_target(tp0[j], tv[j], t);
    err = sqrt_pos(sq3_ref(x[0] - tp[0], x[1] - tp[1], x[2] - tp[2]));
    on_post += err <= eR;
    x[6] = (x[6] + kPi) - kPi;
    x[7] = (x[7] + kPi) - kPi;
    attitude_trig_resid(x + 6, a0, d4, t4, ta);
  };
  for (int s = 0; s < nsteps; s += 4) {
    step();
    step();
    step();
    step();
  }
  double* o = out + e;
  const double r[14] = {x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], x[9], x[10], sum_e, sum_e2, max_e, sum_u};
#pragma unroll
  for (int i = 0; i < 14; ++i) o[i * n] = r[i];
  o[14 * n] = os_max, o[15 * n] = cur;
  o[16 * n] = on_pre, o[17 * n] = on_post, o[18 * n] = os_count, o[19 * n] = z;
}

// ----------------------------------------------------------------- pair
__global__ __launch_bounds__(kBlk) void k_pair(Consts k, Ep in, int64_t n, int nsteps, double* out) {
  const int64_t g = (int64_t)blockIdx.x * kBlk + threadIdx.x;
  const int64_t e = g >> 1;
  const int a = (int)(g & 1);  // 0: roll + y axis, 1: pitch + x axis
  const int h = 1 - a;         // the horizontal axis of this lane
  // (n is even and the grid covers 2n lanes exactly: both lanes of a pair run)
  double ph = in.p0[h * n + e], vh = in.v0[h * n + e], pz = in.p0[2 * n + e], vz = in.v0[2 * n + e];
  const double tph0 = in.tp0[h * n + e], tvh = in.tv[h * n + e], tpz0 = in.tp0[2 * n + e], tvz = in.tv[2 * n + e];
  double tph = tph0, tpz = tpz0;
  double ang = 0.0, w = 0.0, t = 0.0;
  const double Kp = a ? k.K[4] : k.K[2], Kv = a ? k.K[5] : k.K[3];
  // lane selects as arithmetic (one FP64 slot where a select of a double
  // takes two v_cndmask_b32): af = a, nf = 1 - a, exact 0 / 1 factors
  const double af = a, nf = 1.0 - af, am1 = af - 1.0;
  double s0, c0;
  sincos_tilt(ang, &s0, &c0);
  double val;  // lane 0: the tracking error; lane 1: the last command norm (0 before the first)
  {
    const double dh2 = sq(tph - ph), dp2 = swap_pair(dh2);
    const double e2 = add_sq(add_sq(dh2, dp2), sq(tpz - pz));  // (dx^2 + dy^2) + dz^2
    val = a ? 0.0 : sqrt_pos(e2);
  }
  double acc = 0, sum_e2 = 0, max_e = 0, os_max = 0, cur = 0;
  int on_pre = 0, on_post = 0, os_count = 0, z = -(1 << 30);
  const double R = k.rad, eR = k.erad;
  const int W = k.window;
  const RateLin& Rl = k.R;
  const VelLin& L = k.L;
  auto step = [&]() {
    RateCoef rk;
    rk.pin();
    const double a0 = ang;
    // controller: thrust (both lanes), own axis' rate command
    const double u0 = clip_num(k.hover + (k.K[0] * (tpz - pz) + k.K[1] * (tvz - vz)), k.tmin, k.tmax);
    const double ua = clip_num(Kp * (tph - ph) + Kv * (tvh - vh), -k.mr, k.mr);
    // metrics: acc is sum_e on lane 0, sum_u on lane 1 (its val lags a step)
    acc += val;
    sum_e2 = fma(val, val, sum_e2);
    max_e = fmax(max_e, val);
    const bool on = val <= R;
    on_pre += on;
    const bool counted = on & (z > W);
    os_count += counted;
    os_max = counted ? fmax(os_max, cur) : os_max;
    cur = on ? val - R : fmax(cur, val - R);
    z = on ? 1 : z + 1;
    // integrate_yaw0 for this lane's angle and axis
    double sd, cd, cm;
    const double d2 = Rl.h2 * w, d4 = fma(Rl.d4y, w, Rl.d4u * ua);
    rate_sincos(d2, &sd, &cd, rk);
    const double s1 = fma(s0, cd, c0 * sd), c1 = fma(c0, cd, -(s0 * sd));
    const double e3 = fma(Rl.e3y, w, Rl.d3u * ua);
    resid_sincos(e3, &sd, &cm, rk);
    double s2, c2;
    rotate_cm(s1, c1, sd, cm, &s2, &c2);
    rate_sincos(d4, &sd, &cd, rk);
    const double s3 = fma(s0, cd, c0 * sd), c3 = fma(c0, cd, -(s0 * sd));
    const double cs[3] = {c0, c1, c2}, ss[3] = {s0, s1, s2};
    double svh = 0, sph = 0, svz = 0, spz = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double cp = swap_pair(cs[i]);
      const double rh = ss[i] * fma(cp, af, am1);  // pitch: s_pitch c_roll; roll: s_roll * -1
      const double rz = cs[i] * cp;               // c_pitch c_roll
      svh = fma(L.wv[i], rh, svh);
      svz = fma(L.wv[i], rz, svz);
      sph = fma(L.pa[i], rh, sph);
      spz = fma(L.pa[i], rz, spz);
    }
    {
      const double cp = swap_pair(c3);
      const double cr = a ? cp : c3, cq = a ? c3 : cp;  // roll's, pitch's cosine
      const double wc = L.wv[3] * cr;
      svh = fma(a ? wc : -L.wv[3], s3, svh);
      svz = fma(wc, cq, svz);
    }
    const double tm = u0 * k.pl.inv_mass;
    ph = fma(tm, sph, fma(L.pv, vh, ph));
    vh = fma(tm, svh, L.cv * vh);
    pz = fma(tm, spz, fma(L.pv, vz, pz + L.gp));
    vz = fma(tm, svz, fma(L.cv, vz, L.gv));
    ang = fma(Rl.ay, w, fma(Rl.au, ua, ang));
    w = fma(Rl.wy, w, Rl.wu * ua);
    t += k.dt;
    tph = lin_target(tph0, tvh, t);
    tpz = lin_target(tpz0, tvz, t);
    // post-step error (lane 0) and command norm (lane 1) through one sequence
    const double dh2 = sq(ph - tph), dp2 = swap_pair(dh2);
    const double up = swap_pair(ua);
    const double ur = a ? up : ua, uq = a ? ua : up;  // roll's, pitch's command
    const double e2 = add_sq(add_sq(dh2, dp2), sq(pz - tpz));  // dx^2 + dy^2 commutes
    const double un2 = fma(uq, uq, fma(ur, ur, u0 * u0));
    {
      const double xx = fmax(a ? un2 : e2, 0x1p-1000);
      const double y = __builtin_amdgcn_rsq(xx);
      double gg = xx * y, hh = y * 0.5;
      const double r = fma(-hh, gg, 0.5);
      gg = fma(gg, r, gg);
      hh = fma(hh, r, hh);
      double dd = fma(-gg, gg, xx);
      gg = fma(dd, hh, gg);
      dd = fma(-gg, gg, xx);
      val = fma(dd, hh * nf, gg);  // lane 1: sqrt_sum's result (a zero correction)
    }
    on_post += val <= eR;
    ang = (ang + kPi) - kPi;
    double sr, cr;
    tiny_sincos((ang - a0) - d4, &sr, &cr);
    rotate_cm(s3, c3, sr, cr, &s0, &c0);
  };
  for (int s = 0; s < nsteps; s += 4) {
    step();
    step();
    step();
    step();
  }
  acc += a ? val : 0.0;  // lane 1: the last step's command norm
  double* o = out + e;
  o[h * n] = ph, o[(3 + h) * n] = vh;
  if (a == 0) {
    o[2 * n] = pz, o[5 * n] = vz, o[6 * n] = ang, o[8 * n] = w;
    o[10 * n] = acc, o[11 * n] = sum_e2, o[12 * n] = max_e;
    o[14 * n] = os_max, o[15 * n] = cur;
    o[16 * n] = on_pre, o[17 * n] = on_post, o[18 * n] = os_count, o[19 * n] = z;
  } else {
    o[7 * n] = ang, o[9 * n] = w, o[13 * n] = acc;
  }
}

static double urand(uint64_t& s) {  // splitmix64 -> [0, 1)
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (z >> 11) * 0x1.0p-53;
}

int main(int argc, char** argv) {
  const int nsteps = argc > 1 ? atoi(argv[1]) : 3000;
  qt_env_params ep{};
  ep.dt = 0.01, ep.drag_angular = 0.0, ep.drag_linear = 0.1, ep.integrator = 0, ep.gravity = 9.81;
  Consts k{};
  k.R = make_rate_lin(ep);
  k.pl = make_plant(ep, 1.0);
  k.L = make_vel_lin(ep, k.pl);
  const double K[6] = {4.0, 3.0, -1.0, -1.2, 1.0, 1.2};
  memcpy(k.K, K, sizeof K);
  k.hover = 9.81, k.tmin = 0.0, k.tmax = 20.0, k.mr = 3.0, k.dt = ep.dt, k.rad = 0.5, k.erad = 0.5, k.window = 50;
  const int64_t nmax = 65536;
  std::vector<double> h(12 * nmax);
  uint64_t seed = 12345;
  for (int64_t i = 0; i < 3 * nmax; ++i) h[i] = 4.0 * urand(seed) - 2.0;               // p0
  for (int64_t i = 0; i < 3 * nmax; ++i) h[3 * nmax + i] = urand(seed) - 0.5;          // v0
  for (int64_t i = 0; i < 3 * nmax; ++i) h[6 * nmax + i] = 6.0 * urand(seed) - 3.0;    // tp0
  for (int64_t i = 0; i < 3 * nmax; ++i) h[9 * nmax + i] = urand(seed) - 0.5;          // tv
  double *din, *o1, *o2;
  CHECK(hipMalloc(&din, sizeof(double) * 12 * nmax));
  CHECK(hipMalloc(&o1, sizeof(double) * kOut * nmax));
  CHECK(hipMalloc(&o2, sizeof(double) * kOut * nmax));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int64_t n : {8192, 16384, 32768, 65536}) {
    // the inputs of the first n episodes, as [3][n] rows
    std::vector<double> hn(12 * n);
    for (int r = 0; r < 12; ++r)
      for (int64_t i = 0; i < n; ++i) hn[r * n + i] = h[r * nmax + i];
    CHECK(hipMemcpy(din, hn.data(), sizeof(double) * 12 * n, hipMemcpyHostToDevice));
    Ep in{din, din + 3 * n, din + 6 * n, din + 9 * n};
    const int g1 = (int)((n + kBlk - 1) / kBlk), g2 = (int)((2 * n) / kBlk);  // n is a multiple of 128
    float best[2] = {1e30f, 1e30f};
    for (int r = 0; r < 7; ++r) {
      for (int which = 0; which < 2; ++which) {
        CHECK(hipEventRecord(e0));
        if (which == 0)
          hipLaunchKernelGGL(k_one, dim3(g1), dim3(kBlk), 0, 0, k, in, n, nsteps, o1);
        else
          hipLaunchKernelGGL(k_pair, dim3(g2), dim3(kBlk), 0, 0, k, in, n, nsteps, o2);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best[which] = std::min(best[which], ms);
      }
    }
    std::vector<double> a1(kOut * n), a2(kOut * n);
    CHECK(hipMemcpy(a1.data(), o1, sizeof(double) * kOut * n, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(a2.data(), o2, sizeof(double) * kOut * n, hipMemcpyDeviceToHost));
    int64_t diff = 0, nonfinite = 0;
    for (int64_t i = 0; i < kOut * n; ++i) {
      diff += memcmp(&a1[i], &a2[i], sizeof(double)) != 0;
      nonfinite += !std::isfinite(a1[i]);
    }
    int64_t on = 0;
    for (int64_t i = 0; i < n; ++i) on += (int64_t)a1[16 * n + i];
    printf("{\"episodes\": %lld, \"steps\": %d, \"one_ms\": %.4f, \"pair_ms\": %.4f, \"speedup\": %.3f, "
           "\"waves_one\": %d, \"waves_pair\": %d, \"bitwise_equal\": %s, \"differing_values\": %lld, "
           "\"nonfinite\": %lld, \"on_pre_mean\": %.1f}\n",
           (long long)n, nsteps, best[0], best[1], best[0] / best[1], g1 * kBlk / 64, g2 * kBlk / 64,
           diff == 0 ? "true" : "false", (long long)diff, (long long)nonfinite, double(on) / n);
    fflush(stdout);
  }
  return 0;
}
