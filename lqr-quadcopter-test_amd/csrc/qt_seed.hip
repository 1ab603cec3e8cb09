// qt_seed.hip — QuadcopterEnv.reset(seed) draws on the device.
//
// One lane per episode: SeedSequence(seed) -> PCG64, then the draws the
// reference makes from two fresh default_rng(seed) streams
// (quadcopter_env.py:122-137; target_motion.py:318-366):
//   target stream: linear standard_normal(3) | circular uniform(0, 2 pi) |
//                  sinusoidal uniform(0, 2 pi, 3) | figure8, stationary: none
//   env stream:    uniform(-0.5, 0.5, 3) start offset
// Output layout is qt_batch.pattern [4][n] and the reset offset [3][n].
#include <hip/hip_runtime.h>

#include "../../include/quadtrack.h"
#include "qt_rng.hpp"

namespace {

constexpr double kTwoPi = 6.283185307179586;  // 2 * math.pi

__global__ __launch_bounds__(256) void seed_draws_kernel(int64_t n, const int64_t* __restrict__ seeds,
                                                         const int8_t* __restrict__ motion, int32_t motion_default,
                                                         double* pattern, double* offset) {
#pragma clang fp contract(off)
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint64_t seed = (uint64_t)seeds[e];
  const int m = motion ? (int)motion[e] : motion_default;
  const qt::Pcg64 g0 = qt::pcg64_from_seed(seed);
  qt::Pcg64 g = g0;
  double p[3] = {0.0, 0.0, 0.0};
  if (m == QT_MOTION_LINEAR) {
    p[0] = qt::pcg_standard_normal(g);
    p[1] = qt::pcg_standard_normal(g);
    p[2] = qt::pcg_standard_normal(g);
  } else if (m == QT_MOTION_CIRCULAR) {
    p[0] = 0.0 + kTwoPi * qt::pcg_next_double(g);
  } else if (m == QT_MOTION_SINUSOIDAL) {
    p[0] = 0.0 + kTwoPi * qt::pcg_next_double(g);
    p[1] = 0.0 + kTwoPi * qt::pcg_next_double(g);
    p[2] = 0.0 + kTwoPi * qt::pcg_next_double(g);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) pattern[i * n + e] = p[i];
  pattern[3 * n + e] = 0.0;
  g = g0;
#pragma unroll
  for (int i = 0; i < 3; ++i) offset[i * n + e] = -0.5 + 1.0 * qt::pcg_next_double(g);
}

// first k draws of default_rng(seed).uniform(lo[j], hi[j]) per episode
__global__ __launch_bounds__(256) void seed_uniform_kernel(int64_t n, const int64_t* __restrict__ seeds, int32_t k,
                                                           const double* __restrict__ lo,
                                                           const double* __restrict__ hi, double* out) {
#pragma clang fp contract(off)
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  qt::Pcg64 g = qt::pcg64_from_seed((uint64_t)seeds[e]);
  for (int j = 0; j < k; ++j) out[(int64_t)j * n + e] = lo[j] + (hi[j] - lo[j]) * qt::pcg_next_double(g);
}

// Draw vectors first .. first+n-1 of ONE stream default_rng(seed): lane i
// jumps the generator k * (first + i) outputs ahead and draws its k uniforms,
// lo + (hi - lo) * next_double as numpy's uniform forms them.
__global__ __launch_bounds__(256) void stream_uniform_kernel(uint64_t seed, int64_t first, int64_t n, int32_t k,
                                                             const double* __restrict__ lo,
                                                             const double* __restrict__ hi, double* out) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  qt::Pcg64 g = qt::pcg64_from_seed(seed);
  qt::pcg_advance(g, (qt::u128)(uint64_t)(first + i) * (uint64_t)k);
  for (int j = 0; j < k; ++j) out[(int64_t)j * n + i] = lo[j] + (hi[j] - lo[j]) * qt::pcg_next_double(g);
}

}  // namespace

extern "C" int qt_stream_uniform(uint64_t seed, int64_t first, int64_t n, int32_t k, const double* lo,
                                 const double* hi, double* out, void* stream) {
  if (n < 0 || first < 0 || k < 0 || k > 64) return QT_EINVAL;
  if (n == 0 || k == 0) return QT_OK;  // empty: no pointer is read
  if (!lo || !hi || !out) return QT_EINVAL;
  stream_uniform_kernel<<<(int)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(seed, first, n, k, lo, hi, out);
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH;
}

extern "C" int qt_seed_uniform(int64_t n, const int64_t* seeds, int32_t k, const double* lo, const double* hi,
                               double* out, void* stream) {
  if (n < 0 || k < 0 || k > 64) return QT_EINVAL;
  if (n == 0 || k == 0) return QT_OK;  // empty: no pointer is read
  if (!seeds || !lo || !hi || !out) return QT_EINVAL;
  seed_uniform_kernel<<<(int)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(n, seeds, k, lo, hi, out);
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH;
}

extern "C" int qt_seed_draws(int64_t n, const int64_t* seeds, const int8_t* motion, int32_t motion_default,
                             double* pattern, double* offset, void* stream) {
  if (n < 0 || motion_default < 0 || motion_default > 4) return QT_EINVAL;
  if (n == 0) return QT_OK;  // empty: no pointer is read
  if (!seeds || !pattern || !offset) return QT_EINVAL;
  seed_draws_kernel<<<(int)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(n, seeds, motion, motion_default,
                                                                              pattern, offset);
  return hipGetLastError() == hipSuccess ? QT_OK : QT_ELAUNCH;
}
