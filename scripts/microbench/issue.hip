// Issue-rate microbenchmark for the rollout kernel's regime: one wave64 per
// SIMD (1024 waves of 64 lanes on 256 CUs), FP64 VALU streams.  Measures
// cycles per instruction for dependent vs independent v_fma_f64 chains, the
// price of interleaved SALU, of v_cndmask selects and of branches.
// Build: hipcc --offload-arch=gfx950 -O3 issue.hip -o issue
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void dep1(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) x = fma(x, a, b);
  }
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void dep2(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1.0;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x = fma(x, a, b);
      y = fma(y, a, b);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y;
}

__global__ __launch_bounds__(256) void dep4(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = fma(x, a, b);
      y = fma(y, a, b);
      z = fma(z, a, b);
      w = fma(w, a, b);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w;
}

// 16 independent FMAs + 4 SALU per group
__global__ __launch_bounds__(256) void dep4_salu(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = fma(x, a, b);
      y = fma(y, a, b);
      asm volatile("s_nop 0\n s_nop 0" ::);
      z = fma(z, a, b);
      w = fma(w, a, b);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w;
}

// 16 FMAs + 8 v_cndmask (4 double selects) per group
__global__ __launch_bounds__(256) void dep4_sel(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = fma(x, a, b);
      y = fma(y, a, b);
      z = fma(z, a, b);
      w = fma(w, a, b);
      x = x > 1e300 ? y : x;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w;
}

// 16 FMAs + 1 sqrt per group
__global__ __launch_bounds__(256) void dep4_sqrt(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0, s = 0;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = fma(x, a, b);
      y = fma(y, a, b);
      z = fma(z, a, b);
      w = fma(w, a, b);
    }
    s += sqrt(fabs(x) + 1.0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w + s;
}

// 16 FMAs + a per-lane branch that is never taken (the body would clamp)
__global__ __launch_bounds__(256) void dep4_br(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = fma(x, a, b);
      y = fma(y, a, b);
      z = fma(z, a, b);
      w = fma(w, a, b);
    }
    if (x > 1e300) {
      x = x / y * 3.0;
      y = y / z * 3.0;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w;
}

// 16 FMAs + 4 independent selects off the critical chain (results summed late)
__global__ __launch_bounds__(256) void dep4_selind(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0, acc = 0.0;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = fma(x, a, b);
      y = fma(y, a, b);
      z = fma(z, a, b);
      w = fma(w, a, b);
      acc += (z > 1e300) ? 1.0 : 0.0;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w + acc;
}

// 16 FMAs + 1 hand-rolled sqrt (rsq + Newton, no scaling) per group
__device__ __forceinline__ double sqrt_fast(double s) {
  double y = __builtin_amdgcn_rsq(s);
  double g = s * y, h = 0.5 * y;
  double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, s);
  g = fma(d, h, g);
  d = fma(-g, g, s);
  return fma(d, h, g);
}

__global__ __launch_bounds__(256) void dep4_sqrtf(double* out, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0, s = 0;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = fma(x, a, b);
      y = fma(y, a, b);
      z = fma(z, a, b);
      w = fma(w, a, b);
    }
    s += sqrt_fast(fabs(x) + 1.0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w + s;
}

// f32 for comparison: 4 chains
__global__ __launch_bounds__(256) void dep4_f32(float* out, float a, float b) {
  float x = threadIdx.x * 1e-3f, y = x + 1.0f, z = x + 2.0f, w = x + 3.0f;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x = fmaf(x, a, b);
      y = fmaf(y, a, b);
      z = fmaf(z, a, b);
      w = fmaf(w, a, b);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w;
}

template <typename F, typename T>
int run(const char* name, F kern, T* out, int blocks, T a, T b, double instr_per_iter) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  kern<<<blocks, 256>>>(out, a, b);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    kern<<<blocks, 256>>>(out, a, b);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double instr = instr_per_iter * kIters;
  printf("%-10s blocks=%5d  %.4f ms  %.3f ns/instr/wave  (%.2f cyc @2.4GHz)\n", name, blocks, best,
         best * 1e6 / instr, best * 1e6 / instr * 2.4);
  return 0;
}

int main() {
  double* d;
  CHECK(hipMalloc(&d, 1 << 24));
  float* f = (float*)d;
  const double a = 0.999999, b = 1e-7;
  for (int blocks : {256}) {
    run("dep4_br", dep4_br, d, blocks, a, b, 16);
    run("dep4_selind", dep4_selind, d, blocks, a, b, 16);
    run("dep4_sqrtf", dep4_sqrtf, d, blocks, a, b, 16);
  }
  for (int blocks : {256, 512}) {
    run("dep1", dep1, d, blocks, a, b, 16);
    run("dep2", dep2, d, blocks, a, b, 16);
    run("dep4", dep4, d, blocks, a, b, 16);
    run("dep4_salu", dep4_salu, d, blocks, a, b, 16);
    run("dep4_sel", dep4_sel, d, blocks, a, b, 16);
    run("dep4_sqrt", dep4_sqrt, d, blocks, a, b, 16);
    run("dep4_f32", dep4_f32, f, blocks, 0.9999f, 1e-7f, 16);
  }
  CHECK(hipFree(d));
  return 0;
}
