// Per-wave cycle spread of a pure FP64 FMA loop in the rollout kernel's
// regime (1,024 waves = one per SIMD, ~3.6M cycles per wave, like one
// 65,536-episode rollout).  Question: do some CUs take more cycles for the
// same instruction stream (the rollout kernel shows ~4% of CUs per launch at
// +8%), i.e. is the rollout's tail a property of the chip or of the kernel?
// Build: hipcc --offload-arch=gfx950 -O3 tail.hip -o tail
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

struct Stamp {
  unsigned long long t0, t1, hw, xcc;
};

__global__ __launch_bounds__(256) void k_fma(double* out, Stamp* st, double a, double b, int iters) {
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0, p = x + 4.0, q = x + 5.0, r = x + 6.0,
         s = x + 7.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      asm volatile(
          "v_fma_f64 %0, %0, %8, %9\n"
          "v_fma_f64 %1, %1, %8, %9\n"
          "v_fma_f64 %2, %2, %8, %9\n"
          "v_fma_f64 %3, %3, %8, %9\n"
          "v_fma_f64 %4, %4, %8, %9\n"
          "v_fma_f64 %5, %5, %8, %9\n"
          "v_fma_f64 %6, %6, %8, %9\n"
          "v_fma_f64 %7, %7, %8, %9\n"
          : "+v"(x), "+v"(y), "+v"(z), "+v"(w), "+v"(p), "+v"(q), "+v"(r), "+v"(s)
          : "v"(a), "v"(b));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  out[gid] = x + y + z + w + p + q + r + s;
  if ((threadIdx.x & 63) == 0)
    st[gid >> 6] = Stamp{t0, t1, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4),
                         (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20)};
}

int main() {
  const int blocks = 256, nw = blocks * 4, iters = 3600000 / 260;  // ~3.6M cycles at 4 cycles per FMA
  double* out;
  Stamp* st;
  CHECK(hipMalloc(&out, sizeof(double) * nw * 64));
  CHECK(hipMalloc(&st, sizeof(Stamp) * nw));
  for (int r = 0; r < 300; ++r) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, st, 0.999, 1e-3, iters);
  CHECK(hipDeviceSynchronize());
  for (int rep = 0; rep < 6; ++rep) {
    hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, st, 0.999, 1e-3, iters);
    CHECK(hipDeviceSynchronize());
    std::vector<Stamp> h(nw);
    CHECK(hipMemcpy(h.data(), st, sizeof(Stamp) * nw, hipMemcpyDeviceToHost));
    std::vector<double> cyc;
    for (auto& s : h) cyc.push_back(double(s.t1 - s.t0));
    std::vector<double> srt = cyc;
    std::sort(srt.begin(), srt.end());
    const double med = srt[nw / 2];
    int slow = 0, slow_xcc[16] = {0};
    for (int i = 0; i < nw; ++i)
      if (cyc[i] > 1.03 * med) ++slow, ++slow_xcc[h[i].xcc & 15];
    printf("rep %d: cycles p50 %.0f p90 %.0f p99 %.0f max %.0f (max/p50 %.4f); waves > 1.03 p50: %d, by XCD:", rep,
           med, srt[nw * 9 / 10], srt[nw * 99 / 100], srt[nw - 1], srt[nw - 1] / med, slow);
    for (int x = 0; x < 8; ++x) printf(" %d", slow_xcc[x]);
    printf("\n");
  }
  return 0;
}
