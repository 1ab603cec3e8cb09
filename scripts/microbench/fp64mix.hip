// Issue cost of FP64 instruction forms for a lone wave per SIMD (1,024 waves),
// 8 independent chains: v_fma_f64 (VOP3, 3 VGPR sources), v_fmac_f64 (VOP2),
// v_mul_f64, v_add_f64, v_fma_f64 with an inline constant, and v_fma_f64 with
// an SGPR operand.  Prints shader cycles per instruction (s_memtime, median
// over waves).  Build: hipcc --offload-arch=gfx950 -O3 fp64mix.hip -o fp64mix
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

constexpr int kIters = 4096;

#define BODY8(INSN, EXTRA)                                                                                      \
  asm volatile(INSN " %0, %0, %8" EXTRA "\n" INSN " %1, %1, %8" EXTRA "\n" INSN " %2, %2, %8" EXTRA "\n" INSN \
               " %3, %3, %8" EXTRA "\n" INSN " %4, %4, %8" EXTRA "\n" INSN " %5, %5, %8" EXTRA "\n" INSN         \
               " %6, %6, %8" EXTRA "\n" INSN " %7, %7, %8" EXTRA "\n"                                           \
               : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)                \
               : "v"(a), "v"(b), "s"(sc))

#define KERNEL(NAME, INSN, EXTRA)                                                                            \
  __global__ __launch_bounds__(256) void NAME(double* out, unsigned long long* st, double a, double b,      \
                                              double sc) {                                                   \
    double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,       \
           x6 = x0 + 6, x7 = x0 + 7;                                                                        \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                             \
    for (int i = 0; i < kIters; ++i) {                                                                       \
      BODY8(INSN, EXTRA);                                                                                    \
      BODY8(INSN, EXTRA);                                                                                    \
      BODY8(INSN, EXTRA);                                                                                    \
      BODY8(INSN, EXTRA);                                                                                    \
    }                                                                                                        \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                             \
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;                                                   \
    out[gid] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                                                        \
    if ((threadIdx.x & 63) == 0) st[gid >> 6] = t1 - t0;                                                     \
  }

KERNEL(k_fma, "v_fma_f64", ", %9")
KERNEL(k_fmac, "v_fmac_f64", "")
KERNEL(k_mul, "v_mul_f64", "")
KERNEL(k_add, "v_add_f64", "")
KERNEL(k_fma_const, "v_fma_f64", ", 1.0")
KERNEL(k_fma_sgpr, "v_fma_f64", ", %10")

typedef void (*Kern)(double*, unsigned long long*, double, double, double);

int main() {
  struct K {
    const char* name;
    Kern k;
  } ks[] = {{"v_fma_f64 v,v,v", k_fma},   {"v_fmac_f64 v,v", k_fmac},     {"v_mul_f64 v,v", k_mul},
            {"v_add_f64 v,v", k_add},     {"v_fma_f64 v,v,1.0", k_fma_const}, {"v_fma_f64 v,v,s", k_fma_sgpr}};
  const int blocks = 256, nw = blocks * 4;
  double* out;
  unsigned long long* st;
  CHECK(hipMalloc(&out, sizeof(double) * nw * 64));
  CHECK(hipMalloc(&st, sizeof(unsigned long long) * nw));
  for (int r = 0; r < 200; ++r) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, st, 0.999, 1e-3, 0.5);
  CHECK(hipDeviceSynchronize());
  for (auto& kk : ks) {
    hipLaunchKernelGGL(kk.k, dim3(blocks), dim3(256), 0, 0, out, st, 0.999, 1e-3, 0.5);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(nw);
    CHECK(hipMemcpy(h.data(), st, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    const double per = double(h[nw / 2]) / kIters;
    printf("%-22s %7.1f cycles / 32-instr iteration = %5.2f cycles per instruction (loop overhead included)\n",
           kk.name, per, per / 32.0);
  }
  return 0;
}
