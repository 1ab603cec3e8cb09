// Issue-cost microbenchmark, round 2: the single-wave-per-SIMD regime of the
// rollout kernel (1,024 waves = one per SIMD), with inline-asm instruction
// streams so that the compiler neither reorders nor removes them.  Each
// kernel stamps s_memtime (shader clock) and s_memrealtime (100 MHz) around
// its loop; cycles per iteration = d(memtime) / iterations (clock independent).
//
// Questions: what does a taken s_branch cost; a SALU instruction; a 64-bit
// move; v_rsq_f64 on the dependency chain; does a half-populated wave (exec
// upper 32 lanes off) run faster; do two waves per SIMD hide a wave's
// non-FP64 slots.
// Build: hipcc --offload-arch=gfx950 -O3 issue2.hip -o issue2
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

constexpr int kIters = 2048;

#define FMA4                                                         \
  asm volatile(                                                      \
      "v_fma_f64 %0, %0, %4, %5\n"                                   \
      "v_fma_f64 %1, %1, %4, %5\n"                                   \
      "v_fma_f64 %2, %2, %4, %5\n"                                   \
      "v_fma_f64 %3, %3, %4, %5\n"                                   \
      : "+v"(x), "+v"(y), "+v"(z), "+v"(w)                           \
      : "v"(a), "v"(b))

#define FMA16 FMA4; FMA4; FMA4; FMA4

struct Stamp {
  unsigned long long t0, t1, r0, r1;
};

__device__ __forceinline__ void stamp_out(Stamp* st, unsigned long long t0, unsigned long long r0, double v,
                                          double* out) {
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  out[gid] = v;
  if ((threadIdx.x & 63) == 0) st[gid >> 6] = Stamp{t0, t1, r0, r1};
}

#define PROLOGUE                                                         \
  if (half && (threadIdx.x & 63) >= 32) return;                         \
  double x = threadIdx.x * 1e-3, y = x + 1.0, z = x + 2.0, w = x + 3.0; \
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();           \
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();

// 16 FP64 FMAs (4 independent chains)
__global__ __launch_bounds__(256) void k_fma(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  for (int i = 0; i < kIters; ++i) {
    FMA16;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + 4 s_nop (SALU issue slots)
__global__ __launch_bounds__(256) void k_salu(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  for (int i = 0; i < kIters; ++i) {
    FMA4;
    asm volatile("s_nop 0\ns_nop 0\ns_nop 0\ns_nop 0" ::);
    FMA4; FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + 1 taken s_branch (to the next instruction)
__global__ __launch_bounds__(256) void k_branch(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  for (int i = 0; i < kIters; ++i) {
    FMA4; FMA4;
    asm volatile("s_branch 1f\n1:" ::);
    FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + 1 not-taken s_cbranch_scc1 (scc = 0 after the compare)
__global__ __launch_bounds__(256) void k_nobranch(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  for (int i = 0; i < kIters; ++i) {
    FMA4; FMA4;
    asm volatile("s_cmp_eq_u32 0, 1\ns_cbranch_scc1 2f\n2:" ::: "scc");
    FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + 4 v_mov_b64
__global__ __launch_bounds__(256) void k_mov64(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  double m0, m1;
  for (int i = 0; i < kIters; ++i) {
    FMA4;
    asm volatile("v_mov_b64 %0, %2\nv_mov_b64 %1, %3\nv_mov_b64 %0, %3\nv_mov_b64 %1, %2" : "=&v"(m0), "=&v"(m1)
                 : "v"(x), "v"(y));
    FMA4; FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w + m0 + m1, out);
}

// + 4 v_cndmask_b32 (32-bit VALU)
__global__ __launch_bounds__(256) void k_b32(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  int c0 = threadIdx.x, c1 = c0 + 1;
  for (int i = 0; i < kIters; ++i) {
    FMA4;
    asm volatile("v_add_u32 %0, %0, %1\nv_add_u32 %1, %1, %0\nv_add_u32 %0, %0, %1\nv_add_u32 %1, %1, %0"
                 : "+v"(c0), "+v"(c1));
    FMA4; FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w + c0 + c1, out);
}

// + 1 v_rsq_f64 whose result feeds the next FMA of chain x
__global__ __launch_bounds__(256) void k_rsq(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  double r;
  for (int i = 0; i < kIters; ++i) {
    FMA4; FMA4;
    asm volatile("v_rsq_f64 %0, %1\nv_fma_f64 %0, %0, %2, %3" : "=&v"(r) : "v"(w), "v"(a), "v"(b));
    asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(r));
    FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + 1 v_rsq_f64 whose result is first read 16 FMAs later (latency hidden,
// only its issue cost left)
__global__ __launch_bounds__(256) void k_rsq_late(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  double r = 1.0;
  for (int i = 0; i < kIters; ++i) {
    asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(r));
    asm volatile("v_rsq_f64 %0, %1" : "=&v"(r) : "v"(w));
    FMA4; FMA4; FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + 1 v_sqrt_f64 whose result is first read 16 FMAs later
__global__ __launch_bounds__(256) void k_sqrt_late(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  double r = 1.0;
  for (int i = 0; i < kIters; ++i) {
    asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(r));
    asm volatile("v_sqrt_f64 %0, %1" : "=&v"(r) : "v"(w));
    FMA4; FMA4; FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + 1 v_rcp_f64 whose result is first read 16 FMAs later
__global__ __launch_bounds__(256) void k_rcp_late(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  double r = 1.0;
  for (int i = 0; i < kIters; ++i) {
    asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(r));
    asm volatile("v_rcp_f64 %0, %1" : "=&v"(r) : "v"(w));
    FMA4; FMA4; FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + 1 v_fma_f64 whose result feeds the very next FMA (FP64 dependency latency)
__global__ __launch_bounds__(256) void k_fmadep(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  double r;
  for (int i = 0; i < kIters; ++i) {
    FMA4; FMA4;
    asm volatile("v_fma_f64 %0, %1, %2, %3\nv_fma_f64 %0, %0, %2, %3" : "=&v"(r) : "v"(w), "v"(a), "v"(b));
    asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(r));
    FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w, out);
}

// + v_cmp_f64 (writes VCC) feeding 2 v_cndmask_b32 (a double select)
__global__ __launch_bounds__(256) void k_sel(double* out, Stamp* st, double a, double b, int half) {
  PROLOGUE
  int s0 = threadIdx.x, s1 = s0 + 7;
  for (int i = 0; i < kIters; ++i) {
    FMA4; FMA4;
    asm volatile(
        "v_cmp_lt_f64 vcc, %2, %3\n"
        "v_cndmask_b32 %0, %0, %1, vcc\n"
        "v_cndmask_b32 %1, %1, %0, vcc\n"
        : "+v"(s0), "+v"(s1) : "v"(x), "v"(y) : "vcc");
    FMA4; FMA4;
  }
  stamp_out(st, t0, r0, x + y + z + w + s0 + s1, out);
}

typedef void (*Kern)(double*, Stamp*, double, double, int);

int main() {
  struct K {
    const char* name;
    Kern k;
    int extra;  // non-FMA instructions per iteration
  } ks[] = {{"fma16", k_fma, 0},          {"fma16+4salu", k_salu, 4}, {"fma16+branch", k_branch, 1},
            {"fma16+cbranch_nt", k_nobranch, 2}, {"fma16+4mov64", k_mov64, 4}, {"fma16+4b32", k_b32, 4},
            {"fma16+rsq(dep)", k_rsq, 3}, {"fma16+rsq(late)", k_rsq_late, 2}, {"fma16+sqrt(late)", k_sqrt_late, 2},
            {"fma16+rcp(late)", k_rcp_late, 2}, {"fma16+fma2dep+add", k_fmadep, 3},  {"fma16+cmp+2cndmask", k_sel, 3}};
  const int maxw = 4096;
  double* out;
  Stamp* st;
  CHECK(hipMalloc(&out, sizeof(double) * maxw * 64));
  CHECK(hipMalloc(&st, sizeof(Stamp) * maxw));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // warm the clock: ~1 s of back-to-back launches
  for (int r = 0; r < 400; ++r) hipLaunchKernelGGL(k_fma, dim3(256), dim3(256), 0, 0, out, st, 0.999, 1e-3, 0);
  CHECK(hipDeviceSynchronize());
  // configurations: (waves per SIMD, half-populated)
  struct Cfg {
    int blocks, half;
    const char* what;
  } cfgs[] = {{256, 0, "1 wave/SIMD x64 lanes"}, {512, 1, "2 waves/SIMD x32 lanes"}, {512, 0, "2 waves/SIMD x64 lanes"}};
  for (auto& kk : ks) {
    for (auto& cf : cfgs) {
      std::vector<float> ms;
      for (int r = 0; r < 7; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(kk.k, dim3(cf.blocks), dim3(256), 0, 0, out, st, 0.999, 1e-3, cf.half);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float t;
        CHECK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      const int nw = cf.blocks * 4;
      std::vector<Stamp> h(nw);
      CHECK(hipMemcpy(h.data(), st, sizeof(Stamp) * nw, hipMemcpyDeviceToHost));
      std::vector<double> cyc, clk;
      for (auto& s : h) {
        if (s.t1 <= s.t0 || s.r1 <= s.r0) continue;
        cyc.push_back(double(s.t1 - s.t0) / kIters);
        clk.push_back(double(s.t1 - s.t0) / double(s.r1 - s.r0) * 100.0);  // MHz
      }
      std::sort(cyc.begin(), cyc.end());
      std::sort(clk.begin(), clk.end());
      const double c = cyc.empty() ? 0 : cyc[cyc.size() / 2], f = clk.empty() ? 0 : clk[clk.size() / 2];
      printf("%-22s %-24s  %7.3f ms  %7.1f cyc/iter  (%5.2f per instr of %d)  clock %6.0f MHz\n", kk.name, cf.what,
             ms[3], c, c / (16 + kk.extra), 16 + kk.extra, f);
    }
  }
  return 0;
}
