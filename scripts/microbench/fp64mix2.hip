// Issue cost of FP64 instruction encodings for a lone wave per SIMD, round 2.
// fp64mix showed VOP3 forms (v_fma / v_mul / v_add _f64, 8-byte encoding) at
// ~5.25 cycles per instruction against ~4.94 for the VOP2 v_fmac_f64 (4 bytes)
// in a 32-instruction loop.  Here: the loop overhead separated from the
// per-instruction cost (32 vs 64 instructions per trip), an alternating
// VOP2 / VOP3 stream (an encoding-size effect would average out, a per-form
// one would not), and the VOP3 stream with two waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 fp64mix2.hip -o fp64mix2
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

// eight independent accumulators x0..x7, multiplier a (v), b (v)
#define FMA3(r) "v_fma_f64 " r ", " r ", %8, %9\n"
#define FMAC(r) "v_fmac_f64 " r ", %8, %9\n"
#define ALL8(M) M("%0") M("%1") M("%2") M("%3") M("%4") M("%5") M("%6") M("%7")
#define MIX8 FMAC("%0") FMA3("%1") FMAC("%2") FMA3("%3") FMAC("%4") FMA3("%5") FMAC("%6") FMA3("%7")
#define OPS : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(a), "v"(b)

#define KERNEL(NAME, BLOCK8, REPS)                                                                     \
  __global__ __launch_bounds__(256) void NAME(double* out, unsigned long long* st, double a, double b) { \
    double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,  \
           x6 = x0 + 6, x7 = x0 + 7;                                                                   \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                        \
    for (int i = 0; i < kIters; ++i) {                                                                  \
      _Pragma("unroll") for (int r = 0; r < REPS; ++r) asm volatile(BLOCK8 OPS);                        \
    }                                                                                                   \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                        \
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;                                              \
    out[gid] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                                                   \
    if ((threadIdx.x & 63) == 0) st[gid >> 6] = t1 - t0;                                                \
  }

KERNEL(k_fmac32, ALL8(FMAC), 4)
KERNEL(k_fmac64, ALL8(FMAC), 8)
KERNEL(k_fma32, ALL8(FMA3), 4)
KERNEL(k_fma64, ALL8(FMA3), 8)
KERNEL(k_mix32, MIX8, 4)
KERNEL(k_mix64, MIX8, 8)

typedef void (*Kern)(double*, unsigned long long*, double, double);

int main() {
  struct K {
    const char* name;
    Kern k;
    int ninst, blocks;
  } ks[] = {{"fmac x32", k_fmac32, 32, 256}, {"fmac x64", k_fmac64, 64, 256},
            {"fma x32", k_fma32, 32, 256},   {"fma x64", k_fma64, 64, 256},
            {"mix x32", k_mix32, 32, 256},   {"mix x64", k_mix64, 64, 256},
            {"fma x64, 2 waves/SIMD", k_fma64, 64, 512}, {"fmac x64, 2 waves/SIMD", k_fmac64, 64, 512}};
  const int maxw = 512 * 4;
  double* out;
  unsigned long long* st;
  CHECK(hipMalloc(&out, sizeof(double) * maxw * 64));
  CHECK(hipMalloc(&st, sizeof(unsigned long long) * maxw));
  for (int r = 0; r < 200; ++r) hipLaunchKernelGGL(k_fma64, dim3(256), dim3(256), 0, 0, out, st, 0.999, 1e-3);
  CHECK(hipDeviceSynchronize());
  for (auto& kk : ks) {
    const int nw = kk.blocks * 4;
    hipLaunchKernelGGL(kk.k, dim3(kk.blocks), dim3(256), 0, 0, out, st, 0.999, 1e-3);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(nw);
    CHECK(hipMemcpy(h.data(), st, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    const double per = double(h[nw / 2]) / kIters;
    printf("%-24s %7.1f cycles per trip, %5.2f per instruction (wave view, loop overhead included)\n", kk.name, per,
           per / kk.ninst);
  }
  return 0;
}
