// qt_rollout_fast.hip — the fast step flavours of the rollout kernel
// (qt_kernels.hpp: kFast, kYaw0).  Built with relaxed NaN handling for the
// device (-fno-honor-nans -mno-amdgpu-ieee, Makefile): a fast flavour runs
// only waves whose every lane starts finite (bit tests at kernel entry,
// all_finite) and stays finite by construction (clipped commands, clamped
// rates, wrapped angles, bounded position updates), so min / max need no
// signalling-NaN canonicalisation of their operands.  The exact flavour and
// every NaN-handling path stay in qt_rollout.hip (IEEE mode).
#define QT_FAST_TU 1
#include <hip/hip_runtime.h>

#ifndef QT_CLOCK_STAMP
#define QT_CLOCK_STAMP 0
#endif
#if QT_CLOCK_STAMP
// Diagnostic clock-stamp build (scripts/clock_stamp.py; -DQT_CLOCK_STAMP=1):
// lane 0 of every wave of a fast-flavour launch records s_memtime (shader
// clock) and s_memrealtime (100 MHz) around its step loop into this buffer of
// its own, which no other code reads; qt_debug_stamps copies it out.  The
// product build has QT_CLOCK_STAMP == 0 and executes no stamp.
constexpr int kStampWaves = 1 << 16;
__device__ unsigned long long g_qt_stamps[kStampWaves][6];  // memtime x2, realtime x2, HW_ID, XCC_ID
#endif

#include "qt_kernels.hpp"
#include "qt_pair.hpp"

namespace qtk {

namespace {
struct FastLaunch {
  template <int MOTION, int KC, bool FF, bool KS>
  static void run(int flavor, bool uni, int grid, hipStream_t s, const qt_env_params& e, const qt_ctrl_params& c,
                  const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps, const LaunchConst& lc) {
    // (uni, the SGPR-resident plant / gain variant, is not instantiated: with
    // the closed-form and launch constants it overflows the 102 SGPRs and
    // spills through v_writelane / v_readlane in the step loop)
    (void)uni;
    if (flavor == kYaw0)
      rollout_kernel<kYaw0, MOTION, KC, FF, KS><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, nullptr, kExact, lc);
    else
      rollout_kernel<kFast, MOTION, KC, FF, KS><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, nullptr, kExact, lc);
  }
};
}  // namespace

struct GroupedLaunch {
  template <int MOTION, int KC, bool FF, bool KS>
  static void run(int grid, hipStream_t s, const qt_env_params& e, const qt_ctrl_params& c, const qt_criteria& cr,
                  const BatchDev& b, const qt_state& st, int nsteps, const LaunchConst& lc) {
    if constexpr (MOTION == -1)  // one kernel per (KC, FF, KS): instantiated through the runtime-motion slot only
      rollout_grouped_kernel<KC, FF, KS><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, lc);
  }
};

void launch_fast(int flavor, bool uni, bool grouped, int kc, bool ff, bool ks, int motion, int grid, hipStream_t s,
                 const qt_env_params& e, const qt_ctrl_params& c, const qt_criteria& cr, const BatchDev& b,
                 const qt_state& st, int nsteps, const LaunchConst& lc) {
  if (grouped && flavor == kYaw0)
    dispatch_rollout<GroupedLaunch>(kc, ff, ks, -1, grid, s, e, c, cr, b, st, nsteps, lc);
  else
    dispatch_rollout<FastLaunch>(kc, ff, ks, motion, flavor, uni, grid, s, e, c, cr, b, st, nsteps, lc);
}

namespace {
template <int MOTION>
void launch_pair_motion(int grid, hipStream_t s, const qt_env_params& e, const qt_ctrl_params& c,
                        const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps,
                        const LaunchConst& lc) {
  if (b.k_per_episode)
    rollout_pair_kernel<MOTION, true><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, lc);
  else
    rollout_pair_kernel<MOTION, false><<<grid, kBlock, 0, s>>>(e, c, cr, b, st, nsteps, lc);
}
}  // namespace

void launch_pair(int motion, int grid, hipStream_t s, const qt_env_params& e, const qt_ctrl_params& c,
                 const qt_criteria& cr, const BatchDev& b, const qt_state& st, int nsteps, const LaunchConst& lc) {
  switch (motion) {
    case QT_MOTION_LINEAR: launch_pair_motion<QT_MOTION_LINEAR>(grid, s, e, c, cr, b, st, nsteps, lc); break;
    case QT_MOTION_CIRCULAR: launch_pair_motion<QT_MOTION_CIRCULAR>(grid, s, e, c, cr, b, st, nsteps, lc); break;
    case QT_MOTION_SINUSOIDAL: launch_pair_motion<QT_MOTION_SINUSOIDAL>(grid, s, e, c, cr, b, st, nsteps, lc); break;
    case QT_MOTION_FIGURE8: launch_pair_motion<QT_MOTION_FIGURE8>(grid, s, e, c, cr, b, st, nsteps, lc); break;
    default: launch_pair_motion<QT_MOTION_STATIONARY>(grid, s, e, c, cr, b, st, nsteps, lc); break;
  }
}

}  // namespace qtk

#if QT_CLOCK_STAMP
extern "C" {
// Diagnostic build only: copy the first `waves` stamp records
// {memtime start, end, realtime start, end} to host memory out[waves][4].
int qt_debug_stamps(unsigned long long* out, int64_t waves) {
  if (!out || waves < 0 || waves > kStampWaves) return QT_EINVAL;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qt_stamps), sizeof(unsigned long long) * 6 * waves) == hipSuccess
             ? QT_OK
             : QT_ELAUNCH;
}
}
#endif
