// qt_pair.hpp — the pair-lane flavour of the yaw-at-rest loop, for batches
// that leave SIMDs without a wave (DESIGN §5 "Small per-GPU batches").
//
// A lone wave issues one instruction per ~4.4 cycles whatever its lanes do, so
// below one wave per SIMD (65,536 episodes on MI355X) a pass costs the same
// 1.25 ms from 4,096 episodes up.  Here one episode runs on a PAIR of lanes
// (2k, 2k + 1 of a wave, 32 episodes per wave): lane a = 0 takes roll and the
// y axis, lane a = 1 pitch and the x axis — the structured gains couple roll
// to y and pitch to x only (compute_action, riccati_lqr.py:864-900) — and both
// lanes take z, the thrust, time and the target.  What crosses between the two
// (DPP quad_perm swaps, pair_swap): the partner's four RK4 stage cosines (the
// thrust direction couples the angles: sin(pitch) cos(roll), -sin(roll),
// cos(pitch) cos(roll)), its rate command and its squared horizontal error
// per step; its position, velocity and angle where the horizon, the vote and
// the finish need the whole state (once per horizon, rare).  The two square
// roots of a step split as well: lane 0's is the tracking error, lane 1's the
// command norm, through one shared sequence.  Per lane ~173 instructions per
// step instead of ~230 (scripts/microbench/split_step.hip): 1.3x for a batch
// of up to one wave per SIMD in pairs (32,768 episodes on MI355X).
//
// Every operation rounds as the one it replaces in run_yaw0 / integrate_yaw0
// (-ffp-contract=on: the same source expressions; products and sums that
// commute, -s == s * -1, (-w) s == w (-s) inside an fma), and a lane's
// results do not depend on the other lanes of its wave (run_yaw0), so the
// pair flavour's results are the one-lane flavour's bit for bit
// (tests/test_gpu_pair.py).
//
// Scope (launch_rollout checks it on the host): the yaw-at-rest flavour with
// structured 6-column LQR gains (shared, or per episode: the tuner's
// candidates), no feed-forward, no per-episode mass or hover thrust, one
// target motion for the whole batch (periodic targets carry their rotor in
// both lanes), no rewards, no motion groups; QT_PAIR=0 turns it off.
#pragma once

#include "qt_kernels.hpp"

namespace qtk {

// The partner lane's value (lanes 2k <-> 2k + 1): two 32-bit DPP moves
// (quad_perm [1, 0, 3, 2]; gfx950 has no 64-bit DPP lane swap).
__device__ __forceinline__ double pair_swap(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// d * d and (h + p) + z^2 without FMA contraction: sq3_ref's roundings
// ((a^2 + b^2) + c^2), the pair's two horizontal squares added in either order
__device__ __forceinline__ double pair_sq(double d) {
#pragma clang fp contract(off)
  return d * d;
}

__device__ __forceinline__ double pair_sq3(double h2, double p2, double dz) {
#pragma clang fp contract(off)
  return (h2 + p2) + dz * dz;
}

// rollout_lane's prologue for one episode: the reset state formed (a fresh
// pass, qt_rollout_fresh) or the stored state loaded.
template <int MOTION>
__device__ __forceinline__ void pair_episode_start(const qt_env_params& e, const BatchDev& b, const qt_state& st,
                                                   const LaunchConst& lc, int64_t ep, const Pattern& pt, double* x,
                                                   Target& tg, double& t, Acc& a) {
  const int64_t n = b.n;
  if (lc.fresh_off) {
    target_state<true>(e, MOTION, pt, 0.0, tg);
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = tg.p[i] + lc.fresh_off[i * n + ep];
#pragma unroll
    for (int i = 3; i < 12; ++i) x[i] = 0.0;
    t = 0.0;
    a = Acc{0, 0, -INFINITY, 0, 0, 0, 0, 0, 0, -1, -1, 0, 0, QT_TERM_RUNNING};
  } else {
#pragma unroll
    for (int i = 0; i < 12; ++i) x[i] = st.x[i * n + ep];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      tg.p[i] = st.target[i * n + ep];
      tg.v[i] = st.target[(3 + i) * n + ep];
      tg.a[i] = st.target[(6 + i) * n + ep];
    }
    t = st.t[ep];
    a = load_acc(st.acc, n, ep);
  }
}

// rollout_lane's wave test for the yaw-at-rest flavour (KC 6, no feed-forward,
// the launch's plant and hover thrust; no integral rows): the same conditions
// on the same values, so the exact pass after this launch takes exactly the
// waves it leaves.
__device__ __forceinline__ bool pair_lane_ok(const qt_env_params& e, const qt_ctrl_params& c, const Gains<6, true>& G,
                                             double hover, const Plant& pl, const double* x, const Target& tg,
                                             double t, const Acc& a) {
  const double integ[3] = {0.0, 0.0, 0.0};
  bool ok = a.term != QT_TERM_RUNNING ||
            (all_finite(G.k, Gains<6, true>::kCount) && all_finite(x, 12) && all_finite(integ, 3) &&
             all_finite(tg.p, 3) && all_finite(tg.v, 3) && all_finite(tg.a, 3) && finite_bits(hover) &&
             finite_bits(pl.inv_mass) && finite_bits(t) && fabs(t) < 1e300);
  for (int i = 9; i < 12; ++i) ok = ok && fabs(x[i]) <= e.max_angular_velocity;
  return ok && x[8] == 0.0 && x[11] == 0.0 && fabs(x[6]) <= kMaxTilt && fabs(x[7]) <= kMaxTilt &&
         fabs(x[9]) <= c.max_rate && fabs(x[10]) <= c.max_rate;
}

// run_yaw0<MOTION, 6, false, true, UNI> (qt_kernels.hpp) for the pair lane `a`
// of one episode: x, tg, t, acc hold the episode's whole launch-start state in
// both lanes; on return lane 0's hold the episode's end state (lane 1's its
// own half).  The loop structure, horizon and vote are run_yaw0's; see there.
template <int MOTION>
__device__ __forceinline__ void run_pair(const qt_env_params& e, const qt_ctrl_params& c, const qt_criteria& cr,
                                         const Pattern& pt, double hover, const Gains<6, true>& G, int a, double* x,
                                         Target& tg, double& t, Acc& acc_out, int nsteps, const LaunchConst& k) {
  // periodic targets carry their rotor (run_yaw0's kRotor; no feed-forward)
  constexpr bool kRotor = MOTION == QT_MOTION_CIRCULAR || MOTION == QT_MOTION_SINUSOIDAL || MOTION == QT_MOTION_FIGURE8;
  constexpr int kNeg = -(1 << 30);
  // The loop's uniforms (closed-form maps, plant, gains, clamps) held in VGPRs
  // (vpin): with them and the launch constants in scalar registers the kernel
  // needs more than a wave's 102 SGPRs and spills them to VGPR lanes, read
  // back with v_readlane in every step.  A pair batch runs one wave per SIMD,
  // so the VGPRs cost no occupancy.
  Plant pl = k.pl;
  VelLin L = k.vl;
  RateLin Rl = k.rl;
  pl.inv_mass = vpin(pl.inv_mass), pl.gz = vpin(pl.gz);
  L.cv = vpin(L.cv), L.pv = vpin(L.pv), L.gv = vpin(L.gv), L.gp = vpin(L.gp);
  for (int i = 0; i < 4; ++i) L.wv[i] = vpin(L.wv[i]);
  for (int i = 0; i < 3; ++i) L.pa[i] = vpin(L.pa[i]);
  Rl.wy = vpin(Rl.wy), Rl.wu = vpin(Rl.wu), Rl.ay = vpin(Rl.ay), Rl.au = vpin(Rl.au), Rl.h2 = vpin(Rl.h2);
  Rl.d3u = vpin(Rl.d3u), Rl.d4y = vpin(Rl.d4y), Rl.d4u = vpin(Rl.d4u), Rl.e3y = vpin(Rl.e3y);
  const double k0 = vpin(G.k[0]), k1 = vpin(G.k[1]), hov = vpin(hover);
  const double tmin = vpin(c.min_thrust), tmax = vpin(c.max_thrust), rmax = vpin(c.max_rate), dt = vpin(e.dt);
  const double cz = vpin(e.center[2]);
  const double R = vpin(cr.target_radius), eR = vpin(e.target_radius);
  const double vm2 = e.max_velocity * e.max_velocity * (1.0 - 1e-14);
  const double pos_up = nextafter(e.max_position, INFINITY);
  const int W = cr.overshoot_window;
  // lane selects as exact 0 / 1 factors where one FP64 slot replaces a select
  const double af = a, nf = 1.0 - af, am1 = af - 1.0;
  // the observation re-derived from t, as run_yaw0 does at launch start
  double rs[3] = {0.0, 0.0, 0.0}, rc[3] = {1.0, 1.0, 1.0};  // carried target rotor
  if constexpr (kRotor) {
    rotor_init<MOTION>(pt, t, rs, rc);
    target_from_rotor<false, MOTION>(e, pt, rs, rc, tg);
  } else {
    target_state<false, true>(e, MOTION, pt, t, tg);
  }
  // this lane's axis and angle: a = 0 roll and y, a = 1 pitch and x
  const double Kp = a ? G.k[4] : G.k[2], Kv = a ? G.k[5] : G.k[3];
  const double cen_h = a ? e.center[0] : e.center[1], ch = a ? pt.c0 : pt.c1;
  double ph = a ? x[0] : x[1], vh = a ? x[3] : x[4], pz = x[2], vz = x[5];
  double ang = a ? x[7] : x[6], w = a ? x[10] : x[9];
  double tph = a ? tg.p[0] : tg.p[1], tvh = a ? tg.v[0] : tg.v[1], tpz = tg.p[2], tvz = tg.v[2];
  Acc& A = acc_out;
  // launch start as run_yaw0: the pre-step error of the current observation
  // (lane 0's val; lane 1's val is the last command norm, 0 before the first),
  // this lane's roll / pitch trig
  double val = a ? 0.0 : sqrt_pos(sq3_ref(tg.p[0] - x[0], tg.p[1] - x[1], tg.p[2] - x[2]));
  double s0, c0;
  sincos_tilt(ang, &s0, &c0);
  int z = A.prev_on == 1 ? 1 : (A.os_streak >= 0 ? A.os_streak + 1 : kNeg);
  double cur = A.os_cur;
  int on_pre = A.on_pre, on_post = A.on_post, os_count = A.os_count;
  double acc = a ? A.sum_u : A.sum_e;  // lane 0: sum_e, lane 1: sum_u
  double sum_e2 = A.sum_e2, max_e = A.max_e, os_max = A.os_max;
  bool stepped = false;
  // the episode's positions, velocities, roll / pitch and their rates from the
  // pair (the horizon, the vote, the finish; x[8] and x[11] stay at rest)
  auto gather = [&](double* xf) {
    const double pp = pair_swap(ph), vp = pair_swap(vh), angp = pair_swap(ang), wp = pair_swap(w);
    xf[0] = a ? ph : pp, xf[1] = a ? pp : ph, xf[2] = pz;
    xf[3] = a ? vh : vp, xf[4] = a ? vp : vh, xf[5] = vz;
    xf[6] = a ? angp : ang, xf[7] = a ? ang : angp;
    xf[9] = a ? wp : w, xf[10] = a ? w : wp;
  };
  double sm, cmx;
  sincos_tilt(kMaxTilt, &sm, &cmx);  // the tilt clamp's trig bounds (tilt_clamp)
  int s = 0;
  while (A.term == QT_TERM_RUNNING && s < nsteps) {
    const int s_0 = s;
    int rem = nsteps - s_0 > (1 << 29) ? (1 << 29) : nsteps - s_0;
    RateCoef rk;
    // CLAMP: the tilt clamp in a no-vote step (run_yaw0's DUAL body)
    auto step = [&](auto vote, auto clamp) -> bool {
      constexpr bool VOTE = decltype(vote)::value, CLAMP = decltype(clamp)::value;
      rk.pin();
      const double a0 = ang;
      // ---- compute_action (riccati_lqr.py:779-967): thrust from z, this lane's rate from its axis
      const double uf0 = k0 * (tpz - pz) + k1 * (tvz - vz);
      const double ufa = Kp * (tph - ph) + Kv * (tvh - vh);
      const double raw0 = hov + uf0;
      const double u0 = clip_num(raw0, tmin, tmax);
      const double ua = clip_num(ufa, -rmax, rmax);
      // ---- the Evaluator's pre-step record (eval.py:142-159): lane 0's err
      // accumulators; lane 1's acc is sum_u, a step behind
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
      // ---- integrate_yaw0 for this lane's angle and axis
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
      double svh = 0.0, sph = 0.0, svz = 0.0, spz = 0.0;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const double cp = pair_swap(cs[i]);
        const double rh = ss[i] * fma(cp, af, am1);  // pitch lane: sin(pitch) cos(roll); roll lane: -sin(roll)
        const double rz = cs[i] * cp;                // cos(pitch) cos(roll)
        svh = fma(L.wv[i], rh, svh);
        svz = fma(L.wv[i], rz, svz);
        sph = fma(L.pa[i], rh, sph);
        spz = fma(L.pa[i], rz, spz);
      }
      {  // stage 4 reaches the velocities only: its weight folded into cos(roll)
        const double cp = pair_swap(c3);
        const double cr = a ? cp : c3, cq = a ? c3 : cp;  // roll's, pitch's cosine
        const double wc = L.wv[3] * cr;
        svh = fma(a ? wc : -L.wv[3], s3, svh);
        svz = fma(wc, cq, svz);
      }
      const double tm = u0 * pl.inv_mass;
      ph = fma(tm, sph, fma(L.pv, vh, ph));
      pz = fma(tm, spz, fma(L.pv, vz, pz + L.gp));
      vh = fma(tm, svh, L.cv * vh);
      vz = fma(tm, svz, fma(L.cv, vz, L.gv));
      ang = fma(Rl.ay, w, fma(Rl.au, ua, ang));
      w = fma(Rl.wy, w, Rl.wu * ua);
      const double t0 = t;
      t += dt;
      if constexpr (kRotor) {  // the rotor turned by one step (rotor_advance), the whole target from it
        rotor_advance<MOTION>(k, (t - t0) - dt, rs, rc);
        target_from_rotor<false, MOTION>(e, pt, rs, rc, tg);
        tph = a ? tg.p[0] : tg.p[1], tvh = a ? tg.v[0] : tg.v[1], tpz = tg.p[2], tvz = tg.v[2];
      } else if constexpr (MOTION == QT_MOTION_LINEAR) {  // target_state (linear): center + c t
        tph = cen_h + ch * t;
        tpz = cz + pt.c2 * t;
        tvh = ch, tvz = pt.c2;
      } else {  // stationary: the fixed point
        tph = cen_h, tpz = cz, tvh = 0.0, tvz = 0.0;
      }
      // ---- post-step error (lane 0; the env's on-target count and the next
      // pre-step error) and this step's command norm (lane 1), one root
      const double dh2 = pair_sq(ph - tph), dp2 = pair_swap(dh2);
      const double up = pair_swap(ua);
      const double ur = a ? up : ua, uq = a ? ua : up;  // roll's, pitch's command
      const double e2 = pair_sq3(dh2, dp2, pz - tpz);
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
        val = fma(dd, hh * nf, gg);  // lane 0: sqrt_pos(e2); lane 1: sqrt_sum(un2) (a zero correction)
      }
      on_post += val <= eR;
      // ---- angle wrap, carried trig (attitude_trig_resid), the tilt clamp of a voted step
      ang = (ang + kPi) - kPi;
      {
        double sr, cr;
        tiny_sincos((ang - a0) - d4, &sr, &cr);
        rotate_cm(s3, c3, sr, cr, &s0, &c0);
      }
      if constexpr (VOTE || CLAMP) {
        ang = clip_num(ang, -kMaxTilt, kMaxTilt);
        s0 = clip_num(s0, -sm, sm);
        c0 = fmax(c0, cmx);
      }
      if constexpr (!VOTE) return false;
      --rem;
      double xf[12];
      gather(xf);
      const double stop_m = fmax(
          fmax(fmax(fabs(xf[0]), fmax(fabs(xf[1]), fabs(xf[2]))) - pos_up, (xf[3] * xf[3] + xf[4] * xf[4] + xf[5] * xf[5]) - vm2),
          fmax(t - e.max_episode_time, -(double)rem));
      return __builtin_amdgcn_ballot_w64(stop_m >= 0.0) != 0;
    };
    do {
      double xf[12];
      gather(xf);
      int H = yaw0_horizon<true, false>(e, k.hz, L, pl, xf, t, rem);
      bool clamp_body = false;  // wave-uniform (H comes from ballots)
      if constexpr (kRotor) {  // run_yaw0's DUAL (the one-lane fresh pass takes it for periodic LQR loops)
        if (H < k.hz.dual_below) {
          const int H2 = yaw0_horizon<false, false>(e, k.hz, L, pl, xf, t, rem);
          if (H2 > H) H = H2, clamp_body = true;
        }
      }
      using F = std::false_type;
      using T = std::true_type;
      if (kRotor && clamp_body) {
        for (int j = 4; j <= H; j += 4) {
          step(F{}, T{});
          step(F{}, T{});
          step(F{}, T{});
          step(F{}, T{});
        }
        if (H & 2) {
          step(F{}, T{});
          step(F{}, T{});
        }
      } else {
        for (int j = 4; j <= H; j += 4) {
          step(F{}, F{});
          step(F{}, F{});
          step(F{}, F{});
          step(F{}, F{});
        }
        if (H & 2) {
          step(F{}, F{});
          step(F{}, F{});
        }
      }
      rem -= H;
      const int nv = H > 0 ? 0 : (k.hz.on ? kVotedBurst : (1 << 30));
      bool stop = false;
      for (int j = 0; j < nv && !stop; ++j) stop = step(T{}, F{});
      if (stop) break;
    } while (true);
    const int ran = (nsteps - s_0 > (1 << 29) ? (1 << 29) : nsteps - s_0) - rem;
    s += ran;
    A.steps += ran;
    stepped = true;
    z = z <= 0 ? kNeg : z;
    // finish the last step exactly: the velocity clamp, per-episode termination
    double xf[12];
    gather(xf);
    clamp_velocity(e, xf);
    vh = a ? xf[3] : xf[4], vz = xf[5];
    A.term = termination_fast(e, t, xf);
  }
  // lane 1's last command norm, then sum_u to lane 0
  acc += a ? val : 0.0;
  const double acc_p = pair_swap(acc);
  A.sum_e = a ? acc_p : acc;
  A.sum_u = a ? acc : acc_p;
  A.sum_e2 = sum_e2, A.max_e = max_e, A.os_max = os_max;
  if (stepped) {
    A.on_pre = on_pre, A.on_post = on_post, A.os_count = os_count;
    A.prev_on = z == 1 ? 1 : 0;
    A.os_streak = z >= 2 ? z - 1 : -1;
    A.os_cur = cur;
  }
  // the whole end state in both lanes (lane 0 stores it)
  double xf[12];
  gather(xf);
  x[0] = xf[0], x[1] = xf[1], x[2] = xf[2], x[3] = xf[3], x[4] = xf[4], x[5] = xf[5];
  x[6] = xf[6], x[7] = xf[7], x[9] = xf[9], x[10] = xf[10];
  if constexpr (!kRotor) {  // (a periodic target's tg is the last step's whole target already)
    const double tpp = pair_swap(tph), tvp = pair_swap(tvh);
    tg.p[0] = a ? tph : tpp, tg.p[1] = a ? tpp : tph, tg.p[2] = tpz;
    tg.v[0] = a ? tvh : tvp, tg.v[1] = a ? tvp : tvh, tg.v[2] = tvz;
    tg.a[0] = tg.a[1] = tg.a[2] = 0.0;  // target_state without feed-forward (linear, stationary)
  }
}

// One pair-lane wave per 32 episodes; the deferral test runs over the exact
// pass's 64-episode waves (both pair waves of one decide alike), so a wave the
// exact pass skips is one this launch ran whole.  PERK: per-episode gains
// (qt_batch.k_per_episode, the tuner's candidates), else one shared gain.
template <int MOTION, bool PERK>
__global__ __launch_bounds__(kBlock) void rollout_pair_kernel(qt_env_params e, qt_ctrl_params c, qt_criteria cr,
                                                              BatchDev b, qt_state st, int nsteps, LaunchConst lc) {
  const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t n = b.n;
  const double hover = c.hover_thrust;
  const Plant& pl = lc.pl;
  {
    const int64_t te = ((g >> 7) << 6) + (g & 63);  // this lane's episode of the exact pass's wave
    bool ok = true;
    if (te < n) {
      Gains<6, true> G;
      load_gains<6, true, !PERK>(b, te, G);
      const Pattern pt = pattern_of(b, e, MOTION, te);
      double x[12];
      Target tg;
      double t;
      Acc a;
      pair_episode_start<MOTION>(e, b, st, lc, te, pt, x, tg, t, a);
      ok = pair_lane_ok(e, c, G, hover, pl, x, tg, t, a);
    }
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
      if (lc.defer_flag) *lc.defer_flag = lc.epoch;  // the exact pass has work (every lane stores the same value)
      const int64_t ep = g >> 1;
      if (lc.fresh_off && ep < n && (g & 1) == 0) {  // the reset state, for the exact pass (rollout_lane)
        const Pattern pt = pattern_of(b, e, MOTION, ep);
        double x[12];
        Target tg;
        double t;
        Acc a;
        pair_episode_start<MOTION>(e, b, st, lc, ep, pt, x, tg, t, a);
#pragma unroll
        for (int i = 0; i < 12; ++i) st.x[i * n + ep] = x[i];
        if (st.integ) {
#pragma unroll
          for (int i = 0; i < 3; ++i) st.integ[i * n + ep] = 0.0;
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          st.target[i * n + ep] = tg.p[i];
          st.target[(3 + i) * n + ep] = tg.v[i];
          st.target[(6 + i) * n + ep] = tg.a[i];
        }
        st.t[ep] = t;
        store_acc(st.acc, n, ep, a);
      }
      return;
    }
  }
  const int64_t ep = g >> 1;
  if (ep >= n) return;  // both lanes of a pair leave together
  const int a = (int)(g & 1);
  Gains<6, true> G;
  load_gains<6, true, !PERK>(b, ep, G);
  const Pattern pt = pattern_of(b, e, MOTION, ep);
  double x[12];
  Target tg;
  double t;
  Acc acc;
  pair_episode_start<MOTION>(e, b, st, lc, ep, pt, x, tg, t, acc);
  run_pair<MOTION>(e, c, cr, pt, hover, G, a, x, tg, t, acc, nsteps, lc);
  if (a) return;
  if (MOTION == QT_MOTION_CIRCULAR || MOTION == QT_MOTION_SINUSOIDAL || MOTION == QT_MOTION_FIGURE8) {
    // the stored observation carries the reference's acceleration (rollout_lane)
    Target full;
    target_state<true>(e, MOTION, pt, t, full);
#pragma unroll
    for (int i = 0; i < 3; ++i) tg.a[i] = full.a[i];
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) st.x[i * n + ep] = x[i];
  if (lc.fresh_off && st.integ) {  // a fresh pass stores the zeros qt_reset would (rollout_lane)
#pragma unroll
    for (int i = 0; i < 3; ++i) st.integ[i * n + ep] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    st.target[i * n + ep] = tg.p[i];
    st.target[(3 + i) * n + ep] = tg.v[i];
    st.target[(6 + i) * n + ep] = tg.a[i];
  }
  st.t[ep] = t;
  store_acc(st.acc, n, ep, acc);
  if (lc.met) store_metrics(cr, acc, t, lc.met, n, ep);  // a fresh pass: the metrics rows (rollout_lane)
}

}  // namespace qtk
