// qloco_force.hip -- batched Go1 force-distribution QP (gfx950).
//
// Replaces Dynamiccclass::force_distribution + force_opt + solve_grf_opt +
// Solve (go1_rt_control/src/whole_body_dynamics/dynmics_compute.cpp:141-445),
// called every 1 kHz servo tick at servo.cpp:1224-1228 (sim) and
// torque_mode.cpp:1364-1367 (hardware).  One instance per 16-lane group:
// the group builds G = 2(alpha A'A + (beta+gamma) I), g0, the swing-leg
// equality pattern CE and the shared friction/bound rows CI in LDS, then
// runs the Goldfarb-Idnani solver of qloco_gi_core.hpp on them.  The
// skew_hat comma-operator bug (:379-381) and the F_prev = grf_opt coupling
// (:305) are reproduced; a NaN solution falls back to F_leg_guess (:364-367).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

#include "qloco_gi_core.hpp"

namespace qloco {

struct ForceArgs {
  double mass, alpha, beta, gamma, fz_max, mu;
  int64_t batch;
  const double *com_des, *leg_des, *F_force_des, *rfoot_des, *lfoot_des;
  const double *base_p, *feet_p, *FT_total_des, *y_coef;
  const int *mode, *right_support;
  double *F_leg_ref, *grf_opt, *F_leg_guess;
  int *qp_solution, *status, *iters;
  // grouped dispatch (qloco_force_qp_solve_ordered): position -> robot, and
  // the per-robot iteration count carried to the next call's grouping
  const int *list;
  int *prev_it;
};

// Robots grouped by control flow before the launch.  The four 16-lane
// groups of a wave run each other's divergent paths: which swing-leg
// equality rows exist (pattern) and how many active-set iterations the solve
// takes.  With the synthetic mixed-gait batch in its given order 0.736 ms per
// 65,536 robots; grouped by pattern on the host 0.515 ms; by pattern, then by
// iteration count 0.422 ms (profiles/r5w_force_qp_order.txt).  The servo
// calls force_opt every tick with the robot's member state (grf_opt, F_leg_ref),
// so the previous call's iteration count is kept per robot in the caller's
// workspace and predicts this call's; class = pattern * 16 + min(prev, 15).
// Every robot's arithmetic is unchanged (groups never share data), so the
// results are bit-identical to the ungrouped launch.
constexpr int kForcePatterns = 5, kForceItBins = 16, kForceClasses = kForcePatterns * kForceItBins;
static_assert(kForceClasses == QLOCO_FORCE_CLASSES, "qloco_common.hpp");

// The swing-leg equality patterns AA (dynmics_compute.cpp:310-350): 0 = none
// (rs = 2 or other modes), 1 = mode 102 rs 0 (FL, RR zero), 2 = mode 102
// rs 1 (FR, RL), 3 = mode 101 rs 0 (FR, RR), 4 = mode 101 rs 1 (FL, RL);
// 12x12 column-major, in constant memory (identical for every robot).
__constant__ double c_force_CE[5][144];

// Per group: A (6x12) is built in the solver's R and G in its J (both are
// free until the solve starts: the solver copies G's lower triangle into R
// before it forms J, and A is dead once G and g0 are built); g0 lives in the solver's z (first written by
// update_z in the equality loop, after the last reads of g0: the x0 solve and
// f = g0'x / 2); the inequality rows are generated (ForceCi), F_leg_guess
// stays in the owning lanes' registers, ce0 is the constant zero vector and
// the solution is read from gi.x.  With R packed and the per-constraint
// state in registers (qloco_gi_core.hpp) a group needs 2.47 KB: an 8-robot
// block (8-lane groups) 19.8 KB, eight blocks per CU -- the two waves per
// SIMD the register budget allows; a 4-robot block (16-lane groups) 9.9 KB.
template <int FG>
struct ForceLds {
  struct Grp {
    GiLdsT<12, 24, 12> gi;
  } g[FG];
};

__constant__ double c_force_zeros[16];

// swing-leg equality pattern of (gait mode, right_support), dynmics_compute.cpp:310-350
__device__ __forceinline__ int force_pattern(int mode, int rs) {
  if (mode == 102) return rs == 0 ? 1 : rs == 1 ? 2 : 0;
  if (mode == 101) return rs == 0 ? 3 : rs == 1 ? 4 : 0;
  return 0;
}
__device__ __forceinline__ int force_class(const int *mode, const int *rs, const int *prev, int64_t i) {
  const unsigned it = (unsigned)prev[i];
  return force_pattern(mode[i], rs[i]) * kForceItBins + (int)(it < kForceItBins ? it : kForceItBins - 1);
}

// class sizes: an LDS histogram per block, one global add per (block, class)
__global__ __launch_bounds__(256) void force_count_kernel(int64_t batch, const int *mode, const int *rs,
                                                          const int *prev, int *count) {
  __shared__ int h[kForceClasses];
  for (int k = threadIdx.x; k < kForceClasses; k += 256) h[k] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < batch) atomicAdd(&h[force_class(mode, rs, prev, i)], 1);
  __syncthreads();
  for (int k = threadIdx.x; k < kForceClasses; k += 256)
    if (h[k]) atomicAdd(&count[k], h[k]);
}

// positions: class offset (exclusive prefix of the sizes) + this block's
// range in the class (one global add per (block, class)) + the robot's rank
// in the block's share; the order inside a class is immaterial
__global__ __launch_bounds__(256) void force_scatter_kernel(int64_t batch, const int *mode, const int *rs,
                                                            const int *prev, const int *count, int *cursor,
                                                            int *list) {
  __shared__ int off[kForceClasses], h[kForceClasses], base[kForceClasses];
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int k = 0; k < kForceClasses; ++k) {
      off[k] = acc;
      acc += count[k];
    }
  }
  for (int k = threadIdx.x; k < kForceClasses; k += 256) h[k] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int c = 0, r = 0;
  if (i < batch) {
    c = force_class(mode, rs, prev, i);
    r = atomicAdd(&h[c], 1);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < kForceClasses; k += 256)
    if (h[k]) base[k] = atomicAdd(&cursor[k], h[k]);
  __syncthreads();
  if (i < batch) list[off[c] + base[c] + r] = (int)i;
}

// CI = -qp_H' and ci0 = qp_h of Dynamiccclass (dynmics_compute.cpp:75-98):
// per leg i, constraint rows 2i / 2i+1 bound fz in [0, fz_max], rows 8+2i,
// 8+2i+1 and 16+2i, 16+2i+1 the x / y friction pyramid with mu.  CI(v, c) is
// generated from (v, c) -- the same doubles the matrix holds (0, +-1, mu),
// so every dot product over it is unchanged.
struct ForceCi {
  double mu, fz_max;
  __device__ __forceinline__ double a(int v, int c, int) const {
    const int grp = c >> 3, i = (c & 7) >> 1, lo = (c & 1) == 0;
    if (v == 3 * i + 2) return grp == 0 ? (lo ? 1.0 : -1.0) : mu;
    if (grp > 0 && v == 3 * i + grp - 1) return lo ? 1.0 : -1.0;
    return 0.0;
  }
  __device__ __forceinline__ double b(int c) const { return (c < 8 && (c & 1)) ? fz_max : 0.0; }
};

__device__ __forceinline__ double sq(double v) { return v * v; }

// dynmics_compute.cpp:141-261 (scalar, executed redundantly by the group).
// Both gait branches are evaluated and the result selected per entry: with
// per-branch stores the compiler sinks them into one dynamically indexed
// store and R lands in scratch (a per-lane spill written back to HBM).
__device__ __forceinline__ void force_distribution(const double *com_des, const double *leg_des,
                                                   const double *F, int mode, double y_coefficient,
                                                   const double *rfoot_des, const double *lfoot_des,
                                                   double (&R)[12] /* F_leg_ref 3x4 col-major, in/out */) {
  // mode 101 (:155-182): distance ratios
  double p1[12];
#define FRC(r, c) p1[(c)*3 + (r)]
  {
    const double body_FR_dis = sqrt(sq(com_des[0] - leg_des[0]) + sq(com_des[1] - leg_des[1]) + sq(com_des[2] - leg_des[2]));
    const double body_FL_dis = sqrt(sq(com_des[0] - leg_des[3]) + sq(com_des[1] - leg_des[4]) + sq(com_des[2] - leg_des[5]));
    const double body_RR_dis = sqrt(sq(com_des[0] - leg_des[6]) + sq(com_des[1] - leg_des[7]) + sq(com_des[2] - leg_des[8]));
    const double body_RL_dis = sqrt(sq(com_des[0] - leg_des[9]) + sq(com_des[1] - leg_des[10]) + sq(com_des[2] - leg_des[11]));
    double f_double;
    f_double = F[0] * body_FL_dis / (body_FL_dis + body_RL_dis);
    FRC(0, 3) = f_double;
    FRC(0, 1) = F[0] - f_double;
    f_double = F[1] * body_FL_dis / (body_FL_dis + body_RL_dis) * y_coefficient;
    FRC(1, 3) = f_double;
    FRC(1, 1) = F[1] * y_coefficient - f_double;
    f_double = F[2] * body_FL_dis / (body_FL_dis + body_RL_dis);
    FRC(2, 3) = f_double;
    FRC(2, 1) = F[2] - f_double;
    f_double = F[3] * body_FR_dis / (body_FR_dis + body_RR_dis);
    FRC(0, 2) = f_double;
    FRC(0, 0) = F[3] - f_double;
    f_double = F[4] * body_FR_dis / (body_FR_dis + body_RR_dis) * y_coefficient;
    FRC(1, 2) = f_double;
    FRC(1, 0) = F[4] * y_coefficient - f_double;
    f_double = F[5] * body_FR_dis / (body_FR_dis + body_RR_dis);
    FRC(2, 2) = f_double;
    FRC(2, 0) = F[5] - f_double;
  }
#undef FRC
  // mode 102 (:185-246): projection ratios clamped to [0, 1]
  double p2[12];
#define FRC(r, c) p2[(c)*3 + (r)]
  {
    double f_double;
    const double v0 = leg_des[9] - leg_des[0], v1 = leg_des[10] - leg_des[1], v2 = leg_des[11] - leg_des[2];
    const double c0 = lfoot_des[0] - leg_des[0], c1 = lfoot_des[1] - leg_des[1], c2 = lfoot_des[2] - leg_des[2];
    const double rlleg_dis = sqrt(sq(v0) + sq(v1) + sq(v2));
    const double com_rleg_dis = v0 * c0 + v1 * c1 + v2 * c2;
    const double raw = com_rleg_dis / rlleg_dis;
    const double raw1 = raw < 1.0 ? raw : 1.0;
    const double rleg_com = raw1 > 0.0 ? raw1 : 0.0;
    f_double = F[0] * rleg_com;
    FRC(0, 3) = f_double;
    FRC(0, 0) = F[0] - f_double;
    f_double = F[1] * rleg_com * y_coefficient;
    FRC(1, 3) = f_double;
    FRC(1, 0) = F[1] * y_coefficient - f_double;
    f_double = F[2] * rleg_com;
    FRC(2, 3) = f_double;
    FRC(2, 0) = F[2] - f_double;
    const double w0 = leg_des[6] - leg_des[3], w1 = leg_des[7] - leg_des[4], w2 = leg_des[8] - leg_des[5];
    const double e0 = rfoot_des[0] - leg_des[3], e1 = rfoot_des[1] - leg_des[4], e2 = rfoot_des[2] - leg_des[5];
    const double rlleg_disx = sqrt(sq(w0) + sq(w1) + sq(w2));
    const double com_rleg_disx = w0 * e0 + w1 * e1 + w2 * e2;
    const double rawx = com_rleg_disx / rlleg_disx;
    const double raw1x = rawx < 1.0 ? rawx : 1.0;
    const double rleg_comx = raw1x > 0.0 ? raw1x : 0.0;
    f_double = F[3] * rleg_comx;
    FRC(0, 2) = f_double;
    FRC(0, 1) = F[3] - f_double;
    f_double = F[4] * rleg_comx * y_coefficient;
    FRC(1, 2) = f_double;
    FRC(1, 1) = F[4] * y_coefficient - f_double;
    f_double = F[5] * rleg_comx;
    FRC(2, 2) = f_double;
    FRC(2, 1) = F[5] - f_double;
  }
#undef FRC
  // other modes: F_leg_ref unchanged (:247-250)
#pragma unroll
  for (int k = 0; k < 12; ++k) R[k] = mode == 101 ? p1[k] : (mode == 102 ? p2[k] : R[k]);
}

// Waves per SIMD the register budget targets.  Two: 239 VGPRs, no scratch.
// Three (168 VGPRs) was 1.5 % faster (0.721 vs 0.734 ms at 65,536 robots)
// but spills 96 VGPRs -- 340 B of scratch per lane, 370 MB of HBM writes per
// launch against 58 MB of algorithmic traffic (profiles/r3ft_traffic_force_
// qp_b65536_wpe3.json) -- so the spill-free budget is the shipped one.
constexpr int kForceWpe = 2;
template <int GW>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kForceWpe))) void force_qp_kernel(
    const ForceArgs a) {
  constexpr int FG = 64 / GW, VL = (12 + GW - 1) / GW;
  __shared__ ForceLds<FG> S;
  const int lane = threadIdx.x, grp = lane / GW, li = lane % GW;
  const int64_t pos = (int64_t)blockIdx.x * FG + grp;
  if (pos >= a.batch) return;
  const int64_t inst = a.list ? a.list[pos] : pos;
  typename ForceLds<FG>::Grp &P = S.g[grp];
  double *const PA = P.gi.R;  // A, 6x12 col-major (dead before the solver clears R)
  double *const PG = P.gi.J;  // G, 12x12 col-major (read once, before J is formed)
  static_assert(sizeof(P.gi.R) >= 72 * sizeof(double), "A fits the packed R");
  double *const Pg0 = P.gi.z;  // g0 (dead before z is first written)

  // ---- force_distribution (state F_leg_ref in/out) -> F_leg_guess
  double Fref[12];
  for (int k = 0; k < 12; ++k) Fref[k] = a.F_leg_ref[inst * 12 + k];
  force_distribution(a.com_des + inst * 3, a.leg_des + inst * 12, a.F_force_des + inst * 6,
                     a.mode[inst], a.y_coef[inst], a.rfoot_des + inst * 3, a.lfoot_des + inst * 3,
                     Fref);
  // this lane's entries by a static select chain: indexing Fref by li would put
  // the array in scratch (a per-lane spill of 96 B, written back to HBM)
  double guess[VL];  // F_leg_guess entries li + GW v (only their lane reads them)
#pragma unroll
  for (int v = 0; v < VL; ++v) {
    guess[v] = Fref[0];
#pragma unroll
    for (int k = 1; k < 12; ++k) guess[v] = (li + GW * v == k) ? Fref[k] : guess[v];
  }
  // ---- force_opt: A (6x12, col-major) with the skew_hat quirk (:274-298)
#pragma unroll
  for (int v = 0; v < VL; ++v) {
    const int r = li + GW * v;
    if (r < 12)
      for (int k = 0; k < 6; ++k) PA[r * 6 + k] = 0.0;
  }
  GI_SYNC();
  if (li < 4) {
    const int leg = li;
    const double *bp = a.base_p + inst * 3;
    const double *fp = a.feet_p + inst * 12 + 3 * leg;
    const double v0 = bp[0] - fp[0];  // skew_hat uses vec_w[0] everywhere (comma operator)
    for (int k = 0; k < 3; ++k) PA[(3 * leg + k) * 6 + k] = 1.0;
    // W rows [0,-a,a],[a,0,-a],[-a,a,0]
    const double W[3][3] = {{0.0, -v0, v0}, {v0, 0.0, -v0}, {-v0, v0, 0.0}};
    for (int r = 0; r < 3; ++r)
      for (int k = 0; k < 3; ++k) PA[(3 * leg + k) * 6 + 3 + r] = W[r][k];
  }
  GI_SYNC();
  // G = 2 (alpha A'A + (beta+gamma) I), then (G' + G)/2 ; g0 (:300-305).
  // A'A(r,c) and A'A(c,r) are the same products summed in the same order, so G
  // is exactly symmetric and (G' + G)/2 = (x + x)/2 = x bit for bit: the
  // symmetrisation is the identity and is not executed.
#pragma unroll
  for (int v = 0; v < VL; ++v) {
    const int r = li + GW * v;
    if (r < 12) {
      for (int c = 0; c < 12; ++c) {
        double ata = 0.0;
        for (int k = 0; k < 6; ++k) ata += PA[r * 6 + k] * PA[c * 6 + k];
        PG[c * 12 + r] = 2.0 * (a.alpha * ata + (r == c ? (a.beta + a.gamma) : 0.0));
      }
    }
  }
  GI_SYNC();
#pragma unroll
  for (int v = 0; v < VL; ++v) {
    const int r = li + GW * v;
    if (r < 12) {
      double atf = 0.0;
      const double *FT = a.FT_total_des + inst * 6;
      for (int k = 0; k < 6; ++k) atf += PA[r * 6 + k] * FT[k];
      Pg0[r] = -2.0 * (a.alpha * atf + a.beta * guess[v] + a.gamma * a.grf_opt[inst * 12 + r]);
    }
  }
  GI_SYNC();
  // swing-leg equality pattern AA (:310-350)
  const int pat = force_pattern(a.mode[inst], a.right_support[inst]);
  double f;
  int st, it;
  gi_solve_group<GW>(P.gi, li, 12, 12, 24, PG, 12, Pg0, c_force_CE[pat], c_force_zeros,
                 ForceCi{a.mu, a.fz_max}, P.gi.x,
                 f, st, it);
  GI_SYNC();
  // QPBaseClass::solveQP: success iff no NaN (go1_rt_control QPBaseClass.cpp:116-142); Solve / fallback
  bool ok = true;
  for (int k = 0; k < 12; ++k) ok = ok && !isnan(P.gi.x[k]);
#pragma unroll
  for (int v = 0; v < VL; ++v) {
    const int r = li + GW * v;
    if (r < 12) {
      a.grf_opt[inst * 12 + r] = ok ? P.gi.x[r] : guess[v];
      a.F_leg_guess[inst * 12 + r] = guess[v];
      a.F_leg_ref[inst * 12 + r] = guess[v];  // = Fref (F_leg_guess := F_leg_ref, :251-260)
    }
  }
  if (li == 0) {
    if (a.qp_solution) a.qp_solution[inst] = ok ? 1 : 0;
    if (a.status) a.status[inst] = st;
    if (a.iters) a.iters[inst] = it;
    if (a.prev_it) a.prev_it[inst] = it;
  }
}

// dynmics_compute.cpp:109-138, one thread per (instance, leg)
__global__ void joint_torque_kernel(int64_t batch, const double *Jaco, const int *swing,
                                    const double *p_des, const double *p_est,
                                    const double *pv_des, const double *pv_est,
                                    const double *F_leg_ref, double *tau) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= batch * 4) return;
  const int64_t inst = t >> 2;
  const int leg = (int)(t & 3);
  const double swing_kp = 1.0, swing_kd = 0.01;             // :37-38
  const double gcomp = (leg & 1) ? 0.80 : -0.80;            // :39-41 row 0
  const double *J = Jaco + t * 9;
  double f[3];
  if (swing[t]) {
    for (int k = 0; k < 3; ++k)
      f[k] = swing_kp * (p_des[t * 3 + k] - p_est[t * 3 + k]) +
             swing_kd * (pv_des[t * 3 + k] - pv_est[t * 3 + k]);
  } else {
    for (int k = 0; k < 3; ++k) f[k] = F_leg_ref[inst * 12 + leg * 3 + k];
  }
  for (int r = 0; r < 3; ++r) {
    double acc = 0.0;
    for (int k = 0; k < 3; ++k) acc += J[r * 3 + k] * f[k];
    tau[t * 3 + r] = -acc + (r == 0 ? gcomp : 0.0);
  }
}

// unitree_legged_real torque_mode.cpp:1370-1384 (the hardware loop after
// force_opt), one thread per (instance, leg): the stand-up ramp blends
// grf_opt with the leg's stand-up GRF, tau_ff = -J' F_opt, no gravity
// compensation; the product summed in joint_torque_kernel's order
__global__ void hw_torque_ff_kernel(int64_t batch, const double *Jaco, const double *grf_opt,
                                    const double *grf_base, const int *dynamic_count, double *tau) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= batch * 4) return;
  const int64_t inst = t >> 2;
  const double x = dynamic_count[inst] / 500.0;
  double rate = x * x;  // pow(x, 2), :1370 (both correctly rounded)
  if (rate >= 1) rate = 1;
  const double *J = Jaco + t * 9;
  double f[3];
  for (int k = 0; k < 3; ++k) {
    const double b = grf_base[t * 3 + k];
    f[k] = (rate * (grf_opt[t * 3 + k] - b)) + b;
  }
  for (int r = 0; r < 3; ++r) {
    double acc = 0.0;
    for (int k = 0; k < 3; ++k) acc += J[r * 3 + k] * f[k];
    tau[t * 3 + r] = -acc;
  }
}

}  // namespace qloco

using namespace qloco;

extern "C" void qloco_force_params_default(qloco_force_params *p);
extern "C" void qloco_force_params_hw(qloco_force_params *p) {
  qloco_force_params_default(p);
  p->mass = 14.0;  // gait::mass, unitree_legged_real robot_const_para_config.cpp:28 (dynmics_compute.cpp:31)
  p->mu = 0.5;     // unitree_legged_real dynmics_compute.cpp:65
}

extern "C" int qloco_hw_torque_ff(int64_t batch, const double *Jaco, const double *grf_opt,
                                  const double *grf_base, const int32_t *dynamic_count, double *tau,
                                  void *stream) {
  if (batch < 0 || (batch > 0 && (!Jaco || !grf_opt || !grf_base || !dynamic_count || !tau)))
    return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  const int64_t threads = batch * 4;
  hipLaunchKernelGGL(hw_torque_ff_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, batch, Jaco, grf_opt, grf_base, (const int *)dynamic_count, tau);
  QLOCO_HIP_CHECK(hipGetLastError(), "hw_torque_ff_kernel launch");
  return QLOCO_OK;
}

extern "C" void qloco_force_params_default(qloco_force_params *p) {
  p->mass = 12.0;
  p->alpha = 10000.0;
  p->beta = 1000.0;
  p->gamma = 10.0;
  p->fz_max = 160.0;
  p->mu = 0.25;
}

// c_force_CE, once per device
// Robots per wave: eight 8-lane groups (force_qp_kernel<8>), grouped or not
// (65,536 robots: 0.298 vs 0.454 ms grouped, 0.528 vs 0.778 ms ungrouped
// against four 16-lane groups, profiles/r6ac_force_qp_group_width_ab.txt).
// The results are bit-identical either way (qloco_gi_core.hpp);
// qloco_force_set_group_width / QLOCO_FORCE_GW=16 select the 16-lane kernel.
static std::atomic<int> g_force_gw{[] {
  const char *e = getenv("QLOCO_FORCE_GW");
  return (e && atoi(e) == 16) ? 16 : 8;
}()};

extern "C" int qloco_force_set_group_width(int gw) {
  if (gw != 8 && gw != 16) return QLOCO_ERR_ARG;
  return g_force_gw.exchange(gw);
}

static int force_ce_upload() {
  static std::mutex mu;
  static bool done[256] = {};
  int dev = 0;
  QLOCO_HIP_CHECK(hipGetDevice(&dev), "hipGetDevice");
  std::lock_guard<std::mutex> lock(mu);
  if (dev >= 0 && dev < 256 && done[dev]) return QLOCO_OK;
  double CE[5][144];
  memset(CE, 0, sizeof(CE));
  const int zz[5][2] = {{-1, -1}, {1, 2}, {0, 3}, {0, 2}, {1, 3}};
  for (int q = 1; q < 5; ++q)
    for (int k = 0; k < 3; ++k) {
      const int z0 = zz[q][0], z1 = zz[q][1];
      CE[q][(3 * z0 + k) * 12 + 3 * z0 + k] = 1.0;
      CE[q][(3 * z1 + k) * 12 + 3 * z1 + k] = 1.0;
    }
  QLOCO_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_force_CE), CE, sizeof(CE)), "c_force_CE upload");
  if (dev >= 0 && dev < 256) done[dev] = true;
  return QLOCO_OK;
}

extern "C" int64_t qloco_force_order_ws_len(int64_t batch) {
  return batch < 0 ? -1 : 2 * batch + 2 * kForceClasses;
}

extern "C" int qloco_force_qp_solve_ordered(const qloco_force_params *prm, int64_t batch,
                                            const double *com_des, const double *leg_des,
                                            const double *F_force_des, const double *rfoot_des,
                                            const double *lfoot_des, const double *base_p,
                                            const double *feet_p, const double *FT_total_des,
                                            const int32_t *mode, const int32_t *right_support,
                                            const double *y_coef, double *F_leg_ref, double *grf_opt,
                                            double *F_leg_guess, int32_t *qp_solution, int32_t *status,
                                            int32_t *iters, int32_t *order_ws, void *stream) {
  if (!prm || batch < 0) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  if (!com_des || !leg_des || !F_force_des || !rfoot_des || !lfoot_des || !base_p || !feet_p ||
      !FT_total_des || !mode || !right_support || !y_coef || !F_leg_ref || !grf_opt ||
      !F_leg_guess)
    return QLOCO_ERR_ARG;
  ForceArgs a;
  memset(&a, 0, sizeof(a));
  a.mass = prm->mass;
  a.alpha = prm->alpha;
  a.beta = prm->beta;
  a.gamma = prm->gamma;
  a.fz_max = prm->fz_max;
  a.mu = prm->mu;
  a.batch = batch;
  a.com_des = com_des;
  a.leg_des = leg_des;
  a.F_force_des = F_force_des;
  a.rfoot_des = rfoot_des;
  a.lfoot_des = lfoot_des;
  a.base_p = base_p;
  a.feet_p = feet_p;
  a.FT_total_des = FT_total_des;
  a.y_coef = y_coef;
  a.mode = mode;
  a.right_support = right_support;
  a.F_leg_ref = F_leg_ref;
  a.grf_opt = grf_opt;
  a.F_leg_guess = F_leg_guess;
  a.qp_solution = qp_solution;
  a.status = status;
  a.iters = iters;
  const int rc = force_ce_upload();
  if (rc != QLOCO_OK) return rc;
  const hipStream_t st = (hipStream_t)stream;
  if (order_ws) {  // workspace layout: prev iterations [B], list [B], counts, cursors
    if (batch > INT32_MAX) return QLOCO_ERR_ARG;
    int *prev = order_ws, *list = order_ws + batch, *cnt = order_ws + 2 * batch;
    QLOCO_HIP_CHECK(hipMemsetAsync(cnt, 0, 2 * kForceClasses * sizeof(int), st), "force order reset");
    const unsigned cb = (unsigned)((batch + 255) / 256);
    hipLaunchKernelGGL(force_count_kernel, dim3(cb), dim3(256), 0, st, batch, mode, right_support,
                       (const int *)prev, cnt);
    QLOCO_HIP_CHECK(hipGetLastError(), "force_count_kernel launch");
    hipLaunchKernelGGL(force_scatter_kernel, dim3(cb), dim3(256), 0, st, batch, mode, right_support,
                       (const int *)prev, (const int *)cnt, cnt + kForceClasses, list);
    QLOCO_HIP_CHECK(hipGetLastError(), "force_scatter_kernel launch");
    a.list = list;
    a.prev_it = prev;
  }
  if (g_force_gw.load(std::memory_order_relaxed) == 16) {
    const unsigned blocks = (unsigned)((batch + 3) / 4);
    hipLaunchKernelGGL(force_qp_kernel<16>, dim3(blocks), dim3(64), 0, st, a);
  } else {
    const unsigned blocks = (unsigned)((batch + 7) / 8);
    hipLaunchKernelGGL(force_qp_kernel<8>, dim3(blocks), dim3(64), 0, st, a);
  }
  QLOCO_HIP_CHECK(hipGetLastError(), "force_qp_kernel launch");
  return QLOCO_OK;
}

extern "C" int qloco_force_qp_solve(const qloco_force_params *prm, int64_t batch,
                                    const double *com_des, const double *leg_des,
                                    const double *F_force_des, const double *rfoot_des,
                                    const double *lfoot_des, const double *base_p,
                                    const double *feet_p, const double *FT_total_des,
                                    const int32_t *mode, const int32_t *right_support,
                                    const double *y_coef, double *F_leg_ref, double *grf_opt,
                                    double *F_leg_guess, int32_t *qp_solution, int32_t *status,
                                    int32_t *iters, void *stream) {
  return qloco_force_qp_solve_ordered(prm, batch, com_des, leg_des, F_force_des, rfoot_des, lfoot_des,
                                      base_p, feet_p, FT_total_des, mode, right_support, y_coef,
                                      F_leg_ref, grf_opt, F_leg_guess, qp_solution, status, iters,
                                      nullptr, stream);
}

extern "C" int qloco_joint_torques(int64_t batch, const double *Jaco, const int32_t *swing,
                                   const double *p_des, const double *p_est,
                                   const double *pv_des, const double *pv_est,
                                   const double *F_leg_ref, double *tau, void *stream) {
  if (batch < 0 || (batch > 0 && (!Jaco || !swing || !p_des || !p_est || !pv_des || !pv_est ||
                                  !F_leg_ref || !tau)))
    return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  const int64_t threads = batch * 4;
  hipLaunchKernelGGL(joint_torque_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, batch, Jaco, swing, p_des, p_est, pv_des, pv_est,
                     F_leg_ref, tau);
  QLOCO_HIP_CHECK(hipGetLastError(), "joint_torque_kernel launch");
  return QLOCO_OK;
}

