// qloco_kin.hip -- batched Go1 leg kinematics: forward
// kinematics + Jacobian and damped-Newton inverse kinematics, fp64 like the
// reference, one leg per lane.
//
// Replaces Kinematicclass (go1_rt_control/src/kinematics/Kinematics.cpp):
//   Forward_kinematics   :63-142   hip frame
//   Forward_kinematics_g :145-229  world frame (servo.cpp:734-741 per leg)
//   Inverse_kinematics   :233-267  10 steps, stop when det_angle.maxCoeff() < 1e-4
//                                  (the signed step -- reproduced as written)
//   Inverse_kinematics_g :270-304  15 steps, stop when |det_pos|^2 <= 1e-6
//                                  (servo.cpp:1038-1051, Jacobian_kin read after)
// The reference's expanded trigonometric polynomials are evaluated from the
// kinematic chain (S = tl sin qt + cl sin(qt+qc), L = tl cos qt + cl cos(qt+qc),
// p_world = body_P + R p_local, J_world = R J_local with R = Rz Ry Rx of
// body_R): 3 (+3) sincos per evaluation instead of ~60 trig calls, equal in
// real arithmetic, so results match to rounding (oracle/kinematics.c).
//
// Memory: AoS fp64 rows (q / pos n*3, J n*9 col-major, leg n int32) are read
// and written by consecutive lanes, so a wave touches one contiguous span per
// array.  The FK kernel is HBM-bound (≈ 68 B in + 96 B out per leg with J);
// IK adds ≤ 15 FK evaluations + 3x3 solves per leg on the same traffic.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "qloco.h"
#include "qloco_common.hpp"

namespace qloco {
namespace {

struct LegConst {
  double ox, oy, ty, tl, cl;
};

// Kinematics.cpp:31-41 (0 FR, 1 FL, 2 RR, 3 RL)
__device__ __forceinline__ LegConst leg_const(int flag) {
  LegConst k;
  k.ox = (flag == 0 || flag == 1) ? 0.1881 : -0.1881;
  k.oy = (flag == 0 || flag == 2) ? -0.04675 : 0.04675;
  k.ty = (flag == 0 || flag == 2) ? -0.08 : 0.08;
  k.tl = -0.213;
  k.cl = -0.213;
  return k;
}

// hip-frame foot position and Jacobian (column c = d/dq_c), column-major
__device__ __forceinline__ void fk_local(const LegConst &k, const double q[3], double p[3],
                                         double J[9]) {
  double sh, ch, st, ct, stc, ctc;
  sincos(q[0], &sh, &ch);
  sincos(q[1], &st, &ct);
  sincos(q[1] + q[2], &stc, &ctc);
  const double S = k.tl * st + k.cl * stc, L = k.tl * ct + k.cl * ctc;
  p[0] = k.ox + S;
  p[1] = k.oy + k.ty * ch - L * sh;
  p[2] = k.ty * sh + L * ch;
  J[0] = 0.0;
  J[1] = -k.ty * sh - L * ch;
  J[2] = k.ty * ch - L * sh;
  J[3] = L;
  J[4] = S * sh;
  J[5] = -S * ch;
  J[6] = k.cl * ctc;
  J[7] = k.cl * stc * sh;
  J[8] = -k.cl * stc * ch;
}

// R = Rz(yaw) Ry(pitch) Rx(roll), column-major
__device__ __forceinline__ void body_rot(const double e[3], double R[9]) {
  double sr, cr, sp, cp, sy, cy;
  sincos(e[0], &sr, &cr);
  sincos(e[1], &sp, &cp);
  sincos(e[2], &sy, &cy);
  R[0] = cy * cp;
  R[1] = sy * cp;
  R[2] = -sp;
  R[3] = cy * sp * sr - sy * cr;
  R[4] = sy * sp * sr + cy * cr;
  R[5] = cp * sr;
  R[6] = cy * sp * cr + sy * sr;
  R[7] = sy * sp * cr - cy * sr;
  R[8] = cp * cr;
}

// FK (+ J) in the hip frame or, with R / P, in the world frame
__device__ __forceinline__ void fk(const LegConst &k, bool global, const double R[9],
                                   const double P[3], const double q[3], double p[3],
                                   double J[9]) {
  double pl[3], Jl[9];
  fk_local(k, q, pl, Jl);
  if (!global) {
#pragma unroll
    for (int i = 0; i < 3; ++i) p[i] = pl[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) J[i] = Jl[i];
    return;
  }
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    p[r] = P[r] + (R[r] * pl[0] + R[3 + r] * pl[1] + R[6 + r] * pl[2]);
#pragma unroll
    for (int c = 0; c < 3; ++c)
      J[3 * c + r] = R[r] * Jl[3 * c] + R[3 + r] * Jl[3 * c + 1] + R[6 + r] * Jl[3 * c + 2];
  }
}

// Eigen Matrix3d::inverse() cofactor order (oracle/kinematics.c inv3)
__device__ __forceinline__ double cof3(const double A[9], int i, int j) {
  const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return A[3 * j1 + i1] * A[3 * j2 + i2] - A[3 * j2 + i1] * A[3 * j1 + i2];
}

__global__ __launch_bounds__(256) void leg_fk_kernel(int n, const double *__restrict__ q,
                                                     const int32_t *__restrict__ leg,
                                                     const double *__restrict__ body_p,
                                                     const double *__restrict__ body_r,
                                                     double *__restrict__ pos,
                                                     double *__restrict__ jac) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const LegConst k = leg_const(leg[i]);
  const bool global = body_p != nullptr;
  double R[9], P[3] = {0.0, 0.0, 0.0};
  if (global) {
    const double e[3] = {body_r[3 * i], body_r[3 * i + 1], body_r[3 * i + 2]};
    body_rot(e, R);
#pragma unroll
    for (int r = 0; r < 3; ++r) P[r] = body_p[3 * i + r];
  }
  const double qi[3] = {q[3 * i], q[3 * i + 1], q[3 * i + 2]};
  double p[3], J[9];
  fk(k, global, R, P, qi, p, J);
#pragma unroll
  for (int r = 0; r < 3; ++r) pos[3 * i + r] = p[r];
  if (jac) {
#pragma unroll
    for (int c = 0; c < 9; ++c) jac[9 * i + c] = J[c];
  }
}

__global__ __launch_bounds__(256) void leg_ik_kernel(
    int n, const double *__restrict__ pos_des, const double *__restrict__ q_ini,
    const int32_t *__restrict__ leg, const double *__restrict__ body_p,
    const double *__restrict__ body_r, double *__restrict__ q_out, double *__restrict__ pos,
    double *__restrict__ jac, int32_t *__restrict__ updates) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const LegConst k = leg_const(leg[i]);
  const bool global = body_p != nullptr;
  double R[9], P[3] = {0.0, 0.0, 0.0};
  if (global) {
    const double e[3] = {body_r[3 * i], body_r[3 * i + 1], body_r[3 * i + 2]};
    body_rot(e, R);
#pragma unroll
    for (int r = 0; r < 3; ++r) P[r] = body_p[3 * i + r];
  }
  const double pd[3] = {pos_des[3 * i], pos_des[3 * i + 1], pos_des[3 * i + 2]};
  double qd[3] = {q_ini[3 * i], q_ini[3 * i + 1], q_ini[3 * i + 2]};
  double p[3], J[9];
  fk(k, global, R, P, qd, p, J);
  const double lamda = 0.5;  // Kinematics.cpp:52
  const int steps = global ? 15 : 10;
  int nup = 0;
  for (int j = 0; j < steps; ++j) {
    const double dp[3] = {pd[0] - p[0], pd[1] - p[1], pd[2] - p[2]};
    const double c0 = cof3(J, 0, 0), c1 = cof3(J, 1, 0), c2 = cof3(J, 2, 0);
    const double invdet = 1.0 / (c0 * J[0] + c1 * J[1] + c2 * J[2]);
    double Ji[9];
    Ji[0] = c0 * invdet;
    Ji[3] = c1 * invdet;
    Ji[6] = c2 * invdet;
#pragma unroll
    for (int r = 1; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) Ji[3 * c + r] = cof3(J, c, r) * invdet;
    double da[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
      da[r] = (lamda * Ji[r]) * dp[0] + (lamda * Ji[3 + r]) * dp[1] + (lamda * Ji[6 + r]) * dp[2];
    const bool stop = global ? (fabs(dp[0] * dp[0] + dp[1] * dp[1] + dp[2] * dp[2]) <= 0.000001)
                             : (fmax(fmax(da[0], da[1]), da[2]) < 0.0001);
    if (stop) break;
#pragma unroll
    for (int r = 0; r < 3; ++r) qd[r] += da[r];
    ++nup;
    fk(k, global, R, P, qd, p, J);
  }
#pragma unroll
  for (int r = 0; r < 3; ++r) q_out[3 * i + r] = qd[r];
  if (pos) {
#pragma unroll
    for (int r = 0; r < 3; ++r) pos[3 * i + r] = p[r];
  }
  if (jac) {
#pragma unroll
    for (int c = 0; c < 9; ++c) jac[9 * i + c] = J[c];
  }
  if (updates) updates[i] = nup;
}

}  // namespace
}  // namespace qloco

using namespace qloco;

extern "C" int qloco_leg_fk(int64_t n, const double *q, const int32_t *leg, const double *body_p,
                            const double *body_r, double *pos, double *jac, void *stream) {
  if (n < 0 || n > INT32_MAX || (n > 0 && (!q || !leg || !pos)) || ((body_p == nullptr) != (body_r == nullptr)))
    return QLOCO_ERR_ARG;
  if (n == 0) return QLOCO_OK;
  hipLaunchKernelGGL(leg_fk_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (int)n, q, leg, body_p, body_r, pos, jac);
  QLOCO_HIP_CHECK(hipGetLastError(), "leg_fk_kernel launch");
  return QLOCO_OK;
}

extern "C" int qloco_leg_ik(int64_t n, const double *pos_des, const double *q_ini,
                            const int32_t *leg, const double *body_p, const double *body_r,
                            double *q_out, double *pos, double *jac, int32_t *updates,
                            void *stream) {
  if (n < 0 || n > INT32_MAX || (n > 0 && (!pos_des || !q_ini || !leg || !q_out)) ||
      ((body_p == nullptr) != (body_r == nullptr)))
    return QLOCO_ERR_ARG;
  if (n == 0) return QLOCO_OK;
  hipLaunchKernelGGL(leg_ik_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (int)n, pos_des, q_ini, leg, body_p, body_r, q_out, pos,
                     jac, updates);
  QLOCO_HIP_CHECK(hipGetLastError(), "leg_ik_kernel launch");
  return QLOCO_OK;
}
