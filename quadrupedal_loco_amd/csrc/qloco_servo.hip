// qloco_servo.hip -- the go1 servo loop's force block, batched (gfx950).
//
// Replaces servo.cpp:1052-1243 (+ the end-of-loop update :1318) of
// unitree_ros/go1_rt_control/src/servo_control: the call-site glue that
// fixes the force QP's inputs -- leg positions, the
// body-relative desired feet and their finite-difference velocity, F_sum,
// the left/right force split F_lr_predict with rleg_com, the swing flags --
// around Dynamiccclass::force_distribution + force_opt (qloco_force.hip) and
// compute_joint_torques for the four legs.  Three launches on one stream:
//   servo_glue_kernel   one robot per lane (fp64, no FMA contraction, the
//                       restatement's operation order: oracle/servo_block.c)
//   force_qp_kernel     qloco_force_qp_solve on the glue's F_lr_predict / F_sum
//   joint_torque_kernel qloco_joint_torques with the swing flags and velocities
// The Dynamiccclass members (F_leg_ref, grf_opt) and the loop's own state
// (swing flags, relative_des_old, v_relative) live in a device workspace.
#include <math.h>
#include <string.h>

#include "qloco_common.hpp"

namespace qloco {
namespace servo {

constexpr double DTX = 0.005;   // gait::t_program_cyclic (go1_rt_control Robotpara :51)
constexpr double MASS = 12.0;   // gait::mass (:29)
constexpr double G = 9.8;       // gait::_g (:48)
// Momentum_sum, servo.cpp:375-377 (row-major)
__constant__ double c_momentum[9] = {2 * 0.0168352186, 2 * 0.0004636141, 2 * 0.0002367952,
                                     2 * 0.0004636141, 2 * 0.0656071082, 2 * 3.6671e-05,
                                     2 * 0.0002367952, 2 * 3.6671e-05,   2 * 0.0742720659};

struct Ws {  // byte offsets
  int64_t fref, grf, guess, rel, rold, vrel, fsum, flr, swing, qps, st, ord, total;
};
__host__ __device__ inline Ws layout(int64_t B) {
  auto al = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
  Ws w;
  w.fref = 0;
  w.grf = al(w.fref + 8 * 12 * B);
  w.guess = al(w.grf + 8 * 12 * B);
  w.rel = al(w.guess + 8 * 12 * B);
  w.rold = al(w.rel + 8 * 12 * B);
  w.vrel = al(w.rold + 8 * 12 * B);
  w.fsum = al(w.vrel + 8 * 12 * B);
  w.flr = al(w.fsum + 8 * 6 * B);
  w.swing = al(w.flr + 8 * 6 * B);
  w.qps = al(w.swing + 4 * 4 * B);
  w.st = al(w.qps + 4 * B);
  w.ord = al(w.st + 4 * B);  // the force QP's grouping workspace (qloco_force_order_ws_len)
  w.total = al(w.ord + 4 * (2 * B + 2 * QLOCO_FORCE_CLASSES));
  return w;
}

struct GlueArgs {
  int64_t B;
  char *ws;
  const double *coma, *com, *rfoot, *lfoot, *body_p, *foot;
  const int32_t *rs, *mode, *loop;
  double *F_sum_out, *FLR_out;
  int32_t *swing_out;
};

__global__ __launch_bounds__(256) void servo_glue_kernel(const GlueArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.B) return;
  const Ws L = layout(a.B);
  double *rel = reinterpret_cast<double *>(a.ws + L.rel) + r * 12;
  double *rold = reinterpret_cast<double *>(a.ws + L.rold) + r * 12;
  double *vrel = reinterpret_cast<double *>(a.ws + L.vrel) + r * 12;
  double *Fs = reinterpret_cast<double *>(a.ws + L.fsum) + r * 6;
  double *Fl = reinterpret_cast<double *>(a.ws + L.flr) + r * 6;
  int32_t *sw = reinterpret_cast<int32_t *>(a.ws + L.swing) + r * 4;
  const double *bp = a.body_p + r * 3, *fd = a.foot + r * 12, *ca = a.coma + r * 3;
  const double *cd = a.com + r * 3, *rf = a.rfoot + r * 3, *lf = a.lfoot + r * 3;
  // relative desired feet and their velocity (:1060-1070); old updated last (:1318)
  double rd[12];
  for (int l = 0; l < 4; ++l)
    for (int k = 0; k < 3; ++k) rd[3 * l + k] = fd[3 * l + k] - bp[k];
  if (a.loop[r] > 0)
    for (int k = 0; k < 12; ++k) vrel[k] = (rd[k] - rold[k]) / DTX;
  for (int k = 0; k < 12; ++k) {
    rel[k] = rd[k];
    rold[k] = rd[k];
  }
  // F_sum (:1080-1088)
  double F_sum[6];
  F_sum[0] = MASS * ca[0];
  F_sum[1] = MASS * ca[1];
  F_sum[2] = MASS * G + MASS * ca[2];
  for (int i = 0; i < 3; ++i)
    F_sum[3 + i] = c_momentum[3 * i + 0] * ca[0] + c_momentum[3 * i + 1] * ca[1] +
                   c_momentum[3 * i + 2] * ca[2];
  // rleg_com (:1097-1111), pow(v, 2) as v * v (oracle/servo_block.c)
  const double v0 = lf[0] - rf[0], v1 = lf[1] - rf[1], v2 = lf[2] - rf[2];
  const double c0 = cd[0] - rf[0], c1 = cd[1] - rf[1], c2 = cd[2] - rf[2];
  const double rlleg_dis = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
  const double com_rleg_dis = v0 * c0 + v1 * c1 + v2 * c2;
  const double raw = com_rleg_dis / rlleg_dis;
  const double raw1 = (1.0 < raw) ? 1.0 : raw;        // std::min(raw, 1.0)
  const double rleg_com = (raw1 < 0.0) ? 0.0 : raw1;  // std::max(raw1, 0.0)
  // F_lr_predict + swing flags (:1120-1209); other gait modes keep the flags
  const int rs = a.rs[r], mode = a.mode[r];
  double F[6];
  int s0 = sw[0], s1 = sw[1], s2 = sw[2], s3 = sw[3];
  if (rs == 0) {
    F[0] = F_sum[0]; F[1] = F_sum[1]; F[2] = F_sum[2]; F[3] = 0; F[4] = 0; F[5] = 0;
    if (mode == 101) { s0 = 1; s2 = 1; s1 = 0; s3 = 0; }
    else if (mode == 102) { s0 = 0; s3 = 0; s1 = 1; s2 = 1; }
    else if (mode == 103) { s0 = 1; s1 = 1; s2 = 0; s3 = 0; }
  } else if (rs == 1) {
    F[0] = 0; F[1] = 0; F[2] = 0; F[3] = F_sum[0]; F[4] = F_sum[1]; F[5] = F_sum[2];
    if (mode == 101) { s0 = 0; s2 = 0; s1 = 1; s3 = 1; }
    else if (mode == 102) { s0 = 1; s3 = 1; s1 = 0; s2 = 0; }
    else if (mode == 103) { s0 = 0; s1 = 0; s2 = 1; s3 = 1; }
  } else {
    F[0] = F_sum[0] * rleg_com; F[3] = F_sum[0] - F[0];
    F[1] = F_sum[1] * rleg_com; F[4] = F_sum[1] - F[1];
    F[2] = F_sum[2] * rleg_com; F[5] = F_sum[2] - F[2];
    s0 = s1 = s2 = s3 = 0;
  }
  sw[0] = s0; sw[1] = s1; sw[2] = s2; sw[3] = s3;
  for (int k = 0; k < 6; ++k) {
    Fs[k] = F_sum[k];
    Fl[k] = F[k];
  }
  if (a.F_sum_out)
    for (int k = 0; k < 6; ++k) a.F_sum_out[r * 6 + k] = F_sum[k];
  if (a.FLR_out)
    for (int k = 0; k < 6; ++k) a.FLR_out[r * 6 + k] = F[k];
  if (a.swing_out) {
    a.swing_out[r * 4 + 0] = s0;
    a.swing_out[r * 4 + 1] = s1;
    a.swing_out[r * 4 + 2] = s2;
    a.swing_out[r * 4 + 3] = s3;
  }
}

__global__ void servo_init_kernel(int64_t B, char *ws) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = layout(B).total / 4;
  if (i < n) reinterpret_cast<int32_t *>(ws)[i] = 0;
}

}  // namespace servo
}  // namespace qloco

using namespace qloco;

extern "C" int64_t qloco_servo_workspace_bytes(int64_t batch) {
  if (batch < 0) return -1;
  return servo::layout(batch).total;
}

extern "C" int qloco_servo_init(int64_t batch, void *workspace, void *stream) {
  if (batch < 0 || (batch > 0 && !workspace)) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  const int64_t n = servo::layout(batch).total / 4;
  hipLaunchKernelGGL(servo::servo_init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, batch, (char *)workspace);
  QLOCO_HIP_CHECK(hipGetLastError(), "servo_init_kernel launch");
  return QLOCO_OK;
}

extern "C" int qloco_servo_force_block(
    const qloco_force_params *prm, int64_t batch, void *workspace, const double *coma_des,
    const double *com_des, const double *rfoot_des, const double *lfoot_des,
    const double *body_p_des, const double *foot_des, const int32_t *right_support,
    const int32_t *gait_mode, const double *y_offset, const int32_t *loop_count,
    const double *Jaco, const double *foot_rel_mea, const double *v_est_rel, double *F_sum,
    double *Force_L_R, double *grf_opt, double *tau, int32_t *swing, int32_t *qp_solution,
    int32_t *status, void *stream) {
  if (!prm || batch < 0) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  if (!workspace || !coma_des || !com_des || !rfoot_des || !lfoot_des || !body_p_des ||
      !foot_des || !right_support || !gait_mode || !y_offset || !loop_count || !Jaco ||
      !foot_rel_mea || !v_est_rel || !grf_opt || !tau)
    return QLOCO_ERR_ARG;
  const servo::Ws L = servo::layout(batch);
  char *w = (char *)workspace;
  const hipStream_t st = (hipStream_t)stream;
  servo::GlueArgs g;
  g.B = batch;
  g.ws = w;
  g.coma = coma_des;
  g.com = com_des;
  g.rfoot = rfoot_des;
  g.lfoot = lfoot_des;
  g.body_p = body_p_des;
  g.foot = foot_des;
  g.rs = right_support;
  g.mode = gait_mode;
  g.loop = loop_count;
  g.F_sum_out = F_sum;
  g.FLR_out = Force_L_R;
  g.swing_out = swing;
  hipLaunchKernelGGL(servo::servo_glue_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256),
                     0, st, g);
  QLOCO_HIP_CHECK(hipGetLastError(), "servo_glue_kernel launch");
  // Dynam.force_distribution(body_p_des, leg_position, Force_L_R, gait_mode, y_offset,
  // rfoot_des, lfoot_des); Dynam.force_opt(body_p_des, FR..RL_foot_des, F_sum, gait_mode,
  // right_support, y_offset)  (:1216-1228)
  double *fref = (double *)(w + L.fref), *grf = (double *)(w + L.grf);
  int rc = qloco_force_qp_solve_ordered(prm, batch, body_p_des, foot_des, (const double *)(w + L.flr),
                                        rfoot_des, lfoot_des, body_p_des, foot_des,
                                        (const double *)(w + L.fsum), gait_mode, right_support, y_offset,
                                        fref, grf, (double *)(w + L.guess),
                                        qp_solution ? qp_solution : (int32_t *)(w + L.qps),
                                        status ? status : (int32_t *)(w + L.st), nullptr,
                                        (int32_t *)(w + L.ord), stream);
  if (rc != QLOCO_OK) return rc;
  // compute_joint_torques for FR, FL, RR, RL (:1232-1243)
  rc = qloco_joint_torques(batch, Jaco, (const int32_t *)(w + L.swing), (const double *)(w + L.rel),
                           foot_rel_mea, (const double *)(w + L.vrel), v_est_rel, fref, tau, stream);
  if (rc != QLOCO_OK) return rc;
  QLOCO_HIP_CHECK(hipMemcpyAsync(grf_opt, grf, sizeof(double) * 12 * batch,
                                 hipMemcpyDeviceToDevice, st),
                  "grf_opt copy");
  return QLOCO_OK;
}
