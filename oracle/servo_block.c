/*
 * servo_block.c -- restatement of the go1 servo loop's force block
 * (unitree_ros/go1_rt_control/src/servo_control/servo.cpp:1052-1243 and the
 * end-of-loop update :1318), double precision: the call-site glue that fixes
 * the force QP's inputs around
 * Dynamiccclass::force_distribution / force_opt / compute_joint_torques.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).  Parity unpinned (the
 * reference needs ROS / Eigen); the QP parts are force_qp.c's restatement.
 *
 *   leg_position = [FR; FL; RR; RL] desired feet (:1053-1057)
 *   foot_relative_des = foot_des - body_p_des (:1060-1063); when the loop
 *     count > 0, v_relative = (relative_des - relative_des_old) / dtx
 *     (:1064-1070), dtx = gait::t_program_cyclic = 0.005 (go1_rt_control
 *     Robotpara :51; servo.cpp:567)
 *   F_sum = [m a_d; m g + m a_dz; Momentum_sum a_d] (:1080-1088),
 *     Momentum_sum = 2 x Go1 trunk inertia (:375-377), m = 12, g = 9.8
 *   rleg_com = clamp(<lfoot - rfoot, com - rfoot> / |lfoot - rfoot|, 0, 1)
 *     (:1097-1111)
 *   F_lr_predict and the swing flags by right_support / gait_mode
 *     (:1120-1209; a gait_mode outside 101-103 with right_support 0/1 leaves
 *     the flags as they were -- member state)
 *   force_distribution(body_p_des, leg_position, F_lr_predict, ...),
 *   force_opt(body_p_des, feet, F_sum, ...), compute_joint_torques x 4
 *     (:1216-1243), then relative_des_old = relative_des (:1318).
 * pow(v, 2) of :1107 is taken as the exactly rounded square v * v (glibc's
 * pow differs from it by one ulp on ~0.1 % of inputs); the GPU kernel uses
 * the same product, so the two agree bit for bit.
 */
#include "qloco_oracle.h"

#include <math.h>
#include <string.h>

static const double SERVO_DTX = 0.005, SERVO_MASS = 12.0, SERVO_G = 9.8;
static const double MOMENTUM_SUM[9] = {  /* row-major, servo.cpp:375-377 */
    2 * 0.0168352186, 2 * 0.0004636141, 2 * 0.0002367952,
    2 * 0.0004636141, 2 * 0.0656071082, 2 * 3.6671e-05,
    2 * 0.0002367952, 2 * 3.6671e-05,   2 * 0.0742720659};

void qo_servo_init(qo_servo_state *s) {
  memset(s, 0, sizeof(*s));
  qo_dyn_init(&s->dyn);
}

void qo_servo_free(qo_servo_state *s) { qo_dyn_free(&s->dyn); }

int qo_servo_force_block(qo_servo_state *s, const qo_force_params *prm, const double coma_des[3],
                         const double com_des[3], const double rfoot_des[3],
                         const double lfoot_des[3], const double body_p_des[3],
                         const double foot_des[12], int right_support, int gait_mode,
                         double y_offset, int loop_count, const double Jaco[36],
                         const double rel_mea[12], const double v_est[12], double F_sum[6],
                         double Force_L_R[6], double *rleg_com_out, double grf_opt[12],
                         double tau[12], int swing_out[4], int *eqp_status) {
  double rel_des[12];
  for (int l = 0; l < 4; ++l)
    for (int k = 0; k < 3; ++k) rel_des[3 * l + k] = foot_des[3 * l + k] - body_p_des[k];
  if (loop_count > 0)
    for (int k = 0; k < 12; ++k) s->v_rel[k] = (rel_des[k] - s->rel_des_old[k]) / SERVO_DTX;
  F_sum[0] = SERVO_MASS * coma_des[0];
  F_sum[1] = SERVO_MASS * coma_des[1];
  F_sum[2] = SERVO_MASS * SERVO_G + SERVO_MASS * coma_des[2];
  for (int r = 0; r < 3; ++r)
    F_sum[3 + r] = MOMENTUM_SUM[3 * r + 0] * coma_des[0] + MOMENTUM_SUM[3 * r + 1] * coma_des[1] +
                   MOMENTUM_SUM[3 * r + 2] * coma_des[2];
  const double vrl[3] = {lfoot_des[0] - rfoot_des[0], lfoot_des[1] - rfoot_des[1],
                         lfoot_des[2] - rfoot_des[2]};
  const double vcr[3] = {com_des[0] - rfoot_des[0], com_des[1] - rfoot_des[1],
                         com_des[2] - rfoot_des[2]};
  const double rlleg_dis = sqrt(vrl[0] * vrl[0] + vrl[1] * vrl[1] + vrl[2] * vrl[2]);
  const double com_rleg_dis = vrl[0] * vcr[0] + vrl[1] * vcr[1] + vrl[2] * vcr[2];
  const double raw = com_rleg_dis / rlleg_dis;
  const double raw1 = (1.0 < raw) ? 1.0 : raw;           /* std::min(raw, 1.0) */
  const double rleg_com = (raw1 < 0.0) ? 0.0 : raw1;     /* std::max(raw1, 0.0) */
  double F[6];
  int *sw = s->swing; /* FR, FL, RR, RL */
  if (right_support == 0) {
    F[0] = F_sum[0]; F[1] = F_sum[1]; F[2] = F_sum[2]; F[3] = 0; F[4] = 0; F[5] = 0;
    if (gait_mode == 101) { sw[0] = 1; sw[2] = 1; sw[1] = 0; sw[3] = 0; }
    else if (gait_mode == 102) { sw[0] = 0; sw[3] = 0; sw[1] = 1; sw[2] = 1; }
    else if (gait_mode == 103) { sw[0] = 1; sw[1] = 1; sw[2] = 0; sw[3] = 0; }
  } else if (right_support == 1) {
    F[0] = 0; F[1] = 0; F[2] = 0; F[3] = F_sum[0]; F[4] = F_sum[1]; F[5] = F_sum[2];
    if (gait_mode == 101) { sw[0] = 0; sw[2] = 0; sw[1] = 1; sw[3] = 1; }
    else if (gait_mode == 102) { sw[0] = 1; sw[3] = 1; sw[1] = 0; sw[2] = 0; }
    else if (gait_mode == 103) { sw[0] = 0; sw[1] = 0; sw[2] = 1; sw[3] = 1; }
  } else {
    F[0] = F_sum[0] * rleg_com; F[3] = F_sum[0] - F[0];
    F[1] = F_sum[1] * rleg_com; F[4] = F_sum[1] - F[1];
    F[2] = F_sum[2] * rleg_com; F[5] = F_sum[2] - F[2];
    sw[0] = sw[1] = sw[2] = sw[3] = 0;
  }
  memcpy(Force_L_R, F, sizeof(F));
  if (rleg_com_out) *rleg_com_out = rleg_com;
  qo_force_distribution(&s->dyn, body_p_des, foot_des, F, gait_mode, y_offset, rfoot_des,
                        lfoot_des);
  const int ok = qo_force_opt(&s->dyn, prm, body_p_des, foot_des, foot_des + 3, foot_des + 6,
                              foot_des + 9, F_sum, gait_mode, right_support, y_offset,
                              eqp_status, NULL);
  memcpy(grf_opt, s->dyn.grf_opt, sizeof(double) * 12);
  for (int l = 0; l < 4; ++l)
    qo_compute_joint_torques(&s->dyn, Jaco + 9 * l, sw[l], rel_des + 3 * l, rel_mea + 3 * l,
                             s->v_rel + 3 * l, v_est + 3 * l, l, tau + 3 * l);
  memcpy(s->rel_des_old, rel_des, sizeof(rel_des));
  if (swing_out) memcpy(swing_out, sw, sizeof(int) * 4);
  return ok;
}

/* Batch driver for the CPU baseline: n robots, row layout of
 * qloco_servo_force_block (states: n initialised records). */
void qo_servo_batch(int64_t n, qo_servo_state *states, const qo_force_params *prm,
                    const double *coma, const double *com, const double *rfoot,
                    const double *lfoot, const double *body_p, const double *foot,
                    const int32_t *rs, const int32_t *mode, const double *y,
                    const int32_t *loop, const double *Jaco, const double *rel_mea,
                    const double *v_est, double *grf_opt, double *tau) {
  for (int64_t b = 0; b < n; ++b) {
    double Fs[6], Fl[6];
    qo_servo_force_block(&states[b], prm, coma + 3 * b, com + 3 * b, rfoot + 3 * b,
                         lfoot + 3 * b, body_p + 3 * b, foot + 12 * b, rs[b], mode[b], y[b],
                         loop[b], Jaco + 36 * b, rel_mea + 12 * b, v_est + 12 * b, Fs, Fl, NULL,
                         grf_opt + 12 * b, tau + 12 * b, NULL, NULL);
  }
}
