/*
 * a1_qp.c -- restatement of the A1 single-step force QP, the
 * `stance_leg_control_type == 0` branch of A1RobotControl::compute_grf
 * (unitree_ros/a1_cpp_open_source/src/A1RobotControl.cpp:383-450) with the
 * constraint matrix, weights and bounds its constructor fixes (:8-49).
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).  The QP goes through the
 * OSQP-algorithm restatement in admm.c with OSQP's default settings: the
 * reference builds a fresh OsqpEigen::Solver per call with only verbosity
 * off and warm start off (:421-433), so every solve is a cold start.
 *
 * Per-robot state record (QO_A1_STATE_LEN doubles, A1CtrlStates fields):
 *   [0:3]  root_pos          [3:6]  root_pos_d
 *   [6:9]  root_euler        [9:12] root_euler_d
 *   [12:15] root_lin_vel (world)    [15:18] root_lin_vel_d (body)
 *   [18:21] root_ang_vel (world)    [21:24] root_ang_vel_d (body)
 *   [24:33] root_rot_mat   (col-major)
 *   [33:42] root_rot_mat_z (col-major)
 *   [42:54] foot_pos_abs (3x4 col-major, legs FL, FR, RL, RR)
 */
#include "qloco_oracle.h"

#include <math.h>
#include <string.h>

void qo_a1_params_default(qo_a1_params *p) {
  /* gains: A1CtrlStates::reset() (A1CtrlStates.h:123-126); mass :39 */
  const double kpl[3] = {1000.0, 1000.0, 1000.0}, kdl[3] = {200.0, 70.0, 120.0};
  const double kpa[3] = {650.0, 35.0, 1.0}, kda[3] = {4.5, 4.5, 30.0};
  memcpy(p->kp_linear, kpl, sizeof(kpl));
  memcpy(p->kd_linear, kdl, sizeof(kdl));
  memcpy(p->kp_angular, kpa, sizeof(kpa));
  memcpy(p->kd_angular, kda, sizeof(kda));
  p->robot_mass = 15.0;
  /* A1RobotControl ctor (A1RobotControl.cpp:12-16) */
  const double q[6] = {1.0, 1.0, 1.0, 400.0, 400.0, 100.0};
  memcpy(p->q_diag, q, sizeof(q));
  p->r = 1e-3;
  p->mu = 0.7;
  p->f_min = 0.0;
  p->f_max = 180.0;
}

/* Utils::skew (utils/Utils.cpp:35-41), column-major */
static void skew(const double v[3], double S[9]) {
  S[0] = 0.0;   S[3] = -v[2]; S[6] = v[1];
  S[1] = v[2];  S[4] = 0.0;   S[7] = -v[0];
  S[2] = -v[1]; S[5] = v[0];  S[8] = 0.0;
}

void qo_a1_qp_build(const qo_a1_params *p, const double *s, const uint8_t contacts[4],
                    double root_acc[6], double H[144], double g[12], double A[240],
                    double l[20], double u[20]) {
  const double *pos = s, *pos_d = s + 3, *eul = s + 6, *eul_d = s + 9;
  const double *lv = s + 12, *lv_d = s + 15, *av = s + 18, *av_d = s + 21;
  const double *R = s + 24, *Rz = s + 33, *feet = s + 42;
  /* euler error with the yaw wrap (:330-337) */
  double ee[3];
  for (int k = 0; k < 3; ++k) ee[k] = eul_d[k] - eul[k];
  if (ee[2] > 3.1415926 * 1.5) ee[2] = eul_d[2] - 3.1415926 * 2 - eul[2];
  else if (ee[2] < -3.1415926 * 1.5) ee[2] = eul_d[2] + 3.1415926 * 2 - eul[2];
  /* root_acc (:384-397): R^T v is sum_k R(k,r) v_k */
  double vb[3], wb[3], t[3];
  for (int r = 0; r < 3; ++r) {
    vb[r] = R[3 * r + 0] * lv[0] + R[3 * r + 1] * lv[1] + R[3 * r + 2] * lv[2];
    wb[r] = R[3 * r + 0] * av[0] + R[3 * r + 1] * av[1] + R[3 * r + 2] * av[2];
  }
  for (int k = 0; k < 3; ++k) t[k] = p->kd_linear[k] * (lv_d[k] - vb[k]);
  for (int r = 0; r < 3; ++r) {
    root_acc[r] = p->kp_linear[r] * (pos_d[r] - pos[r]);
    root_acc[r] += R[r] * t[0] + R[3 + r] * t[1] + R[6 + r] * t[2];
    root_acc[3 + r] = p->kp_angular[r] * ee[r];
    root_acc[3 + r] += p->kd_angular[r] * (av_d[r] - wb[r]);
  }
  root_acc[2] += p->robot_mass * 9.8;
  /* inertia_inv (6 x 12): [I; Rz^T skew(foot_i)] per leg (:399-405) */
  double inv[72];
  memset(inv, 0, sizeof(inv));
  for (int i = 0; i < 4; ++i) {
    double S[9];
    skew(feet + 3 * i, S);
    for (int c = 0; c < 3; ++c) {
      inv[(3 * i + c) * 6 + c] = 1.0;
      for (int r = 0; r < 3; ++r) /* (Rz^T S)(r,c) = sum_k Rz(k,r) S(k,c) */
        inv[(3 * i + c) * 6 + 3 + r] =
            Rz[3 * r + 0] * S[3 * c + 0] + Rz[3 * r + 1] * S[3 * c + 1] + Rz[3 * r + 2] * S[3 * c + 2];
    }
  }
  /* H = R I + inv' Q inv (:406-409); g = -inv' Q root_acc (:411).  OSQP
   * reads only the upper triangle of the Hessian it is handed (OsqpEigen
   * passes triu(P)), so H is built on r <= c and mirrored. */
  for (int c = 0; c < 12; ++c) {
    for (int r = 0; r <= c; ++r) {
      double a = 0.0;
      for (int k = 0; k < 6; ++k) a += inv[r * 6 + k] * p->q_diag[k] * inv[c * 6 + k];
      H[c * 12 + r] = a + (r == c ? p->r : 0.0);
      H[r * 12 + c] = H[c * 12 + r];
    }
    double a = 0.0;
    for (int k = 0; k < 6; ++k) a += inv[c * 6 + k] * p->q_diag[k] * root_acc[k];
    g[c] = -a;
  }
  /* linearMatrix (20 x 12) and bounds (ctor :28-49, contact flags :414-419) */
  memset(A, 0, sizeof(double) * 240);
  for (int i = 0; i < 4; ++i) {
    A[(2 + 3 * i) * 20 + i] = 1.0;
    const int r0 = 4 + 4 * i;
    A[(3 * i) * 20 + r0] = 1.0;
    A[(2 + 3 * i) * 20 + r0] = -p->mu;
    A[(3 * i) * 20 + r0 + 1] = -1.0;
    A[(2 + 3 * i) * 20 + r0 + 1] = -p->mu;
    A[(1 + 3 * i) * 20 + r0 + 2] = 1.0;
    A[(2 + 3 * i) * 20 + r0 + 2] = -p->mu;
    A[(1 + 3 * i) * 20 + r0 + 3] = -1.0;
    A[(2 + 3 * i) * 20 + r0 + 3] = -p->mu;
    const double cf = contacts[i] ? 1.0 : 0.0;
    l[i] = cf * p->f_min;
    u[i] = cf * p->f_max;
    for (int k = 0; k < 4; ++k) {
      l[r0 + k] = -1e30; /* -OsqpEigen::INFTY */
      u[r0 + k] = 0.0;
    }
  }
}

int qo_a1_compute_grf(const qo_a1_params *p, const qo_admm_settings *st, const double *s,
                      const uint8_t contacts[4], double forces_body[12], double x[12],
                      qo_admm_info *info) {
  double acc[6], H[144], g[12], A[240], l[20], u[20], xs[12];
  qo_a1_qp_build(p, s, contacts, acc, H, g, A, l, u);
  const int status = qo_admm_solve(st, 12, 20, H, g, A, l, u, xs, NULL, info);
  const double *R = s + 24;
  /* foot_forces_grf(:, i) = root_rot_mat^T * QPSolution.segment<3>(3i) (:445-449) */
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 3; ++r)
      forces_body[3 * i + r] =
          R[3 * r + 0] * xs[3 * i] + R[3 * r + 1] * xs[3 * i + 1] + R[3 * r + 2] * xs[3 * i + 2];
  if (x) memcpy(x, xs, sizeof(xs));
  return status;
}
