/*
 * kinematics.c -- CPU restatement of the Go1 leg kinematics (TEST
 * INFRASTRUCTURE ONLY, see qloco_oracle.h).  SURVEY.md §8f row 4.
 *
 * Reference: go1_rt_control/src/kinematics/Kinematics.cpp
 *   constants            :29-55   leg offsets (+-0.1881, +-0.04675), thigh_y
 *                                 (+-0.08), thigh / calf length -0.213, lamda 0.5
 *   Forward_kinematics   :63-142  hip-frame foot position + 3x3 Jacobian
 *   Forward_kinematics_g :145-229 world frame: body_P + R(body_R) * (...)
 *   Inverse_kinematics   :233-267 10 damped Newton steps; quirk: the stop
 *                                 test is det_angle.maxCoeff() < 1e-4 on the
 *                                 SIGNED step (:249), not its norm
 *   Inverse_kinematics_g :270-304 15 steps, stop on |det_pos|^2 <= 1e-6 (:286)
 *
 * The reference writes every coordinate as one expanded trigonometric
 * polynomial.  They are restated here from the kinematic chain instead:
 * with S = tl sin(qt) + cl sin(qt+qc) and L = tl cos(qt) + cl cos(qt+qc),
 *   p_local = (ox + S, oy + ty cos(qh) - L sin(qh), ty sin(qh) + L cos(qh)),
 * and, with R = Rz(yaw) Ry(pitch) Rx(roll) of body_R = (roll, pitch, yaw),
 *   p_world = body_P + R p_local,  J_world = R J_local.
 * This equals the reference's expansions exactly in real arithmetic (the
 * sin/cos sum identities), so results agree up to rounding (~1e-15), not bit
 * for bit.  Eigen's Matrix3d::inverse() is restated with its cofactor
 * expansion.  Leg flags: 0 FR, 1 FL, 2 RR, 3 RL.  Matrices column-major.
 */
#include <math.h>
#include <string.h>

#include "qloco_oracle.h"

/* Kinematics.cpp:31-41 */
static void leg_consts(int flag, double c[5]) {
  c[0] = (flag == 0 || flag == 1) ? 0.1881 : -0.1881;     /* leg_offset_x */
  c[1] = (flag == 0 || flag == 2) ? -0.04675 : 0.04675;   /* leg_offset_y */
  c[2] = (flag == 0 || flag == 2) ? -0.08 : 0.08;         /* thigh_y */
  c[3] = -0.213;                                          /* thigh_length */
  c[4] = -0.213;                                          /* calf_length */
}

/* Forward_kinematics (:105-138) restated from the chain */
void qo_leg_fk(const double q[3], int flag, double pos[3], double J[9]) {
  double k[5];
  leg_consts(flag, k);
  const double ox = k[0], oy = k[1], ty = k[2], tl = k[3], cl = k[4];
  const double sh = sin(q[0]), ch = cos(q[0]);
  const double st = sin(q[1]), ct = cos(q[1]);
  const double stc = sin(q[1] + q[2]), ctc = cos(q[1] + q[2]);
  const double S = tl * st + cl * stc, L = tl * ct + cl * ctc;
  pos[0] = ox + S;
  pos[1] = oy + ty * ch - L * sh;
  pos[2] = ty * sh + L * ch;
  /* column 0: d/d q_hip, column 1: d/d q_thigh, column 2: d/d q_calf */
  J[0] = 0.0;
  J[1] = -ty * sh - L * ch;
  J[2] = ty * ch - L * sh;
  J[3] = L;
  J[4] = S * sh;
  J[5] = -S * ch;
  J[6] = cl * ctc;
  J[7] = cl * stc * sh;
  J[8] = -cl * stc * ch;
}

/* R = Rz(y) Ry(p) Rx(r), column-major */
static void body_rot(const double body_R[3], double R[9]) {
  const double sr = sin(body_R[0]), cr = cos(body_R[0]);
  const double sp = sin(body_R[1]), cp = cos(body_R[1]);
  const double sy = sin(body_R[2]), cy = cos(body_R[2]);
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

/* Forward_kinematics_g (:187-225): body_P + R p_local, J = R J_local */
void qo_leg_fk_g(const double body_P[3], const double body_R[3], const double q[3], int flag,
                 double pos[3], double J[9]) {
  double pl[3], Jl[9], R[9];
  qo_leg_fk(q, flag, pl, Jl);
  body_rot(body_R, R);
  for (int r = 0; r < 3; r++) {
    pos[r] = body_P[r] + (R[r] * pl[0] + R[3 + r] * pl[1] + R[6 + r] * pl[2]);
    for (int c = 0; c < 3; c++)
      J[3 * c + r] = R[r] * Jl[3 * c] + R[3 + r] * Jl[3 * c + 1] + R[6 + r] * Jl[3 * c + 2];
  }
}

/* Eigen's Matrix3d::inverse() (size-3 path of Eigen/src/LU/InverseImpl.h):
 * cof(i,j) = m(i1,j1) m(i2,j2) - m(i1,j2) m(i2,j1), i1 = (i+1)%3, i2 = (i+2)%3
 * (same for j); det = sum_i cof(i,0) m(i,0); inverse(r,c) = cof(c,r) / det. */
static double cof3(const double A[9], int i, int j) {
  const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return A[3 * j1 + i1] * A[3 * j2 + i2] - A[3 * j2 + i1] * A[3 * j1 + i2];
}
static void inv3(const double A[9], double Ai[9]) {
  const double c0 = cof3(A, 0, 0), c1 = cof3(A, 1, 0), c2 = cof3(A, 2, 0);
  const double det = c0 * A[0] + c1 * A[1] + c2 * A[2];
  const double invdet = 1.0 / det;
  Ai[0] = c0 * invdet;
  Ai[3] = c1 * invdet;
  Ai[6] = c2 * invdet;
  for (int r = 1; r < 3; r++)
    for (int c = 0; c < 3; c++) Ai[3 * c + r] = cof3(A, c, r) * invdet;
}

/* Inverse_kinematics (:233-267, body_P = body_R = NULL) and
 * Inverse_kinematics_g (:270-304).  Returns the number of Newton updates;
 * pos / J are the FK and Jacobian at the returned q (the last evaluation,
 * which is what the callers read from Jacobian_kin afterwards). */
int qo_leg_ik(const double *body_P, const double *body_R, const double pos_des[3],
              const double q_ini[3], int flag, double q_des[3], double pos[3], double J[9]) {
  const int global = body_P != 0 && body_R != 0;
  const double lamda = 0.5; /* :52 */
  const int steps = global ? 15 : 10;
  double Ji[9], det_pos[3], det_angle[3];
  if (global)
    qo_leg_fk_g(body_P, body_R, q_ini, flag, pos, J);
  else
    qo_leg_fk(q_ini, flag, pos, J);
  memcpy(q_des, q_ini, 3 * sizeof(double));
  int updates = 0;
  for (int j = 0; j < steps; j++) {
    for (int r = 0; r < 3; r++) det_pos[r] = pos_des[r] - pos[r];
    inv3(J, Ji);
    /* lamda * J^-1 * det_pos: the matrix is scaled first, then the product */
    for (int r = 0; r < 3; r++)
      det_angle[r] = (lamda * Ji[r]) * det_pos[0] + (lamda * Ji[3 + r]) * det_pos[1] +
                     (lamda * Ji[6 + r]) * det_pos[2];
    int stop;
    if (global) {
      stop = fabs(det_pos[0] * det_pos[0] + det_pos[1] * det_pos[1] + det_pos[2] * det_pos[2]) <= 0.000001;
    } else {
      double mx = det_angle[0];
      if (det_angle[1] > mx) mx = det_angle[1];
      if (det_angle[2] > mx) mx = det_angle[2];
      stop = mx < 0.0001;
    }
    if (stop) break;
    for (int r = 0; r < 3; r++) q_des[r] += det_angle[r];
    updates++;
    if (global)
      qo_leg_fk_g(body_P, body_R, q_des, flag, pos, J);
    else
      qo_leg_fk(q_des, flag, pos, J);
  }
  return updates;
}

/* Batch drivers for the CPU baseline timing (bench_kin.py): n legs, row
 * layout as the C ABI (q / pos n*3, J n*9, leg n; body_p / body_r n*3 or
 * NULL).  Single thread. */
void qo_leg_fk_batch(int64_t n, const double *q, const int32_t *leg, const double *body_p,
                     const double *body_r, double *pos, double *J) {
  for (int64_t i = 0; i < n; i++) {
    if (body_p)
      qo_leg_fk_g(body_p + 3 * i, body_r + 3 * i, q + 3 * i, leg[i], pos + 3 * i, J + 9 * i);
    else
      qo_leg_fk(q + 3 * i, leg[i], pos + 3 * i, J + 9 * i);
  }
}

void qo_leg_ik_batch(int64_t n, const double *pos_des, const double *q_ini, const int32_t *leg,
                     const double *body_p, const double *body_r, double *q, double *pos, double *J,
                     int32_t *updates) {
  for (int64_t i = 0; i < n; i++)
    updates[i] = qo_leg_ik(body_p ? body_p + 3 * i : 0, body_r ? body_r + 3 * i : 0,
                           pos_des + 3 * i, q_ini + 3 * i, leg[i], q + 3 * i, pos + 3 * i, J + 9 * i);
}
