/*
 * force_qp.c -- restatement of the Go1 12-force distribution QP
 * (Dynamiccclass, unitree_ros/go1_rt_control/src/whole_body_dynamics/
 * dynmics_compute.cpp), double precision, quirks kept.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).  Parity unpinned.
 */
#include "qloco_oracle.h"

#include <math.h>
#include <string.h>

#define FRC(m, r, c) ((m)[(c) * 3 + (r)]) /* 3x4 col-major */

void qo_force_params_default(qo_force_params *p) {
  p->mass = 12.0;     /* dynmics_compute.cpp:31 */
  p->alpha = 10000.0; /* :61 */
  p->beta = 1000.0;   /* :62 */
  p->gamma = 10.0;    /* :63 */
  p->fz_max = 160.0;  /* :64 */
  p->mu = 0.25;       /* :65 (HW copy: 0.5) */
}

void qo_dyn_init(qo_dyn_state *s) {
  memset(s, 0, sizeof(*s));
  s->qp_solution = 1;                 /* :52 */
  s->ws = qo_eqp_create(12, 12, 24);  /* resizeQP(12,12,24), :46-49 */
}

void qo_dyn_free(qo_dyn_state *s) {
  qo_eqp_destroy(s->ws);
  s->ws = NULL;
}

static double sq(double v) { return v * v; }

/* dynmics_compute.cpp:141-261 */
void qo_force_distribution(qo_dyn_state *s, const double com_des[3],
                           const double leg_des[12], const double F[6], int mode,
                           double y_coefficient, const double rfoot_des[3],
                           const double lfoot_des[3]) {
  double body_FR_dis = sqrt(sq(com_des[0] - leg_des[0]) + sq(com_des[1] - leg_des[1]) + sq(com_des[2] - leg_des[2]));
  double body_FL_dis = sqrt(sq(com_des[0] - leg_des[3]) + sq(com_des[1] - leg_des[4]) + sq(com_des[2] - leg_des[5]));
  double body_RR_dis = sqrt(sq(com_des[0] - leg_des[6]) + sq(com_des[1] - leg_des[7]) + sq(com_des[2] - leg_des[8]));
  double body_RL_dis = sqrt(sq(com_des[0] - leg_des[9]) + sq(com_des[1] - leg_des[10]) + sq(com_des[2] - leg_des[11]));
  double f_double;
  double *R = s->F_leg_ref;
  if (mode == 101) { /* bipedal, :155-182 */
    f_double = F[0] * body_FL_dis / (body_FL_dis + body_RL_dis);
    FRC(R, 0, 3) = f_double;
    FRC(R, 0, 1) = F[0] - f_double;
    f_double = F[1] * body_FL_dis / (body_FL_dis + body_RL_dis) * y_coefficient;
    FRC(R, 1, 3) = f_double;
    FRC(R, 1, 1) = F[1] * y_coefficient - f_double;
    f_double = F[2] * body_FL_dis / (body_FL_dis + body_RL_dis);
    FRC(R, 2, 3) = f_double;
    FRC(R, 2, 1) = F[2] - f_double;

    f_double = F[3] * body_FR_dis / (body_FR_dis + body_RR_dis);
    FRC(R, 0, 2) = f_double;
    FRC(R, 0, 0) = F[3] - f_double;
    f_double = F[4] * body_FR_dis / (body_FR_dis + body_RR_dis) * y_coefficient;
    FRC(R, 1, 2) = f_double;
    FRC(R, 1, 0) = F[4] * y_coefficient - f_double;
    f_double = F[5] * body_FR_dis / (body_FR_dis + body_RR_dis);
    FRC(R, 2, 2) = f_double;
    FRC(R, 2, 0) = F[5] - f_double;
  } else if (mode == 102) { /* trotting, :185-246 */
    double v0 = leg_des[9] - leg_des[0], v1 = leg_des[10] - leg_des[1], v2 = leg_des[11] - leg_des[2];
    double c0 = lfoot_des[0] - leg_des[0], c1 = lfoot_des[1] - leg_des[1], c2 = lfoot_des[2] - leg_des[2];
    double rlleg_dis = sqrt(sq(v0) + sq(v1) + sq(v2));
    double com_rleg_dis = v0 * c0 + v1 * c1 + v2 * c2;
    double raw = com_rleg_dis / rlleg_dis;
    double raw1 = raw < 1.0 ? raw : 1.0;            /* std::min(raw, 1.0) */
    double rleg_com = raw1 > 0.0 ? raw1 : 0.0;      /* std::max(raw1, 0.0) */
    f_double = F[0] * rleg_com;
    FRC(R, 0, 3) = f_double;
    FRC(R, 0, 0) = F[0] - f_double;
    f_double = F[1] * rleg_com * y_coefficient;
    FRC(R, 1, 3) = f_double;
    FRC(R, 1, 0) = F[1] * y_coefficient - f_double;
    f_double = F[2] * rleg_com;
    FRC(R, 2, 3) = f_double;
    FRC(R, 2, 0) = F[2] - f_double;

    double w0 = leg_des[6] - leg_des[3], w1 = leg_des[7] - leg_des[4], w2 = leg_des[8] - leg_des[5];
    double e0 = rfoot_des[0] - leg_des[3], e1 = rfoot_des[1] - leg_des[4], e2 = rfoot_des[2] - leg_des[5];
    double rlleg_disx = sqrt(sq(w0) + sq(w1) + sq(w2));
    double com_rleg_disx = w0 * e0 + w1 * e1 + w2 * e2;
    double rawx = com_rleg_disx / rlleg_disx;
    double raw1x = rawx < 1.0 ? rawx : 1.0;
    double rleg_comx = raw1x > 0.0 ? raw1x : 0.0;
    f_double = F[3] * rleg_comx;
    FRC(R, 0, 2) = f_double;
    FRC(R, 0, 1) = F[3] - f_double;
    f_double = F[4] * rleg_comx * y_coefficient;
    FRC(R, 1, 2) = f_double;
    FRC(R, 1, 1) = F[4] * y_coefficient - f_double;
    f_double = F[5] * rleg_comx;
    FRC(R, 2, 2) = f_double;
    FRC(R, 2, 1) = F[5] - f_double;
  } /* other modes: F_leg_ref untouched (:247-250) */
  for (int i = 0; i < 12; ++i) s->F_leg_guess[i] = R[i]; /* :256-259 */
}

/* skew_hat with the comma-operator bug: vec_w[2,0] == vec_w[0] (:375-384) */
static void skew_hat_quirk(const double v[3], double W[9] /* col-major */) {
  double a = v[0];
  /* rows: [0,-a,a],[a,0,-a],[-a,a,0] */
  W[0 + 0 * 3] = 0;  W[0 + 1 * 3] = -a; W[0 + 2 * 3] = a;
  W[1 + 0 * 3] = a;  W[1 + 1 * 3] = 0;  W[1 + 2 * 3] = -a;
  W[2 + 0 * 3] = -a; W[2 + 1 * 3] = a;  W[2 + 2 * 3] = 0;
}

int qo_force_opt(qo_dyn_state *s, const qo_force_params *prm, const double base_p[3],
                 const double FR_p[3], const double FL_p[3], const double RR_p[3],
                 const double RL_p[3], const double FT[6], int mode,
                 int right_support, double y_coefficient, int *eqp_status,
                 int *iters) {
  (void)y_coefficient; /* unused by force_opt in the reference */
  double A[6 * 12];    /* 6x12 col-major */
  memset(A, 0, sizeof(A));
  const double *feet[4] = {FR_p, FL_p, RR_p, RL_p};
  for (int leg = 0; leg < 4; ++leg) {
    for (int k = 0; k < 3; ++k) A[(3 * leg + k) * 6 + k] = 1.0; /* A_unit, :279-282 */
    double c[3] = {base_p[0] - feet[leg][0], base_p[1] - feet[leg][1], base_p[2] - feet[leg][2]};
    double W[9];
    skew_hat_quirk(c, W);
    for (int r = 0; r < 3; ++r)
      for (int k = 0; k < 3; ++k) A[(3 * leg + k) * 6 + 3 + r] = W[k * 3 + r];
  }
  /* Q_goal = 2 (alpha A'A + (beta+gamma) I); Q_goal1 = (Q'+Q)/2  (:300-301) */
  double G[144], g0[12];
  for (int c = 0; c < 12; ++c)
    for (int r = 0; r < 12; ++r) {
      double ata = 0.0;
      for (int k = 0; k < 6; ++k) ata += A[r * 6 + k] * A[c * 6 + k];
      G[c * 12 + r] = 2.0 * (prm->alpha * ata + (r == c ? (prm->beta + prm->gamma) : 0.0));
    }
  double Gs[144];
  for (int c = 0; c < 12; ++c)
    for (int r = 0; r < 12; ++r) Gs[c * 12 + r] = (G[r * 12 + c] + G[c * 12 + r]) / 2.0;
  /* q_goal = -2 (alpha A' FT + beta F_guess + gamma grf_opt)  (:305) */
  for (int r = 0; r < 12; ++r) {
    double atf = 0.0;
    for (int k = 0; k < 6; ++k) atf += A[r * 6 + k] * FT[k];
    g0[r] = -2.0 * (prm->alpha * atf + prm->beta * s->F_leg_guess[r] + prm->gamma * s->grf_opt[r]);
  }
  /* equality pattern AA (12x12) and bb = 0 (:310-350) */
  double CE[144], ce0[12];
  memset(CE, 0, sizeof(CE));
  memset(ce0, 0, sizeof(ce0));
  int zero_legs[2] = {-1, -1};
  if (mode == 102) {
    if (right_support == 0) { zero_legs[0] = 1; zero_legs[1] = 2; }      /* FL, RR */
    else if (right_support == 1) { zero_legs[0] = 0; zero_legs[1] = 3; } /* FR, RL */
  } else if (mode == 101) {
    if (right_support == 0) { zero_legs[0] = 0; zero_legs[1] = 2; }      /* FR, RR */
    else if (right_support == 1) { zero_legs[0] = 1; zero_legs[1] = 3; } /* FL, RL */
  }
  for (int z = 0; z < 2; ++z)
    if (zero_legs[z] >= 0)
      for (int k = 0; k < 3; ++k) {
        int idx = 3 * zero_legs[z] + k;
        CE[idx * 12 + idx] = 1.0;
      }
  /* qp_H / qp_h (:75-98) -> CI = -qp_H', ci0 = qp_h (:419-420) */
  double qpH[24 * 12], qph[24];
  memset(qpH, 0, sizeof(qpH));
  memset(qph, 0, sizeof(qph));
  for (int i = 0; i < 4; i++) {
    qpH[(3 * i + 2) * 24 + 2 * i] = -1;
    qpH[(3 * i + 2) * 24 + 2 * i + 1] = 1;
    qph[2 * i + 1] = prm->fz_max;
  }
  for (int i = 0; i < 4; i++) {
    qpH[(3 * i) * 24 + 8 + 2 * i] = -1;
    qpH[(3 * i + 2) * 24 + 8 + 2 * i] = -prm->mu;
    qpH[(3 * i) * 24 + 8 + 2 * i + 1] = 1;
    qpH[(3 * i + 2) * 24 + 8 + 2 * i + 1] = -prm->mu;
  }
  for (int i = 0; i < 4; i++) {
    qpH[(3 * i + 1) * 24 + 16 + 2 * i] = -1;
    qpH[(3 * i + 2) * 24 + 16 + 2 * i] = -prm->mu;
    qpH[(3 * i + 1) * 24 + 16 + 2 * i + 1] = 1;
    qpH[(3 * i + 2) * 24 + 16 + 2 * i + 1] = -prm->mu;
  }
  double CI[12 * 24]; /* n x m col-major: CI(v, c) = -qpH(c, v) */
  for (int c = 0; c < 24; ++c)
    for (int v = 0; v < 12; ++v) CI[c * 12 + v] = -qpH[v * 24 + c];
  double X[12];
  memcpy(X, s->grf_opt, sizeof(X)); /* _X = grf_opt (:391) */
  int st = QO_OK;
  qo_eqp_solve(s->ws, Gs, g0, CE, ce0, CI, qph, X, &st, iters);
  if (eqp_status) *eqp_status = st;
  /* QPBaseClass::solveQP: success iff no NaN in X (go1_rt_control QPBaseClass.cpp:116-142) */
  int ok = 1;
  for (int i = 0; i < 12; ++i)
    if (isnan(X[i])) { ok = 0; break; }
  s->qp_solution = ok;
  memcpy(s->grf_opt, X, sizeof(X)); /* Solve: grf_opt = _X (:440-443) */
  if (!s->qp_solution) memcpy(s->grf_opt, s->F_leg_guess, sizeof(X)); /* :364-367 */
  return s->qp_solution;
}

void qo_compute_joint_torques(const qo_dyn_state *s, const double J[9], int swing_flag,
                              const double p_des[3], const double p_est[3],
                              const double pv_des[3], const double pv_est[3],
                              int leg_number, double tau[3]) {
  static const double swing_kp = 1.0, swing_kd = 0.01;             /* :37-38 */
  static const double gcomp[4] = {-0.80, 0.80, -0.80, 0.80};       /* :39-41 row 0 */
  double f[3];
  if (swing_flag) {
    for (int k = 0; k < 3; ++k) f[k] = swing_kp * (p_des[k] - p_est[k]) + swing_kd * (pv_des[k] - pv_est[k]);
  } else {
    for (int k = 0; k < 3; ++k) f[k] = FRC(s->F_leg_ref, k, leg_number);
  }
  for (int r = 0; r < 3; ++r) {
    double acc = 0.0;
    for (int k = 0; k < 3; ++k) acc += J[r * 3 + k] * f[k]; /* (J')(r,k) = J(k,r) */
    tau[r] = -acc + (r == 0 ? gcomp[leg_number] : 0.0);
  }
}

/* The hardware loop's feed-forward after force_opt (unitree_legged_real
 * torque_mode.cpp:1370-1384): the stand-up ramp rate = min((dynamic_count /
 * 500)^2, 1) blends each leg's grf_opt with the leg's stand-up GRF (FR_GRF ..
 * RL_GRF, set at :1057-1058), then Torque_ff_GRF = -J' F_opt per leg -- no
 * gravity compensation (the sim's compute_joint_torques adds it).  Legs in the
 * servo order FR, FL, RR, RL; J 3x3 col-major per leg; the product summed in
 * compute_joint_torques' order. */
void qo_hw_torque_ff(const double Jaco[36], const double grf_opt[12], const double grf_base[12],
                     int32_t dynamic_count, double tau[12]) {
  double rate = pow(dynamic_count / 500.0, 2); /* :1370 */
  if (rate >= 1) rate = 1;                     /* :1371-1374 */
  for (int l = 0; l < 4; ++l) {
    double f[3];
    for (int k = 0; k < 3; ++k)
      f[k] = (rate * (grf_opt[3 * l + k] - grf_base[3 * l + k])) + grf_base[3 * l + k]; /* :1376-1379 */
    const double *J = Jaco + 9 * l;
    for (int r = 0; r < 3; ++r) {
      double acc = 0.0;
      for (int k = 0; k < 3; ++k) acc += J[r * 3 + k] * f[k];
      tau[3 * l + r] = -acc; /* :1381-1384 */
    }
  }
}

/* Batch driver for the CPU baseline (tools/bench_qp.py): servo.cpp:1224-1228
 * (force_distribution then force_opt) for n robots, row layout of
 * qloco_force_qp_solve, one persistent Dynamiccclass per robot in `states`
 * (n records, qo_dyn_init'ed by the caller).  Single thread. */
void qo_force_batch(int64_t n, qo_dyn_state *states, const qo_force_params *prm,
                    const double *com_des, const double *leg_des, const double *F_force_des,
                    const double *rfoot_des, const double *lfoot_des, const double *base_p,
                    const double *feet_p, const double *FT_total_des, const int32_t *mode,
                    const int32_t *right_support, const double *y_coef, double *grf_opt) {
  for (int64_t b = 0; b < n; ++b) {
    qo_dyn_state *s = &states[b];
    qo_force_distribution(s, com_des + 3 * b, leg_des + 12 * b, F_force_des + 6 * b, mode[b],
                          y_coef[b], rfoot_des + 3 * b, lfoot_des + 3 * b);
    const double *f = feet_p + 12 * b;
    qo_force_opt(s, prm, base_p + 3 * b, f, f + 3, f + 6, f + 9, FT_total_des + 6 * b, mode[b],
                 right_support[b], y_coef[b], NULL, NULL);
    memcpy(grf_opt + 12 * b, s->grf_opt, sizeof(double) * 12);
  }
}
