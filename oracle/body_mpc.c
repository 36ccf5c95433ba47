/*
 * body_mpc.c -- restatement of the QP part of the rt body-inclination MPC,
 * PRMPCClass (unitree_ros/rt_mpc_qp/src/FastMPC/PRMPCClass.cpp), double.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).  Parity unpinned.
 *
 * Covered: Initialize (schedule + prediction matrices, :157-374),
 * body_theta_mpc (:379-714), Indexfind (:716-738), Matrix_ps/pu (:741-796),
 * solve_body_rotation/Solve (:799-849).  Robot constants from
 * rt_mpc_qp/src/Robotpara/robot_const_para_config.cpp:8-47.
 * The 16 CI columns 32..47 that the reference never writes (:813-816,
 * :826-829; Eigen leaves them uninitialised) are treated as zero (inert).
 */
#include "qloco_oracle.h"

#include <math.h>
#include <string.h>

#define NH QO_NH
#define NT (2 * QO_NH)
#define NI (12 * QO_NH) /* resizeQP(_Nt, 0, 12*_nh), :355-360 */

/* 2x2 / 2x1 helpers, col-major */
static void mat2_mul(const double A[4], const double B[4], double C[4]) {
  double c00 = A[0] * B[0] + A[2] * B[1];
  double c10 = A[1] * B[0] + A[3] * B[1];
  double c01 = A[0] * B[2] + A[2] * B[3];
  double c11 = A[1] * B[2] + A[3] * B[3];
  C[0] = c00; C[1] = c10; C[2] = c01; C[3] = c11;
}

/* Matrix_ps, :741-763: row i = c * a^(i+1) */
static void matrix_ps(const double a[4], const double c[2], double out[NH * 2]) {
  for (int i = 0; i < NH; i++) {
    double A[4] = {1, 0, 0, 1};
    for (int j = 1; j < i + 2; j++) mat2_mul(A, a, A);
    out[0 * NH + i] = c[0] * A[0] + c[1] * A[1];
    out[1 * NH + i] = c[0] * A[2] + c[1] * A[3];
  }
}

/* Matrix_pu, :765-796: (i-1,j-1) = c * a^(i-j) * b, j <= i */
static void matrix_pu(const double a[4], const double b[2], const double c[2],
                      double out[NH * NH]) {
  memset(out, 0, sizeof(double) * NH * NH);
  for (int i = 1; i < NH + 1; i++)
    for (int j = 1; j < i + 1; j++) {
      double A[4] = {1, 0, 0, 1};
      if (j != i)
        for (int k = 1; k < i - j + 1; k++) mat2_mul(A, a, A);
      double ca0 = c[0] * A[0] + c[1] * A[1];
      double ca1 = c[0] * A[2] + c[1] * A[3];
      out[(j - 1) * NH + (i - 1)] = ca0 * b[0] + ca1 * b[1];
    }
}

void qo_body_init(qo_body_state *s) {
  memset(s, 0, sizeof(*s));
  const double dt_slow = 0.025, dt_fast = 0.01, tstep = 0.7; /* gait:: :8-9,26 */
  s->dt_mpc = dt_fast;
  s->j_ini = 12 * 0.1 * 0.1;   /* J_ini, :11 */
  s->mass = 12;                /* gait::mass, :32 */
  s->g = 9.8;                  /* _ggg(0,0) = gait::g, PRMPCClass.cpp:166 */
  /* _tx schedule, :172-178 */
  s->tx[0] = 0.0;
  for (int i = 1; i < QO_FOOTSTEPS; i++) {
    s->tx[i] = s->tx[i - 1] + tstep;
    s->tx[i] = round(s->tx[i] / dt_slow) * dt_slow - 0.00001;
  }
  s->nstepx = (int)round(tstep / dt_fast);                         /* :172 */
  s->nsum_mpc = (int)floor(s->tx[QO_FOOTSTEPS - 1] / dt_fast);     /* :185 */
  /* prediction model, :198-220 */
  s->a[0] = 1; s->a[1] = 0; s->a[2] = dt_fast; s->a[3] = 1;
  s->b[0] = pow(dt_fast, 2) / 2; s->b[1] = dt_fast;
  const double cp[2] = {1, 0}, cv[2] = {0, 1};
  matrix_ps(s->a, cp, s->pps);
  matrix_ps(s->a, cv, s->pvs);
  matrix_pu(s->a, s->b, cp, s->ppu);
  matrix_pu(s->a, s->b, cv, s->pvu);
  for (int c = 0; c < NH; ++c)
    for (int r = 0; r < NH; ++r) {
      double a1 = 0, a2 = 0;
      for (int k = 0; k < NH; ++k) {
        a1 += s->pvu[r * NH + k] * s->pvu[c * NH + k];
        a2 += s->ppu[r * NH + k] * s->ppu[c * NH + k];
      }
      s->pvu_2[c * NH + r] = a1;
      s->ppu_2[c * NH + r] = a2;
    }
  /* bounds, :227-250 */
  s->thetax_max = 10 * M_PI / 180; s->thetax_min = -10 * M_PI / 180;
  s->thetay_max = 10 * M_PI / 180; s->thetay_min = -10 * M_PI / 180;
  s->torque_max = 20 / s->j_ini; s->torque_min = -20 / s->j_ini;
  /* ZMP box with the local FOOT_LENGTH/WIDTH = 0.02 override (:161-162,253-256) */
  s->zmpx_max = 0.02 / 2 + 0; s->zmpx_min = -(0.02 / 2 - 0);
  s->zmpy_max = 0.02 / 2;     s->zmpy_min = -0.02 / 2;
  /* go1 weights, :280-287 */
  s->Rthetax = 100; s->Rthetay = 100;
  s->alphathetax = 10; s->alphathetay = 10;
  s->beltathetax = 5000000000.0; s->beltathetay = 5000000000.0;
  s->gama_zmpx = 5000; s->gama_zmpy = 5000;
  s->qp_solution = 1;
  s->ws = qo_eqp_create(NT, 0, NI);
}

void qo_body_free(qo_body_state *s) {
  qo_eqp_destroy(s->ws);
  s->ws = NULL;
}

/* :716-738, xyz = 0 branch (the only one body_theta_mpc uses) */
int qo_body_indexfind(const qo_body_state *s, double goal) {
  int j = 0;
  while (j < QO_FOOTSTEPS && goal >= s->tx[j]) j++;
  return j - 1;
}

#define R2(m, r, c) ((m)[(c) * 2 + (r)])
#define R3(m, r, c) ((m)[(c) * 3 + (r)])

int qo_body_theta_mpc(qo_body_state *s, int i, const double bodyangle_state[4],
                      const double zmp_ref[10], const double angle_ref[10],
                      const double rfoot_ref[10], const double lfoot_ref[10],
                      const double comacc_ref[15], const double Nrtfoorpr_gen[9],
                      double com_traj[14], int *eqp_status) {
  (void)Nrtfoorpr_gen;
  if (eqp_status) *eqp_status = QO_OK;
  const int off = (int)round(1.0 / s->dt_mpc); /* height_offset_time / dt, :395 */
  if (i >= off) {
    i -= off;
    if (i < (s->nsum_mpc - NH)) {
      double t_f0 = (i + 1) * s->dt_mpc, t_f3 = (i + NH) * s->dt_mpc; /* :406 */
      s->bjx1 = qo_body_indexfind(s, t_f0) + 1;
      s->bjx2 = qo_body_indexfind(s, t_f3) + 1;
      int t_yu = (i + 1) % s->nstepx;
      s->t_yu = t_yu;
      double copx[NH], copy[NH];
      /* CoP reference by support parity (:427-499) */
      const double *sup = lfoot_ref, *oth = rfoot_ref;
      if (s->bjx1 >= 2 && (s->bjx1 % 2 != 0)) { sup = rfoot_ref; oth = lfoot_ref; }
      for (int k = 0; k < NH; ++k) { copx[k] = R2(sup, 0, k); copy[k] = R2(sup, 1, k); }
      if (s->bjx1 >= 2 && !((t_yu + NH - 1) < s->nstepx)) {
        int t_yu_k = (t_yu + NH) - s->nstepx;
        for (int jx = 1; jx <= t_yu_k; jx++) {
          copx[NH - jx] = R2(oth, 0, NH - jx);
          copy[NH - jx] = R2(oth, 1, NH - jx);
        }
      }
      /* :504-515 */
      double pth[NH];
      for (int jx = 0; jx < NH; jx++) pth[jx] = s->j_ini / (s->mass * (R3(comacc_ref, 2, jx) + s->g));
      double G[NT * NT], g0[NT];
      memset(G, 0, sizeof(G));
      for (int c = 0; c < NH; ++c)
        for (int r = 0; r < NH; ++r) {
          double I = (r == c) ? 1.0 : 0.0;
          double pp = pth[r] * pth[c]; /* pthetax*pthetax' (diagonal -> only r==c) */
          if (r != c) pp = 0.0;
          double wx = s->Rthetax / 2 * I + s->alphathetax / 2 * s->pvu_2[c * NH + r] +
                      s->beltathetax / 2 * s->ppu_2[c * NH + r] + s->gama_zmpy / 2 * pp;
          double wy = s->Rthetay / 2 * I + s->alphathetay / 2 * s->pvu_2[c * NH + r] +
                      s->beltathetay / 2 * s->ppu_2[c * NH + r] + s->gama_zmpx / 2 * pp;
          G[c * NT + r] = 2 * wx;
          G[(c + NH) * NT + (r + NH)] = 2 * wy;
        }
      double det_px[NH], det_py[NH];
      for (int k = 0; k < NH; ++k) {
        det_px[k] = R2(zmp_ref, 0, k) - copx[k];
        det_py[k] = R2(zmp_ref, 1, k) - copy[k];
      }
      /* q_goal, :523-526 */
      for (int r = 0; r < NH; ++r) {
        double pvs_tx = 0, pps_tx = 0, pvs_ty = 0, pps_ty = 0;
        double vx = 0, px = 0, vy = 0, py = 0, refx = 0, refy = 0;
        for (int k = 0; k < NH; ++k) {
          pvs_tx = s->pvs[k] * s->thetaxk[0] + s->pvs[NH + k] * s->thetaxk[1];
          pps_tx = s->pps[k] * s->thetaxk[0] + s->pps[NH + k] * s->thetaxk[1];
          pvs_ty = s->pvs[k] * s->thetayk[0] + s->pvs[NH + k] * s->thetayk[1];
          pps_ty = s->pps[k] * s->thetayk[0] + s->pps[NH + k] * s->thetayk[1];
          vx += s->pvu[r * NH + k] * pvs_tx;   /* (pvu')(r,k) = pvu(k,r) */
          px += s->ppu[r * NH + k] * pps_tx;
          vy += s->pvu[r * NH + k] * pvs_ty;
          py += s->ppu[r * NH + k] * pps_ty;
          refx += s->ppu[r * NH + k] * R2(angle_ref, 0, k);
          refy += s->ppu[r * NH + k] * R2(angle_ref, 1, k);
        }
        g0[r] = s->alphathetax * vx + s->beltathetax * px - s->beltathetax * refx +
                s->gama_zmpy * pth[r] * det_py[r];
        g0[NH + r] = s->alphathetay * vy + s->beltathetay * py - s->beltathetay * refy +
                     s->gama_zmpx * (-pth[r]) * det_px[r];
      }
      /* constraints, :541-561 and :805-825 */
      double CI[NT * NI], ci0[NI];
      memset(CI, 0, sizeof(CI));
      memset(ci0, 0, sizeof(ci0));
      double ppsx[NH], ppsy[NH];
      for (int k = 0; k < NH; ++k) {
        ppsx[k] = s->pps[k] * s->thetaxk[0] + s->pps[NH + k] * s->thetaxk[1];
        ppsy[k] = s->pps[k] * s->thetayk[0] + s->pps[NH + k] * s->thetayk[1];
      }
      for (int row = 0; row < NH; ++row) {
        for (int v = 0; v < NH; ++v) {
          double pu = s->ppu[v * NH + row];               /* (ppu*Sj)(row, v) */
          CI[(0 * NH + row) * NT + v] = -pu;              /* -q_upx'  */
          CI[(1 * NH + row) * NT + v] = pu;               /* -q_lowx' */
          CI[(2 * NH + row) * NT + NH + v] = -pu;         /* -q_upy'  */
          CI[(3 * NH + row) * NT + NH + v] = pu;          /* -q_lowy' */
        }
        CI[(4 * NH + row) * NT + row] = -s->j_ini;        /* -t_upx'  */
        CI[(5 * NH + row) * NT + row] = s->j_ini;         /* -t_lowx' */
        CI[(6 * NH + row) * NT + NH + row] = -s->j_ini;   /* -t_upy'  */
        CI[(7 * NH + row) * NT + NH + row] = s->j_ini;    /* -t_lowy' */
        ci0[0 * NH + row] = s->thetax_max - ppsx[row];
        ci0[1 * NH + row] = -s->thetax_min + ppsx[row];
        ci0[2 * NH + row] = s->thetay_max - ppsy[row];
        ci0[3 * NH + row] = -s->thetay_min + ppsy[row];
        ci0[4 * NH + row] = s->torque_max;
        ci0[5 * NH + row] = -s->torque_min;
        ci0[6 * NH + row] = s->torque_max;
        ci0[7 * NH + row] = -s->torque_min;
      }
      double X[NT];
      memcpy(X, s->V_ini, sizeof(X)); /* _X = _V_ini, :803 */
      int st = QO_OK;
      qo_eqp_solve(s->ws, G, g0, NULL, NULL, CI, ci0, X, &st, NULL);
      if (eqp_status) *eqp_status = st;
      int ok = 1;
      for (int k = 0; k < NT; ++k)
        if (isnan(X[k])) { ok = 0; break; }
      s->qp_solution = ok;
      memcpy(s->V_ini, X, sizeof(X)); /* Solve: _V_ini = _X, :844-847 */

      /* post-processing, :567-617 */
      const double *a = s->a, *b = s->b;
      double thax0 = s->V_ini[0], thay0 = s->V_ini[NH];
      double a0x = a[0] * s->thetaxk[0] + a[2] * s->thetaxk[1]; /* a.row(0)*thetaxk */
      double a0y = a[0] * s->thetayk[0] + a[2] * s->thetayk[1];
      if (!s->qp_solution) {
        thax0 = (s->thetaxk[0] - a0x) / b[0];
        thay0 = (s->thetayk[0] - a0y) / b[0];
      } else {
        double nx0 = a0x + b[0] * thax0;
        if (nx0 > s->thetax_max) thax0 = (s->thetax_max - a0x) / b[0];
        else if (nx0 < s->thetax_min) thax0 = (s->thetax_min - a0x) / b[0];
        double ny0 = a0y + b[0] * thay0;
        if (ny0 > s->thetay_max) thay0 = (s->thetay_max - a0y) / b[0];
        else if (ny0 < s->thetay_min) thay0 = (s->thetay_min - a0y) / b[0];
      }
      s->V_ini[0] = thax0;  /* :621-622 */
      s->V_ini[NH] = thay0;
      double txk_tmp[2] = {a[0] * s->thetaxk[0] + a[2] * s->thetaxk[1] + b[0] * thax0,
                           a[1] * s->thetaxk[0] + a[3] * s->thetaxk[1] + b[1] * thax0};
      double tyk_tmp[2] = {a[0] * s->thetayk[0] + a[2] * s->thetayk[1] + b[0] * thay0,
                           a[1] * s->thetayk[0] + a[3] * s->thetayk[1] + b[1] * thay0};
      s->torquex_real[0] = s->j_ini * thax0; /* :633-634 */
      s->torquey_real[0] = s->j_ini * thay0;
      for (int jj = 0; jj < NH; jj++) { /* :636-655 */
        double tax = s->V_ini[jj], tay = s->V_ini[NH + jj];
        double x0 = a[0] * s->thetaxk[0] + a[2] * s->thetaxk[1] + b[0] * tax;
        double x1 = a[1] * s->thetaxk[0] + a[3] * s->thetaxk[1] + b[1] * tax;
        s->thetaxk[0] = x0; s->thetaxk[1] = x1;
        s->thetax[jj] = x0;
        double y0 = a[0] * s->thetayk[0] + a[2] * s->thetayk[1] + b[0] * tay;
        double y1 = a[1] * s->thetayk[0] + a[3] * s->thetayk[1] + b[1] * tay;
        s->thetayk[0] = y0; s->thetayk[1] = y1;
        s->thetay[jj] = y0;
        double den = s->mass * (s->g + R3(comacc_ref, 2, jj));
        s->zmpx_real[jj] = R2(zmp_ref, 0, jj) - s->j_ini * tay / den;
        s->zmpy_real[jj] = R2(zmp_ref, 1, jj) + s->j_ini * tax / den;
      }
      s->thetaxk[0] = txk_tmp[0]; s->thetaxk[1] = txk_tmp[1]; /* :659-660 */
      s->thetayk[0] = tyk_tmp[0]; s->thetayk[1] = tyk_tmp[1];
      /* lambda feedback with all lambdas 0 (:664-692), restated literally */
      const double lx = 0.0, lvx = 0.0, ly = 0.0, lvy = 0.0;
      s->thetaxk[0] = lx * bodyangle_state[0] + (1 - lx) * s->thetaxk[0];
      s->thetaxk[1] = lvx * bodyangle_state[1] + (1 - lvx) * s->thetaxk[1];
      s->thetayk[0] = (ly * bodyangle_state[2] + (1 - ly) * s->thetayk[0]);
      s->thetayk[1] = (lvy * bodyangle_state[3] + (1 - lvy) * s->thetayk[1]);
    }
  }
  /* :696-709 */
  com_traj[0] = s->thetax[0];
  com_traj[1] = s->thetay[0];
  com_traj[2] = s->torquex_real[0];
  com_traj[3] = s->torquey_real[0];
  com_traj[4] = s->zmpx_real[0];
  com_traj[5] = s->zmpy_real[0];
  com_traj[6] = s->thetax[1];
  com_traj[7] = s->thetay[1];
  com_traj[8] = s->zmpx_real[1];
  com_traj[9] = s->zmpy_real[1];
  com_traj[10] = s->thetax[2];
  com_traj[11] = s->thetay[2];
  com_traj[12] = s->zmpx_real[2];
  com_traj[13] = s->zmpy_real[2];
  return s->qp_solution;
}
