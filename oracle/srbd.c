/*
 * srbd.c -- literal restatement of the SRBD convex-MPC condensed-QP build
 * (unitree_ros/a1_cpp_open_source/src/ConvexMpc.cpp and the MPC branch of
 * A1RobotControl::compute_grf, A1RobotControl.cpp:452-600), double.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).  Parity unpinned.
 *
 * This is deliberately the dense, as-written algorithm (A_qp by repeated
 * products, B_qp blocks, H = B_qp' Q B_qp + R as a dense triple product):
 * it is the checker for the GPU build, which uses closed forms instead.
 */
#include "qloco_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define INFTY 1e30 /* OsqpEigen::INFTY == OSQP_INFTY (OSQP v0.6 default) */

void qo_srbd_A_c(double yaw, double A_c[169]) { /* ConvexMpc.cpp:111-133 */
  memset(A_c, 0, sizeof(double) * 169);
  double c = cos(yaw), s = sin(yaw);
  /* block(0,6) = [[c,s,0],[-s,c,0],[0,0,1]] */
  A_c[6 * 13 + 0] = c;  A_c[7 * 13 + 0] = s;
  A_c[6 * 13 + 1] = -s; A_c[7 * 13 + 1] = c;
  A_c[8 * 13 + 2] = 1;
  for (int k = 0; k < 3; ++k) A_c[(9 + k) * 13 + 3 + k] = 1; /* block(3,9) = I */
  A_c[12 * 13 + 11] = 1;                                      /* A_c(11, NUM_DOF) */
}

/* Eigen Matrix3d::inverse (cofactor form) */
static void inv3(const double m[9], double o[9]) {
#define E(r, c) m[(c) * 3 + (r)]
  double c00 = E(1, 1) * E(2, 2) - E(1, 2) * E(2, 1);
  double c10 = E(1, 2) * E(2, 0) - E(1, 0) * E(2, 2);
  double c20 = E(1, 0) * E(2, 1) - E(1, 1) * E(2, 0);
  double det = E(0, 0) * c00 + E(0, 1) * c10 + E(0, 2) * c20;
  double id = 1.0 / det;
  o[0 * 3 + 0] = c00 * id;
  o[0 * 3 + 1] = c10 * id;
  o[0 * 3 + 2] = c20 * id;
  o[1 * 3 + 0] = (E(0, 2) * E(2, 1) - E(0, 1) * E(2, 2)) * id;
  o[1 * 3 + 1] = (E(0, 0) * E(2, 2) - E(0, 2) * E(2, 0)) * id;
  o[1 * 3 + 2] = (E(0, 1) * E(2, 0) - E(0, 0) * E(2, 1)) * id;
  o[2 * 3 + 0] = (E(0, 1) * E(1, 2) - E(0, 2) * E(1, 1)) * id;
  o[2 * 3 + 1] = (E(0, 2) * E(1, 0) - E(0, 0) * E(1, 2)) * id;
  o[2 * 3 + 2] = (E(0, 0) * E(1, 1) - E(0, 1) * E(1, 0)) * id;
#undef E
}

static void mm(int M, int K, int N, const double *A, int lda, const double *B, int ldb,
               double *C, int ldc) { /* C = A*B, col-major */
  for (int c = 0; c < N; ++c)
    for (int r = 0; r < M; ++r) {
      double acc = 0.0;
      for (int k = 0; k < K; ++k) acc += A[(size_t)k * lda + r] * B[(size_t)c * ldb + k];
      C[(size_t)c * ldc + r] = acc;
    }
}

void qo_srbd_B_c(double mass, const double I[9], const double R[9], const double feet[12],
                 double B_c[156]) { /* ConvexMpc.cpp:135-147 */
  memset(B_c, 0, sizeof(double) * 156);
  double RI[9], Iw[9], Rt[9], Iwi[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) Rt[c * 3 + r] = R[r * 3 + c];
  mm(3, 3, 3, R, 3, I, 3, RI, 3);
  mm(3, 3, 3, RI, 3, Rt, 3, Iw, 3);
  inv3(Iw, Iwi);
  for (int i = 0; i < 4; ++i) {
    const double *v = feet + 3 * i;
    double S[9] = {0, v[2], -v[1], -v[2], 0, v[0], v[1], -v[0], 0}; /* Utils::skew, col-major */
    double T[9];
    mm(3, 3, 3, Iwi, 3, S, 3, T, 3);
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) {
        B_c[(3 * i + c) * 13 + 6 + r] = T[c * 3 + r];
        B_c[(3 * i + c) * 13 + 9 + r] = (r == c) ? (1.0 / mass) : 0.0;
      }
  }
}

void qo_srbd_discretize(const double A_c[169], const double B_c[156], double dt,
                        double A_d[169], double B_d[156]) { /* ConvexMpc.cpp:149-160 */
  for (int c = 0; c < 13; ++c)
    for (int r = 0; r < 13; ++r) A_d[c * 13 + r] = (r == c ? 1.0 : 0.0) + A_c[c * 13 + r] * dt;
  for (int i = 0; i < 156; ++i) B_d[i] = B_c[i] * dt;
}

void qo_srbd_constraints(const qo_srbd_spec *sp, double *C) { /* ConvexMpc.cpp:47-59 */
  int N = sp->N, m = 20 * N, n = 12 * N;
  memset(C, 0, sizeof(double) * (size_t)m * n);
  for (int i = 0; i < 4 * N; ++i) {
    C[(size_t)(3 * i) * m + 5 * i + 0] = 1;
    C[(size_t)(3 * i) * m + 5 * i + 1] = 1;
    C[(size_t)(3 * i + 1) * m + 5 * i + 2] = 1;
    C[(size_t)(3 * i + 1) * m + 5 * i + 3] = 1;
    C[(size_t)(3 * i + 2) * m + 5 * i + 4] = 1;
    C[(size_t)(3 * i + 2) * m + 5 * i + 0] = sp->mu;
    C[(size_t)(3 * i + 2) * m + 5 * i + 1] = -sp->mu;
    C[(size_t)(3 * i + 2) * m + 5 * i + 2] = sp->mu;
    C[(size_t)(3 * i + 2) * m + 5 * i + 3] = -sp->mu;
  }
}

void qo_srbd_qp_mats(const qo_srbd_spec *sp, const double A_d[169], const double *B_d_list,
                     const double x0[13], const double *x_ref, const uint8_t *contacts,
                     int contacts_per_step, double *Aqp_o, double *Bqp_o, double *H,
                     double *g, double *lb, double *ub) {
  const int N = sp->N, nx = 13 * N, nu = 12 * N;
  double *Aqp = (double *)calloc((size_t)nx * 13, sizeof(double));
  double *Bqp = (double *)calloc((size_t)nx * nu, sizeof(double));
  double tmp[156];
  /* A_qp / B_qp, ConvexMpc.cpp:188-205 */
  for (int i = 0; i < N; ++i) {
    if (i == 0) {
      for (int c = 0; c < 13; ++c)
        for (int r = 0; r < 13; ++r) Aqp[(size_t)c * nx + r] = A_d[c * 13 + r];
    } else {
      mm(13, 13, 13, Aqp + 13 * (i - 1), nx, A_d, 13, Aqp + 13 * i, nx);
    }
    for (int j = 0; j < i + 1; ++j) {
      const double *Bj = B_d_list + 156 * j;
      if (i - j == 0) {
        for (int c = 0; c < 12; ++c)
          for (int r = 0; r < 13; ++r) Bqp[(size_t)(12 * j + c) * nx + 13 * i + r] = Bj[c * 13 + r];
      } else {
        mm(13, 13, 12, Aqp + 13 * (i - j - 1), nx, Bj, 13, tmp, 13);
        for (int c = 0; c < 12; ++c)
          for (int r = 0; r < 13; ++r) Bqp[(size_t)(12 * j + c) * nx + 13 * i + r] = tmp[c * 13 + r];
      }
    }
  }
  /* dense H = B' Q B + R, ConvexMpc.cpp:207-215 (Q = diag(2 q_w), R = diag(2 r_w), :18-45) */
  if (H) {
    double *QB = (double *)malloc(sizeof(double) * (size_t)nx * nu);
    for (int c = 0; c < nu; ++c)
      for (int r = 0; r < nx; ++r) QB[(size_t)c * nx + r] = 2.0 * sp->q_w[r % 13] * Bqp[(size_t)c * nx + r];
    for (int c = 0; c < nu; ++c)
      for (int r = 0; r < nu; ++r) {
        double acc = 0.0;
        for (int k = 0; k < nx; ++k) acc += Bqp[(size_t)r * nx + k] * QB[(size_t)c * nx + k];
        H[(size_t)c * nu + r] = acc;
      }
    for (int i = 0; i < nu; ++i) H[(size_t)i * nu + i] += 2.0 * sp->r_w[i % 12];
    free(QB);
  }
  /* g = B' Q (A_qp x0 - x_d), :219-221 */
  if (g) {
    double *e = (double *)malloc(sizeof(double) * nx);
    for (int r = 0; r < nx; ++r) {
      double acc = 0.0;
      for (int k = 0; k < 13; ++k) acc += Aqp[(size_t)k * nx + r] * x0[k];
      e[r] = 2.0 * sp->q_w[r % 13] * (acc - x_ref[r]);
    }
    for (int c = 0; c < nu; ++c) {
      double acc = 0.0;
      for (int k = 0; k < nx; ++k) acc += Bqp[(size_t)c * nx + k] * e[k];
      g[c] = acc;
    }
    free(e);
  }
  /* bounds, :223-249 (fz_min = 0, fz_max = 180 are set inside calculate_qp_mats) */
  if (lb && ub) {
    for (int k = 0; k < N; ++k)
      for (int i = 0; i < 4; ++i) {
        double c = contacts[contacts_per_step ? 4 * k + i : i] ? 1.0 : 0.0;
        double *l = lb + 20 * k + 5 * i, *u = ub + 20 * k + 5 * i;
        l[0] = 0; l[1] = -INFTY; l[2] = 0; l[3] = -INFTY; l[4] = sp->fz_min * c;
        u[0] = INFTY; u[1] = 0; u[2] = INFTY; u[3] = 0; u[4] = sp->fz_max * c;
      }
  }
  if (Aqp_o) memcpy(Aqp_o, Aqp, sizeof(double) * (size_t)nx * 13);
  if (Bqp_o) memcpy(Bqp_o, Bqp, sizeof(double) * (size_t)nx * nu);
  free(Aqp);
  free(Bqp);
}

void qo_srbd_build_instance(const qo_srbd_spec *sp, const double x0[13], const double *x_ref,
                            const double *feet, int feet_per_step, const uint8_t *contacts,
                            int contacts_per_step, double *H, double *g, double *lb,
                            double *ub) {
  const int N = sp->N;
  double A_c[169], A_d[169], B_c[156];
  double *B_d = (double *)malloc(sizeof(double) * 156 * N);
  /* yaw-only "rotation" that overwrites root_rot_mat, A1RobotControl.cpp:502-510 */
  double c = cos(x0[2]), s = sin(x0[2]);
  double R[9] = {c, -s, 0, s, c, 0, 0, 0, 1}; /* rows [[c,s,0],[-s,c,0],[0,0,1]] */
  qo_srbd_A_c(x0[2], A_c);                    /* :512 */
  for (int k = 0; k < N; ++k) {               /* :518-549 */
    qo_srbd_B_c(sp->mass, sp->inertia, R, feet + (feet_per_step ? 12 * k : 0), B_c);
    qo_srbd_discretize(A_c, B_c, sp->dt, A_d, B_d + 156 * k);
  }
  qo_srbd_qp_mats(sp, A_d, B_d, x0, x_ref, contacts, contacts_per_step, NULL, NULL, H, g, lb,
                  ub);
  free(B_d);
}
