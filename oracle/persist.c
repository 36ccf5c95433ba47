/*
 * persist.c -- the reference's persistent OSQP solver for the SRBD MPC,
 * restated on the stance-only QP (TEST INFRASTRUCTURE ONLY, see
 * qloco_oracle.h).
 *
 * A1RobotControl keeps ONE OsqpEigen::Solver per controller
 * (A1RobotControl.h:67).  The first MPC tick sets it up with warm start on
 * (A1RobotControl.cpp:557-569: setWarmStart(true), initSolver); every later
 * tick calls updateHessianMatrix / updateGradient / updateLowerBound /
 * updateUpperBound and solve() (:570-577).  In OSQP v0.6 that is
 *   osqp_update_P      unscale_data, new P, scale_data (Ruiz from scratch,
 *                      the cost scale seeing the PREVIOUS q), refactor with
 *                      the current rho_vec
 *   osqp_update_lin_cost   q = c * (D q_new)
 *   osqp_update_*_bound    l, u = E l_new, E u_new; update_rho_vec
 *   osqp_solve         no cold start: the scaled x, z, y of the last solve
 *                      as they are; rho as adapted by the last solve
 The literal 12N-variable QP (literal = 1, the reference's call): the
 * Hessian pattern does not depend on the contacts, so every call after the
 * first is the update path above; the new bounds re-type the fz rows whose
 * contact flag changed (update_rho_vec: l == u -> equality, 1e3 rho), which
 * set_rho_vec inside qo_admm_solve_ex does from the new bounds.
 * The stance-only reduction (literal = 0, the fast kernels' problem, DESIGN.md
 * §3) changes dimensions with the stance set.  Same stance set as the last
 * call: the update path (QO_ADMM_RESUME).  Changed stance set: the analogue
 * of OsqpEigen's re-initialisation branch for a changed problem structure
 * (getPrimal/DualVariable, clearSolver, initSolver, setPrimal/DualVariable):
 * fresh setup (settings rho) warm-started from the last unscaled solution
 * (QO_ADMM_WARM), variables / rows that were not stance starting at 0 -- a
 * documented deviation from the reference.  First call: cold.
 *
 * Record layout (doubles, full index: variable 12k + 3i + c, row 20k + 5i + r):
 *   [0,12N) xs   [12N,32N) zs   [32N,52N) ys      scaled iterates
 *   [52N,64N) xu [64N,84N) yu                     unscaled solution
 *   [84N,96N) qp (unscaled q of the last call)   [96N,100N) contacts (0/1)
 *   [100N] rho   [100N+1] 1 after the first call (0 = fresh record)
 */
#include "qloco_oracle.h"

#include <stdlib.h>
#include <string.h>

int qo_srbd_persist_step(double *rec, const qo_srbd_spec *sp, const qo_admm_settings *st,
                         const float *x0f, const float *xrf, const float *ftf, int feet_per_step,
                         const uint8_t *contacts, int contacts_per_step, double *u,
                         qo_admm_info *info) {
  return qo_srbd_persist_step_ex(rec, sp, st, x0f, xrf, ftf, feet_per_step, contacts,
                                 contacts_per_step, 0, u, info);
}

int qo_srbd_persist_step_ex(double *rec, const qo_srbd_spec *sp, const qo_admm_settings *st,
                            const float *x0f, const float *xrf, const float *ftf,
                            int feet_per_step, const uint8_t *contacts, int contacts_per_step,
                            int literal, double *u, qo_admm_info *info) {
  const int N = sp->N, nu = 12 * N, nc = 20 * N;
  double *xs = rec, *zs = rec + 12 * N, *ys = rec + 32 * N, *xu = rec + 52 * N;
  double *yu = rec + 64 * N, *qp = rec + 84 * N, *ct = rec + 96 * N;
  double *rho = rec + 100 * N, *calls = rec + 100 * N + 1;
  double x0[13];
  for (int k = 0; k < 13; ++k) x0[k] = x0f[k];
  double *xr = (double *)malloc(sizeof(double) * 13 * N);
  for (int k = 0; k < 13 * N; ++k) xr[k] = xrf[k];
  const int nft = feet_per_step ? 12 * N : 12;
  double *ft = (double *)malloc(sizeof(double) * nft);
  for (int k = 0; k < nft; ++k) ft[k] = ftf[k];
  uint8_t *c = (uint8_t *)malloc(4 * N);
  for (int k = 0; k < 4 * N; ++k) c[k] = contacts[contacts_per_step ? k : (k & 3)] ? 1 : 0;
  double *H = (double *)malloc(sizeof(double) * nu * nu), *g = (double *)malloc(sizeof(double) * nu);
  double *lb = (double *)malloc(sizeof(double) * nc), *ub = (double *)malloc(sizeof(double) * nc);
  double *C = (double *)malloc(sizeof(double) * nc * nu);
  qo_srbd_build_instance(sp, x0, xr, ft, feet_per_step, c, 1, H, g, lb, ub);
  qo_srbd_constraints(sp, C);
  /* stance reduction: variables and rows of stance (step, leg) pairs;
   * the literal QP keeps every pair (ConvexMpc.cpp:227-249, A1RobotControl.cpp:560-567) */
  int *vi = (int *)malloc(sizeof(int) * nu), *ri = (int *)malloc(sizeof(int) * nc);
  int n = 0, m = 0;
  for (int k = 0; k < 4 * N; ++k)
    if (literal || c[k]) {
      for (int j = 0; j < 3; ++j) vi[n++] = 3 * k + j;
      for (int j = 0; j < 5; ++j) ri[m++] = 5 * k + j;
    }
  double *P = (double *)malloc(sizeof(double) * (n ? n * n : 1));
  double *q = (double *)malloc(sizeof(double) * (n ? n : 1));
  double *A = (double *)malloc(sizeof(double) * (n > 0 && m > 0 ? n * m : 1));
  double *l = (double *)malloc(sizeof(double) * (m ? m : 1));
  double *uu = (double *)malloc(sizeof(double) * (m ? m : 1));
  for (int a = 0; a < n; ++a) {
    q[a] = g[vi[a]];
    for (int b = 0; b < n; ++b) P[(size_t)b * n + a] = H[(size_t)vi[b] * nu + vi[a]];
    for (int r = 0; r < m; ++r) A[(size_t)a * m + r] = C[(size_t)vi[a] * nc + ri[r]];
  }
  for (int r = 0; r < m; ++r) {
    l[r] = lb[ri[r]];
    uu[r] = ub[ri[r]];
  }
  int same = *calls > 0.0;
  /* the literal problem's structure never changes: after the first call every
   * call is OsqpEigen's update path (updateHessianMatrix finds the pattern of
   * hessian = dense_hessian.sparseView() unchanged, ConvexMpc.cpp:211-215) */
  if (!literal)
    for (int k = 0; k < 4 * N && same; ++k) same = (ct[k] != 0.0) == (c[k] != 0);
  double *ix = (double *)calloc(n ? n : 1, sizeof(double)), *iz = (double *)calloc(m ? m : 1, sizeof(double));
  double *iy = (double *)calloc(m ? m : 1, sizeof(double)), *iq = (double *)calloc(n ? n : 1, sizeof(double));
  qo_admm_init in;
  memset(&in, 0, sizeof(in));
  if (same) {
    in.mode = QO_ADMM_RESUME;
    for (int a = 0; a < n; ++a) { ix[a] = xs[vi[a]]; iq[a] = qp[vi[a]]; }
    for (int r = 0; r < m; ++r) { iz[r] = zs[ri[r]]; iy[r] = ys[ri[r]]; }
    in.x = ix; in.z = iz; in.y = iy; in.rho = *rho; in.q_scale = iq;
  } else if (*calls > 0.0) {
    in.mode = QO_ADMM_WARM;
    for (int a = 0; a < n; ++a) ix[a] = xu[vi[a]];
    for (int r = 0; r < m; ++r) iy[r] = yu[ri[r]];
    in.x = ix; in.y = iy;
  } else {
    in.mode = QO_ADMM_COLD;
  }
  double *ox = (double *)malloc(sizeof(double) * (n ? n : 1)), *oz = (double *)malloc(sizeof(double) * (m ? m : 1));
  double *oy = (double *)malloc(sizeof(double) * (m ? m : 1)), *xo = (double *)malloc(sizeof(double) * (n ? n : 1));
  double *yo = (double *)malloc(sizeof(double) * (m ? m : 1));
  qo_admm_state out = {ox, oz, oy, 0.0};
  qo_admm_info inf;
  memset(&inf, 0, sizeof(inf));
  int status = QO_OK;
  if (n > 0) {
    status = qo_admm_solve_ex(st, n, m, P, q, A, l, uu, &in, &out, xo, yo, &inf);
  } else {
    out.rho = same ? *rho : st->rho;
  }
  /* store the record: zeros outside the stance set */
  memset(rec, 0, sizeof(double) * QO_SRBD_PERSIST_LEN(N));
  for (int a = 0; a < n; ++a) { xs[vi[a]] = ox[a]; xu[vi[a]] = xo[a]; }
  for (int r = 0; r < m; ++r) { zs[ri[r]] = oz[r]; ys[ri[r]] = oy[r]; yu[ri[r]] = yo[r]; }
  for (int j = 0; j < nu; ++j) qp[j] = g[j];
  for (int k = 0; k < 4 * N; ++k) ct[k] = c[k];
  *rho = out.rho;
  *calls = 1.0;  /* written after the memset */
  if (u) {
    memset(u, 0, sizeof(double) * nu);
    for (int a = 0; a < n; ++a) u[vi[a]] = xo[a];
  }
  if (info) *info = inf;
  free(xr); free(ft); free(c); free(H); free(g); free(lb); free(ub); free(C); free(vi); free(ri);
  free(P); free(q); free(A); free(l); free(uu); free(ix); free(iz); free(iy); free(iq);
  free(ox); free(oz); free(oy); free(xo); free(yo);
  return status;
}
