/*
 * admm.c -- restatement of the OSQP ADMM algorithm that the reference calls
 * through OsqpEigen for the SRBD MPC (A1RobotControl.cpp:557-578;
 * test_mpc.cpp:131-151), plus an exact-optimum wrapper around the
 * EiQuadProg restatement.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).
 *
 * THIRD-PARTY ALGORITHM: OSQP is not vendored under /root/reference and its
 * version is unpinned (find_package(OsqpEigen REQUIRED)).  We
 * restate the published OSQP v0.6.x algorithm with its default settings:
 *   rho 0.1, sigma 1e-6, alpha 1.6, eps_abs = eps_rel = 1e-3,
 *   eps_prim_inf = eps_dual_inf = 1e-4, max_iter 4000, check_termination 25,
 *   scaling 10 (modified Ruiz), adaptive_rho on (tolerance 5), polish off.
 * OSQP's default adaptive_rho_interval = 0 picks the interval from the setup
 * time when built with PROFILING (non-deterministic); we use the
 * deterministic non-PROFILING rule, 4 * check_termination = 100.
 * The KKT system [[P+sigma I, A'],[A, -diag(1/rho)]] is solved in its
 * reduced form (P + sigma I + A' diag(rho) A) by dense Cholesky -- the same
 * linear algebra as OSQP's QDLDL path, different factorisation.
 * Parity for this path is unpinned: no reference test pins OSQP outputs.
 */
#include "qloco_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define OSQP_INFTY 1e30
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define RHO_TOL 1e-4
#define OSQP_DIVISION_TOL (1.0 / OSQP_INFTY)

void qo_admm_settings_default(qo_admm_settings *s) {
  s->rho = 0.1;
  s->sigma = 1e-6;
  s->alpha = 1.6;
  s->eps_abs = 1e-3;
  s->eps_rel = 1e-3;
  s->eps_prim_inf = 1e-4;
  s->eps_dual_inf = 1e-4;
  s->max_iter = 4000;
  s->check_termination = 25;
  s->scaling = 10;
  s->adaptive_rho = 1;
  s->adaptive_rho_interval = 0;
  s->adaptive_rho_tolerance = 5.0;
  s->warm_start = 0;
}

static double vnorm(const double *v, int n) {
  double m = 0.0;
  for (int i = 0; i < n; ++i) m = fmax(m, fabs(v[i]));
  return m;
}
static double vsnorm(const double *s, const double *v, int n) {
  double m = 0.0;
  for (int i = 0; i < n; ++i) m = fmax(m, fabs(s[i] * v[i]));
  return m;
}
static void limit_scaling(double *D, int n) {
  for (int i = 0; i < n; ++i) {
    D[i] = D[i] < MIN_SCALING ? 1.0 : D[i];
    D[i] = D[i] > MAX_SCALING ? MAX_SCALING : D[i];
  }
}

/* dense Cholesky, lower, in place; returns 0 if not PD */
static int chol(int n, double *K) {
  for (int k = 0; k < n; ++k) {
    double x = K[(size_t)k * n + k];
    for (int j = 0; j < k; ++j) x -= K[(size_t)j * n + k] * K[(size_t)j * n + k];
    if (!(x > 0.0)) return 0;
    double l = sqrt(x);
    K[(size_t)k * n + k] = l;
    for (int r = k + 1; r < n; ++r) {
      double a = K[(size_t)k * n + r];
      for (int j = 0; j < k; ++j) a -= K[(size_t)j * n + r] * K[(size_t)j * n + k];
      K[(size_t)k * n + r] = a / l;
    }
  }
  return 1;
}
static void chol_solve(int n, const double *L, double *b) {
  for (int i = 0; i < n; ++i) {
    double a = b[i];
    for (int j = 0; j < i; ++j) a -= L[(size_t)j * n + i] * b[j];
    b[i] = a / L[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double a = b[i];
    for (int j = i + 1; j < n; ++j) a -= L[(size_t)i * n + j] * b[j];
    b[i] = a / L[(size_t)i * n + i];
  }
}

typedef struct {
  int n, m;
  double *P, *q, *A, *l, *u;   /* scaled data */
  double *D, *E, *Dinv, *Einv, c, cinv;
  double *rho_vec, *rho_inv;
  int *ctype;
  double *K;                   /* Cholesky factor of the reduced KKT */
  double rho, sigma;
  /* A in CSC (OSQP stores A sparse): column j has rows ai[ap[j]..ap[j+1]) */
  int *ap, *ai;
  double *ax;
} admm_ws;

/* refresh the CSC values from the (scaled) dense A */
static void csc_build(admm_ws *w) {
  int nnz = 0;
  for (int j = 0; j < w->n; ++j) {
    w->ap[j] = nnz;
    for (int i = 0; i < w->m; ++i) {
      double a = w->A[(size_t)j * w->m + i];
      if (a != 0.0) { w->ai[nnz] = i; w->ax[nnz] = a; nnz++; }
    }
  }
  w->ap[w->n] = nnz;
}
static void csc_Ax(const admm_ws *w, const double *x, double *y) {
  for (int i = 0; i < w->m; ++i) y[i] = 0.0;
  for (int j = 0; j < w->n; ++j)
    for (int k = w->ap[j]; k < w->ap[j + 1]; ++k) y[w->ai[k]] += w->ax[k] * x[j];
}
static void csc_Aty(const admm_ws *w, const double *y, double *x) {
  for (int j = 0; j < w->n; ++j) {
    double a = 0.0;
    for (int k = w->ap[j]; k < w->ap[j + 1]; ++k) a += w->ax[k] * y[w->ai[k]];
    x[j] = a;
  }
}

static void build_factor(admm_ws *w) {
  int n = w->n;
  for (int c = 0; c < n; ++c)
    for (int r = 0; r < n; ++r) w->K[(size_t)c * n + r] = w->P[(size_t)c * n + r] + (r == c ? w->sigma : 0.0);
  /* + A' diag(rho) A: sum over rows shared by columns r, c */
  for (int c = 0; c < n; ++c)
    for (int r = 0; r < n; ++r) {
      int kr = w->ap[r], kc = w->ap[c];
      double a = 0.0;
      while (kr < w->ap[r + 1] && kc < w->ap[c + 1]) {
        if (w->ai[kr] == w->ai[kc]) { a += w->ax[kr] * w->rho_vec[w->ai[kr]] * w->ax[kc]; kr++; kc++; }
        else if (w->ai[kr] < w->ai[kc]) kr++;
        else kc++;
      }
      w->K[(size_t)c * n + r] += a;
    }
  chol(n, w->K);
}

static void set_rho_vec(admm_ws *w) {
  w->rho = fmin(fmax(w->rho, RHO_MIN), RHO_MAX);
  for (int i = 0; i < w->m; ++i) {
    if (w->l[i] < -OSQP_INFTY * MIN_SCALING && w->u[i] > OSQP_INFTY * MIN_SCALING) {
      w->ctype[i] = -1;
      w->rho_vec[i] = RHO_MIN;
    } else if (w->u[i] - w->l[i] < RHO_TOL) {
      w->ctype[i] = 1;
      w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->rho;
    } else {
      w->ctype[i] = 0;
      w->rho_vec[i] = w->rho;
    }
    w->rho_inv[i] = 1.0 / w->rho_vec[i];
  }
}

static void update_rho(admm_ws *w, double rho_new) {
  w->rho = fmin(fmax(rho_new, RHO_MIN), RHO_MAX);
  for (int i = 0; i < w->m; ++i) {
    if (w->ctype[i] == 0) w->rho_vec[i] = w->rho;
    else if (w->ctype[i] == 1) w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->rho;
    w->rho_inv[i] = 1.0 / w->rho_vec[i];
  }
  build_factor(w);
}

/* modified Ruiz equilibration, OSQP scaling.c scale_data */
static void scale_data(admm_ws *w, int iters) {
  int n = w->n, m = w->m;
  double *Dt = (double *)malloc(sizeof(double) * n), *Et = (double *)malloc(sizeof(double) * (m ? m : 1));
  w->c = 1.0;
  for (int j = 0; j < n; ++j) w->D[j] = 1.0;
  for (int i = 0; i < m; ++i) w->E[i] = 1.0;
  for (int it = 0; it < iters; ++it) {
    for (int j = 0; j < n; ++j) {
      double a = 0.0;
      for (int r = 0; r < n; ++r) a = fmax(a, fabs(w->P[(size_t)j * n + r]));
      for (int i = 0; i < m; ++i) a = fmax(a, fabs(w->A[(size_t)j * m + i]));
      Dt[j] = a;
    }
    for (int i = 0; i < m; ++i) {
      double a = 0.0;
      for (int j = 0; j < n; ++j) a = fmax(a, fabs(w->A[(size_t)j * m + i]));
      Et[i] = a;
    }
    limit_scaling(Dt, n);
    limit_scaling(Et, m);
    for (int j = 0; j < n; ++j) Dt[j] = 1.0 / sqrt(Dt[j]);
    for (int i = 0; i < m; ++i) Et[i] = 1.0 / sqrt(Et[i]);
    for (int c = 0; c < n; ++c)
      for (int r = 0; r < n; ++r) w->P[(size_t)c * n + r] *= Dt[r] * Dt[c];
    for (int c = 0; c < n; ++c)
      for (int i = 0; i < m; ++i) w->A[(size_t)c * m + i] *= Et[i] * Dt[c];
    for (int j = 0; j < n; ++j) w->q[j] *= Dt[j];
    for (int j = 0; j < n; ++j) w->D[j] *= Dt[j];
    for (int i = 0; i < m; ++i) w->E[i] *= Et[i];
    /* cost scaling */
    double mean = 0.0;
    for (int j = 0; j < n; ++j) {
      double a = 0.0;
      for (int r = 0; r < n; ++r) a = fmax(a, fabs(w->P[(size_t)j * n + r]));
      mean += a;
    }
    mean /= n;
    double qn = vnorm(w->q, n);
    limit_scaling(&qn, 1);
    double ct = fmax(mean, qn);
    limit_scaling(&ct, 1);
    ct = 1.0 / ct;
    for (size_t k = 0; k < (size_t)n * n; ++k) w->P[k] *= ct;
    for (int j = 0; j < n; ++j) w->q[j] *= ct;
    w->c *= ct;
  }
  w->cinv = 1.0 / w->c;
  for (int j = 0; j < n; ++j) w->Dinv[j] = 1.0 / w->D[j];
  for (int i = 0; i < m; ++i) w->Einv[i] = 1.0 / w->E[i];
  for (int i = 0; i < m; ++i) { w->l[i] *= w->E[i]; w->u[i] *= w->E[i]; }
  free(Dt);
  free(Et);
}

int qo_admm_solve(const qo_admm_settings *st, int n, int m, const double *P0, const double *q0,
                  const double *A0, const double *l0, const double *u0, double *xo, double *yo,
                  qo_admm_info *info) {
  qo_admm_init in;
  memset(&in, 0, sizeof(in));
  in.mode = st->warm_start ? QO_ADMM_WARM : QO_ADMM_COLD;
  in.x = xo;
  in.y = yo;
  return qo_admm_solve_ex(st, n, m, P0, q0, A0, l0, u0, &in, NULL, xo, yo, info);
}

int qo_admm_solve_ex(const qo_admm_settings *st, int n, int m, const double *P0, const double *q0,
                     const double *A0, const double *l0, const double *u0, const qo_admm_init *in,
                     qo_admm_state *out, double *xo, double *yo, qo_admm_info *info) {
  admm_ws W, *w = &W;
  memset(w, 0, sizeof(W));
  w->n = n; w->m = m;
  w->P = (double *)malloc(sizeof(double) * (size_t)n * n); memcpy(w->P, P0, sizeof(double) * (size_t)n * n);
  w->q = (double *)malloc(sizeof(double) * n); memcpy(w->q, q0, sizeof(double) * n);
  w->A = (double *)malloc(sizeof(double) * (size_t)m * n); memcpy(w->A, A0, sizeof(double) * (size_t)m * n);
  w->l = (double *)malloc(sizeof(double) * m); memcpy(w->l, l0, sizeof(double) * m);
  w->u = (double *)malloc(sizeof(double) * m); memcpy(w->u, u0, sizeof(double) * m);
  w->D = (double *)malloc(sizeof(double) * n); w->Dinv = (double *)malloc(sizeof(double) * n);
  w->E = (double *)malloc(sizeof(double) * m); w->Einv = (double *)malloc(sizeof(double) * m);
  w->rho_vec = (double *)malloc(sizeof(double) * m); w->rho_inv = (double *)malloc(sizeof(double) * m);
  w->ctype = (int *)malloc(sizeof(int) * m);
  w->K = (double *)malloc(sizeof(double) * (size_t)n * n);
  w->ap = (int *)malloc(sizeof(int) * (n + 1));
  w->ai = (int *)malloc(sizeof(int) * (size_t)m * n);
  w->ax = (double *)malloc(sizeof(double) * (size_t)m * n);
  double *x = (double *)calloc(n, sizeof(double)), *xp = (double *)calloc(n, sizeof(double));
  double *z = (double *)calloc(m, sizeof(double)), *zp = (double *)calloc(m, sizeof(double));
  double *y = (double *)calloc(m, sizeof(double)), *dy = (double *)calloc(m, sizeof(double));
  double *dx = (double *)calloc(n, sizeof(double)), *xt = (double *)calloc(n, sizeof(double));
  double *zt = (double *)calloc(m, sizeof(double)), *Ax = (double *)calloc(m, sizeof(double));
  double *Px = (double *)calloc(n, sizeof(double)), *Aty = (double *)calloc(n, sizeof(double));
  double *rp = (double *)calloc(m, sizeof(double)), *rd = (double *)calloc(n, sizeof(double));
  double *tm = (double *)calloc(m > n ? m : n, sizeof(double));

  w->sigma = st->sigma;
  /* QO_ADMM_RESUME (OSQP's update path, osqp_update_P + osqp_update_lin_cost
   * + osqp_update_{lower,upper}_bound on a live workspace): scale_data runs
   * on the new P with the PREVIOUS q still in place (update_P precedes
   * update_lin_cost), so the cost scale c sees the old gradient; the new q
   * is then scaled as c * (D q_new); the adapted rho of the last solve stays */
  const int resume = in && in->mode == QO_ADMM_RESUME;
  w->rho = resume ? in->rho : st->rho;
  if (resume && in->q_scale) memcpy(w->q, in->q_scale, sizeof(double) * n);
  if (st->scaling) scale_data(w, st->scaling);
  else {
    w->c = w->cinv = 1.0;
    for (int j = 0; j < n; ++j) w->D[j] = w->Dinv[j] = 1.0;
    for (int i = 0; i < m; ++i) w->E[i] = w->Einv[i] = 1.0;
  }
  if (resume && in->q_scale) {
    for (int j = 0; j < n; ++j) {
      w->q[j] = w->D[j] * q0[j];
      w->q[j] *= w->c;
    }
  }
  csc_build(w);
  set_rho_vec(w);
  build_factor(w);
  int interval = st->adaptive_rho_interval;
  if (st->adaptive_rho && !interval)
    interval = st->check_termination ? 4 * st->check_termination : 100; /* ADAPTIVE_RHO_FIXED */

  if (in && in->mode == QO_ADMM_WARM) { /* osqp_warm_start: x by Dinv, y by Einv*c, z = A x */
    for (int j = 0; j < n; ++j) x[j] = in->x[j] * w->Dinv[j];
    for (int i = 0; i < m; ++i) y[i] = in->y[i] * w->Einv[i] * w->c;
    csc_Ax(w, x, z);
  } else if (resume) { /* warm_start on a live workspace: the scaled iterates as they are */
    memcpy(x, in->x, sizeof(double) * n);
    memcpy(z, in->z, sizeof(double) * m);
    memcpy(y, in->y, sizeof(double) * m);
  }

  int iter, status = QO_MAX_ITER, can_check = 0, rho_updates = 0;
  double pri_res = 0, dua_res = 0;
  /* residuals in the scaled space + their unscaled norms (update_info) */
#define UPDATE_INFO()                                                                    \
  do {                                                                                   \
    csc_Ax(w, x, Ax);                                                                    \
    for (int i = 0; i < m; ++i) rp[i] = Ax[i] - z[i];                                    \
    pri_res = vsnorm(w->Einv, rp, m);                                                    \
    csc_Aty(w, y, Aty);                                                                  \
    for (int j = 0; j < n; ++j) {                                                        \
      double a = 0.0;                                                                    \
      for (int r = 0; r < n; ++r) a += w->P[(size_t)r * n + j] * x[r];                   \
      Px[j] = a;                                                                         \
      rd[j] = w->q[j] + a + Aty[j];                                                      \
    }                                                                                    \
    dua_res = w->cinv * vsnorm(w->Dinv, rd, n);                                          \
  } while (0)

  for (iter = 1; iter <= st->max_iter; ++iter) {
    memcpy(xp, x, sizeof(double) * n);
    memcpy(zp, z, sizeof(double) * m);
    /* update_xz_tilde (reduced KKT) */
    for (int i = 0; i < m; ++i) tm[i] = w->rho_vec[i] * zp[i] - y[i];
    csc_Aty(w, tm, xt);
    for (int j = 0; j < n; ++j) xt[j] += w->sigma * xp[j] - w->q[j];
    chol_solve(n, w->K, xt);
    csc_Ax(w, xt, zt);
    /* update_x, update_z, update_y */
    for (int j = 0; j < n; ++j) {
      x[j] = st->alpha * xt[j] + (1.0 - st->alpha) * xp[j];
      dx[j] = x[j] - xp[j];
    }
    for (int i = 0; i < m; ++i) {
      double v = st->alpha * zt[i] + (1.0 - st->alpha) * zp[i] + w->rho_inv[i] * y[i];
      z[i] = fmin(fmax(v, w->l[i]), w->u[i]);
    }
    for (int i = 0; i < m; ++i) {
      dy[i] = w->rho_vec[i] * (st->alpha * zt[i] + (1.0 - st->alpha) * zp[i] - z[i]);
      y[i] += dy[i];
    }
    can_check = st->check_termination && (iter % st->check_termination == 0);
    if (can_check) {
      UPDATE_INFO();
      double eps_p = st->eps_abs + st->eps_rel * fmax(vsnorm(w->Einv, z, m), vsnorm(w->Einv, Ax, m));
      double eps_d = st->eps_abs +
                     st->eps_rel * w->cinv *
                         fmax(fmax(vsnorm(w->Dinv, w->q, n), vsnorm(w->Dinv, Aty, n)), vsnorm(w->Dinv, Px, n));
      if (pri_res < eps_p && dua_res < eps_d) { status = QO_OK; break; }
      /* primal/dual infeasibility detection cannot trigger for the SRBD QP
       * (x = 0 is feasible and P is positive definite); not restated. */
    }
    if (st->adaptive_rho && interval && (iter % interval == 0)) {
      if (!can_check) UPDATE_INFO();
      /* compute_rho_estimate: scaled residual vectors rp, rd */
      double p = vnorm(rp, m) / (fmax(vnorm(z, m), vnorm(Ax, m)) + OSQP_DIVISION_TOL);
      double d = vnorm(rd, n) / (fmax(fmax(vnorm(w->q, n), vnorm(Aty, n)), vnorm(Px, n)) + OSQP_DIVISION_TOL);
      double rho_new = w->rho * sqrt(p / (d + OSQP_DIVISION_TOL));
      rho_new = fmin(fmax(rho_new, RHO_MIN), RHO_MAX);
      if (rho_new > w->rho * st->adaptive_rho_tolerance || rho_new < w->rho / st->adaptive_rho_tolerance) {
        update_rho(w, rho_new);
        rho_updates++;
      }
    }
  }
  if (iter > st->max_iter) {
    iter = st->max_iter;
    if (!can_check) UPDATE_INFO();
    double eps_p = 10 * st->eps_abs + 10 * st->eps_rel * fmax(vsnorm(w->Einv, z, m), vsnorm(w->Einv, Ax, m));
    double eps_d = 10 * st->eps_abs + 10 * st->eps_rel * w->cinv *
                                          fmax(fmax(vsnorm(w->Dinv, w->q, n), vsnorm(w->Dinv, Aty, n)), vsnorm(w->Dinv, Px, n));
    status = (pri_res < eps_p && dua_res < eps_d) ? QO_SOLVED_INACCURATE : QO_MAX_ITER;
  }
  /* objective (scaled space * cinv == unscaled) */
  double obj = 0.0;
  for (int j = 0; j < n; ++j) {
    double a = 0.0;
    for (int r = 0; r < n; ++r) a += w->P[(size_t)r * n + j] * x[r];
    obj += 0.5 * a * x[j] + w->q[j] * x[j];
  }
  obj *= w->cinv;
  if (out) {
    memcpy(out->x, x, sizeof(double) * n);
    memcpy(out->z, z, sizeof(double) * m);
    memcpy(out->y, y, sizeof(double) * m);
    out->rho = w->rho;
  }
  for (int j = 0; j < n; ++j) xo[j] = w->D[j] * x[j];
  if (yo)
    for (int i = 0; i < m; ++i) yo[i] = w->cinv * w->E[i] * y[i];
  if (info) {
    info->iters = iter;
    info->rho_updates = rho_updates;
    info->status = status;
    info->obj = obj;
    info->pri_res = pri_res;
    info->dua_res = dua_res;
    info->rho_final = w->rho;
  }
  free(w->P); free(w->q); free(w->A); free(w->l); free(w->u); free(w->D); free(w->Dinv);
  free(w->E); free(w->Einv); free(w->rho_vec); free(w->rho_inv); free(w->ctype); free(w->K);
  free(w->ap); free(w->ai); free(w->ax);
  free(x); free(xp); free(z); free(zp); free(y); free(dy); free(dx); free(xt); free(zt);
  free(Ax); free(Px); free(Aty); free(rp); free(rd); free(tm);
  return status;
}

int qo_exact_solve(int n, int m, const double *P, const double *q, const double *A,
                   const double *l, const double *u, double *x, int *iters) {
  /* rows with l == u -> equalities (CE), finite one-sided bounds -> CI */
  int ne = 0, ni = 0;
  for (int i = 0; i < m; ++i) {
    if (l[i] == u[i]) { ne++; continue; }
    if (l[i] > -1e20) ni++;
    if (u[i] < 1e20) ni++;
  }
  double *CE = (double *)calloc((size_t)n * (ne ? ne : 1), sizeof(double));
  double *ce0 = (double *)calloc(ne ? ne : 1, sizeof(double));
  double *CI = (double *)calloc((size_t)n * (ni ? ni : 1), sizeof(double));
  double *ci0 = (double *)calloc(ni ? ni : 1, sizeof(double));
  int e = 0, k = 0;
  for (int i = 0; i < m; ++i) {
    if (l[i] == u[i]) {
      int zero = 1;
      for (int j = 0; j < n; ++j) { CE[(size_t)e * n + j] = A[(size_t)j * m + i]; if (A[(size_t)j * m + i] != 0.0) zero = 0; }
      ce0[e] = -l[i];
      if (!zero) e++;
      continue;
    }
    if (l[i] > -1e20) {
      for (int j = 0; j < n; ++j) CI[(size_t)k * n + j] = A[(size_t)j * m + i];
      ci0[k++] = -l[i];
    }
    if (u[i] < 1e20) {
      for (int j = 0; j < n; ++j) CI[(size_t)k * n + j] = -A[(size_t)j * m + i];
      ci0[k++] = u[i];
    }
  }
  double *G = (double *)malloc(sizeof(double) * (size_t)n * n);
  memcpy(G, P, sizeof(double) * (size_t)n * n);
  qo_eqp_ws *ws = qo_eqp_create(n, e, k);
  int st = QO_OK;
  qo_eqp_solve(ws, G, q, CE, ce0, CI, ci0, x, &st, iters);
  qo_eqp_destroy(ws);
  free(G); free(CE); free(ce0); free(CI); free(ci0);
  return st;
}
