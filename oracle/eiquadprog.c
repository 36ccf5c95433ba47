/*
 * eiquadprog.c -- restatement of the reference's Eigen::QP (Goldfarb-Idnani
 * dual active-set) in plain C, double precision, control flow kept 1:1
 * including the index quirks listed in SURVEY.md §8a-a20.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).  Parity unpinned.
 *
 * Follows rt_mpc_qp/src/utils/EiQuadProg/EiQuadProg.cpp (identical copies
 * in go1_rt_control, mosek_nlp_kmp and the HW tree):
 *   resize               :4-28      add_constraint   :30-93
 *   delete_constraint    :95-170    solve_quadprog2  :172-491
 *   solve_quadprog       :493-513   distance / compute_d / update_z /
 *   update_r             EiQuadProg.hpp:100-134
 */
#include "qloco_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

struct qo_eqp_ws {
  int n, p, m;
  double *R, *J, *L;                    /* n*n col-major */
  double *s, *z, *r, *d, *np, *u, *x_old, *u_old;
  int *A, *A_old, *iai, *iaexcl;
};

#define M2(a, r, c, ld) ((a)[(size_t)(c) * (ld) + (r)])

qo_eqp_ws *qo_eqp_create(int n, int p, int m) {
  qo_eqp_ws *w = (qo_eqp_ws *)calloc(1, sizeof(*w));
  int mp = m + p;
  w->n = n; w->p = p; w->m = m;
  w->R = (double *)calloc((size_t)n * n, sizeof(double));
  w->J = (double *)calloc((size_t)n * n, sizeof(double));
  w->L = (double *)calloc((size_t)n * n, sizeof(double));
  w->s = (double *)calloc(mp + 1, sizeof(double));
  w->z = (double *)calloc(n, sizeof(double));
  w->r = (double *)calloc(mp + 1, sizeof(double));
  w->d = (double *)calloc(n, sizeof(double));
  w->np = (double *)calloc(n, sizeof(double));
  w->u = (double *)calloc(mp + 1, sizeof(double));
  w->x_old = (double *)calloc(n, sizeof(double));
  w->u_old = (double *)calloc(mp + 1, sizeof(double));
  /* Eigen leaves these uninitialised (EiQuadProg.cpp:22-25); we zero them. */
  w->A = (int *)calloc(mp + 1, sizeof(int));
  w->A_old = (int *)calloc(mp + 1, sizeof(int));
  w->iai = (int *)calloc(mp + 1, sizeof(int));
  w->iaexcl = (int *)calloc(mp + 1, sizeof(int));
  return w;
}

void qo_eqp_destroy(qo_eqp_ws *w) {
  if (!w) return;
  free(w->R); free(w->J); free(w->L); free(w->s); free(w->z); free(w->r);
  free(w->d); free(w->np); free(w->u); free(w->x_old); free(w->u_old);
  free(w->A); free(w->A_old); free(w->iai); free(w->iaexcl);
  free(w);
}

/* EiQuadProg.hpp:100-118 */
static double eqp_distance(double a, double b) {
  double a1 = fabs(a), b1 = fabs(b), t;
  if (a1 > b1) { t = b1 / a1; return a1 * sqrt(1.0 + t * t); }
  if (b1 > a1) { t = a1 / b1; return b1 * sqrt(1.0 + t * t); }
  return a1 * sqrt(2.0);
}

/* d = J' np  (EiQuadProg.hpp:121-124) */
static void compute_d(int n, double *d, const double *J, const double *np) {
  for (int c = 0; c < n; ++c) {
    double acc = 0.0;
    for (int r = 0; r < n; ++r) acc += M2(J, r, c, n) * np[r];
    d[c] = acc;
  }
}
/* z = J(:, iq:) d(iq:)  (EiQuadProg.hpp:126-129) */
static void update_z(int n, double *z, const double *J, const double *d, int iq) {
  for (int r = 0; r < n; ++r) {
    double acc = 0.0;
    for (int c = iq; c < n; ++c) acc += M2(J, r, c, n) * d[c];
    z[r] = acc;
  }
}
/* r(0:iq) = triu(R(0:iq,0:iq)) \ d(0:iq)  (EiQuadProg.hpp:131-134) */
static void update_r(int n, const double *R, double *r, const double *d, int iq) {
  for (int i = iq - 1; i >= 0; --i) {
    double acc = d[i];
    for (int j = i + 1; j < iq; ++j) acc -= M2(R, i, j, n) * r[j];
    r[i] = acc / M2(R, i, i, n);
  }
}

/* EiQuadProg.cpp:30-93 */
static int add_constraint(qo_eqp_ws *w, int *iq, double *R_norm) {
  int n = w->n, j, k;
  double cc, ss, h, t1, t2, xny;
  double *d = w->d, *J = w->J, *R = w->R;
  for (j = n - 1; j >= *iq + 1; j--) {
    cc = d[j - 1];
    ss = d[j];
    h = eqp_distance(cc, ss);
    if (h == 0.0) continue;
    d[j] = 0.0;
    ss = ss / h;
    cc = cc / h;
    if (cc < 0.0) {
      cc = -cc;
      ss = -ss;
      d[j - 1] = -h;
    } else {
      d[j - 1] = h;
    }
    xny = ss / (1.0 + cc);
    for (k = 0; k < n; k++) {
      t1 = M2(J, k, j - 1, n);
      t2 = M2(J, k, j, n);
      M2(J, k, j - 1, n) = t1 * cc + t2 * ss;
      M2(J, k, j, n) = xny * (t1 + M2(J, k, j - 1, n)) - t2;
    }
  }
  (*iq)++;
  for (k = 0; k < *iq; ++k) M2(R, k, *iq - 1, n) = d[k];
  if (fabs(d[*iq - 1]) <= DBL_EPSILON * (*R_norm)) return 0; /* degenerate */
  if (fabs(d[*iq - 1]) > *R_norm) *R_norm = fabs(d[*iq - 1]);
  return 1;
}

/* EiQuadProg.cpp:95-170.  Returns 0 when the reference would read the
 * uninitialised `qq` (constraint l not found in positions [p, iq)). */
static int delete_constraint(qo_eqp_ws *w, int p, int *iq, int l) {
  int n = w->n, i, j, k, qq = -1;
  double cc, ss, h, xny, t1, t2;
  double *R = w->R, *J = w->J, *u = w->u;
  int *A = w->A;
  for (i = p; i < *iq; i++)
    if (A[i] == l) { qq = i; break; }
  if (qq < 0) return 0; /* reference: UB (uninitialised qq) */
  for (i = qq; i < *iq - 1; i++) {
    A[i] = A[i + 1];
    u[i] = u[i + 1];
    for (k = 0; k < n; ++k) M2(R, k, i, n) = M2(R, k, i + 1, n);
  }
  A[*iq - 1] = A[*iq];
  u[*iq - 1] = u[*iq];
  A[*iq] = 0;
  u[*iq] = 0.0;
  for (j = 0; j < *iq; j++) M2(R, j, *iq - 1, n) = 0.0;
  (*iq)--;
  if (*iq == 0) return 1;
  for (j = qq; j < *iq; j++) {
    cc = M2(R, j, j, n);
    ss = M2(R, j + 1, j, n);
    h = eqp_distance(cc, ss);
    if (h == 0.0) continue;
    cc = cc / h;
    ss = ss / h;
    M2(R, j + 1, j, n) = 0.0;
    if (cc < 0.0) {
      M2(R, j, j, n) = -h;
      cc = -cc;
      ss = -ss;
    } else {
      M2(R, j, j, n) = h;
    }
    xny = ss / (1.0 + cc);
    for (k = j + 1; k < *iq; k++) {
      t1 = M2(R, j, k, n);
      t2 = M2(R, j + 1, k, n);
      M2(R, j, k, n) = t1 * cc + t2 * ss;
      M2(R, j + 1, k, n) = xny * (t1 + M2(R, j, k, n)) - t2;
    }
    for (k = 0; k < n; k++) {
      t1 = M2(J, k, j, n);
      t2 = M2(J, k, j + 1, n);
      M2(J, k, j, n) = t1 * cc + t2 * ss;
      M2(J, k, j + 1, n) = xny * (M2(J, k, j, n) + t1) - t2;
    }
  }
  return 1;
}

/* Eigen LLT<MatrixXd,Lower>::compute restated as an unblocked left-looking
 * Cholesky on the lower triangle (Eigen reads only the lower part).
 * Returns 0 if not positive definite. */
static int llt_lower(int n, const double *G, double *L) {
  memset(L, 0, sizeof(double) * (size_t)n * n);
  for (int c = 0; c < n; ++c)
    for (int r = c; r < n; ++r) M2(L, r, c, n) = M2(G, r, c, n);
  for (int k = 0; k < n; ++k) {
    double x = M2(L, k, k, n);
    for (int j = 0; j < k; ++j) x -= M2(L, k, j, n) * M2(L, k, j, n);
    if (!(x > 0.0)) return 0;
    double lkk = sqrt(x);
    M2(L, k, k, n) = lkk;
    for (int r = k + 1; r < n; ++r) {
      double acc = M2(L, r, k, n);
      for (int j = 0; j < k; ++j) acc -= M2(L, r, j, n) * M2(L, k, j, n);
      M2(L, r, k, n) = acc / lkk;
    }
  }
  return 1;
}

static int col_is_zero(const double *C, int n, int i) {
  for (int r = 0; r < n; ++r)
    if (M2(C, r, i, n) != 0.0) return 0;
  return 1;
}

static double dotcol(const double *C, int n, int i, const double *x) {
  double acc = 0.0;
  for (int r = 0; r < n; ++r) acc += M2(C, r, i, n) * x[r];
  return acc;
}

double qo_eqp_solve(qo_eqp_ws *w, double *G, const double *g0, const double *CE,
                    const double *ce0, const double *CI, const double *ci0,
                    double *x, int *status, int *iters) {
  const double inf = INFINITY;
  int n = w->n, p = w->p, m = w->m;
  int i, k, l, ip, me, mi, iq, iter = 0;
  double f_value, psi, c1, c2, sum, ss, R_norm, t, t1, t2;
  double *R = w->R, *J = w->J, *L = w->L, *s = w->s, *z = w->z, *r = w->r,
         *d = w->d, *np = w->np, *u = w->u;
  int *A = w->A, *iai = w->iai, *iaexcl = w->iaexcl;
  if (status) *status = QO_OK;

  /* solve_quadprog: EiQuadProg.cpp:493-513 */
  c1 = 0.0;
  for (i = 0; i < n; ++i) c1 += M2(G, i, i, n);
  if (!llt_lower(n, G, L)) {
    if (status) *status = QO_NOT_PD;
    if (iters) *iters = 0;
    return inf;
  }
  memcpy(G, L, sizeof(double) * (size_t)n * n); /* G is overwritten (hpp:45-48) */

  /* solve_quadprog2: EiQuadProg.cpp:172-491 */
  me = p;
  mi = m;
  memset(d, 0, sizeof(double) * n);
  memset(R, 0, sizeof(double) * (size_t)n * n);
  R_norm = 1.0;
  /* J = U^-1 = L^-T (upper triangular), :213-214 */
  memset(J, 0, sizeof(double) * (size_t)n * n);
  for (int c = 0; c < n; ++c) {
    /* solve L' J(:,c) = e_c by back substitution */
    for (int rr = n - 1; rr >= 0; --rr) {
      double acc = (rr == c) ? 1.0 : 0.0;
      for (int j = rr + 1; j < n; ++j) acc -= M2(L, j, rr, n) * M2(J, j, c, n);
      M2(J, rr, c, n) = acc / M2(L, rr, rr, n);
    }
  }
  c2 = 0.0;
  for (i = 0; i < n; ++i) c2 += M2(J, i, i, n);

  /* x = -G^-1 g0 via the factor, :227-230 */
  for (i = 0; i < n; ++i) {
    double acc = g0[i];
    for (int j = 0; j < i; ++j) acc -= M2(L, i, j, n) * x[j];
    x[i] = acc / M2(L, i, i, n);
  }
  for (i = n - 1; i >= 0; --i) {
    double acc = x[i];
    for (int j = i + 1; j < n; ++j) acc -= M2(L, j, i, n) * x[j];
    x[i] = acc / M2(L, i, i, n);
  }
  for (i = 0; i < n; ++i) x[i] = -x[i];
  f_value = 0.0;
  for (i = 0; i < n; ++i) f_value += g0[i] * x[i];
  f_value *= 0.5;

  /* equality constraints, :237-276 (quirk: me = p counts skipped columns,
   * and the marker is stored at A(i), not A(iq)) */
  iq = 0;
  for (i = 0; i < me; i++) {
    if (col_is_zero(CE, n, i)) continue;
    for (k = 0; k < n; ++k) np[k] = M2(CE, k, i, n);
    compute_d(n, d, J, np);
    update_z(n, z, J, d, iq);
    update_r(n, R, r, d, iq);
    t2 = 0.0;
    double zz = 0.0, znp = 0.0, npx = 0.0;
    for (k = 0; k < n; ++k) { zz += z[k] * z[k]; znp += z[k] * np[k]; npx += np[k] * x[k]; }
    if (fabs(zz) > DBL_EPSILON) t2 = (-npx - ce0[i]) / znp;
    for (k = 0; k < n; ++k) x[k] += t2 * z[k];
    u[iq] = t2;
    for (k = 0; k < iq; ++k) u[k] -= t2 * r[k];
    f_value += 0.5 * (t2 * t2) * znp;
    A[i] = -i - 1;
    if (!add_constraint(w, &iq, &R_norm)) {
      if (status) *status = QO_DEGENERATE;
      if (iters) *iters = iter;
      return f_value;
    }
  }

  for (i = 0; i < mi; i++) iai[i] = i;

l1:
  iter++;
  for (i = me; i < iq; i++) { /* quirk: starts at me, :288-292 */
    ip = A[i];
    iai[ip] = -1;
  }
  ss = 0.0;
  psi = 0.0;
  ip = 0;
  for (i = 0; i < mi; i++) {
    iaexcl[i] = 1;
    sum = dotcol(CI, n, i, x) + ci0[i];
    s[i] = sum;
    psi += (sum < 0.0) ? sum : 0.0;
  }
  if (fabs(psi) <= mi * DBL_EPSILON * c1 * c2 * 100.0) {
    if (iters) *iters = iter;
    return f_value;
  }
  for (i = 0; i < iq; ++i) { w->u_old[i] = u[i]; w->A_old[i] = A[i]; }
  memcpy(w->x_old, x, sizeof(double) * n);

l2:
  for (i = 0; i < mi; i++) {
    if (s[i] < ss && iai[i] != -1 && iaexcl[i]) {
      ss = s[i];
      ip = i;
    }
  }
  if (ss >= 0.0) {
    if (iters) *iters = iter;
    return f_value;
  }
  for (k = 0; k < n; ++k) np[k] = M2(CI, k, ip, n);
  u[iq] = 0.0;
  A[iq] = ip;

l2a:
  compute_d(n, d, J, np);
  update_z(n, z, J, d, iq);
  update_r(n, R, r, d, iq);
  l = 0;
  t1 = inf;
  for (k = me; k < iq; k++) { /* quirk: starts at me, :370-378 */
    double tmp;
    if (r[k] > 0.0 && ((tmp = u[k] / r[k]) < t1)) {
      t1 = tmp;
      l = A[k];
    }
  }
  {
    double zz = 0.0, znp = 0.0;
    for (k = 0; k < n; ++k) { zz += z[k] * z[k]; znp += z[k] * np[k]; }
    if (fabs(zz) > DBL_EPSILON)
      t2 = -s[ip] / znp;
    else
      t2 = inf;
    t = (t1 < t2) ? t1 : t2;
    if (t >= inf) {
      if (status) *status = QO_INFEASIBLE;
      if (iters) *iters = iter;
      return inf;
    }
    if (t2 >= inf) {
      for (k = 0; k < iq; ++k) u[k] -= t * r[k];
      u[iq] += t;
      iai[l] = l;
      if (!delete_constraint(w, p, &iq, l)) {
        if (status) *status = QO_UB_PATH;
        if (iters) *iters = iter;
        return f_value;
      }
      goto l2a;
    }
    for (k = 0; k < n; ++k) x[k] += t * z[k];
    f_value += t * znp * (0.5 * t + u[iq]);
    for (k = 0; k < iq; ++k) u[k] -= t * r[k];
    u[iq] += t;
  }
  if (t == t2) {
    if (!add_constraint(w, &iq, &R_norm)) {
      iaexcl[ip] = 0;
      if (!delete_constraint(w, p, &iq, ip)) {
        if (status) *status = QO_UB_PATH;
        if (iters) *iters = iter;
        return f_value;
      }
      for (i = 0; i < m; i++) iai[i] = i;
      for (i = 0; i < iq; i++) {
        A[i] = w->A_old[i];
        if (A[i] < 0 || A[i] >= m) { /* reference: out-of-range write, UB */
          if (status) *status = QO_UB_PATH;
          if (iters) *iters = iter;
          return f_value;
        }
        iai[A[i]] = -1;
        u[i] = w->u_old[i];
      }
      memcpy(x, w->x_old, sizeof(double) * n);
      goto l2;
    } else {
      iai[ip] = -1;
    }
    goto l1;
  }
  /* partial step: drop constraint l, :477-490 */
  iai[l] = l;
  if (!delete_constraint(w, p, &iq, l)) {
    if (status) *status = QO_UB_PATH;
    if (iters) *iters = iter;
    return f_value;
  }
  s[ip] = dotcol(CI, n, ip, x) + ci0[ip];
  goto l2a;
}
