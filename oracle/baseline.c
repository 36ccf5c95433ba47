/*
 * baseline.c -- batch driver over the oracle: builds each SRBD instance
 * (srbd.c) and solves it with the ADMM restatement (CPU-A) or the exact
 * EiQuadProg restatement (CPU-B), one pthread per requested core, each
 * thread on a contiguous slice of instances.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h): it is the checker in the
 * parity tests and the timed `cpu_baseline` leg of bench.py.
 */
#include "qloco_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
  const qo_srbd_spec *sp;
  const qo_admm_settings *st;
  int solver;
  int64_t lo, hi;
  const float *x0, *x_ref, *feet;
  int feet_per_step;
  const uint8_t *contacts;
  int contacts_per_step;
  double *u, *obj;
  int *iters, *status;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  const int N = j->sp->N, n = 12 * N, m = 20 * N;
  double *H = malloc(sizeof(double) * n * n), *g = malloc(sizeof(double) * n);
  double *lb = malloc(sizeof(double) * m), *ub = malloc(sizeof(double) * m);
  double *C = malloc(sizeof(double) * (size_t)m * n), *x = malloc(sizeof(double) * n);
  double *y = malloc(sizeof(double) * m);
  double *x0 = malloc(sizeof(double) * 13), *xr = malloc(sizeof(double) * 13 * N);
  double *ft = malloc(sizeof(double) * 12 * N);
  qo_srbd_constraints(j->sp, C);
  for (int64_t t = j->lo; t < j->hi; ++t) {
    for (int k = 0; k < 13; ++k) x0[k] = j->x0[13 * t + k];
    for (int k = 0; k < 13 * N; ++k) xr[k] = j->x_ref[(int64_t)13 * N * t + k];
    int nf = j->feet_per_step ? 12 * N : 12;
    for (int k = 0; k < nf; ++k) ft[k] = j->feet[(int64_t)nf * t + k];
    const uint8_t *ct = j->contacts + (int64_t)(j->contacts_per_step ? 4 * N : 4) * t;
    qo_srbd_build_instance(j->sp, x0, xr, ft, j->feet_per_step, ct, j->contacts_per_step, H, g, lb, ub);
    int it = 0, stt;
    double obj = 0;
    if (j->solver == 0) {
      qo_admm_info info;
      memset(x, 0, sizeof(double) * n);
      memset(y, 0, sizeof(double) * m);
      stt = qo_admm_solve(j->st, n, m, H, g, C, lb, ub, x, y, &info);
      it = info.iters;
      obj = info.obj;
    } else {
      stt = qo_exact_solve(n, m, H, g, C, lb, ub, x, &it);
      for (int a = 0; a < n; ++a) {
        double s = 0;
        for (int b = 0; b < n; ++b) s += H[(size_t)b * n + a] * x[b];
        obj += 0.5 * s * x[a] + g[a] * x[a];
      }
    }
    if (j->u) memcpy(j->u + (int64_t)n * t, x, sizeof(double) * n);
    if (j->iters) j->iters[t] = it;
    if (j->status) j->status[t] = stt;
    if (j->obj) j->obj[t] = obj;
  }
  free(H); free(g); free(lb); free(ub); free(C); free(x); free(y); free(x0); free(xr); free(ft);
  return NULL;
}

int qo_srbd_batch(const qo_srbd_spec *sp, const qo_admm_settings *st, int solver, int64_t count,
                  const float *x0, const float *x_ref, const float *feet, int feet_per_step,
                  const uint8_t *contacts, int contacts_per_step, double *u, int *iters,
                  int *status, double *obj, int nthreads, double *seconds) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > count) nthreads = (int)(count > 0 ? count : 1);
  pthread_t *th = malloc(sizeof(pthread_t) * nthreads);
  job_t *jobs = malloc(sizeof(job_t) * nthreads);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int i = 0; i < nthreads; ++i) {
    job_t *j = &jobs[i];
    j->sp = sp; j->st = st; j->solver = solver;
    j->lo = count * i / nthreads; j->hi = count * (i + 1) / nthreads;
    j->x0 = x0; j->x_ref = x_ref; j->feet = feet; j->feet_per_step = feet_per_step;
    j->contacts = contacts; j->contacts_per_step = contacts_per_step;
    j->u = u; j->obj = obj; j->iters = iters; j->status = status;
    pthread_create(&th[i], NULL, worker, j);
  }
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (seconds) *seconds = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  free(th);
  free(jobs);
  return 0;
}
