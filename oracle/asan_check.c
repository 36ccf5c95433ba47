/*
 * asan_check.c -- sanitizer driver for the oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Built by `make -C oracle asan` together with every oracle source under
 * -fsanitize=address,undefined (oracle/_build_asan/asan_check) and run by
 * tests/test_sanitizers.py.  It walks the restated reference paths that
 * emulate reference undefined behaviour or index arithmetic near array ends:
 * EiQuadProg with zero CE columns and the `qq` search (EiQuadProg.cpp:105-110,
 * :240-268), the force QP over every mode / support pattern across ticks
 * (F_prev coupling), the rt node tick over a long walk (Indexfind past the
 * 27-step schedule, _footxyz_real(., _bjxx-2), the body QP's inert CI
 * columns), the SRBD build + ADMM + exact + persistent solver, the A1 QP,
 * the servo force block, leg kinematics and the NLP contact phase.
 *
 *   asan_check DIR     DIR holds rt_msgs.bin (int32 T, B; then per tick
 *                      B*100 /MPC/Gait + B*25 /control2rtmpc/state doubles)
 *                      and force.bin (int32 B; then per robot 52 doubles +
 *                      2 int32: mode, right_support), written by the test.
 * Prints one summary line; exit 0 when every path ran.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qloco_oracle.h"

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static double urand(void) { /* splitmix64 -> [0, 1) */
  rs = qo_splitmix64(rs);
  return (double)(rs >> 11) * (1.0 / 9007199254740992.0);
}
static double U(double lo, double hi) { return lo + (hi - lo) * urand(); }

static void *load(const char *dir, const char *name, size_t *bytes) {
  char path[4096];
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  void *p = malloc((size_t)n);
  if (fread(p, 1, (size_t)n, f) != (size_t)n) { free(p); fclose(f); return NULL; }
  fclose(f);
  *bytes = (size_t)n;
  return p;
}

static int check_eiquadprog(void) {
  int runs = 0;
  for (int t = 0; t < 200; ++t) {
    const int n = 12, p = 12, m = 24;
    double G[144], g0[12], CE[144], ce0[12], CI[288], ci0[24], x[12];
    double Mr[144];
    for (int k = 0; k < 144; ++k) Mr[k] = U(-1, 1);
    for (int c = 0; c < n; ++c)
      for (int r = 0; r < n; ++r) {
        double a = (r == c) ? 4.0 : 0.0;
        for (int k = 0; k < n; ++k) a += Mr[k * n + r] * Mr[k * n + c];
        G[c * n + r] = a;
      }
    for (int k = 0; k < n; ++k) g0[k] = U(-5, 5);
    memset(CE, 0, sizeof(CE));
    /* swing-leg style equality blocks: some columns identity, some zero */
    const int pat = t % 4;
    for (int c = 0; c < p; ++c)
      if (((c / 3) + pat) % 2 == 0) CE[c * n + c] = 1.0;
    for (int k = 0; k < p; ++k) ce0[k] = 0.0;
    for (int k = 0; k < n * m; ++k) CI[k] = U(-1, 1);
    for (int k = 0; k < m; ++k) ci0[k] = U(0.5, 3.0);
    qo_eqp_ws *ws = qo_eqp_create(n, p, m);
    int st = 0, it = 0;
    qo_eqp_solve(ws, G, g0, CE, ce0, CI, ci0, x, &st, &it);
    qo_eqp_destroy(ws);
    runs++;
  }
  return runs;
}

static int check_force_qp(const char *dir) {
  size_t bytes = 0;
  unsigned char *buf = (unsigned char *)load(dir, "force.bin", &bytes);
  if (!buf) return -1;
  int32_t B;
  memcpy(&B, buf, 4);
  const size_t rec = 52 * 8 + 8;
  if (bytes != 4 + (size_t)B * rec) { free(buf); return -1; }
  qo_force_params prm;
  qo_force_params_default(&prm);
  qo_dyn_state s;
  qo_dyn_init(&s);
  int runs = 0;
  for (int tick = 0; tick < 3; ++tick)
    for (int b = 0; b < B; ++b) {
      double d[52];
      int32_t mr[2];
      memcpy(d, buf + 4 + (size_t)b * rec, 52 * 8);
      memcpy(mr, buf + 4 + (size_t)b * rec + 52 * 8, 8);
      /* com_des 0:3 leg_des 3:15 F 15:21 rfoot 21:24 lfoot 24:27 base 27:30
       * feet 30:42 FT 42:48 y 48 (49..51 pad) */
      qo_force_distribution(&s, d, d + 3, d + 15, mr[0], d[48], d + 21, d + 24);
      int est = 0, it = 0;
      qo_force_opt(&s, &prm, d + 27, d + 30, d + 33, d + 36, d + 39, d + 42, mr[0], mr[1], d[48],
                   &est, &it);
      double tau[3], J[9], pd[3] = {0.1, 0.0, -0.3}, pe[3] = {0.1, 0.01, -0.29}, v[3] = {0, 0, 0};
      for (int k = 0; k < 9; ++k) J[k] = U(-0.3, 0.3);
      for (int leg = 0; leg < 4; ++leg) qo_compute_joint_torques(&s, J, leg & 1, pd, pe, v, v, leg, tau);
      runs++;
    }
  qo_dyn_free(&s);
  free(buf);
  return runs;
}

static int check_rt(const char *dir) {
  size_t bytes = 0;
  unsigned char *buf = (unsigned char *)load(dir, "rt_msgs.bin", &bytes);
  if (!buf) return -1;
  int32_t T, B;
  memcpy(&T, buf, 4);
  memcpy(&B, buf + 4, 4);
  const size_t per = (size_t)B * 125 * 8;
  if (bytes != 8 + (size_t)T * per) { free(buf); return -1; }
  qo_rt *rt = qo_rt_create_n(B);
  double *traj = malloc(sizeof(double) * B * 100), *nrt = malloc(sizeof(double) * B * 25);
  double *gen = malloc(sizeof(double) * B * 60);
  int32_t *sched = malloc(sizeof(int32_t) * B * QO_RT_SCHED);
  double *gait = malloc(sizeof(double) * B * 100), *ctrl = malloc(sizeof(double) * B * 25);
  for (int t = 0; t < T; ++t) {
    memcpy(gait, buf + 8 + (size_t)t * per, (size_t)B * 100 * 8);
    memcpy(ctrl, buf + 8 + (size_t)t * per + (size_t)B * 100 * 8, (size_t)B * 25 * 8);
    qo_rt_tick_n(rt, B, gait, ctrl, traj, nrt, gen, sched);
  }
  qo_rt_destroy_n(rt, B);
  free(traj); free(nrt); free(gen); free(sched); free(gait); free(ctrl); free(buf);
  return T * B;
}

static int check_srbd(void) {
  int runs = 0;
  const int Ns[3] = {1, 4, 10};
  for (int gi = 0; gi < 3; ++gi) {
    const int N = Ns[gi];
    qo_srbd_spec sp;
    memset(&sp, 0, sizeof(sp));
    sp.N = N; sp.dt = 0.0025; sp.mass = 12.0;
    const double I[9] = {0.0336704372, 0.0009272282, 0.0004735904, 0.0009272282, 0.1312142164,
                         7.3342e-05, 0.0004735904, 7.3342e-05, 0.1485441318};
    memcpy(sp.inertia, I, sizeof(I));
    const double q[13] = {20, 10, 1, 0, 0, 420, 0.05, 0.05, 0.05, 30, 30, 10, 0};
    memcpy(sp.q_w, q, sizeof(q));
    for (int k = 0; k < 12; ++k) sp.r_w[k] = 1e-7;
    sp.mu = 0.3; sp.fz_min = 0.0; sp.fz_max = 180.0;
    qo_admm_settings st;
    qo_admm_settings_default(&st);
    for (int gait = 0; gait < 4; ++gait) {
      float x0[13], *xr = malloc(sizeof(float) * 13 * N), ft[12];
      uint8_t *ct = malloc(4 * N);
      qo_gen_srbd(20261015, N, 0.0025, gait, 7, 1, x0, xr, ft, ct);
      const int nu = 12 * N, nc = 20 * N;
      double x0d[13], *xrd = malloc(sizeof(double) * 13 * N), ftd[12];
      for (int k = 0; k < 13; ++k) x0d[k] = x0[k];
      for (int k = 0; k < 13 * N; ++k) xrd[k] = xr[k];
      for (int k = 0; k < 12; ++k) ftd[k] = ft[k];
      double *H = malloc(sizeof(double) * nu * nu), *g = malloc(sizeof(double) * nu);
      double *lb = malloc(sizeof(double) * nc), *ub = malloc(sizeof(double) * nc);
      double *C = malloc(sizeof(double) * nc * nu), *u = malloc(sizeof(double) * nu);
      double *y = malloc(sizeof(double) * nc);
      qo_srbd_build_instance(&sp, x0d, xrd, ftd, 0, ct, 1, H, g, lb, ub);
      qo_srbd_constraints(&sp, C);
      qo_admm_info info;
      qo_admm_solve(&st, nu, nc, H, g, C, lb, ub, u, y, &info);
      int it = 0;
      qo_exact_solve(nu, nc, H, g, C, lb, ub, u, &it);
      double *rec = calloc(QO_SRBD_PERSIST_LEN(N), sizeof(double));
      for (int tick = 0; tick < 4; ++tick) {
        if (tick == 2)
          for (int k = 0; k < 4 * N; ++k) ct[k] = (uint8_t)(1 - ct[k]);
        qo_srbd_persist_step(rec, &sp, &st, x0, xr, ft, 0, ct, 1, u, &info);
      }
      free(rec); free(xr); free(ct); free(xrd); free(H); free(g); free(lb); free(ub); free(C);
      free(u); free(y);
      runs++;
    }
  }
  return runs;
}

static int check_a1(void) {
  qo_a1_params p;
  qo_a1_params_default(&p);
  qo_admm_settings st;
  qo_admm_settings_default(&st);
  int runs = 0;
  for (int t = 0; t < 64; ++t) {
    double s[QO_A1_STATE_LEN];
    memset(s, 0, sizeof(s));
    const double yaw = U(-3.1, 3.1);
    s[5] = 0.3; s[2] = 0.28; s[8] = yaw; s[11] = yaw + (t % 3 == 0 ? 2 * 3.14159265 : 0.1);
    for (int k = 12; k < 24; ++k) s[k] = U(-0.3, 0.3);
    const double c = cos(yaw), sn = sin(yaw);
    const double R[9] = {c, sn, 0, -sn, c, 0, 0, 0, 1};
    memcpy(s + 24, R, sizeof(R));
    memcpy(s + 33, R, sizeof(R));
    const double fb[12] = {0.17, 0.15, -0.3, 0.17, -0.15, -0.3, -0.17, 0.15, -0.3, -0.17, -0.15, -0.3};
    memcpy(s + 42, fb, sizeof(fb));
    uint8_t ct[4] = {(uint8_t)(t & 1), (uint8_t)((t >> 1) & 1), (uint8_t)((t >> 2) & 1), 1};
    double f[12], x[12];
    qo_admm_info info;
    qo_a1_compute_grf(&p, &st, s, ct, f, x, &info);
    runs++;
  }
  return runs;
}

static int check_servo(void) {
  qo_force_params prm;
  qo_force_params_default(&prm);
  qo_servo_state s;
  qo_servo_init(&s);
  int runs = 0;
  for (int t = 0; t < 60; ++t) {
    double coma[3] = {U(-1, 1), U(-1, 1), U(-1, 1)}, com[3] = {0, 0, 0.3};
    double rf[3] = {0.0, -0.13, 0.0}, lf[3] = {0.0, 0.13, 0.0}, bp[3] = {0, 0, 0.3};
    double foot[12], J[36], rel[12], v[12];
    for (int k = 0; k < 12; ++k) { foot[k] = U(-0.2, 0.2); rel[k] = U(-0.3, 0.3); v[k] = U(-0.1, 0.1); }
    for (int k = 0; k < 36; ++k) J[k] = U(-0.3, 0.3);
    double F[6], FLR[6], rl, grf[12], tau[12];
    int sw[4], est;
    const int mode = 101 + (t % 4);
    qo_servo_force_block(&s, &prm, coma, com, rf, lf, bp, foot, t % 3, mode, 0.01, t, J, rel, v, F,
                         FLR, &rl, grf, tau, sw, &est);
    runs++;
  }
  qo_servo_free(&s);
  return runs;
}

static int check_kin_support(void) {
  int runs = 0;
  for (int t = 0; t < 400; ++t) {
    const double q[3] = {U(-0.5, 0.5), U(0.2, 1.4), U(-2.5, -0.9)};
    const double bp[3] = {U(-1, 1), U(-1, 1), U(0.2, 0.4)}, br[3] = {U(-0.2, 0.2), U(-0.2, 0.2), U(-3, 3)};
    double pos[3], J[9], qd[3], p2[3], J2[9];
    qo_leg_fk_g(bp, br, q, t & 3, pos, J);
    const double q0[3] = {0.0, 0.87, -1.5};
    qo_leg_ik(bp, br, pos, q0, t & 3, qd, p2, J2);
    qo_leg_fk(q, t & 3, pos, J);
    qo_leg_ik(NULL, NULL, pos, q0, t & 3, qd, p2, J2);
    runs++;
  }
  /* contact phase: schedules past their end, grid points, t_int beyond the horizon */
  enum { NS = 64 };
  double ts[NS * 27], tx[NS * 27];
  int32_t ti[NS], te[NS], bjxx[NS], bjx1[NS], rsup[NS];
  for (int b = 0; b < NS; ++b) {
    tx[b * 27] = 0.0;
    for (int i = 0; i < 27; ++i) ts[b * 27 + i] = U(0.45, 1.0);
    for (int i = 1; i < 27; ++i) tx[b * 27 + i] = tx[b * 27 + i - 1] + ts[b * 27 + i - 1];
    ti[b] = (int32_t)(U(0, 1.2) * tx[b * 27 + 26] / 0.025);
    te[b] = (int32_t)((tx[b * 27 + 26] - 1.4) / 0.025);
  }
  qo_support_phase(NS, ts, tx, ti, te, bjxx, bjx1, rsup);
  return runs + NS;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: asan_check DIR\n");
    return 2;
  }
  const int e = check_eiquadprog();
  const int f = check_force_qp(argv[1]);
  const int r = check_rt(argv[1]);
  const int s = check_srbd();
  const int a = check_a1();
  const int v = check_servo();
  const int k = check_kin_support();
  printf("asan_check: eiquadprog %d, force_qp %d, rt %d, srbd %d, a1 %d, servo %d, kin+support %d\n",
         e, f, r, s, a, v, k);
  return (f < 0 || r < 0) ? 3 : 0;
}
