/*
 * rt_tick.c -- restatement of one iteration of the rt_mpc_qp node loop
 * (unitree_ros/rt_mpc_qp/src/gait_fast.cpp:505-735) together with the
 * PRMPCClass reference generators it calls, double precision.
 *
 * TEST INFRASTRUCTURE ONLY (see qloco_oracle.h).  Parity unpinned: the
 * reference cannot be compiled here (Eigen, Armadillo, ROS absent) and holds
 * no fixtures for these functions; tests/rt_ref.py is an independent second
 * transcription the tests hold this file to.
 *
 * Covered:
 *   gait_fast.cpp   callbacks :79-110, xget_position_interpolation :113-372,
 *                   main() state init :384-502, loop body :505-735
 *                   (/rtMPC/traj and /rt2nrt/state packing :633-729, :519-527)
 *   PRMPCClass.cpp  Initialize (reference-generation part) :46-190,
 *                   XGetSolution_position_mod3 :1170-1261,
 *                   solve_AAA_inv_mod1 :1344-1362, Foot_trajectory_solve_mod2
 *                   :1756-2195, FootStepInputs :2198-2222, solve_AAA_inv2
 *                   :2225-2237, XGetSolution_Foot_rotation :2255-2380,
 *                   Indexfind :716-738; body_theta_mpc via body_mpc.c.
 *
 * Quirks reproduced: rfoot_mpc_ref row 1 is never written and row 0 ends up
 * holding the y coordinate (gait_fast.cpp:585-586, 606-607); t_int grows by
 * floor(count/2) every tick (:517, int32 wrap-around); mpc_gait_flag is the
 * truncated /MPC/Gait[99] (:85); the traj timing slot [86] (ros::Time
 * duration, :707-714) is written as 0; stale _bjx1 / foot-array entries are
 * carried between calls exactly as the members are.
 * Reference UB made defined: Nrtfoorpr_gen indices outside the 27-step
 * arrays (:1758-1772 write unchecked) are ignored; Indexfind stops at 27.
 * Dead state not kept: the FootL/FootR/rpy interpolation vectors of
 * gait_fast.cpp (their *_inter outputs are commented out, :133-136).
 */
#include "qloco_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define NS QO_FOOTSTEPS
#define NH QO_NH

enum { RX = 0, RY, RZ, RVX, RVY, RVZ, RAX, RAY, RAZ, LX, LY, LZ, LVX, LVY, LVZ, LAX, LAY, LAZ };

struct qo_rt {
  qo_body_state body; /* PRMPCClass QP part; body.tx / body.bjx1 are shared members */
  /* PRMPCClass reference-generation members (PRMPCClass.h:86-125) */
  double ts[NS], td[NS], lift[NS], stepwidth0, tdsp_ratio, footx_max;
  double fxyz[3][NS]; /* _footxyz_real */
  int t_end_footstep, bjxx;
  double tx_total, ry_left_right;
  double foot[18][10];
  double Rfoot_r[15], Lfoot_r[15]; /* 3x5 col-major */
  double AAA_inv_mod[16];          /* col-major */
  /* gait_fast.cpp globals */
  int count_in_rt_loop, count_in_rt_mpc, count_inteplotation, t_int, mpc_gait_flag_old;
  double COM_in1[3], COM_in2[3], COMxyz_ref[3], COMv_ref[3], COM_ref2[3];
  double COMacc_in1[3], COMacc_in2[3], COMacc_ref[3], COMacc_ref2[3];
  double zmp_in1[3], zmp_in2[3], zmpxyz_ref[3], zmp_ref2[3];
  double dcm_in1[3], dcm_in2[3], dcmxyz_ref[3], dcm_ref2[3];
  double rpy_mpc_body[21], comacc_inter[21], zmp_inter[21], dcm_inter[21];
  double foorpr_gen[30], foortheta_gen[30], body_thetax[3], bodyangle_mpc[14];
  double state_feedback[25], state_to_MPC[25];
};

static const double DT_SLOW = 0.025, DT_FAST = 0.01, TSTEP = 0.7; /* gait:: :8-9,26 */
static const double HALF_HIP = 0.12675;                            /* :19 */

/* std::pow(t, 3) / pow(t, 2) of the reference (PRMPCClass.cpp:1199-1211,
 * :1901-1906, :2227-2230) as a compensated cube (error-free products via
 * fma, one final rounding) and an exact-rounded square: glibc's pow is only
 * <1 ulp, which the ill-conditioned cubic fits (solve_AAA_inv2 near the
 * swing's knot crossings) amplify, so every restatement (this file, the
 * GPU kernel, tests/rt_ref.py) uses these same primitives. */
static double sq(double x) { return x * x; }
static double cube(double x) {
  const double p = x * x, e = fma(x, x, -p);
  const double hi = p * x, lo = fma(p, x, -hi);
  return hi + (lo + e * x);
}

/* Dense 4x4 inverse, Gauss-Jordan with partial pivoting (Eigen's
 * Matrix4d::inverse() restated; agreement to rounding, not bit-exact).
 * A, Ainv row-major. */
void qo_inv4(const double A[16], double Ainv[16]) {
  double M[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      M[r][c] = A[r * 4 + c];
      M[r][4 + c] = (r == c) ? 1.0 : 0.0;
    }
  for (int k = 0; k < 4; ++k) {
    int p = k;
    for (int r = k + 1; r < 4; ++r)
      if (fabs(M[r][k]) > fabs(M[p][k])) p = r;
    if (p != k)
      for (int c = 0; c < 8; ++c) {
        double t = M[k][c];
        M[k][c] = M[p][c];
        M[p][c] = t;
      }
    double piv = M[k][k];
    for (int c = 0; c < 8; ++c) M[k][c] = M[k][c] / piv;
    for (int r = 0; r < 4; ++r) {
      if (r == k) continue;
      double f = M[r][k];
      for (int c = 0; c < 8; ++c) M[r][c] = M[r][c] - f * M[k][c];
    }
  }
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) Ainv[r * 4 + c] = M[r][4 + c];
}

/* solve_AAA_inv_mod1, :1344-1362 (t = -dt, 0, dt, 2dt with _dt = dt_mpc_slow) */
static void aaa_inv_mod(double out_colmajor[16]) {
  const double t[4] = {-DT_SLOW, 0, DT_SLOW, 2 * DT_SLOW};
  double A[16], Ai[16];
  for (int r = 0; r < 4; ++r) {
    A[r * 4 + 0] = cube(t[r]);
    A[r * 4 + 1] = sq(t[r]);
    A[r * 4 + 2] = (t[r]);
    A[r * 4 + 3] = 1;
  }
  qo_inv4(A, Ai);
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) out_colmajor[c * 4 + r] = Ai[r * 4 + c];
}

/* solve_AAA_inv2, :2225-2237; returns row-major */
static void aaa_inv2(const double tp[3], double Ai[16]) {
  double A[16] = {cube(tp[0]), sq(tp[0]), (tp[0]), 1,
                  cube(tp[1]), sq(tp[1]), (tp[1]), 1,
                  cube(tp[2]), sq(tp[2]), (tp[2]), 1,
                  3 * sq(tp[2]), 2 * (tp[2]), 1.0, 0};
  qo_inv4(A, Ai);
}

/* Indexfind xyz = 0 (:716-738) on the robot's current _tx */
static int indexfind(const qo_rt *s, double goal) { return qo_body_indexfind(&s->body, goal); }

static void recompute_tx(qo_rt *s) { /* :1773-1779 (also Initialize :172-178) */
  for (int i = 0; i < NS; ++i) s->td[i] = s->tdsp_ratio * s->ts[i];
  s->body.tx[0] = 0.0;
  for (int i = 1; i < NS; i++) {
    s->body.tx[i] = s->body.tx[i - 1] + s->ts[i - 1];
    s->body.tx[i] = round(s->body.tx[i] / DT_SLOW) * DT_SLOW - 0.00001;
  }
}

qo_rt *qo_rt_create_n(int64_t n) {
  qo_rt *arr = (qo_rt *)calloc((size_t)n, sizeof(qo_rt));
  for (int64_t b = 0; b < n; ++b) {
    qo_rt *s = &arr[b];
    qo_body_init(&s->body);
    /* FootStepInputs(2*HALF_HIP, 0, 0, 0.015), :48-53 and :2198-2222 */
    const double stepwidth = 2 * HALF_HIP, lift_height = 0.015;
    double steplength[NS], sw[NS], sh[NS];
    for (int i = 0; i < NS; ++i) {
      steplength[i] = 0.0; /* steplengthx = 0 (all entries, incl. the /2 one) */
      sw[i] = stepwidth;
      sh[i] = 0.0;
      s->lift[i] = lift_height;
    }
    sw[0] = sw[0] / 2;
    s->lift[NS - 1] = 0;
    s->lift[NS - 2] = 0;
    s->lift[NS - 3] = lift_height / 2;
    s->lift[NS - 4] = lift_height;
    s->stepwidth0 = sw[0];
    /* _footx/y/z_ref and _footxyz_real, :111-123 */
    double fx = 0, fy = 0, fz = 0;
    s->fxyz[0][0] = s->fxyz[1][0] = s->fxyz[2][0] = 0;
    for (int i = 1; i < NS; i++) {
      fx = fx + steplength[i - 1];
      fy = fy + (int)pow(-1, i - 1) * sw[i - 1];
      fz = fz + sh[i - 1];
      s->fxyz[0][i] = fx;
      s->fxyz[1][i] = fy;
      s->fxyz[2][i] = fz;
    }
    s->bjxx = 0;
    /* foot arrays, :131-138 */
    for (int k = 0; k < 10; ++k) {
      s->foot[LY][k] = sw[0];
      s->foot[RY][k] = -sw[0];
    }
    s->ry_left_right = 0;
    s->footx_max = 0.15;
    /* schedule, :168-185 */
    s->tdsp_ratio = 0.1;
    for (int i = 0; i < NS; ++i) s->ts[i] = TSTEP;
    recompute_tx(s);
    s->t_end_footstep = (int)round((s->body.tx[NS - 1] - 3 * TSTEP) / DT_FAST);
    s->tx_total = s->body.tx[NS - 1];
    aaa_inv_mod(s->AAA_inv_mod);
    /* gait_fast.cpp main(), :384-502 */
    s->COM_in1[2] = s->COM_in2[2] = s->COMxyz_ref[2] = s->COM_ref2[2] = 0.309458;
    s->rpy_mpc_body[2] = s->COM_ref2[2];
    for (int j = 0; j < 5; j++) {
      s->foorpr_gen[1 + 6 * j] = -HALF_HIP;
      s->foorpr_gen[4 + 6 * j] = HALF_HIP;
    }
  }
  return arr;
}

void qo_rt_destroy_n(qo_rt *arr, int64_t n) {
  if (!arr) return;
  for (int64_t b = 0; b < n; ++b) qo_body_free(&arr[b].body);
  free(arr);
}

/* XGetSolution_position_mod3, :1170-1261 */
static void position_mod3(const qo_rt *s, int walktime, double dt_sample, const double in1[3],
                          const double in2[3], const double ref[3], const double ref2[3],
                          double out[21]) {
  memset(out, 0, sizeof(double) * 21);
  if (walktime > s->t_end_footstep) return;
  for (int jx = 0; jx < NH; jx++) {
    double t_cur = (walktime * dt_sample + jx * dt_sample);
    double tp[4] = {cube(t_cur), sq(t_cur), (t_cur), 1.0};
    double tv[4] = {3 * sq(t_cur), 2 * (t_cur), 1, 0};
    double ta[4] = {6 * (t_cur), 2, 0, 0};
    /* row vectors times _AAA_inv_mod (left to right), then times temp */
    double rp[4], rv[4], ra[4];
    for (int c = 0; c < 4; ++c) {
      double ap = 0, av = 0, aa = 0;
      for (int k = 0; k < 4; ++k) {
        ap += tp[k] * s->AAA_inv_mod[c * 4 + k];
        av += tv[k] * s->AAA_inv_mod[c * 4 + k];
        aa += ta[k] * s->AAA_inv_mod[c * 4 + k];
      }
      rp[c] = ap;
      rv[c] = av;
      ra[c] = aa;
    }
    for (int ax = 0; ax < 3; ++ax) {
      double temp[4] = {in1[ax], in2[ax], ref[ax], ref2[ax]};
      double p = 0, v = 0, a = 0;
      for (int k = 0; k < 4; ++k) {
        p += rp[k] * temp[k];
        v += rv[k] * temp[k];
        a += ra[k] * temp[k];
      }
      if (jx == 0) {
        out[ax] = p;
        out[3 + ax] = v;
        out[6 + ax] = a;
      } else {
        out[8 + 3 * jx - 2 + ax] = p;
      }
    }
  }
}

static void set3(double d[3], double a, double b, double c) { d[0] = a; d[1] = b; d[2] = c; }

/* xget_position_interpolation, gait_fast.cpp:113-372 (live vectors only) */
static void interpolation(qo_rt *s, const double *g, int mpc_gait_flag) {
  const int n_t_int = (int)floor(DT_SLOW / DT_FAST); /* :475 */
  s->count_inteplotation += 1;
  if (s->t_int > 2) { /* :118-139 */
    position_mod3(s, s->count_inteplotation, DT_FAST, s->COM_in1, s->COM_in2, s->COMxyz_ref,
                  s->COM_ref2, s->rpy_mpc_body);
    position_mod3(s, s->count_inteplotation, DT_FAST, s->COMacc_in1, s->COMacc_in2,
                  s->COMacc_ref, s->COMacc_ref2, s->comacc_inter);
    position_mod3(s, s->count_inteplotation, DT_FAST, s->zmp_in1, s->zmp_in2, s->zmpxyz_ref,
                  s->zmp_ref2, s->zmp_inter);
    position_mod3(s, s->count_inteplotation, DT_FAST, s->dcm_in1, s->dcm_in2, s->dcmxyz_ref,
                  s->dcm_ref2, s->dcm_inter);
  }
  if (s->count_inteplotation % n_t_int == 0) { /* :143-371 */
    memcpy(s->COM_in1, s->COM_in2, 24);
    memcpy(s->COM_in2, s->COMxyz_ref, 24);
    memcpy(s->zmp_in1, s->zmp_in2, 24);
    memcpy(s->zmp_in2, s->zmpxyz_ref, 24);
    memcpy(s->dcm_in1, s->dcm_in2, 24);
    memcpy(s->dcm_in2, s->dcmxyz_ref, 24);
    memcpy(s->COMacc_in1, s->COMacc_in2, 24);
    memcpy(s->COMacc_in2, s->COMacc_ref, 24);
    const double dt = DT_SLOW;
    if (mpc_gait_flag > s->mpc_gait_flag_old) { /* :170-250 */
      set3(s->COMxyz_ref, g[0], g[1], g[2]);
      set3(s->COMv_ref, g[36], g[37], g[38]);
      for (int k = 0; k < 3; ++k) s->COM_ref2[k] = s->COMxyz_ref[k] + s->COMv_ref[k] * dt;
      set3(s->COMacc_ref, g[39], g[40], g[41]);
      set3(s->COMacc_ref2, g[80], g[81], g[82]);
      s->zmpxyz_ref[0] = g[12];
      s->zmpxyz_ref[1] = g[13];
      s->zmp_ref2[0] = g[42];
      s->zmp_ref2[1] = g[43];
      s->dcmxyz_ref[0] = g[34];
      s->dcmxyz_ref[1] = g[35];
      s->dcm_ref2[0] = g[44];
      s->dcm_ref2[1] = g[45];
    } else { /* :251-367 */
      set3(s->COMxyz_ref, g[0], g[1], g[2]);
      set3(s->COMv_ref, g[36], g[37], g[38]);
      for (int k = 0; k < 3; ++k) s->COMxyz_ref[k] += s->COMv_ref[k] * dt;
      for (int k = 0; k < 3; ++k) s->COMv_ref[k] += g[39 + k] * dt;
      for (int k = 0; k < 3; ++k) s->COM_ref2[k] = s->COMxyz_ref[k] + s->COMv_ref[k] * dt;
      set3(s->COMacc_ref, g[80], g[81], g[82]);
      set3(s->COMacc_ref2, g[83], g[84], g[85]);
      s->zmpxyz_ref[0] = g[42];
      s->zmpxyz_ref[1] = g[43];
      s->zmp_ref2[0] = g[76];
      s->zmp_ref2[1] = g[77];
      s->dcmxyz_ref[0] = g[44];
      s->dcmxyz_ref[1] = g[45];
      s->dcm_ref2[0] = g[78];
      s->dcm_ref2[1] = g[79];
    }
    s->count_inteplotation = 0;
    s->mpc_gait_flag_old = mpc_gait_flag;
  }
}

#define F(a, k) (s->foot[a][k])

/* one swing-foot axis of Foot_trajectory_solve_mod2 (:1875-1934 / :2052-2111):
 * cubic through (t_plan[0], prev), (t_plan[1], mid), (t_plan[2], end) with
 * zero end velocity, evaluated at t_des */
static void swing_axis(qo_rt *s, const double Ai[16], double t_des, int p, int v, int a, int k,
                       double mid, double end) {
  double plan[4] = {F(p, k - 1), mid, end, 0};
  double co[4];
  for (int r = 0; r < 4; ++r) {
    double acc = 0;
    for (int c = 0; c < 4; ++c) acc += Ai[r * 4 + c] * plan[c];
    co[r] = acc;
  }
  double tp[4] = {cube(t_des), sq(t_des), (t_des), 1};
  double tv[4] = {3 * sq(t_des), 2 * (t_des), 1, 0};
  double ta[4] = {6 * (t_des), 2, 0, 0};
  double xp = 0, xv = 0, xa = 0;
  for (int c = 0; c < 4; ++c) {
    xp += tp[c] * co[c];
    xv += tv[c] * co[c];
    xa += ta[c] * co[c];
  }
  F(p, k) = xp;
  F(v, k) = xv;
  F(a, k) = xa;
}

/* Foot_trajectory_solve_mod2, PRMPCClass.cpp:1756-2195 */
static void foot_traj_mod2(qo_rt *s, int j_indexx, int stopwalking, const double nrt[9],
                           double out[30]) {
  int bjxx_nrt = (int)nrt[0];
  if (bjxx_nrt >= 0 && bjxx_nrt + 1 < NS) { /* :1758-1764 (unchecked in the reference) */
    s->fxyz[0][bjxx_nrt] = nrt[1];
    s->fxyz[0][bjxx_nrt + 1] = nrt[2];
    s->fxyz[1][bjxx_nrt] = nrt[3];
    s->fxyz[1][bjxx_nrt + 1] = nrt[4];
    s->fxyz[2][bjxx_nrt] = nrt[5];
    s->fxyz[2][bjxx_nrt + 1] = nrt[6];
  }
  int bjx_period_nrt = (int)nrt[7];
  if (nrt[8] > 0 && bjx_period_nrt >= 0 && bjx_period_nrt < NS) s->ts[bjx_period_nrt] = nrt[8];
  recompute_tx(s);
  s->t_end_footstep = (int)round((s->body.tx[NS - 1] - 2 * TSTEP) / DT_FAST); /* :1780 */
  s->tx_total = s->body.tx[NS - 1];
  memset(out, 0, sizeof(double) * 30);
  int *bjx1 = &s->body.bjx1;
  for (int j_index = j_indexx; j_index < j_indexx + NH; j_index++) {
    const int k = j_index - j_indexx + 1;
    if (j_index <= s->t_end_footstep) { /* :1790-1799 */
      s->bjxx = indexfind(s, j_index * DT_FAST) + 1;
      *bjx1 = indexfind(s, (j_index + 1) * DT_FAST) + 1;
    }
    if (stopwalking || (j_index > s->t_end_footstep)) /* :1801-1807 */
      for (int i_t = *bjx1 + 1; i_t < NS; i_t++) s->lift[i_t] = 0;
    for (int i_t = 24; i_t < NS; i_t++) s->lift[i_t] = 0; /* :1809-1811 */
    s->fxyz[1][0] = -s->stepwidth0;                       /* :1814 */
    if ((*bjx1 >= 2) && (j_index <= s->t_end_footstep)) {
      const int b1 = *bjx1, bx = s->bjxx;
      /* _bjxx-2 < 0 is reachable only with a step period under 0.1 s (the DSP
       * window td = 0.1 ts shorter than one tick); the reference then reads
       * out of bounds -- defined here as index 0 */
      const int bm = bx >= 2 ? bx - 2 : 0;
      /* support leg holds (:1866-1876 / :2003-2008); swing leg = other */
      const int sx = (b1 % 2 == 0) ? LX : RX; /* support */
      const int wx = (b1 % 2 == 0) ? RX : LX; /* swing   */
      for (int ax = 0; ax < 3; ++ax) {
        F(sx + ax, k) = F(sx + ax, k - 1);
        F(sx + ax, k + 1) = F(sx + ax, k - 1);
      }
      const double rt = round(s->body.tx[b1 - 1] / DT_FAST);
      if ((j_index + 1 - rt) * DT_FAST < s->td[b1 - 1]) { /* double support */
        for (int ax = 0; ax < 3; ++ax) {
          F(wx + ax, k) = F(wx + ax, k - 1);
          F(wx + ax, k + 1) = F(wx + ax, k - 1);
        }
      } else {
        double t_des = (j_index + 1 - rt + 1) * DT_FAST;
        double tp[3];
        tp[0] = t_des - DT_FAST;
        tp[1] = (s->td[b1 - 1] + s->ts[b1 - 1]) / 2 + 0.0001;
        tp[2] = s->ts[b1 - 1] - (2 * DT_FAST + 0.001);
        if (fabs(t_des - s->ts[b1 - 1]) <= (DT_FAST)) {
          for (int ax = 0; ax < 3; ++ax) {
            F(wx + ax, k) = s->fxyz[ax][bx];
            F(wx + ax, k + 1) = s->fxyz[ax][bx];
          }
        } else {
          double Ai[16];
          aaa_inv2(tp, Ai);
          swing_axis(s, Ai, t_des, wx + 0, wx + 3, wx + 6, k,
                     (s->fxyz[0][bm] + s->fxyz[0][bx]) / 2, s->fxyz[0][bx]);
          if ((j_index + 1 - rt) * DT_FAST < s->td[b1 - 1] + DT_FAST)
            s->ry_left_right = (s->fxyz[1][bx] + s->fxyz[1][bm]) / 2;
          swing_axis(s, Ai, t_des, wx + 1, wx + 4, wx + 7, k, s->ry_left_right, s->fxyz[1][bx]);
          /* std::max(a, b) returns a unless a < b */
          const double zmax = (s->fxyz[2][bm] < s->fxyz[2][bx]) ? s->fxyz[2][bx]
                                                                   : s->fxyz[2][bm];
          swing_axis(s, Ai, t_des, wx + 2, wx + 5, wx + 8, k, zmax + s->lift[b1 - 1],
                     s->fxyz[2][bx]);
          for (int ax = 0; ax < 3; ++ax)
            F(wx + ax, k + 1) = F(wx + ax, k) + DT_FAST * F(wx + 3 + ax, k);
        }
      }
    } else {
      if (j_index > s->t_end_footstep) { /* :2152-2160 */
        for (int ax = 0; ax < 3; ++ax) {
          F(RX + ax, k) = F(RX + ax, k - 1);
          F(LX + ax, k) = F(LX + ax, k - 1);
        }
      } else { /* :2163-2166 */
        F(RY, k) = -s->stepwidth0;
        F(LY, k) = s->stepwidth0;
      }
    }
  }
  for (int j = 0; j < 5; j++) { /* :2170-2178 */
    out[0 + 6 * j] = F(RX, j + 1);
    out[1 + 6 * j] = F(RY, j + 1);
    out[2 + 6 * j] = F(RZ, j + 1);
    out[3 + 6 * j] = F(LX, j + 1);
    out[4 + 6 * j] = F(LY, j + 1);
    out[5 + 6 * j] = F(LZ, j + 1);
  }
  for (int a = 0; a < 18; ++a) F(a, 0) = F(a, 1); /* :2180-2197 */
}

/* XGetSolution_Foot_rotation, PRMPCClass.cpp:2255-2380 */
static void foot_rotation(qo_rt *s, int walktimex, double dt_sample, double out[30]) {
  memset(out, 0, sizeof(double) * 30);
  int *bjx1 = &s->body.bjx1;
  for (int walktime = walktimex; walktime < walktimex + NH; walktime++) {
    const int c = walktime - walktimex;
    if (walktime <= s->t_end_footstep) {
      s->bjxx = indexfind(s, walktime * DT_FAST) + 1;
      *bjx1 = indexfind(s, (walktime + 1) * DT_FAST) + 1;
    }
    const int b1 = *bjx1;
    if ((b1 >= 2) && (walktime <= s->t_end_footstep)) {
      /* t_desxx (:2271) is only read inside this branch */
      double t_desxx = (walktime + 1) * dt_sample - (s->body.tx[b1 - 1] + 2 * s->td[b1 - 1] / 4);
      const double ts = s->ts[b1 - 1], td = s->td[b1 - 1];
      const double ph = t_desxx + 2 * td / 4;
      const double dx = s->fxyz[0][b1] - s->fxyz[0][b1 - 1];
      double *r = (b1 % 2 == 0) ? s->Rfoot_r : s->Lfoot_r;
      if (b1 % 2 == 0) /* right foot roll, :2279 */
        r[c * 3 + 0] = -0.065 * (1 - cos(2 * M_PI / (ts) * (ph)));
      else /* left foot roll, :2321 */
        r[c * 3 + 0] = 0.075 * (1 - cos(2 * M_PI / (ts) * (ph)));
      if (ph >= (ts / 2)) {
        if (dx > 0)
          r[c * 3 + 1] = 0.075 * dx / (s->footx_max) * (cos(4 * M_PI / (ts) * (ph)) - 1);
      } else {
        r[c * 3 + 1] = 0;
      }
    }
    out[0 + 6 * c] = s->Rfoot_r[c * 3 + 0];
    out[1 + 6 * c] = s->Rfoot_r[c * 3 + 1];
    out[2 + 6 * c] = s->Rfoot_r[0 * 3 + 2];
    out[3 + 6 * c] = s->Lfoot_r[c * 3 + 0];
    out[4 + 6 * c] = s->Lfoot_r[c * 3 + 1];
    out[5 + 6 * c] = s->Lfoot_r[0 * 3 + 2];
  }
}

/* gait_fast.cpp loop body :512-735, after the subscriber callbacks :79-110
 * applied the latest /MPC/Gait (gait) and /control2rtmpc/state (ctrl). */
static void rt_tick(qo_rt *s, const double *gait, const double *ctrl, double *traj, double *nrt,
                    double *gen, int32_t *sched) {
  /* callbacks */
  const int mpc_gait_flag = (int)gait[99];
  const double *Nrt = gait + 86;
  for (int jx = 1; jx < 25; jx++) s->state_feedback[jx] = ctrl[jx];
  const double bodyangle_state[4] = {s->state_feedback[10], s->state_feedback[11],
                                     s->state_feedback[13], s->state_feedback[14]};
  const int n_t_int = (int)floor(DT_SLOW / DT_FAST);
  int body_status = -1, flags = 0;
  if (ctrl[0] > 0) {
    s->count_in_rt_loop += 1;
    s->t_int = (int32_t)((uint32_t)s->t_int + (uint32_t)(int)floor(s->count_in_rt_loop / n_t_int));
    s->state_feedback[0] = s->t_int;
    for (int jx = 0; jx < 25; jx++) s->state_to_MPC[jx] = s->state_feedback[jx]; /* :522-527 */
    flags |= 1;
    if (mpc_gait_flag > 0) {
      s->count_in_rt_mpc += 1;
      interpolation(s, gait, mpc_gait_flag);
      if (s->count_in_rt_mpc * DT_FAST > 1.0) { /* _height_offset_timex = 1 */
        int foot_i = (int)(s->count_in_rt_mpc - (int)1.0 / DT_FAST);
        foot_traj_mod2(s, foot_i, 0, Nrt, s->foorpr_gen);
        foot_rotation(s, foot_i, DT_FAST, s->foortheta_gen);
      }
      s->zmpxyz_ref[2] = 0.0; /* _Zsc = {l,r}foot_inter(2) = 0 (:557-566) */
      double zmp_ref[10], angle_ref[10], rfoot_ref[10], lfoot_ref[10], comacc_ref[15];
      memset(rfoot_ref, 0, sizeof(rfoot_ref));
      memset(comacc_ref, 0, sizeof(comacc_ref));
      for (int j = 0; j < 5; j++) { /* :568-616 */
        if (j == 0) {
          zmp_ref[0] = s->zmp_inter[0];
          zmp_ref[1] = s->zmp_inter[1];
        } else {
          zmp_ref[2 * j] = s->zmp_inter[8 + 3 * j - 2];
          zmp_ref[2 * j + 1] = s->zmp_inter[8 + 3 * j - 1];
        }
        rfoot_ref[2 * j] = s->foorpr_gen[j * 6 + 1]; /* row 0 overwritten by y */
        lfoot_ref[2 * j] = s->foorpr_gen[j * 6 + 3];
        lfoot_ref[2 * j + 1] = s->foorpr_gen[j * 6 + 4];
        angle_ref[2 * j] = (s->foortheta_gen[j * 6] + s->foortheta_gen[j * 6 + 3]) / 5;
        angle_ref[2 * j + 1] = (s->foortheta_gen[j * 6 + 1] + s->foortheta_gen[j * 6 + 4]) / 5;
        comacc_ref[3 * j + 2] = (j == 0) ? s->comacc_inter[2] : s->comacc_inter[8 + 3 * j];
      }
      s->body_thetax[0] = angle_ref[0];
      s->body_thetax[1] = angle_ref[1];
      int st = QO_OK;
      qo_body_theta_mpc(&s->body, s->count_in_rt_mpc, bodyangle_state, zmp_ref, angle_ref,
                        rfoot_ref, lfoot_ref, comacc_ref, Nrt, s->bodyangle_mpc, &st);
      body_status = st;
    }
  }
  /* low_mpc_gait_inte, :633-714 and the /rtMPC/traj message :716-729 */
  double inte[51];
  memset(inte, 0, sizeof(inte));
  for (int k = 0; k < 3; ++k) inte[k] = s->rpy_mpc_body[k];
  for (int k = 0; k < 3; ++k) inte[3 + k] = s->body_thetax[k];
  inte[6] = s->foorpr_gen[3];
  inte[7] = s->foorpr_gen[4];
  inte[8] = s->foorpr_gen[5];
  inte[9] = s->foorpr_gen[0];
  inte[10] = s->foorpr_gen[1];
  inte[11] = s->foorpr_gen[2];
  inte[12] = s->zmp_inter[0];
  inte[13] = s->zmp_inter[1];
  inte[14] = s->zmpxyz_ref[2];
  /* 15..26 F_L, F_R, M_L, M_R stay zero */
  inte[27] = gait[27];
  inte[28] = s->foortheta_gen[3];
  inte[29] = s->foortheta_gen[4];
  inte[30] = s->foortheta_gen[5];
  inte[31] = s->foortheta_gen[0];
  inte[32] = s->foortheta_gen[1];
  inte[33] = s->foortheta_gen[2];
  inte[34] = s->dcm_inter[0];
  inte[35] = s->dcm_inter[1];
  for (int k = 0; k < 14; ++k) inte[36 + k] = s->bodyangle_mpc[k];
  inte[50] = 0.0; /* t_fast_mpc: wall-clock duration, not reproduced */
  memset(traj, 0, sizeof(double) * 100);
  for (int jx = 0; jx < 36; jx++) traj[jx] = gait[jx];
  for (int jx = 36; jx <= 86; jx++) traj[jx] = inte[jx - 36];
  traj[98] = (int)s->tx_total / 0.001; /* (int) _tx_total / gait::t_program_cyclic */
  traj[99] = s->count_in_rt_loop;
  for (int jx = 0; jx < 25; jx++) nrt[jx] = s->state_to_MPC[jx];
  if (gen) {
    memcpy(gen, s->foorpr_gen, sizeof(double) * 30);
    memcpy(gen + 30, s->foortheta_gen, sizeof(double) * 30);
  }
  if (sched) {
    sched[0] = s->body.bjx1;
    sched[1] = s->bjxx;
    sched[2] = s->t_end_footstep;
    sched[3] = s->count_in_rt_mpc;
    sched[4] = s->t_int;
    sched[5] = body_status;
    sched[6] = flags; /* bit 0: /rt2nrt/state published this tick */
    sched[7] = s->body.bjx2;
  }
}

void qo_rt_tick_n(qo_rt *arr, int64_t n, const double *gait, const double *ctrl, double *traj,
                  double *nrt, double *gen, int32_t *sched) {
  for (int64_t b = 0; b < n; ++b)
    rt_tick(&arr[b], gait + b * 100, ctrl + b * 25, traj + b * 100, nrt + b * 25,
            gen ? gen + b * 60 : NULL, sched ? sched + b * QO_RT_SCHED : NULL);
}
