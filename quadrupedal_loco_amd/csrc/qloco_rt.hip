// qloco_rt.hip -- batched rt_mpc_qp node tick (gfx950), SURVEY.md §8f rows 2-3.
//
// One tick = one iteration of the rt node's 100 Hz loop for B robots
// (unitree_ros/rt_mpc_qp/src/gait_fast.cpp:505-735): the subscriber
// callbacks on the latest /MPC/Gait and /control2rtmpc/state messages
// (:79-110), the loop counters and /rt2nrt/state (:512-527), the cubic
// interpolation of the slow-MPC references (xget_position_interpolation,
// :113-372 -> PRMPCClass::XGetSolution_position_mod3, PRMPCClass.cpp:
// 1170-1261), the contact schedule and swing-foot generator
// (Foot_trajectory_solve_mod2, :1756-2195, with Indexfind :716-738), the
// foot rotation generator (XGetSolution_Foot_rotation, :2255-2380), the
// body-MPC reference packing (:557-616), body_theta_mpc (qloco_body.hip)
// and the /rtMPC/traj message (:633-729).
//
// Three launches on one stream:
//   rt_pre_kernel    one robot per lane: everything before body_theta_mpc;
//                    writes the body kernel's reference arrays and run mask
//   body_mpc_kernel  8 robots per wave (8-lane Goldfarb-Idnani groups), on
//                    each robot's own _tx schedule
//   rt_post_kernel   one robot per lane: packs /rtMPC/traj, /rt2nrt/state
//
// State lives in one device workspace: the node/generator members in
// 64-robot tiles, field-major inside a tile (field f of robot r at
// d[(r / 64) * F_DOUBLES * 64 + f * 64 + r % 64]: every lane access of a
// field is one coalesced 512-byte row per wave, and the field offsets are
// compile-time constants, so the compiler can tell fields apart and batch
// loads across the stores of other fields), the body-MPC records
// (QLOCO_BODY_STATE_LEN doubles per robot, shared with qloco_body_mpc_step)
// and per-tick scratch.  fp64 throughout, compiled without FMA contraction
// so the schedule arithmetic follows the restatement (oracle/rt_tick.c)
// operation for operation; schedule integers are bit-exact.
//
// Reference quirks kept (see oracle/rt_tick.c): rfoot_mpc_ref row 0 holds
// the y coordinate and row 1 stays 0; t_int += floor(count/2) (int32 wrap);
// mpc_gait_flag = (int) /MPC/Gait[99]; traj[86] (the node's own wall-clock
// duration) is 0; stale member values carried between calls.
#include <math.h>
#include <string.h>

#include "qloco_common.hpp"

namespace qloco {

int body_mpc_launch(int64_t batch, const int32_t *i, const double *bodyangle_state,
                    const double *zmp_ref, const double *angle_ref, const double *rfoot_ref,
                    const double *lfoot_ref, const double *comacc_ref, double *state,
                    double *com_traj, int32_t *status, const double *tx, int64_t tx_stride,
                    int64_t tx_tile, const int32_t *run, int64_t ref_ld, hipStream_t stream);

namespace rt {

constexpr int NS = 27;  // _footstepsnumber
constexpr int NH = 4;   // _nh
constexpr double DT_SLOW = 0.025, DT_FAST = 0.01, TSTEP = 0.7, HALF_HIP = 0.12675;
constexpr double STEPWIDTH0 = 2 * HALF_HIP / 2, TDSP_RATIO = 0.1, FOOTX_MAX = 0.15;

// double fields (SoA offsets, in units of B)
enum : int {
  F_TS = 0,
  F_TD = F_TS + NS,
  F_LIFT = F_TD + NS,
  F_TX = F_LIFT + NS,
  F_FXYZ = F_TX + NS,       // _footxyz_real(a, i) at F_FXYZ + a*NS + i
  F_TXTOT = F_FXYZ + 3 * NS,
  F_RYLR = F_TXTOT + 1,
  F_FOOT = F_RYLR + 1,      // foot array a (RX..LAZ), index k (0..5) at F_FOOT + a*6 + k
  F_RFR = F_FOOT + 18 * 6,  // _Rfoot_r (3x5 col-major)
  F_LFR = F_RFR + 15,
  F_COM = F_LFR + 15,       // COM_in1, COM_in2, COMxyz_ref, COM_ref2, COMv_ref
  F_ACC = F_COM + 15,       // COMacc_in1, _in2, _ref, _ref2
  F_ZMP = F_ACC + 12,       // zmp_in1, _in2, zmpxyz_ref, zmp_ref2
  F_DCM = F_ZMP + 12,       // dcm_in1, _in2, dcmxyz_ref, dcm_ref2
  F_RPY = F_DCM + 12,       // rpy_mpc_body (21)
  F_CACC = F_RPY + 21,      // comacc_inter
  F_ZINT = F_CACC + 21,     // zmp_inter
  F_DINT = F_ZINT + 21,     // dcm_inter
  F_FOORPR = F_DINT + 21,   // foorpr_gen (30)
  F_FTHETA = F_FOORPR + 30, // foortheta_gen (30)
  F_BTHX = F_FTHETA + 30,   // body_thetax(0..1)
  F_NRT = F_BTHX + 2,       // state_to_MPC (25)
  F_DOUBLES = F_NRT + 25
};
// int fields
enum : int { I_LOOP = 0, I_MPC, I_INT, I_TINT, I_FLAGOLD, I_TEND, I_BJXX, I_INTS };
enum { RX = 0, RY, RZ, RVX, RVY, RVZ, RAX, RAY, RAZ, LX, LY, LZ, LVX, LVY, LVZ, LAX, LAY, LAZ };

// body_theta_mpc reference record per robot (doubles): bodyangle_state,
// zmp_mpc_ref, bodyangle_mpc_ref, rfoot_mpc_ref, lfoot_mpc_ref (Eigen 2x5
// col-major), comacc_mpc_ref (3x5)
enum : int { RF_BAS = 0, RF_ZMP = 4, RF_ANG = 14, RF_RFT = 24, RF_LFT = 34, RF_ACC = 44,
             RF_USED = 59, RF_LD = 64 };
constexpr int TL = 64;  // robots per state tile (one wave)
struct Ws {  // byte offsets into the workspace
  int64_t d, n, body, ref, ct, bi, run, st, total;
};
__host__ __device__ inline Ws layout(int64_t B) {
  Ws w;
  auto al = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
  const int64_t Bt = (B + TL - 1) / TL * TL;  // whole tiles
  w.d = 0;
  w.n = al(w.d + 8 * F_DOUBLES * Bt);
  w.body = al(w.n + 4 * I_INTS * Bt);
  w.ref = al(w.body + 8 * QLOCO_BODY_STATE_LEN * B);
  w.ct = al(w.ref + 8 * RF_LD * B);
  w.bi = al(w.ct + 8 * 14 * B);
  w.run = al(w.bi + 4 * B);
  w.st = al(w.run + 4 * B);
  w.total = al(w.st + 4 * B);
  return w;
}

struct RtArgs {
  int64_t B;
  char *ws;
  const double *gait, *ctrl;
  double *traj, *nrt, *gen;
  int32_t *sched;
  double aaa_inv_mod[16];  // solve_AAA_inv_mod1 (:1344-1362), col-major
};

// per-lane view of one robot's tiled state
struct Robot {
  double *__restrict__ d;
  int32_t *__restrict__ n;
  __device__ Robot(char *ws, const Ws &L, int64_t r)
      : d(reinterpret_cast<double *>(ws + L.d) + (r / TL) * (F_DOUBLES * TL) + r % TL),
        n(reinterpret_cast<int32_t *>(ws + L.n) + (r / TL) * (I_INTS * TL) + r % TL) {}
  __device__ double &D(int f) const { return d[f * TL]; }
  __device__ int32_t &I(int f) const { return n[f * TL]; }
  __device__ double &foot(int a, int k) const { return D(F_FOOT + a * 6 + k); }
  __device__ double &fxyz(int a, int i) const { return D(F_FXYZ + a * NS + i); }
};

// Indexfind, xyz = 0 (:716-738), bounded at the 27 steps
__device__ __forceinline__ int indexfind(const Robot &R, double goal) {
  int j = 0;
  while (j < NS && goal >= R.D(F_TX + j)) j++;
  return j - 1;
}
// The same scan for a non-decreasing sequence of goals: _tx is non-decreasing
// (every _ts > 0, and round(tx/dt)*dt - 1e-5 never decreases), so every
// j < the previous answer + 1 still satisfies goal >= _tx(j) and the scan may
// resume there -- the result equals the reference's scan from 0.
struct IndexScan {
  int j = 0;
  __device__ __forceinline__ int operator()(const Robot &R, double goal) {
    while (j < NS && goal >= R.D(F_TX + j)) j++;
    return j - 1;
  }
};

// std::pow(t, 3) / pow(t, 2) as in oracle/rt_tick.c: compensated cube (fma
// error-free products, one final rounding), exact-rounded square
__host__ __device__ inline double sq(double x) { return x * x; }
__host__ __device__ inline double cube(double x) {
  const double p = x * x, e = fma(x, x, -p);
  const double hi = p * x, lo = fma(p, x, -hi);
  return hi + (lo + e * x);
}

// Dense 4x4 inverse, Gauss-Jordan with partial pivoting (row-major), the
// same algorithm and operation order as oracle/rt_tick.c:qo_inv4
__host__ __device__ inline void inv4(const double A[16], double Ai[16]) {
  // every index static (pivot search by value, row swap by selects), so the
  // 4x8 tableau stays in registers
  double M[4][8];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      M[r][c] = A[r * 4 + c];
      M[r][4 + c] = (r == c) ? 1.0 : 0.0;
    }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int p = k;
    double best = fabs(M[k][k]);
#pragma unroll
    for (int r = k + 1; r < 4; ++r) {
      const double v = fabs(M[r][k]);
      if (v > best) {
        best = v;
        p = r;
      }
    }
#pragma unroll
    for (int r = k + 1; r < 4; ++r)
      if (p == r)
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const double t = M[k][c];
          M[k][c] = M[r][c];
          M[r][c] = t;
        }
    const double piv = M[k][k];
#pragma unroll
    for (int c = 0; c < 8; ++c) M[k][c] = M[k][c] / piv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r == k) continue;
      const double f = M[r][k];
#pragma unroll
      for (int c = 0; c < 8; ++c) M[r][c] = M[r][c] - f * M[k][c];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) Ai[r * 4 + c] = M[r][4 + c];
}

__device__ void recompute_tx(const Robot &R) {  // :1773-1779
  for (int i = 0; i < NS; ++i) R.D(F_TD + i) = TDSP_RATIO * R.D(F_TS + i);
  double t = 0.0;
  R.D(F_TX) = 0.0;
  for (int i = 1; i < NS; i++) {
    t = t + R.D(F_TS + i - 1);
    t = round(t / DT_SLOW) * DT_SLOW - 0.00001;
    R.D(F_TX + i) = t;
  }
}

// XGetSolution_position_mod3 (:1170-1261): 4 horizon points of the cubic
// through (in1, in2, ref, ref2) at t = -dt, 0, dt, 2dt (dt = dt_mpc_slow)
__device__ void position_mod3(const RtArgs &a, const Robot &R, int walktime, int f_in,
                              int f_out, int t_end) {
  // com_inte.setZero(): entries 18..20 are never written below (jx < 4) and
  // stay 0 from init; 0..17 are all overwritten
  if (walktime > t_end) {
    for (int k = 0; k < 21; ++k) R.D(f_out + k) = 0.0;
    return;
  }
  double in[4][3];
  for (int q = 0; q < 4; ++q)
    for (int ax = 0; ax < 3; ++ax) in[q][ax] = R.D(f_in + 3 * q + ax);
#pragma unroll
  for (int jx = 0; jx < NH; jx++) {
    const double t_cur = (walktime * DT_FAST + jx * DT_FAST);
    const double tp[4] = {cube(t_cur), sq(t_cur), (t_cur), 1.0};
    const double tv[4] = {3 * sq(t_cur), 2 * (t_cur), 1, 0};
    const double ta[4] = {6 * (t_cur), 2, 0, 0};
    double rp[4], rv[4], ra[4];
    for (int c = 0; c < 4; ++c) {
      double ap = 0, av = 0, aa = 0;
      for (int k = 0; k < 4; ++k) {
        ap += tp[k] * a.aaa_inv_mod[c * 4 + k];
        av += tv[k] * a.aaa_inv_mod[c * 4 + k];
        aa += ta[k] * a.aaa_inv_mod[c * 4 + k];
      }
      rp[c] = ap;
      rv[c] = av;
      ra[c] = aa;
    }
    for (int ax = 0; ax < 3; ++ax) {
      double p = 0, v = 0, acc = 0;
      for (int k = 0; k < 4; ++k) {
        p += rp[k] * in[k][ax];
        v += rv[k] * in[k][ax];
        acc += ra[k] * in[k][ax];
      }
      if (jx == 0) {
        R.D(f_out + ax) = p;
        R.D(f_out + 3 + ax) = v;
        R.D(f_out + 6 + ax) = acc;
      } else {
        R.D(f_out + 8 + 3 * jx - 2 + ax) = p;
      }
    }
  }
}

// one swing-foot axis (:1903-1951 right / :2069-2118 left): the cubic
// through (start, mid, end) and zero end velocity, evaluated at t_des
__device__ __forceinline__ void swing_axis(const double Ai[16], double t_des, double start,
                                           double mid, double end, double &xp, double &xv,
                                           double &xa) {
  const double plan[4] = {start, mid, end, 0};
  double co[4];
  for (int r = 0; r < 4; ++r) {
    double s = 0;
    for (int c = 0; c < 4; ++c) s += Ai[r * 4 + c] * plan[c];
    co[r] = s;
  }
  const double tp[4] = {cube(t_des), sq(t_des), (t_des), 1};
  const double tv[4] = {3 * sq(t_des), 2 * (t_des), 1, 0};
  const double ta[4] = {6 * (t_des), 2, 0, 0};
  xp = 0;
  xv = 0;
  xa = 0;
  for (int c = 0; c < 4; ++c) {
    xp += tp[c] * co[c];
    xv += tv[c] * co[c];
    xa += ta[c] * co[c];
  }
}

// Foot_trajectory_solve_mod2 (PRMPCClass.cpp:1756-2195), _stopwalking = false
__device__ void foot_traj_mod2(const Robot &R, int j_indexx, const double nrt[9], int &bjx1,
                               int &bjxx, int &t_end, int sched_xx[NH], int sched_x1[NH]) {
  const int bjxx_nrt = (int)nrt[0];
  if (bjxx_nrt >= 0 && bjxx_nrt + 1 < NS) {  // :1758-1764 (unchecked in the reference)
    R.fxyz(0, bjxx_nrt) = nrt[1];
    R.fxyz(0, bjxx_nrt + 1) = nrt[2];
    R.fxyz(1, bjxx_nrt) = nrt[3];
    R.fxyz(1, bjxx_nrt + 1) = nrt[4];
    R.fxyz(2, bjxx_nrt) = nrt[5];
    R.fxyz(2, bjxx_nrt + 1) = nrt[6];
  }
  const int bjx_period_nrt = (int)nrt[7];
  // _td and _tx are pure functions of _ts (:1773-1779), recomputed by the
  // reference on every call; they only change when this call changed _ts
  if (nrt[8] > 0 && bjx_period_nrt >= 0 && bjx_period_nrt < NS &&
      R.D(F_TS + bjx_period_nrt) != nrt[8]) {
    R.D(F_TS + bjx_period_nrt) = nrt[8];
    recompute_tx(R);
  }
  t_end = (int)round((R.D(F_TX + NS - 1) - 2 * TSTEP) / DT_FAST);  // :1780
  R.D(F_TXTOT) = R.D(F_TX + NS - 1);
  // The four passes below are restated with their memory traffic regrouped
  // (same arithmetic, same order of operations):
  //  * _footxyz_real(1, 0) = -stepwidth is written at the head of every pass
  //    (:1814) -- written once here, before anything reads it;
  //  * the schedule of all passes first (Indexfind only reads _tx, which no
  //    pass writes), then every data-dependent load of all passes in one
  //    batch (_tx/_td/_ts/_lift_height_ref at bjx1-1, _footxyz_real at bjxx
  //    and bjxx-2): a pass that swings has j_index <= _t_end_footstep, and
  //    the lift zeroing of :1801-1807 only runs in passes with j_index >
  //    _t_end_footstep, which come after it, so the lift it reads is the
  //    stored one, or 0 from :1809-1811 for steps 24..26;
  //  * the foot positions at k - 1 and _ry_left_right carried in registers
  //    from pass to pass instead of stored and re-read.
  R.fxyz(1, 0) = -STEPWIDTH0;  // :1814
  int xx[NH], x1[NH];
  {
    IndexScan scan;  // goals j*dt, (j+1)*dt, (j+1)*dt, ... never decrease
    // and across ticks: resume near last tick's answer when goal >= _tx(j0-1)
    // (then every earlier entry passes too, _tx being non-decreasing), so
    // the scan costs O(1) loads however far the robot has walked
    {
      const int j0 = bjxx - 1;
      if (j0 >= 1 && j0 <= NS && j_indexx <= t_end && j_indexx * DT_FAST >= R.D(F_TX + j0 - 1))
        scan.j = j0;
    }
#pragma unroll
    for (int kk = 1; kk <= NH; ++kk) {
      const int j_index = j_indexx + kk - 1;
      if (j_index <= t_end) {  // :1790-1799
        bjxx = scan(R, j_index * DT_FAST) + 1;
        bjx1 = scan(R, (j_index + 1) * DT_FAST) + 1;
      }
      xx[kk - 1] = sched_xx[kk - 1] = bjxx;
      x1[kk - 1] = sched_x1[kk - 1] = bjx1;
    }
  }
  double txb[NH], tdb[NH], tsb[NH], lfb[NH], fx[NH][3], fm[NH][3];
#pragma unroll
  for (int kk = 1; kk <= NH; ++kk) {
    const int q = kk - 1, j_index = j_indexx + q;
    if ((x1[q] >= 2) && (j_index <= t_end)) {
      const int b1 = x1[q], bx = xx[q];
      const int bm = bx >= 2 ? bx - 2 : 0;  // reference UB below 0 (oracle/rt_tick.c)
      txb[q] = R.D(F_TX + b1 - 1);
      tdb[q] = R.D(F_TD + b1 - 1);
      tsb[q] = R.D(F_TS + b1 - 1);
      lfb[q] = (b1 - 1 >= 24) ? 0.0 : R.D(F_LIFT + b1 - 1);
      for (int ax = 0; ax < 3; ++ax) {
        fx[q][ax] = R.fxyz(ax, bx);
        fm[q][ax] = R.fxyz(ax, bm);
      }
    } else {
      txb[q] = tdb[q] = tsb[q] = lfb[q] = 0.0;
      for (int ax = 0; ax < 3; ++ax) fx[q][ax] = fm[q][ax] = 0.0;
    }
  }
  // foot positions at k - 1: right x, y, z then left x, y, z
  double pos[6];
  for (int ax = 0; ax < 3; ++ax) {
    pos[ax] = R.foot(RX + ax, 0);
    pos[3 + ax] = R.foot(LX + ax, 0);
  }
  double rylr = R.D(F_RYLR);
#pragma unroll
  for (int kk = 1; kk <= NH; ++kk) {
    const int q = kk - 1, j_index = j_indexx + q, k = kk;
    const int b1 = x1[q];
    if (j_index > t_end)  // :1801-1807
      for (int i_t = b1 + 1; i_t < NS; i_t++) R.D(F_LIFT + i_t) = 0;
    for (int i_t = 24; i_t < NS; i_t++) R.D(F_LIFT + i_t) = 0;  // :1809-1811
    if ((b1 >= 2) && (j_index <= t_end)) {
      const bool even = (b1 % 2 == 0);
      const int sx = even ? LX : RX;  // support leg holds
      const int wx = even ? RX : LX;  // swing leg
      const int sp = even ? 3 : 0, wp = even ? 0 : 3;  // their slots in pos
      for (int ax = 0; ax < 3; ++ax) {
        const double h = pos[sp + ax];
        R.foot(sx + ax, k) = h;
        R.foot(sx + ax, k + 1) = h;
      }
      const double rt = round(txb[q] / DT_FAST);
      if ((j_index + 1 - rt) * DT_FAST < tdb[q]) {  // double support
        for (int ax = 0; ax < 3; ++ax) {
          const double h = pos[wp + ax];
          R.foot(wx + ax, k) = h;
          R.foot(wx + ax, k + 1) = h;
        }
      } else {
        const double t_des = (j_index + 1 - rt + 1) * DT_FAST;
        double tp[3];
        tp[0] = t_des - DT_FAST;
        tp[1] = (tdb[q] + tsb[q]) / 2 + 0.0001;
        tp[2] = tsb[q] - (2 * DT_FAST + 0.001);
        if (fabs(t_des - tsb[q]) <= (DT_FAST)) {
          for (int ax = 0; ax < 3; ++ax) {
            const double e = fx[q][ax];
            R.foot(wx + ax, k) = e;
            R.foot(wx + ax, k + 1) = e;
            pos[wp + ax] = e;
          }
        } else {
          const double A[16] = {cube(tp[0]), sq(tp[0]), (tp[0]), 1,
                                cube(tp[1]), sq(tp[1]), (tp[1]), 1,
                                cube(tp[2]), sq(tp[2]), (tp[2]), 1,
                                3 * sq(tp[2]), 2 * (tp[2]), 1.0, 0};
          double Ai[16];
          inv4(A, Ai);  // solve_AAA_inv2 (:2225-2237)
          if ((j_index + 1 - rt) * DT_FAST < tdb[q] + DT_FAST)
            rylr = (fx[q][1] + fm[q][1]) / 2;
          const double z0 = fm[q][2], z1 = fx[q][2];
          const double zmax = (z0 < z1) ? z1 : z0;  // std::max
          const double mid[3] = {(fm[q][0] + fx[q][0]) / 2, rylr, zmax + lfb[q]};
          for (int ax = 0; ax < 3; ++ax) {
            double xp, xv, xa;
            swing_axis(Ai, t_des, pos[wp + ax], mid[ax], fx[q][ax], xp, xv, xa);
            R.foot(wx + ax, k) = xp;
            R.foot(wx + 3 + ax, k) = xv;
            R.foot(wx + 6 + ax, k) = xa;
            R.foot(wx + ax, k + 1) = xp + DT_FAST * xv;
            pos[wp + ax] = xp;
          }
        }
      }
    } else {
      if (j_index > t_end) {  // :2152-2160
        for (int ax = 0; ax < 3; ++ax) {
          R.foot(RX + ax, k) = pos[ax];
          R.foot(LX + ax, k) = pos[3 + ax];
        }
      } else {  // :2163-2166; the other axes keep their stored values
        R.foot(RY, k) = -STEPWIDTH0;
        R.foot(LY, k) = STEPWIDTH0;
        pos[1] = -STEPWIDTH0;
        pos[4] = STEPWIDTH0;
        pos[0] = R.foot(RX, k);
        pos[2] = R.foot(RZ, k);
        pos[3] = R.foot(LX, k);
        pos[5] = R.foot(LZ, k);
      }
    }
  }
  R.D(F_RYLR) = rylr;
  for (int j = 0; j < 5; j++) {  // :2170-2178
    R.D(F_FOORPR + 0 + 6 * j) = R.foot(RX, j + 1);
    R.D(F_FOORPR + 1 + 6 * j) = R.foot(RY, j + 1);
    R.D(F_FOORPR + 2 + 6 * j) = R.foot(RZ, j + 1);
    R.D(F_FOORPR + 3 + 6 * j) = R.foot(LX, j + 1);
    R.D(F_FOORPR + 4 + 6 * j) = R.foot(LY, j + 1);
    R.D(F_FOORPR + 5 + 6 * j) = R.foot(LZ, j + 1);
  }
  for (int f = 0; f < 18; ++f) R.foot(f, 0) = R.foot(f, 1);  // :2180-2197
}

// XGetSolution_Foot_rotation (PRMPCClass.cpp:2255-2380)
// the Indexfind calls here repeat Foot_trajectory_solve_mod2's (same goals,
// same _tx, same _t_end_footstep test), so their results are reused
__device__ void foot_rotation(const Robot &R, int walktimex, int &bjx1, int &bjxx, int t_end,
                              const int sched_xx[NH], const int sched_x1[NH]) {
#pragma unroll
  for (int c = 0; c < NH; ++c) {
    const int walktime = walktimex + c;
    if (walktime <= t_end) {
      bjxx = sched_xx[c];
      bjx1 = sched_x1[c];
    }
    const int b1 = bjx1;
    if ((b1 >= 2) && (walktime <= t_end)) {
      const double tsb = R.D(F_TS + b1 - 1), tdb = R.D(F_TD + b1 - 1);
      const double t_desxx = (walktime + 1) * DT_FAST - (R.D(F_TX + b1 - 1) + 2 * tdb / 4);
      const double ph = t_desxx + 2 * tdb / 4;
      const double dx = R.fxyz(0, b1) - R.fxyz(0, b1 - 1);
      const int fr = (b1 % 2 == 0) ? F_RFR : F_LFR;
      if (b1 % 2 == 0)
        R.D(fr + c * 3 + 0) = -0.065 * (1 - cos(2 * M_PI / (tsb) * (ph)));
      else
        R.D(fr + c * 3 + 0) = 0.075 * (1 - cos(2 * M_PI / (tsb) * (ph)));
      if (ph >= (tsb / 2)) {
        if (dx > 0) R.D(fr + c * 3 + 1) = 0.075 * dx / (FOOTX_MAX) * (cos(4 * M_PI / (tsb) * (ph)) - 1);
      } else {
        R.D(fr + c * 3 + 1) = 0;
      }
    }
    R.D(F_FTHETA + 0 + 6 * c) = R.D(F_RFR + c * 3 + 0);
    R.D(F_FTHETA + 1 + 6 * c) = R.D(F_RFR + c * 3 + 1);
    R.D(F_FTHETA + 2 + 6 * c) = R.D(F_RFR + 2);
    R.D(F_FTHETA + 3 + 6 * c) = R.D(F_LFR + c * 3 + 0);
    R.D(F_FTHETA + 4 + 6 * c) = R.D(F_LFR + c * 3 + 1);
    R.D(F_FTHETA + 5 + 6 * c) = R.D(F_LFR + 2);
  }
}

__device__ __forceinline__ void copy3(const Robot &R, int dst, int src) {
  for (int k = 0; k < 3; ++k) R.D(dst + k) = R.D(src + k);
}

// xget_position_interpolation (gait_fast.cpp:113-372), live vectors only
__device__ void interpolation(const RtArgs &a, const Robot &R, const double *g, int flag,
                              int t_int, int t_end) {
  int cnt = R.I(I_INT) + 1;
  if (t_int > 2) {
    position_mod3(a, R, cnt, F_COM, F_RPY, t_end);
    position_mod3(a, R, cnt, F_ACC, F_CACC, t_end);
    position_mod3(a, R, cnt, F_ZMP, F_ZINT, t_end);
    position_mod3(a, R, cnt, F_DCM, F_DINT, t_end);
  }
  if (cnt % 2 == 0) {  // n_t_int = floor(0.025 / 0.01) = 2
    copy3(R, F_COM + 0, F_COM + 3);
    copy3(R, F_COM + 3, F_COM + 6);
    copy3(R, F_ZMP + 0, F_ZMP + 3);
    copy3(R, F_ZMP + 3, F_ZMP + 6);
    copy3(R, F_DCM + 0, F_DCM + 3);
    copy3(R, F_DCM + 3, F_DCM + 6);
    copy3(R, F_ACC + 0, F_ACC + 3);
    copy3(R, F_ACC + 3, F_ACC + 6);
    const double dt = DT_SLOW;
    if (flag > R.I(I_FLAGOLD)) {  // :170-250
      for (int k = 0; k < 3; ++k) {
        R.D(F_COM + 6 + k) = g[k];
        R.D(F_COM + 12 + k) = g[36 + k];
        R.D(F_COM + 9 + k) = R.D(F_COM + 6 + k) + R.D(F_COM + 12 + k) * dt;
        R.D(F_ACC + 6 + k) = g[39 + k];
        R.D(F_ACC + 9 + k) = g[80 + k];
      }
      R.D(F_ZMP + 6) = g[12];
      R.D(F_ZMP + 7) = g[13];
      R.D(F_ZMP + 9) = g[42];
      R.D(F_ZMP + 10) = g[43];
      R.D(F_DCM + 6) = g[34];
      R.D(F_DCM + 7) = g[35];
      R.D(F_DCM + 9) = g[44];
      R.D(F_DCM + 10) = g[45];
    } else {  // :251-367
      for (int k = 0; k < 3; ++k) {
        double ref = g[k], v = g[36 + k];
        ref += v * dt;
        v += g[39 + k] * dt;
        R.D(F_COM + 6 + k) = ref;
        R.D(F_COM + 12 + k) = v;
        R.D(F_COM + 9 + k) = ref + v * dt;
        R.D(F_ACC + 6 + k) = g[80 + k];
        R.D(F_ACC + 9 + k) = g[83 + k];
      }
      R.D(F_ZMP + 6) = g[42];
      R.D(F_ZMP + 7) = g[43];
      R.D(F_ZMP + 9) = g[76];
      R.D(F_ZMP + 10) = g[77];
      R.D(F_DCM + 6) = g[44];
      R.D(F_DCM + 7) = g[45];
      R.D(F_DCM + 9) = g[78];
      R.D(F_DCM + 10) = g[79];
    }
    cnt = 0;
    R.I(I_FLAGOLD) = flag;
  }
  R.I(I_INT) = cnt;
}

// body_theta_mpc reference record slot k (RF_* layout) of robot R, from the
// generator outputs (gait_fast.cpp:568-616): zmp from zmp_inter, rfoot row 0
// = the y entry (assigned twice, :585-586) and row 1 never set, lfoot x/y,
// body angle = (right + left foot rotation) / 5, comacc row 2 only
__device__ __forceinline__ double ref_slot(const Robot &R, const double *ctrl, int k) {
  if (k < RF_ZMP) return ctrl[k < 2 ? 10 + k : 11 + k];  // state_feedback(10, 11, 13, 14)
  if (k < RF_ANG) {
    const int e = k - RF_ZMP, j = e >> 1, rr = e & 1;
    return j == 0 ? R.D(F_ZINT + rr) : R.D(F_ZINT + 8 + 3 * j - 2 + rr);
  }
  if (k < RF_RFT) {
    const int e = k - RF_ANG, j = e >> 1, rr = e & 1;
    return (R.D(F_FTHETA + j * 6 + rr) + R.D(F_FTHETA + j * 6 + 3 + rr)) / 5;
  }
  if (k < RF_LFT) {
    const int e = k - RF_RFT, j = e >> 1, rr = e & 1;
    return rr == 0 ? R.D(F_FOORPR + j * 6 + 1) : 0.0;
  }
  if (k < RF_ACC) {
    const int e = k - RF_LFT, j = e >> 1, rr = e & 1;
    return R.D(F_FOORPR + j * 6 + 3 + rr);
  }
  const int e = k - RF_ACC, j = e / 3, rr = e - 3 * j;
  if (rr != 2) return 0.0;
  return j == 0 ? R.D(F_CACC + 2) : R.D(F_CACC + 8 + 3 * j);
}

constexpr int PRE_R = 64;           // robots per block (one state tile)
constexpr int PRE_T = 2 * PRE_R;    // wave 0: callbacks + interpolation, wave 1: foot generators
constexpr int STG_C = 16;           // slots per transpose chunk
constexpr int STG_LD = 17;          // LDS row stride (doubles): odd, conflict-free column reads

// One tile of 64 robots per block, two waves: the loop counters, the
// published state and the four cubic interpolations (wave 0) and the foot
// trajectory / rotation generators (wave 1) read and write disjoint fields,
// so they run side by side; what both need from the previous tick
// (count_in_mpc, _t_end_footstep) is read before either writes.  Then both
// waves write the body-MPC reference records, row-coalesced through LDS.
__global__ __launch_bounds__(PRE_T) void rt_pre_kernel(const RtArgs a) {
  __shared__ double stage[PRE_R * STG_LD];
  const int tid = threadIdx.x, rr = tid & (PRE_R - 1), role = tid >> 6;
  const int64_t B = a.B, r0 = (int64_t)blockIdx.x * PRE_R;
  const int nb = (int)((B - r0) < PRE_R ? (B - r0) : PRE_R);
  const int64_t r = r0 + rr;
  const bool live = rr < nb;
  const Ws L = layout(B);
  Robot R(a.ws, L, r);
  const double *ctrl = a.ctrl + r * QLOCO_CTRL_MSG_LEN;
  const double *g = a.gait + r * QLOCO_GAIT_MSG_LEN;
  double *body = reinterpret_cast<double *>(a.ws + L.body) + r * QLOCO_BODY_STATE_LEN;
  // callbacks (:79-110): the loop body runs when /control2rtmpc/state[0] > 0,
  // the MPC part when mpc_gait_flag = (int)/MPC/Gait[99] > 0
  bool pub = false, walk = false;
  int flag = 0, mpc = 0, t_end = 0;
  if (live) {
    flag = (int)g[99];
    pub = ctrl[0] > 0;
    walk = pub && flag > 0;
    if (walk) {
      mpc = R.I(I_MPC) + 1;
      t_end = R.I(I_TEND);
    }
  }
  __syncthreads();  // both waves have read the previous tick's counters
  if (live && role == 0) {
    if (pub) {
      const int loop = R.I(I_LOOP) + 1;
      R.I(I_LOOP) = loop;
      const int t_int = (int)((uint32_t)R.I(I_TINT) + (uint32_t)(int)floor((double)(loop / 2)));
      R.I(I_TINT) = t_int;
      R.D(F_NRT + 0) = t_int;  // state_to_MPC = state_feedback (:519-527)
      for (int k = 1; k < 25; ++k) R.D(F_NRT + k) = ctrl[k];
      if (walk) {
        R.I(I_MPC) = mpc;
        interpolation(a, R, g, flag, t_int, t_end);
        R.D(F_ZMP + 8) = 0.0;  // zmpxyz_ref(2) = _Zsc = {l,r}foot_inter(2) = 0 (:557-566)
        *(reinterpret_cast<int32_t *>(a.ws + L.bi) + r) = mpc;
      }
    }
    *(reinterpret_cast<int32_t *>(a.ws + L.run) + r) = walk ? 1 : 0;
  }
  if (live && role == 1 && walk && mpc * DT_FAST > 1.0) {  // _height_offset_timex = 1 (:537-545)
    double nrt[9];
    for (int k = 0; k < 9; ++k) nrt[k] = g[86 + k];
    const int foot_i = (int)(mpc - (int)1.0 / DT_FAST);
    int bjx1 = (int)body[26], bjxx = R.I(I_BJXX), te = t_end;
    int sxx[NH], sx1[NH];
    foot_traj_mod2(R, foot_i, nrt, bjx1, bjxx, te, sxx, sx1);
    foot_rotation(R, foot_i, bjx1, bjxx, te, sxx, sx1);
    body[26] = bjx1;
    R.I(I_BJXX) = bjxx;
    R.I(I_TEND) = te;
  }
  __syncthreads();  // the foot generator's fields are visible to wave 0
  if (live && role == 0 && walk) {
    // body_thetax(0..1) = bodyangle_mpc_ref(:, 0) (:590-591)
    R.D(F_BTHX + 0) = (R.D(F_FTHETA + 0) + R.D(F_FTHETA + 3)) / 5;
    R.D(F_BTHX + 1) = (R.D(F_FTHETA + 1) + R.D(F_FTHETA + 4)) / 5;
  }
  // the reference record of every robot (read by body_mpc_kernel only where
  // run = 1), written row-coalesced; the two waves take alternate slots
  double *ref = reinterpret_cast<double *>(a.ws + L.ref);
#pragma unroll
  for (int c0 = 0; c0 < RF_USED; c0 += STG_C) {
    const int w = (RF_USED - c0) < STG_C ? (RF_USED - c0) : STG_C;
    if (live)
#pragma unroll
      for (int j = 0; j < STG_C; ++j)
        if (j < w && (j & 1) == role) stage[rr * STG_LD + j] = ref_slot(R, ctrl, c0 + j);
    __syncthreads();
    for (int idx = tid; idx < nb * w; idx += PRE_T) {
      const int q = idx / w, j = idx - q * w;
      ref[(r0 + q) * RF_LD + c0 + j] = stage[q * STG_LD + j];
    }
    __syncthreads();
  }
}

// /rtMPC/traj slot k in [36, 100) of robot R: low_mpc_gait_inte(k - 36)
// (gait_fast.cpp:633-714), the untouched [87, 98), (int)_tx_total/0.001 and
// the loop count (:727-729)
__device__ __forceinline__ double traj_slot(const Robot &R, const double *body, double g27,
                                            int k) {
  const int u = k - 36;
  if (u < 3) return R.D(F_RPY + u);                       // rpy_mpc_body
  if (u < 5) return R.D(F_BTHX + u - 3);                  // body_thetax(0..1)
  if (u == 5) return 0.0;                                 // body_thetax(2)
  if (u < 9) return R.D(F_FOORPR + 3 + (u - 6));          // left foot
  if (u < 12) return R.D(F_FOORPR + (u - 9));             // right foot
  if (u < 14) return R.D(F_ZINT + u - 12);                // zmp_inter(0..1)
  if (u == 14) return R.D(F_ZMP + 8);                     // zmpxyz_ref(2)
  if (u < 27) return 0.0;                                 // F_L, F_R, M_L, M_R
  if (u == 27) return g27;                                // bjx1 of /MPC/Gait[27]
  if (u < 31) return R.D(F_FTHETA + 3 + (u - 28));        // left foot rpy
  if (u < 34) return R.D(F_FTHETA + (u - 31));            // right foot rpy
  if (u < 36) return R.D(F_DINT + u - 34);                // dcm_inter(0..1)
  if (u < 50) return body[12 + (u - 36)];                 // bodyangle_mpc
  if (u == 50) return 0.0;                                // t_fast_mpc (wall clock)
  if (k < 98) return 0.0;
  if (k == 98) return (int)R.D(F_TXTOT) / 0.001;          // (int) _tx_total / t_program_cyclic
  return R.I(I_LOOP);                                     // count_in_rt_loop
}

constexpr int POST_R = 64;             // robots per block (one state tile)
constexpr int POST_P = 4;              // waves per block: slot quarters
constexpr int POST_T = POST_R * POST_P;
constexpr int POST_LD = 65;            // LDS row stride (doubles), odd

// Wave p of the block computes its quarter of the slots for the block's 64
// robots (one state tile: every field read is one coalesced 512-byte row),
// into an LDS copy of the rows; the block then writes whole rows (a wave
// stores 512 contiguous bytes).  Four waves per 64 robots keep four times
// the memory requests in flight of one-robot-per-lane-for-all-slots.
template <int P>
__device__ __forceinline__ void post_part(const Robot &R, const double *body, double g27,
                                          double *st, int rr, bool live) {
  if (!live) return;
#pragma unroll
  for (int j = 0; j < 16; ++j) st[rr * POST_LD + 16 * P + j] = traj_slot(R, body, g27, 36 + 16 * P + j);
}

__global__ __launch_bounds__(POST_T) void rt_post_kernel(const RtArgs a) {
  __shared__ double stage[POST_R * POST_LD];
  const int tid = threadIdx.x, rr = tid & (POST_R - 1), part = tid >> 6;
  const int64_t B = a.B, r0 = (int64_t)blockIdx.x * POST_R;
  const int nb = (int)((B - r0) < POST_R ? (B - r0) : POST_R);
  const int64_t r = r0 + rr;
  const bool live = rr < nb;
  const Ws L = layout(B);
  Robot R(a.ws, L, r);
  const double *body = reinterpret_cast<const double *>(a.ws + L.body) + r * QLOCO_BODY_STATE_LEN;
  // [0, 36): the /MPC/Gait rows copied through (:716-719)
  for (int idx = tid; idx < nb * 36; idx += POST_T) {
    const int q = idx / 36, k = idx - q * 36;
    a.traj[(r0 + q) * QLOCO_TRAJ_MSG_LEN + k] = a.gait[(r0 + q) * QLOCO_GAIT_MSG_LEN + k];
  }
  // [36, 100): low_mpc_gait_inte etc., a quarter per wave
  const double g27 = live ? a.gait[r * QLOCO_GAIT_MSG_LEN + 27] : 0.0;
  switch (part) {  // wave-uniform
    case 0: post_part<0>(R, body, g27, stage, rr, live); break;
    case 1: post_part<1>(R, body, g27, stage, rr, live); break;
    case 2: post_part<2>(R, body, g27, stage, rr, live); break;
    default: post_part<3>(R, body, g27, stage, rr, live); break;
  }
  __syncthreads();
  for (int idx = tid; idx < nb * 64; idx += POST_T) {
    const int q = idx >> 6, j = idx & 63;
    a.traj[(r0 + q) * QLOCO_TRAJ_MSG_LEN + 36 + j] = stage[q * POST_LD + j];
  }
  __syncthreads();
  // /rt2nrt/state (last published state_to_MPC): slots k = part + 4i
  if (live)
    for (int k = part; k < 25; k += POST_P) stage[rr * POST_LD + k] = R.D(F_NRT + k);
  __syncthreads();
  for (int idx = tid; idx < nb * 25; idx += POST_T) {
    const int q = idx / 25, j = idx - q * 25;
    a.nrt[(r0 + q) * QLOCO_NRT_MSG_LEN + j] = stage[q * POST_LD + j];
  }
  if (a.gen) {  // debug dump: foorpr_gen | foortheta_gen (contiguous fields)
    __syncthreads();
    if (live)
      for (int k = part; k < 60; k += POST_P) stage[rr * POST_LD + k] = R.D(F_FOORPR + k);
    __syncthreads();
    for (int idx = tid; idx < nb * 60; idx += POST_T) {
      const int q = idx / 60, j = idx - q * 60;
      a.gen[(r0 + q) * 60 + j] = stage[q * POST_LD + j];
    }
  }
  if (a.sched && live && part == 0) {
    const int32_t run = *(reinterpret_cast<const int32_t *>(a.ws + L.run) + r);
    const int32_t bst = *(reinterpret_cast<const int32_t *>(a.ws + L.st) + r);
    const double *ctrl = a.ctrl + r * QLOCO_CTRL_MSG_LEN;
    int32_t *sp = a.sched + r * QLOCO_RT_SCHED_LEN;
    sp[0] = (int32_t)body[26];
    sp[1] = R.I(I_BJXX);
    sp[2] = R.I(I_TEND);
    sp[3] = R.I(I_MPC);
    sp[4] = R.I(I_TINT);
    sp[5] = run ? bst : -1;
    sp[6] = ctrl[0] > 0 ? 1 : 0;
    sp[7] = (int32_t)body[27];
  }
}

// PRMPCClass() + Initialize() + gait_fast.cpp main() init (:384-502)
__global__ __launch_bounds__(256) void rt_init_kernel(int64_t B, char *ws) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  const Ws L = layout(B);
  Robot R(ws, L, r);
  for (int f = 0; f < F_DOUBLES; ++f) R.D(f) = 0.0;
  for (int f = 0; f < I_INTS; ++f) R.I(f) = 0;
  double *body = reinterpret_cast<double *>(ws + L.body) + r * QLOCO_BODY_STATE_LEN;
  for (int k = 0; k < QLOCO_BODY_STATE_LEN; ++k) body[k] = 0.0;
  body[29] = 1.0;  // qp_solution
  // FootStepInputs(2 * half_hip, 0, 0, 0.015) (:48-53, :2198-2222)
  const double lift = 0.015;
  for (int i = 0; i < NS; ++i) R.D(F_LIFT + i) = lift;
  R.D(F_LIFT + NS - 1) = 0;
  R.D(F_LIFT + NS - 2) = 0;
  R.D(F_LIFT + NS - 3) = lift / 2;
  R.D(F_LIFT + NS - 4) = lift;
  double fy = 0;  // _footxyz_real (:111-123); x and z stay 0 (steplength = stepheight = 0)
  for (int i = 1; i < NS; i++) {
    const double sw = (i - 1 == 0) ? STEPWIDTH0 : 2 * HALF_HIP;
    fy = fy + (int)pow(-1.0, (double)(i - 1)) * sw;
    R.fxyz(1, i) = fy;
  }
  for (int k = 0; k < 6; ++k) {  // :131-138
    R.foot(LY, k) = STEPWIDTH0;
    R.foot(RY, k) = -STEPWIDTH0;
  }
  for (int i = 0; i < NS; ++i) R.D(F_TS + i) = TSTEP;  // :168-185
  recompute_tx(R);
  R.I(I_TEND) = (int)round((R.D(F_TX + NS - 1) - 3 * TSTEP) / DT_FAST);
  R.D(F_TXTOT) = R.D(F_TX + NS - 1);
  const double z_c = 0.309458;  // gait::RobotPara_Z_C (gait_fast.cpp:391-395)
  R.D(F_COM + 2) = R.D(F_COM + 5) = R.D(F_COM + 8) = R.D(F_COM + 11) = z_c;
  R.D(F_RPY + 2) = z_c;
  for (int j = 0; j < 5; j++) {  // :492-496
    R.D(F_FOORPR + 1 + 6 * j) = -HALF_HIP;
    R.D(F_FOORPR + 4 + 6 * j) = HALF_HIP;
  }
}

// Slow planner's contact-phase flag (mosek_nlp_kmp NLPClass; oracle/
// support_phase.c): bjxx / bjx1 from the planner's own _tx after its
// step-timing SQP (NLPClass_sqp.cpp:1029-1039, Indexfind :1105-1142 with
// xyz1, bounded at 27) and Foot_trajectory_solve_mod2's right_support
// (:2076-2090, :2187-2202, :2311-2313).  64 robots per block: the block's
// _ts / _tx rows (27 doubles each, contiguous for consecutive robots) are
// staged through LDS by all 256 threads with coalesced 16-byte loads (a
// 64-robot row block is 13.8 KB, 16-byte aligned), then one lane per robot
// runs the scan out of LDS.
constexpr int SP_T = 64;    // robots per block
constexpr int SP_TH = 256;  // threads per block: 4 per robot for the row loads
constexpr double SP_DT = 0.025;  // NLPClass.h:32
__global__ __launch_bounds__(SP_TH) void support_phase_kernel(int64_t B, const double *ts,
                                                              const double *tx,
                                                              const int32_t *t_int,
                                                              const int32_t *t_end,
                                                              int32_t *bjxx, int32_t *bjx1,
                                                              int32_t *rs) {
  __shared__ __attribute__((aligned(16))) double sts[SP_T * NS], stx[SP_T * NS];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * SP_T;
  const int nb = (int)((B - r0) < SP_T ? (B - r0) : SP_T);
  if (nb == SP_T) {  // whole block: 16-byte loads, all issued before the LDS stores
    constexpr int NV = SP_T * NS / 2, PER = (NV + SP_TH - 1) / SP_TH;
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v *gs = reinterpret_cast<const d2v *>(ts + r0 * NS);
    const d2v *gx = reinterpret_cast<const d2v *>(tx + r0 * NS);
    d2v vs[PER], vx[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int k = tid + q * SP_TH;
      if (k < NV) {
        vs[q] = __builtin_nontemporal_load(gs + k);
        vx[q] = __builtin_nontemporal_load(gx + k);
      }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int k = tid + q * SP_TH;
      if (k < NV) {
        reinterpret_cast<d2v *>(sts)[k] = vs[q];
        reinterpret_cast<d2v *>(stx)[k] = vx[q];
      }
    }
  } else {
    for (int k = tid; k < nb * NS; k += SP_TH) {
      sts[k] = ts[r0 * NS + k];
      stx[k] = tx[r0 * NS + k];
    }
  }
  __syncthreads();
  if (tid >= nb) return;
  const int64_t r = r0 + tid;
  const double *x = stx + tid * NS;
  const int i = t_int[r];
  auto find = [&](double goal) {
    int j = 0;
    while (j < NS && goal >= x[j]) j++;
    return j - 1;
  };
  const int bxx = find(i * SP_DT) + 1;
  const int b1 = find((i + 1) * SP_DT) + 1;
  int f = 2;
  if (b1 >= 2 && i <= t_end[r]) {
    const double td = 0.2 * sts[tid * NS + b1 - 1];
    f = (b1 % 2 == 0) ? 0 : 1;
    if ((i + 1 - round(x[b1 - 1] / SP_DT)) * SP_DT < td) f = 2;
  }
  if (bjxx) bjxx[r] = bxx;
  if (bjx1) bjx1[r] = b1;
  rs[r] = f;
}

static void aaa_inv_mod(double out[16]) {  // :1344-1362
  const double t[4] = {-DT_SLOW, 0, DT_SLOW, 2 * DT_SLOW};
  double A[16], Ai[16];
  for (int r = 0; r < 4; ++r) {
    A[r * 4 + 0] = cube(t[r]);
    A[r * 4 + 1] = sq(t[r]);
    A[r * 4 + 2] = (t[r]);
    A[r * 4 + 3] = 1;
  }
  inv4(A, Ai);
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) out[c * 4 + r] = Ai[r * 4 + c];
}

}  // namespace rt
}  // namespace qloco

using namespace qloco;

extern "C" int64_t qloco_rt_workspace_bytes(int64_t batch) {
  if (batch < 0) return -1;
  return rt::layout(batch).total;
}

extern "C" int qloco_rt_init(int64_t batch, void *workspace, void *stream) {
  if (batch < 0 || (batch > 0 && !workspace)) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  hipLaunchKernelGGL(rt::rt_init_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, batch, (char *)workspace);
  QLOCO_HIP_CHECK(hipGetLastError(), "rt_init_kernel launch");
  return QLOCO_OK;
}

extern "C" int qloco_rt_tick(int64_t batch, void *workspace, const double *gait_msg,
                             const double *ctrl_msg, double *traj_msg, double *nrt_msg,
                             double *gen, int32_t *sched, void *stream) {
  if (batch < 0) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  if (!workspace || !gait_msg || !ctrl_msg || !traj_msg || !nrt_msg) return QLOCO_ERR_ARG;
  if (batch > (int64_t)0x7fffffff * 64) return QLOCO_BAD_SIZE;
  rt::RtArgs a;
  memset(&a, 0, sizeof(a));
  a.B = batch;
  a.ws = (char *)workspace;
  a.gait = gait_msg;
  a.ctrl = ctrl_msg;
  a.traj = traj_msg;
  a.nrt = nrt_msg;
  a.gen = gen;
  a.sched = sched;
  rt::aaa_inv_mod(a.aaa_inv_mod);
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(rt::rt_pre_kernel, dim3((unsigned)((batch + rt::PRE_R - 1) / rt::PRE_R)),
                     dim3(rt::PRE_T), 0, s, a);
  QLOCO_HIP_CHECK(hipGetLastError(), "rt_pre_kernel launch");
  const rt::Ws L = rt::layout(batch);
  char *w = (char *)workspace;
  const int rc = body_mpc_launch(
      batch, (const int32_t *)(w + L.bi), (const double *)(w + L.ref) + rt::RF_BAS,
      (const double *)(w + L.ref) + rt::RF_ZMP, (const double *)(w + L.ref) + rt::RF_ANG,
      (const double *)(w + L.ref) + rt::RF_RFT, (const double *)(w + L.ref) + rt::RF_LFT,
      (const double *)(w + L.ref) + rt::RF_ACC, (double *)(w + L.body),
      (double *)(w + L.ct), (int32_t *)(w + L.st),
      (const double *)(w + L.d) + rt::F_TX * rt::TL, rt::TL, rt::F_DOUBLES * rt::TL,
      (const int32_t *)(w + L.run), rt::RF_LD, s);
  if (rc != QLOCO_OK) return rc;
  hipLaunchKernelGGL(rt::rt_post_kernel, dim3((unsigned)((batch + rt::POST_R - 1) / rt::POST_R)),
                     dim3(rt::POST_T), 0, s, a);
  QLOCO_HIP_CHECK(hipGetLastError(), "rt_post_kernel launch");
  return QLOCO_OK;
}

extern "C" int qloco_support_phase(int64_t batch, const double *ts, const double *tx,
                                   const int32_t *t_int, const int32_t *t_end_footstep,
                                   int32_t *bjxx, int32_t *bjx1, int32_t *right_support,
                                   void *stream) {
  if (batch < 0) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  if (!ts || !tx || !t_int || !t_end_footstep || !right_support) return QLOCO_ERR_ARG;
  if (batch > (int64_t)0x7fffffff * rt::SP_T) return QLOCO_BAD_SIZE;
  hipLaunchKernelGGL(rt::support_phase_kernel,
                     dim3((unsigned)((batch + rt::SP_T - 1) / rt::SP_T)), dim3(rt::SP_TH), 0,
                     (hipStream_t)stream, batch, ts, tx, t_int, t_end_footstep, bjxx, bjx1,
                     right_support);
  QLOCO_HIP_CHECK(hipGetLastError(), "support_phase_kernel launch");
  return QLOCO_OK;
}
