// qloco_body.hip -- batched rt body-inclination MPC step (gfx950).
//
// Replaces PRMPCClass::body_theta_mpc (rt_mpc_qp/src/FastMPC/
// PRMPCClass.cpp:379-714) + Indexfind (:716-738) + solve_body_rotation /
// Solve (:799-849), called at 100 Hz from gait_fast.cpp:620.  Constants of
// PRMPCClass::Initialize (:157-374) are computed once on the host
// (body_constants) and passed by value.  One instance per 8-lane group:
// the group derives the schedule integers (bjx1, bjx2, t_yu -- fp64 compares,
// bit-exact), builds the 8-variable QP in LDS, solves it with the
// Goldfarb-Idnani core and applies the reference's clamping, propagation and
// (all-zero) lambda feedback.  The 16 CI columns the reference never writes
// (:813-816, :826-829) are zero, i.e. inert.
#include <math.h>
#include <string.h>

#include <mutex>

#include "qloco_gi_core.hpp"

namespace qloco {

constexpr int BNH = 4;               // _nh
constexpr int BNT = 2 * BNH;         // _Nt
constexpr int BNI = 12 * BNH;        // resizeQP(_Nt, 0, 12*_nh)
constexpr int BSTEPS = 27;           // _footstepsnumber

struct BodyConsts {
  double tx[BSTEPS];
  int nsum_mpc, nstepx;
  double dt_mpc, j_ini, mass, g;
  double a[4], b[2];
  double pps[BNH * 2], pvs[BNH * 2], ppu[BNH * BNH], pvu[BNH * BNH], ppu_2[BNH * BNH],
      pvu_2[BNH * BNH];
  double thetax_max, thetax_min, thetay_max, thetay_min, torque_max, torque_min;
  double Rthetax, Rthetay, alphathetax, alphathetay, beltathetax, beltathetay, gama_zmpx,
      gama_zmpy;
};

static void mat2_mul(const double A[4], const double B[4], double C[4]) {
  const double c00 = A[0] * B[0] + A[2] * B[1];
  const double c10 = A[1] * B[0] + A[3] * B[1];
  const double c01 = A[0] * B[2] + A[2] * B[3];
  const double c11 = A[1] * B[2] + A[3] * B[3];
  C[0] = c00;
  C[1] = c10;
  C[2] = c01;
  C[3] = c11;
}

// PRMPCClass::Initialize, QP part (PRMPCClass.cpp:157-374) with the gait::
// constants of rt_mpc_qp/src/Robotpara/robot_const_para_config.cpp:8-47.
static void body_constants(BodyConsts &c) {
  memset(&c, 0, sizeof(c));
  const double dt_slow = 0.025, dt_fast = 0.01, tstep = 0.7;
  c.dt_mpc = dt_fast;
  c.j_ini = 12 * 0.1 * 0.1;
  c.mass = 12;
  c.g = 9.8;
  c.tx[0] = 0.0;
  for (int i = 1; i < BSTEPS; i++) {  // :174-178
    c.tx[i] = c.tx[i - 1] + tstep;
    c.tx[i] = round(c.tx[i] / dt_slow) * dt_slow - 0.00001;
  }
  c.nstepx = (int)round(tstep / dt_fast);                   // :172
  c.nsum_mpc = (int)floor(c.tx[BSTEPS - 1] / dt_fast);      // :185
  c.a[0] = 1;
  c.a[1] = 0;
  c.a[2] = dt_fast;
  c.a[3] = 1;
  c.b[0] = pow(dt_fast, 2) / 2;
  c.b[1] = dt_fast;
  const double cp[2] = {1, 0}, cv[2] = {0, 1};
  for (int pass = 0; pass < 2; ++pass) {  // Matrix_ps (:741-763)
    const double *cc = pass == 0 ? cp : cv;
    double *out = pass == 0 ? c.pps : c.pvs;
    for (int i = 0; i < BNH; i++) {
      double A[4] = {1, 0, 0, 1};
      for (int j = 1; j < i + 2; j++) mat2_mul(A, c.a, A);
      out[0 * BNH + i] = cc[0] * A[0] + cc[1] * A[1];
      out[1 * BNH + i] = cc[0] * A[2] + cc[1] * A[3];
    }
  }
  for (int pass = 0; pass < 2; ++pass) {  // Matrix_pu (:765-796)
    const double *cc = pass == 0 ? cp : cv;
    double *out = pass == 0 ? c.ppu : c.pvu;
    for (int i = 1; i < BNH + 1; i++)
      for (int j = 1; j < i + 1; j++) {
        double A[4] = {1, 0, 0, 1};
        if (j != i)
          for (int k = 1; k < i - j + 1; k++) mat2_mul(A, c.a, A);
        const double ca0 = cc[0] * A[0] + cc[1] * A[1];
        const double ca1 = cc[0] * A[2] + cc[1] * A[3];
        out[(j - 1) * BNH + (i - 1)] = ca0 * c.b[0] + ca1 * c.b[1];
      }
  }
  for (int cc = 0; cc < BNH; ++cc)  // :219-220
    for (int r = 0; r < BNH; ++r) {
      double a1 = 0, a2 = 0;
      for (int k = 0; k < BNH; ++k) {
        a1 += c.pvu[r * BNH + k] * c.pvu[cc * BNH + k];
        a2 += c.ppu[r * BNH + k] * c.ppu[cc * BNH + k];
      }
      c.pvu_2[cc * BNH + r] = a1;
      c.ppu_2[cc * BNH + r] = a2;
    }
  c.thetax_max = 10 * M_PI / 180;
  c.thetax_min = -10 * M_PI / 180;
  c.thetay_max = 10 * M_PI / 180;
  c.thetay_min = -10 * M_PI / 180;
  c.torque_max = 20 / c.j_ini;
  c.torque_min = -20 / c.j_ini;
  c.Rthetax = 100;  // go1 weights, :280-287
  c.Rthetay = 100;
  c.alphathetax = 10;
  c.alphathetay = 10;
  c.beltathetax = 5000000000.0;
  c.beltathetay = 5000000000.0;
  c.gama_zmpx = 5000;
  c.gama_zmpy = 5000;
}

struct BodyArgs {
  BodyConsts k;
  int64_t batch;
  const int *i;
  const double *bodyangle_state, *zmp_ref, *angle_ref, *rfoot_ref, *lfoot_ref, *comacc_ref;
  double *state, *com_traj;
  int *status;
  // rt node tick (qloco_rt.hip): the robot's own _tx (Foot_trajectory_solve_mod2
  // rewrites it, PRMPCClass.cpp:1773-1779) at tx[j * tx_stride + inst] or,
  // with tx_tile > 0 (the rt workspace's 64-robot tiles), at
  // tx[(inst / 64) * tx_tile + j * tx_stride + inst % 64], and a mask of the
  // robots whose loop calls body_theta_mpc this tick.  NULL: the Initialize()
  // schedule for every instance / all run.
  const double *tx;
  int64_t tx_stride, tx_tile;
  const int32_t *run;
  // row stride (doubles) of the reference arrays: 0 = packed (4 / 10 / 15);
  // the rt tick keeps all of a robot's references in one 64-double record
  int64_t ref_ld;
};

// constant inequality rows (:541-561, :805-812): CI(:, c) = -[q_upx' q_lowx'
// q_upy' q_lowy' t_upx' t_lowx' t_upy' t_lowy'], columns 32..47 zero.  The
// same for every robot, so it lives in constant memory (set once per device)
// rather than in each workgroup's LDS.
__constant__ double c_body_CI[BNT * BNI];
// The Initialize() constants, also in constant memory: as a by-value kernel
// argument the dynamically indexed struct was materialised in VGPRs.
__constant__ BodyConsts c_body_K;

// Eight robots per wave: one 8-lane Goldfarb-Idnani group per robot, a lane
// per variable (BNT = 8; qloco_gi_core.hpp's results do not depend on the
// group width).
constexpr int kBodyGW = 8, kBodyGroups = 64 / kBodyGW;
struct BodyLds {
  struct Grp {
    double g0[BNT], ci0[BNI], x[BNT];  // G is built in gi.J (read once, before J is formed)
    GiLdsT<BNT, BNI, 0> gi;
  } g[kBodyGroups];
};

// PRMPCClass::Indexfind, xyz = 0 branch (:716-738)
__device__ __forceinline__ int indexfind(const BodyConsts &k, double goal) {
  int j = 0;
  while (j < BSTEPS && goal >= k.tx[j]) j++;
  return j - 1;
}

#define R2(m, r, c) ((m)[(c)*2 + (r)])
#define R3(m, r, c) ((m)[(c)*3 + (r)])

// 2-waves/SIMD register floor (no spills); the LDS of an 8-robot block sets
// the resident waves
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void body_mpc_kernel(const BodyArgs a) {
  __shared__ BodyLds S;
  const BodyConsts &K = c_body_K;
  const int lane = threadIdx.x, grp = lane / kBodyGW, li = lane % kBodyGW;
  const int64_t inst = (int64_t)blockIdx.x * kBodyGroups + grp;
  if (inst >= a.batch) return;
  BodyLds::Grp &P = S.g[grp];
  double *st = a.state + inst * QLOCO_BODY_STATE_LEN;
  const int64_t l10 = a.ref_ld ? a.ref_ld : 10, l15 = a.ref_ld ? a.ref_ld : 15;
  const double *zmp_ref = a.zmp_ref + inst * l10, *angle_ref = a.angle_ref + inst * l10;
  const double *rfoot_ref = a.rfoot_ref + inst * l10, *lfoot_ref = a.lfoot_ref + inst * l10;
  const double *comacc_ref = a.comacc_ref + inst * l15;
  double thetaxk[2] = {st[0], st[1]}, thetayk[2] = {st[2], st[3]};
  int i = a.i[inst];
  int status = QLOCO_OK;
  bool active = false;
  const int off = (int)round(1.0 / K.dt_mpc);  // height_offset_time / dt (:395)
  int bjx1 = (int)st[26], bjx2 = (int)st[27], t_yu = (int)st[28];
  const bool run = a.run ? a.run[inst] != 0 : true;
  if (run && i >= off) {
    i -= off;
    active = i < (K.nsum_mpc - BNH);  // :403
  }
  if (active) {
    const double t_f0 = (i + 1) * K.dt_mpc, t_f3 = (i + BNH) * K.dt_mpc;  // :406
    if (a.tx) {
      // the robot's _tx: lane li of the group holds entries li + 8 q
      // (q < 4), loaded together; Indexfind's stopping index (the first j
      // with goal < _tx(j), 27 if none) is the lowest set bit of the group's
      // ballots -- the same answer as the scan for any _tx, one load round trip
      const double *txr = a.tx + (a.tx_tile > 0 ? (inst >> 6) * a.tx_tile + (inst & 63) : inst);
      constexpr int TQ = (BSTEPS + kBodyGW - 1) / kBodyGW;
      double tq[TQ];
#pragma unroll
      for (int q = 0; q < TQ; ++q) tq[q] = (li + kBodyGW * q < BSTEPS) ? txr[(li + kBodyGW * q) * a.tx_stride] : 0.0;
      auto first_below = [&](double goal) {
        int j = BSTEPS;
#pragma unroll
        for (int q = TQ - 1; q >= 0; --q) {
          const uint64_t m = (__ballot(li + kBodyGW * q < BSTEPS && goal < tq[q]) >> (kBodyGW * grp)) &
                             ((1ull << kBodyGW) - 1);
          if (m) j = kBodyGW * q + __builtin_ctzll(m);
        }
        return j;
      };
      bjx1 = first_below(t_f0);  // Indexfind + 1 = stopping index
      bjx2 = first_below(t_f3);
    } else {
      bjx1 = indexfind(K, t_f0) + 1;
      bjx2 = indexfind(K, t_f3) + 1;
    }
    t_yu = (i + 1) % K.nstepx;
    double copx[BNH], copy[BNH];
    const double *sup = lfoot_ref, *oth = rfoot_ref;  // CoP reference, :427-499
    if (bjx1 >= 2 && (bjx1 % 2 != 0)) {
      sup = rfoot_ref;
      oth = lfoot_ref;
    }
    for (int k = 0; k < BNH; ++k) {
      copx[k] = R2(sup, 0, k);
      copy[k] = R2(sup, 1, k);
    }
    if (bjx1 >= 2 && !((t_yu + BNH - 1) < K.nstepx)) {
      const int t_yu_k = (t_yu + BNH) - K.nstepx;
      for (int jx = 1; jx <= t_yu_k; jx++) {
        copx[BNH - jx] = R2(oth, 0, BNH - jx);
        copy[BNH - jx] = R2(oth, 1, BNH - jx);
      }
    }
    double pth[BNH];
    for (int jx = 0; jx < BNH; jx++) pth[jx] = K.j_ini / (K.mass * (R3(comacc_ref, 2, jx) + K.g));
    // QP data (:505-535), entry sets spread over the 8-lane group (each
    // entry computed exactly as the serial loops of the reference do)
#pragma unroll
    for (int e = li; e < 2 * kBodyGW; e += kBodyGW) {
      const int r = e & 3, c = e >> 2;  // G: entry (r, c) of the two 4x4 blocks
      const double I = (r == c) ? 1.0 : 0.0;  // :511-515
      double pp = pth[r] * pth[c];
      if (r != c) pp = 0.0;
      const double wx = K.Rthetax / 2 * I + K.alphathetax / 2 * K.pvu_2[c * BNH + r] +
                        K.beltathetax / 2 * K.ppu_2[c * BNH + r] + K.gama_zmpy / 2 * pp;
      const double wy = K.Rthetay / 2 * I + K.alphathetay / 2 * K.pvu_2[c * BNH + r] +
                        K.beltathetay / 2 * K.ppu_2[c * BNH + r] + K.gama_zmpx / 2 * pp;
      P.gi.J[c * BNT + r] = 2 * wx;
      P.gi.J[(c + BNH) * BNT + (r + BNH)] = 2 * wy;
      P.gi.J[c * BNT + (r + BNH)] = 0.0;
      P.gi.J[(c + BNH) * BNT + r] = 0.0;
    }
    if (li < BNT) {  // q_goal row li (:523-526): x rows 0..3, y rows 4..7
      const int r = li & 3;
      const bool ya = li >= BNH;
      const double *tk = ya ? thetayk : thetaxk;
      double v = 0, pq = 0, ref = 0;
      for (int k = 0; k < BNH; ++k) {
        const double pvs_t = K.pvs[k] * tk[0] + K.pvs[BNH + k] * tk[1];
        const double pps_t = K.pps[k] * tk[0] + K.pps[BNH + k] * tk[1];
        v += K.pvu[r * BNH + k] * pvs_t;
        pq += K.ppu[r * BNH + k] * pps_t;
        ref += K.ppu[r * BNH + k] * R2(angle_ref, ya ? 1 : 0, k);
      }
      if (!ya) {
        const double det_py = R2(zmp_ref, 1, r) - copy[r];
        P.g0[r] = K.alphathetax * v + K.beltathetax * pq - K.beltathetax * ref +
                  K.gama_zmpy * pth[r] * det_py;
      } else {
        const double det_px = R2(zmp_ref, 0, r) - copx[r];
        P.g0[BNH + r] = K.alphathetay * v + K.beltathetay * pq - K.beltathetay * ref +
                        K.gama_zmpx * (-pth[r]) * det_px;
      }
    }
#pragma unroll
    for (int e = li; e < 2 * kBodyGW; e += kBodyGW) {  // ci0 (:527-535): (row, block pair); entries 32..47 stay 0
      const int row = e & 3, bp = e >> 2;
      const double ppsx = K.pps[row] * thetaxk[0] + K.pps[BNH + row] * thetaxk[1];
      const double ppsy = K.pps[row] * thetayk[0] + K.pps[BNH + row] * thetayk[1];
      double e0, e1;
      if (bp == 0) {
        e0 = K.thetax_max - ppsx;
        e1 = -K.thetax_min + ppsx;
      } else if (bp == 1) {
        e0 = K.thetay_max - ppsy;
        e1 = -K.thetay_min + ppsy;
      } else {
        e0 = K.torque_max;
        e1 = -K.torque_min;
      }
      P.ci0[(2 * bp) * BNH + row] = e0;
      P.ci0[(2 * bp + 1) * BNH + row] = e1;
      P.ci0[8 * BNH + e] = 0.0;
    }
    GI_SYNC();
    double f;
    int it;
    // the serial l2 scan: the butterfly's registers would cost this kernel
    // its third wave per SIMD (176 VGPRs; rt tick +1.3 %, profiles/r6am_gi_l2_butterfly_ab.txt)
    gi_solve_group<kBodyGW, false>(P.gi, li, BNT, 0, BNI, P.gi.J, BNT, P.g0, nullptr, nullptr, c_body_CI, P.ci0, P.x, f,
                   status, it);
    GI_SYNC();
    if (li == 0) {
      bool ok = true;
      for (int k = 0; k < BNT; ++k) ok = ok && !isnan(P.x[k]);
      double V[BNT];
      for (int k = 0; k < BNT; ++k) V[k] = P.x[k];  // Solve: _V_ini = _X (:844-847)
      const double *aa = K.a, *bb = K.b;
      double thax0 = V[0], thay0 = V[BNH];
      const double a0x = aa[0] * thetaxk[0] + aa[2] * thetaxk[1];
      const double a0y = aa[0] * thetayk[0] + aa[2] * thetayk[1];
      if (!ok) {  // :570-579
        thax0 = (thetaxk[0] - a0x) / bb[0];
        thay0 = (thetayk[0] - a0y) / bb[0];
      } else {  // :580-617
        const double nx0 = a0x + bb[0] * thax0;
        if (nx0 > K.thetax_max) thax0 = (K.thetax_max - a0x) / bb[0];
        else if (nx0 < K.thetax_min) thax0 = (K.thetax_min - a0x) / bb[0];
        const double ny0 = a0y + bb[0] * thay0;
        if (ny0 > K.thetay_max) thay0 = (K.thetay_max - a0y) / bb[0];
        else if (ny0 < K.thetay_min) thay0 = (K.thetay_min - a0y) / bb[0];
      }
      V[0] = thax0;
      V[BNH] = thay0;
      const double txk_tmp[2] = {aa[0] * thetaxk[0] + aa[2] * thetaxk[1] + bb[0] * thax0,
                                 aa[1] * thetaxk[0] + aa[3] * thetaxk[1] + bb[1] * thax0};
      const double tyk_tmp[2] = {aa[0] * thetayk[0] + aa[2] * thetayk[1] + bb[0] * thay0,
                                 aa[1] * thetayk[0] + aa[3] * thetayk[1] + bb[1] * thay0};
      double thetax[BNH], thetay[BNH], zmpx[BNH], zmpy[BNH];
      const double torquex0 = K.j_ini * thax0, torquey0 = K.j_ini * thay0;
      for (int jj = 0; jj < BNH; jj++) {  // :636-655
        const double tax = V[jj], tay = V[BNH + jj];
        const double x0 = aa[0] * thetaxk[0] + aa[2] * thetaxk[1] + bb[0] * tax;
        const double x1 = aa[1] * thetaxk[0] + aa[3] * thetaxk[1] + bb[1] * tax;
        thetaxk[0] = x0;
        thetaxk[1] = x1;
        thetax[jj] = x0;
        const double y0 = aa[0] * thetayk[0] + aa[2] * thetayk[1] + bb[0] * tay;
        const double y1 = aa[1] * thetayk[0] + aa[3] * thetayk[1] + bb[1] * tay;
        thetayk[0] = y0;
        thetayk[1] = y1;
        thetay[jj] = y0;
        const double den = K.mass * (K.g + R3(comacc_ref, 2, jj));
        zmpx[jj] = R2(zmp_ref, 0, jj) - K.j_ini * tay / den;
        zmpy[jj] = R2(zmp_ref, 1, jj) + K.j_ini * tax / den;
      }
      thetaxk[0] = txk_tmp[0];
      thetaxk[1] = txk_tmp[1];
      thetayk[0] = tyk_tmp[0];
      thetayk[1] = tyk_tmp[1];
      const double *bs = a.bodyangle_state + inst * (a.ref_ld ? a.ref_ld : 4);  // lambda feedback, all 0 (:664-692)
      const double lx = 0.0, lvx = 0.0, ly = 0.0, lvy = 0.0;
      thetaxk[0] = lx * bs[0] + (1 - lx) * thetaxk[0];
      thetaxk[1] = lvx * bs[1] + (1 - lvx) * thetaxk[1];
      thetayk[0] = (ly * bs[2] + (1 - ly) * thetayk[0]);
      thetayk[1] = (lvy * bs[3] + (1 - lvy) * thetayk[1]);
      st[0] = thetaxk[0];
      st[1] = thetaxk[1];
      st[2] = thetayk[0];
      st[3] = thetayk[1];
      for (int k = 0; k < BNT; ++k) st[4 + k] = V[k];
      const double ct[14] = {thetax[0], thetay[0], torquex0, torquey0, zmpx[0], zmpy[0],
                             thetax[1], thetay[1], zmpx[1],  zmpy[1],  thetax[2], thetay[2],
                             zmpx[2],   zmpy[2]};
      for (int k = 0; k < 14; ++k) st[12 + k] = ct[k];
      st[26] = bjx1;
      st[27] = bjx2;
      st[28] = t_yu;
      st[29] = ok ? 1.0 : 0.0;
    }
  }
  GI_SYNC();
  for (int k = li; k < 14; k += kBodyGW) a.com_traj[inst * 14 + k] = st[12 + k];  // :696-709 (last state otherwise)
  if (li == 0 && a.status) a.status[inst] = active ? status : QLOCO_OK;
}

int body_mpc_launch(int64_t batch, const int32_t *i, const double *bodyangle_state,
                    const double *zmp_ref, const double *angle_ref, const double *rfoot_ref,
                    const double *lfoot_ref, const double *comacc_ref, double *state,
                    double *com_traj, int32_t *status, const double *tx, int64_t tx_stride,
                    int64_t tx_tile, const int32_t *run, int64_t ref_ld, hipStream_t stream);

__global__ void indexfind_kernel(const BodyConsts k, int64_t batch, const double *t, int *j) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < batch) j[idx] = indexfind(k, t[idx]);
}

}  // namespace qloco

using namespace qloco;

extern "C" int qloco_body_state_init_host(int64_t batch, double *state) {
  if (batch < 0 || (batch > 0 && !state)) return QLOCO_ERR_ARG;
  memset(state, 0, sizeof(double) * QLOCO_BODY_STATE_LEN * batch);
  for (int64_t b = 0; b < batch; ++b) state[b * QLOCO_BODY_STATE_LEN + 29] = 1.0;  // qp_solution
  return QLOCO_OK;
}

extern "C" int qloco_body_mpc_step(int64_t batch, const int32_t *i,
                                   const double *bodyangle_state, const double *zmp_ref,
                                   const double *angle_ref, const double *rfoot_ref,
                                   const double *lfoot_ref, const double *comacc_ref,
                                   double *state, double *com_traj, int32_t *status,
                                   void *stream) {
  if (batch < 0) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  if (!i || !bodyangle_state || !zmp_ref || !angle_ref || !rfoot_ref || !lfoot_ref ||
      !comacc_ref || !state || !com_traj)
    return QLOCO_ERR_ARG;
  return body_mpc_launch(batch, i, bodyangle_state, zmp_ref, angle_ref, rfoot_ref, lfoot_ref,
                         comacc_ref, state, com_traj, status, nullptr, 0, 0, nullptr, 0,
                         (hipStream_t)stream);
}

// c_body_CI / c_body_K from the Initialize() constants, once per device
static int body_ci_upload(const BodyConsts &K) {
  static std::mutex mu;
  static bool done[256] = {};
  int dev = 0;
  QLOCO_HIP_CHECK(hipGetDevice(&dev), "hipGetDevice");
  std::lock_guard<std::mutex> lock(mu);
  if (dev >= 0 && dev < 256 && done[dev]) return QLOCO_OK;
  double CI[BNT * BNI];
  memset(CI, 0, sizeof(CI));
  for (int row = 0; row < BNH; ++row) {
    for (int v = 0; v < BNH; ++v) {
      const double pu = K.ppu[v * BNH + row];
      CI[(0 * BNH + row) * BNT + v] = -pu;
      CI[(1 * BNH + row) * BNT + v] = pu;
      CI[(2 * BNH + row) * BNT + BNH + v] = -pu;
      CI[(3 * BNH + row) * BNT + BNH + v] = pu;
    }
    CI[(4 * BNH + row) * BNT + row] = -K.j_ini;
    CI[(5 * BNH + row) * BNT + row] = K.j_ini;
    CI[(6 * BNH + row) * BNT + BNH + row] = -K.j_ini;
    CI[(7 * BNH + row) * BNT + BNH + row] = K.j_ini;
  }
  QLOCO_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_body_CI), CI, sizeof(CI)), "c_body_CI upload");
  QLOCO_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_body_K), &K, sizeof(K)), "c_body_K upload");
  if (dev >= 0 && dev < 256) done[dev] = true;
  return QLOCO_OK;
}

int qloco::body_mpc_launch(int64_t batch, const int32_t *i, const double *bodyangle_state,
                           const double *zmp_ref, const double *angle_ref,
                           const double *rfoot_ref, const double *lfoot_ref,
                           const double *comacc_ref, double *state, double *com_traj,
                           int32_t *status, const double *tx, int64_t tx_stride,
                           int64_t tx_tile, const int32_t *run, int64_t ref_ld,
                           hipStream_t stream) {
  BodyArgs a;
  memset(&a, 0, sizeof(a));
  body_constants(a.k);
  a.batch = batch;
  a.i = i;
  a.bodyangle_state = bodyangle_state;
  a.zmp_ref = zmp_ref;
  a.angle_ref = angle_ref;
  a.rfoot_ref = rfoot_ref;
  a.lfoot_ref = lfoot_ref;
  a.comacc_ref = comacc_ref;
  a.state = state;
  a.com_traj = com_traj;
  a.status = status;
  a.tx = tx;
  a.tx_stride = tx_stride;
  a.tx_tile = tx_tile;
  a.run = run;
  a.ref_ld = ref_ld;
  const int rc = body_ci_upload(a.k);
  if (rc != QLOCO_OK) return rc;
  const unsigned blocks = (unsigned)((batch + kBodyGroups - 1) / kBodyGroups);
  hipLaunchKernelGGL(body_mpc_kernel, dim3(blocks), dim3(64), 0, stream, a);
  QLOCO_HIP_CHECK(hipGetLastError(), "body_mpc_kernel launch");
  return QLOCO_OK;
}

extern "C" int qloco_body_indexfind(int64_t batch, const double *t, int32_t *j_period,
                                    void *stream) {
  if (batch < 0 || (batch > 0 && (!t || !j_period))) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  BodyConsts k;
  body_constants(k);
  hipLaunchKernelGGL(indexfind_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, k, batch, t, j_period);
  QLOCO_HIP_CHECK(hipGetLastError(), "indexfind_kernel launch");
  return QLOCO_OK;
}
