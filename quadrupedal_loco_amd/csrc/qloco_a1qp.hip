// qloco_a1qp.hip -- batched A1 single-step force QP for gfx950 (fp64).
//
// Replaces the `stance_leg_control_type == 0` branch of
// A1RobotControl::compute_grf (unitree_ros/a1_cpp_open_source/src/
// A1RobotControl.cpp:383-450; weights, friction pyramid and bounds fixed in
// the constructor :8-49): root acceleration from PD gains, the 12-variable
// dense Hessian H = R I + inv' Q inv, g = -inv' Q root_acc, a 20-row
// friction-pyramid / normal-force constraint block, and a COLD OSQP solve with
// default settings (a fresh OsqpEigen::Solver per call, warm start off,
// :421-433), then the world-frame solution rotated into the body frame
// (:445-449).
//
// One robot per 16-lane group, four robots per 64-thread workgroup (one
// wavefront): lane v owns variable v (leg v/3, component v%3; lanes 12..15
// pad) -- its column of the (exactly symmetric) P, its row of K^-1 and the
// <= 2 constraint rows of its leg that touch it first (x lane: the two F_x
// pyramid rows, y lane: the two F_y rows, z lane: the normal-force row), so
// A x and A' y are leg-local.  Vectors that every lane needs (K^-1 matvec
// right-hand side, pivot columns, Ruiz factors, P x operands, group
// reductions) go through a per-robot LDS slot; a wavefront's LDS operations
// complete in order, so wave-level fences replace barriers.
//
// fp64 throughout, compiled without FMA contraction and with the oracle's
// (oracle/a1_qp.c, oracle/admm.c) summation orders, so the QP BUILD (H, g, A,
// l, u) is bit-identical to the restatement.  The ADMM is not: the linear
// solve uses an explicit Gauss-Jordan inverse where the oracle uses Cholesky
// solves, so iterates differ by rounding (tests/test_a1qp_gpu.py allows
// 1e-7 relative / 0.5 N and iteration counts within one check interval).
// The fixture tests/golden/a1_qp.npz comes from the repo's own restatement
// (make_a1_golden.py): parity with the reference's OsqpEigen solve is
// unpinned (OSQP is not vendored).
#include <math.h>
#include <string.h>

#include "qloco_common.hpp"

namespace qloco {
namespace a1 {

constexpr int kN = 12;      // variables
constexpr int kGroup = 16;  // lanes per robot
constexpr double kInf = 1e30;       // OSQP_INFTY / OsqpEigen::INFTY
constexpr double kRhoMin = 1e-6, kRhoMax = 1e6, kRhoEq = 1e3, kRhoTol = 1e-4;
constexpr double kDivTol = 1.0 / kInf;

struct Args {
  qloco_a1_params p;
  int64_t batch;
  const double *state;
  const uint8_t *contacts;
  double *forces, *x, *obj;
  int32_t *status, *iters, *rho_updates;
};

struct Slot {  // one robot's LDS
  double vec[kGroup];
  double aux[kGroup];
  double red[8][kGroup];
  double col[kN][6];  // inertia_inv columns
};

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double limit_scaling_d(double d) {
  d = d < 1e-4 ? 1.0 : d;
  return d > 1e4 ? 1e4 : d;
}

// max over the 12 variable lanes of the robot, NV values at once
template <int NV>
__device__ __forceinline__ void gmax(Slot &S, int v, double (&val)[NV]) {
#pragma unroll
  for (int k = 0; k < NV; ++k) S.red[k][v] = val[k];
  wsync();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double m = 0.0;
#pragma unroll
    for (int j = 0; j < kN; ++j) m = fmax(m, S.red[k][j]);
    val[k] = m;
  }
  wsync();
}

__global__ __launch_bounds__(64) void a1_qp_kernel(const Args a) {
  __shared__ __attribute__((aligned(16))) Slot slots[4];
  const int lane = threadIdx.x;
  const int g = lane >> 4, v = lane & 15;
  Slot &S = slots[g];
  const int64_t b_raw = (int64_t)blockIdx.x * 4 + g;
  const bool live = b_raw < a.batch;             // the group's robot exists
  const int64_t b = live ? b_raw : a.batch - 1;  // dead groups recompute the last robot
  const bool valid = v < kN;
  const int leg = valid ? v / 3 : 0, comp = valid ? v - 3 * (v / 3) : 0;
  const int zl = 3 * leg + 2;  // the leg's z lane (slot index)
  const qloco_a1_params &P = a.p;
  const double *s = a.state + b * QLOCO_A1_STATE_LEN;

  // ------------------------------------------------ build (A1RobotControl.cpp:383-419)
  double acc[6];
  {
    const double *pos = s, *pos_d = s + 3, *eul = s + 6, *eul_d = s + 9;
    const double *lv = s + 12, *lv_d = s + 15, *av = s + 18, *av_d = s + 21, *R = s + 24;
    double ee[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) ee[k] = eul_d[k] - eul[k];
    if (ee[2] > 3.1415926 * 1.5) ee[2] = eul_d[2] - 3.1415926 * 2 - eul[2];  // :333-337
    else if (ee[2] < -3.1415926 * 1.5) ee[2] = eul_d[2] + 3.1415926 * 2 - eul[2];
    double vb[3], wb[3], t[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      vb[r] = R[3 * r + 0] * lv[0] + R[3 * r + 1] * lv[1] + R[3 * r + 2] * lv[2];
      wb[r] = R[3 * r + 0] * av[0] + R[3 * r + 1] * av[1] + R[3 * r + 2] * av[2];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = P.kd_linear[k] * (lv_d[k] - vb[k]);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      acc[r] = P.kp_linear[r] * (pos_d[r] - pos[r]);
      acc[r] += R[r] * t[0] + R[3 + r] * t[1] + R[6 + r] * t[2];
      acc[3 + r] = P.kp_angular[r] * ee[r];
      acc[3 + r] += P.kd_angular[r] * (av_d[r] - wb[r]);
    }
    acc[2] += P.robot_mass * 9.8;
  }
  // this lane's column of inertia_inv: [e_comp; Rz^T skew(foot_leg) e_comp] (:399-405)
  double cv[6];
  {
    const double *Rz = s + 33, *f = s + 42 + 3 * leg;
    double Sc[3];  // column comp of skew(f) (Utils.cpp:35-41)
    Sc[0] = comp == 0 ? 0.0 : (comp == 1 ? -f[2] : f[1]);
    Sc[1] = comp == 0 ? f[2] : (comp == 1 ? 0.0 : -f[0]);
    Sc[2] = comp == 0 ? -f[1] : (comp == 1 ? f[0] : 0.0);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      cv[r] = r == comp ? 1.0 : 0.0;
      cv[3 + r] = Rz[3 * r + 0] * Sc[0] + Rz[3 * r + 1] * Sc[1] + Rz[3 * r + 2] * Sc[2];
    }
    if (valid)
#pragma unroll
      for (int k = 0; k < 6; ++k) S.col[v][k] = cv[k];
  }
  wsync();
  // P column v = upper triangle mirrored (OSQP reads triu(P)): entry (r, v) is
  // computed as H(min, max) = sum_k inv(k,min) Q_k inv(k,max) (+ R on the diagonal)
  double Pc[kN];
#pragma unroll
  for (int r = 0; r < kN; ++r) {
    double x = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const double cr = S.col[r][k];
      x += (r < v) ? (cr * P.q_diag[k]) * cv[k] : (cv[k] * P.q_diag[k]) * cr;
    }
    Pc[r] = valid ? x + (r == v ? P.r : 0.0) : (r == v ? 1.0 : 0.0);
  }
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) q += cv[k] * P.q_diag[k] * acc[k];
  q = valid ? -q : 0.0;
  // constraint rows owned by this lane (ctor :28-49, contact bounds :414-419):
  //  x lane: rows [1 0 -mu], [-1 0 -mu] in (-inf, 0];  y lane: the F_y pair;
  //  z lane: [0 0 1] in [c fmin, c fmax] and an inert zero row in [0, 0]
  const bool xy = valid && comp < 2;
  double ra0 = valid ? 1.0 : 0.0, ra1 = xy ? -1.0 : 0.0;
  double rz0 = xy ? -P.mu : 0.0, rz1 = xy ? -P.mu : 0.0;
  const double cflag = a.contacts[b * 4 + leg] ? 1.0 : 0.0;
  double l0 = xy ? -kInf : (valid ? cflag * P.f_min : 0.0), u0 = xy ? 0.0 : (valid ? cflag * P.f_max : 0.0);
  double l1 = xy ? -kInf : 0.0, u1 = 0.0;

  // ------------------------------------------------ modified Ruiz (OSQP scale_data; admm.c)
  double D = 1.0, E0 = 1.0, E1 = 1.0, c = 1.0;
  for (int it = 0; it < P.scaling; ++it) {
    // column norms: |P(:, v)| and the A entries of column v (z lane: + the
    // -mu entries of its leg's four pyramid rows, held by the x / y lanes)
    S.vec[v] = fmax(fabs(rz0), fabs(rz1));
    wsync();
    double cn = 0.0;
#pragma unroll
    for (int r = 0; r < kN; ++r) cn = fmax(cn, fabs(Pc[r]));
    double an = fmax(fabs(ra0), fabs(ra1));
    if (comp == 2) an = fmax(an, fmax(S.vec[3 * leg], S.vec[3 * leg + 1]));
    // admm.c scans P's column then A's column with one running max
    double Dt = valid ? limit_scaling_d(fmax(cn, an)) : 1.0;
    double Et0 = valid ? limit_scaling_d(fmax(fabs(ra0), fabs(rz0))) : 1.0;
    double Et1 = xy ? limit_scaling_d(fmax(fabs(ra1), fabs(rz1))) : 1.0;
    Dt = 1.0 / sqrt(Dt);
    Et0 = 1.0 / sqrt(Et0);
    Et1 = 1.0 / sqrt(Et1);
    wsync();
    S.vec[v] = Dt;
    wsync();
    const double Dz = S.vec[zl];
#pragma unroll
    for (int r = 0; r < kN; ++r) Pc[r] *= S.vec[r] * Dt;
    ra0 *= Et0 * Dt;
    ra1 *= Et1 * Dt;
    rz0 *= Et0 * Dz;
    rz1 *= Et1 * Dz;
    q *= Dt;
    D *= Dt;
    E0 *= Et0;
    E1 *= Et1;
    wsync();
    // cost scaling: mean column inf-norm of the new P, summed in column order
    double cm = 0.0;
#pragma unroll
    for (int r = 0; r < kN; ++r) cm = fmax(cm, fabs(Pc[r]));
    S.vec[v] = cm;
    S.aux[v] = fabs(q);
    wsync();
    double mean = 0.0, qn = 0.0;
#pragma unroll
    for (int j = 0; j < kN; ++j) {
      mean += S.vec[j];
      qn = fmax(qn, S.aux[j]);
    }
    mean /= kN;
    qn = limit_scaling_d(qn);
    double ct = limit_scaling_d(fmax(mean, qn));
    ct = 1.0 / ct;
#pragma unroll
    for (int r = 0; r < kN; ++r) Pc[r] *= ct;
    q *= ct;
    c *= ct;
    wsync();
  }
  const double cinv = 1.0 / c, Dinv = 1.0 / D, Einv0 = 1.0 / E0, Einv1 = 1.0 / E1;
  l0 *= E0;
  u0 *= E0;
  l1 *= E1;
  u1 *= E1;
  // set_rho_vec: no loose rows here; l == u rows (a swing leg's normal force)
  // are equalities with 1e3 rho
  const bool eq0 = valid && (u0 - l0 < kRhoTol);
  const bool eq1 = xy && (u1 - l1 < kRhoTol);
  double rho = fmin(fmax(P.rho, kRhoMin), kRhoMax);
  double rv0 = eq0 ? kRhoEq * rho : rho, rv1 = eq1 ? kRhoEq * rho : rho;

  // K = P + sigma I + A' diag(rho) A (row v), then K^-1 in place (Gauss-Jordan)
  double K[kN];
  auto factor = [&]() {
    // leg-local A' diag(rho) A entries: own rows (x / y / z lane) and, for
    // the z lane, the pyramid rows of its x / y lanes
    const double own = rv0 * ra0 * ra0 + rv1 * ra1 * ra1;
    const double oz = rv0 * ra0 * rz0 + rv1 * ra1 * rz1;
    const double zz = rv0 * rz0 * rz0 + rv1 * rz1 * rz1;
    S.vec[v] = oz;
    S.aux[v] = zz;
    wsync();
    const double ozx = S.vec[3 * leg], ozy = S.vec[3 * leg + 1];
    const double zzx = S.aux[3 * leg], zzy = S.aux[3 * leg + 1];
    wsync();
#pragma unroll
    for (int cc = 0; cc < kN; ++cc) {
      double add = cc == v ? P.sigma : 0.0;
      if (valid && cc / 3 == leg) {
        const int o = cc - 3 * leg;
        if (comp < 2) add += (o == comp) ? own : (o == 2 ? oz : 0.0);
        else add += (o == 2) ? (own + zzx + zzy) : (o == 0 ? ozx : ozy);
      }
      K[cc] = valid ? Pc[cc] + add : (cc == v ? 1.0 : 0.0);
    }
#pragma unroll
    for (int k = 0; k < kN; ++k) {
      const double vk = K[k];
      double e = (v < k) ? -vk : vk;
      if (v == k) {
        e = vk + 1.0;
        S.aux[0] = vk;
      }
      if (valid) S.vec[v] = e;
      wsync();
      const double p = S.aux[0];
      const double gk = (v == k) ? (1.0 - 1.0 / p) : vk / p;
      if (valid)
#pragma unroll
        for (int cc = 0; cc < kN; ++cc) K[cc] -= gk * S.vec[cc];
      wsync();
    }
  };
  factor();

  // ------------------------------------------------ ADMM (OSQP osqp_solve, admm.c)
  double x = 0.0, z0 = 0.0, z1 = 0.0, y0 = 0.0, y1 = 0.0;
  const double alpha = P.alpha, sigma = P.sigma;
  const int ctm = P.check_termination;
  const int interval = (P.adaptive_rho && P.adaptive_rho_interval == 0)
                           ? (ctm ? 4 * ctm : 100)
                           : (P.adaptive_rho ? P.adaptive_rho_interval : 0);
  // A' w for this lane's column: own rows, then (z lane) the pyramid rows of
  // the x lane and the y lane -- CSC row order (fz row i < pyramid rows)
  auto At = [&](double w0, double w1) {
    S.vec[v] = rz0 * w0;
    S.aux[v] = rz1 * w1;
    wsync();
    double r = 0.0 + ra0 * w0;
    r += ra1 * w1;
    if (comp == 2) {
      r = 0.0 + ra0 * w0;
      r += S.vec[3 * leg];
      r += S.aux[3 * leg];
      r += S.vec[3 * leg + 1];
      r += S.aux[3 * leg + 1];
    }
    wsync();
    return valid ? r : 0.0;
  };
  // A x for this lane's rows: (0 + own coefficient * x_own) + z coefficient * x_z
  auto Ax = [&](double xv, double &a0, double &a1) {
    S.vec[v] = xv;
    wsync();
    const double xz = S.vec[zl];
    wsync();
    a0 = (0.0 + ra0 * xv) + rz0 * xz;
    a1 = (0.0 + ra1 * xv) + rz1 * xz;
    if (comp == 2) {
      a0 = 0.0 + ra0 * xv;
      a1 = 0.0;
    }
  };
  // P x for this lane (row v of the symmetric P, summed in column order)
  auto Px = [&](double xv) {
    S.vec[v] = valid ? xv : 0.0;
    wsync();
    double r = 0.0;
#pragma unroll
    for (int j = 0; j < kN; ++j) r += Pc[j] * S.vec[j];
    wsync();
    return valid ? r : 0.0;
  };
  int status = QLOCO_MAX_ITER, iter, rho_updates = 0;
  bool can_check = false;
  // residual state of the last update_info
  double ax0 = 0, ax1 = 0, aty = 0, px = 0, rd = 0, pri = 0, dua = 0;
  auto update_info = [&]() {
    Ax(x, ax0, ax1);
    aty = At(y0, y1);
    px = Px(x);
    rd = valid ? (q + px) + aty : 0.0;
    double nv[2] = {fmax(fabs(Einv0 * (ax0 - z0)), fabs(Einv1 * (ax1 - z1))), fabs(Dinv * rd)};
    gmax<2>(S, v, nv);
    pri = nv[0];
    dua = cinv * nv[1];
  };
  for (iter = 1; iter <= P.max_iter; ++iter) {
    const double xp = x, zp0 = z0, zp1 = z1;
    // update_xz_tilde: xt = K^-1 (A'(rho z - y) + sigma x - q)
    double rhs = At(rv0 * zp0 - y0, rv1 * zp1 - y1);
    rhs += sigma * xp - q;
    S.vec[v] = valid ? rhs : 0.0;
    wsync();
    double xt = 0.0;
#pragma unroll
    for (int j = 0; j < kN; ++j) xt += K[j] * S.vec[j];
    xt = valid ? xt : 0.0;
    wsync();
    double zt0, zt1;
    Ax(xt, zt0, zt1);
    x = alpha * xt + (1.0 - alpha) * xp;
    const double w0 = alpha * zt0 + (1.0 - alpha) * zp0, w1 = alpha * zt1 + (1.0 - alpha) * zp1;
    z0 = fmin(fmax(w0 + (1.0 / rv0) * y0, l0), u0);
    z1 = fmin(fmax(w1 + (1.0 / rv1) * y1, l1), u1);
    y0 += rv0 * (w0 - z0);
    y1 += rv1 * (w1 - z1);
    can_check = ctm && (iter % ctm == 0);
    if (can_check) {
      update_info();
      double nv[5] = {fmax(fabs(Einv0 * z0), fabs(Einv1 * z1)),
                      fmax(fabs(Einv0 * ax0), fabs(Einv1 * ax1)), fabs(Dinv * q),
                      fabs(Dinv * aty), fabs(Dinv * px)};
      gmax<5>(S, v, nv);
      const double eps_p = P.eps_abs + P.eps_rel * fmax(nv[0], nv[1]);
      const double eps_d = P.eps_abs + P.eps_rel * cinv * fmax(fmax(nv[2], nv[3]), nv[4]);
      if (pri < eps_p && dua < eps_d) {
        status = QLOCO_OK;
        break;
      }
    }
    if (P.adaptive_rho && interval && (iter % interval == 0)) {
      if (!can_check) update_info();
      // compute_rho_estimate on the scaled residual vectors
      double nv[7] = {fmax(fabs(ax0 - z0), fabs(ax1 - z1)), fmax(fabs(z0), fabs(z1)),
                      fmax(fabs(ax0), fabs(ax1)), fabs(rd), fabs(q), fabs(aty), fabs(px)};
      gmax<7>(S, v, nv);
      const double pp = nv[0] / (fmax(nv[1], nv[2]) + kDivTol);
      const double dd = nv[3] / (fmax(fmax(nv[4], nv[5]), nv[6]) + kDivTol);
      double rho_new = rho * sqrt(pp / (dd + kDivTol));
      rho_new = fmin(fmax(rho_new, kRhoMin), kRhoMax);
      if (rho_new > rho * P.adaptive_rho_tolerance || rho_new < rho / P.adaptive_rho_tolerance) {
        rho = fmin(fmax(rho_new, kRhoMin), kRhoMax);
        rv0 = eq0 ? kRhoEq * rho : rho;
        rv1 = eq1 ? kRhoEq * rho : rho;
        factor();
        rho_updates++;
      }
    }
  }
  if (iter > P.max_iter) {
    iter = P.max_iter;
    if (!can_check) update_info();
    double nv[5] = {fmax(fabs(Einv0 * z0), fabs(Einv1 * z1)),
                    fmax(fabs(Einv0 * ax0), fabs(Einv1 * ax1)), fabs(Dinv * q), fabs(Dinv * aty),
                    fabs(Dinv * px)};
    gmax<5>(S, v, nv);
    const double ep = 10 * P.eps_abs + 10 * P.eps_rel * fmax(nv[0], nv[1]);
    const double ed = 10 * P.eps_abs + 10 * P.eps_rel * cinv * fmax(fmax(nv[2], nv[3]), nv[4]);
    status = (pri < ep && dua < ed) ? QLOCO_SOLVED_INACCURATE : QLOCO_MAX_ITER;
  }

  // ------------------------------------------------ outputs
  const double pxf = Px(x);
  S.vec[v] = valid ? 0.5 * pxf * x + q * x : 0.0;
  const double xu = D * x;
  S.aux[v] = valid ? xu : 0.0;
  wsync();
  double objv = 0.0;
#pragma unroll
  for (int j = 0; j < kN; ++j) objv += S.vec[j];
  objv *= cinv;
  const bool bad = !isfinite(objv);
  if (bad) status = QLOCO_NAN;
  if (live && valid) {
    // foot_forces_grf(:, leg) = root_rot_mat^T QPSolution.segment<3>(3 leg)
    const double *R = s + 24;
    const double *xl = S.aux + 3 * leg;
    const double f = R[3 * comp + 0] * xl[0] + R[3 * comp + 1] * xl[1] + R[3 * comp + 2] * xl[2];
    a.forces[b * kN + v] = bad ? NAN : f;
    if (a.x) a.x[b * kN + v] = bad ? NAN : xu;
  }
  if (live && v == 0) {
    if (a.status) a.status[b] = status;
    if (a.iters) a.iters[b] = iter;
    if (a.rho_updates) a.rho_updates[b] = rho_updates;
    if (a.obj) a.obj[b] = objv;
  }
}

}  // namespace a1
}  // namespace qloco

extern "C" void qloco_a1_params_default(qloco_a1_params *p) {
  memset(p, 0, sizeof(*p));
  // A1CtrlStates::reset() (A1CtrlStates.h:39, :123-126)
  const double kpl[3] = {1000.0, 1000.0, 1000.0}, kdl[3] = {200.0, 70.0, 120.0};
  const double kpa[3] = {650.0, 35.0, 1.0}, kda[3] = {4.5, 4.5, 30.0};
  for (int k = 0; k < 3; ++k) {
    p->kp_linear[k] = kpl[k];
    p->kd_linear[k] = kdl[k];
    p->kp_angular[k] = kpa[k];
    p->kd_angular[k] = kda[k];
  }
  p->robot_mass = 15.0;
  // A1RobotControl ctor (A1RobotControl.cpp:12-16)
  const double qd[6] = {1.0, 1.0, 1.0, 400.0, 400.0, 100.0};
  for (int k = 0; k < 6; ++k) p->q_diag[k] = qd[k];
  p->r = 1e-3;
  p->mu = 0.7;
  p->f_min = 0.0;
  p->f_max = 180.0;
  // OSQP v0.6 defaults (OsqpEigen::Settings)
  p->rho = 0.1;
  p->sigma = 1e-6;
  p->alpha = 1.6;
  p->eps_abs = 1e-3;
  p->eps_rel = 1e-3;
  p->max_iter = 4000;
  p->check_termination = 25;
  p->scaling = 10;
  p->adaptive_rho = 1;
  p->adaptive_rho_interval = 0;
  p->adaptive_rho_tolerance = 5.0;
}

extern "C" int qloco_a1_qp_solve(const qloco_a1_params *prm, int64_t batch, const double *state,
                                 const uint8_t *contacts, double *forces_body, double *qp_solution,
                                 int32_t *status, int32_t *iters, int32_t *rho_updates,
                                 double *obj, void *stream) {
  if (!prm || batch < 0) return QLOCO_ERR_ARG;
  if (batch == 0) return QLOCO_OK;
  if (!state || !contacts || !forces_body) return QLOCO_ERR_ARG;
  if (prm->max_iter < 1 || prm->scaling < 0 || prm->check_termination < 0 || prm->rho <= 0.0 ||
      prm->sigma <= 0.0 || prm->robot_mass <= 0.0)
    return QLOCO_ERR_ARG;
  qloco::a1::Args a;
  memset(&a, 0, sizeof(a));
  a.p = *prm;
  a.batch = batch;
  a.state = state;
  a.contacts = contacts;
  a.forces = forces_body;
  a.x = qp_solution;
  a.obj = obj;
  a.status = status;
  a.iters = iters;
  a.rho_updates = rho_updates;
  const int64_t blocks = (batch + 3) / 4;
  hipLaunchKernelGGL(qloco::a1::a1_qp_kernel, dim3((unsigned)blocks), dim3(64), 0,
                     (hipStream_t)stream, a);
  QLOCO_HIP_CHECK(hipGetLastError(), "a1_qp_kernel launch");
  return QLOCO_OK;
}
