// test_host.cpp -- GPU test of the C++ host shim (include/qloco.hpp), run by
// tests/test_host_gpu.py.  Checker: the CPU oracle (oracle/, test
// infrastructure, linked here only).  Prints "ALL OK" on success.
//
//  1. Dynamiccclass on BASELINE config 1 (Go1 stand balance: mode 102,
//     right_support 2, homing feet, F_sum = (0,0,117.6,0,0,0)) and a
//     mode/support sweep over 3 ticks: grf_opt vs qo_force_opt within 1e-9.
//  2. QPsolverGpu / QPBaseClassGpu on random QPs vs qo_eqp_solve.
//  3. PRMPCClass::body_theta_mpc over a gait window vs qo_body_theta_mpc;
//     Indexfind bit-exact.
//  5. RtMpcNode (gait_fast.cpp loop) over 400 ticks of scripted messages vs
//     qo_rt_tick_n: schedule integers and /rt2nrt/state bit-exact, /rtMPC/traj
//     within 1e-9 (foot-rotation cos is the device libm's).
//  6. ServoForceBlock (servo.cpp:1052-1243) over 40 ticks vs
//     qo_servo_force_block: F_sum / F_lr_predict / swing bit-exact, grf_opt
//     and torques within 1e-9.
//  4. ConvexMpcBatch::compute_grf on the inputs of the reference harness
//     test_mpc.cpp:18-91 (A1, mass 15, contacts FL, RL): forces within 0.5 N
//     of the exact optimum committed in tests/golden/srbd_test_mpc_kat.npz.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "qloco.hpp"

extern "C" {
#include "qloco_oracle.h"
}

static int g_fail = 0;
#define CHECK(cond, ...)                  \
  do {                                    \
    if (!(cond)) {                        \
      std::printf("FAIL: " __VA_ARGS__);  \
      std::printf("\n");                  \
      ++g_fail;                           \
    }                                     \
  } while (0)

static bool close(double a, double b, double rtol, double atol) {
  return std::fabs(a - b) <= atol + rtol * std::fabs(b);
}

static void test_force_qp() {
  const double homing[12] = {0.150786, -0.12675, 0.0, 0.150786, 0.12675, 0.0,
                             -0.225414, -0.12675, 0.0, -0.225414, 0.12675, 0.0};
  const int B = 8;
  qloco::Dynamiccclass dyn(B);
  std::vector<qo_dyn_state> ref(B);
  qo_force_params prm;
  qo_force_params_default(&prm);
  for (auto &s : ref) qo_dyn_init(&s);
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-0.02, 0.02);
  const int modes[3] = {102, 101, 103};
  for (int tick = 0; tick < 3; ++tick) {
    std::vector<double> base(B * 3), feet(B * 12), F(B * 6), rf(B * 3), lf(B * 3), y(B);
    std::vector<int> mode(B), rs(B);
    for (int b = 0; b < B; ++b) {
      base[b * 3 + 0] = b ? U(rng) : 0.0;
      base[b * 3 + 1] = b ? U(rng) : 0.0;
      base[b * 3 + 2] = 0.309458 + (b ? U(rng) : 0.0);
      for (int k = 0; k < 12; ++k) feet[b * 12 + k] = homing[k] + ((b && k % 3 != 2) ? U(rng) : 0.0);
      const double m = 12.0, az = b ? 10 * U(rng) : 0.0;
      F[b * 6 + 0] = b ? 100 * U(rng) : 0.0;
      F[b * 6 + 1] = b ? 100 * U(rng) : 0.0;
      F[b * 6 + 2] = m * 9.8 + m * az;
      F[b * 6 + 3] = F[b * 6 + 4] = F[b * 6 + 5] = 0.0;
      mode[b] = b ? modes[(b + tick) % 3] : 102;
      rs[b] = b ? (b + tick) % 3 : 2;  // b = 0: BASELINE config 1 (double support)
      y[b] = mode[b] == 101 ? 0.75 : (mode[b] == 102 ? 0.0 : 0.11);
      for (int c = 0; c < 3; ++c) {
        rf[b * 3 + c] = 0.5 * (feet[b * 12 + c] + feet[b * 12 + 9 + c]);
        lf[b * 3 + c] = 0.5 * (feet[b * 12 + 3 + c] + feet[b * 12 + 6 + c]);
      }
    }
    for (int b = 0; b < B; ++b) {  // servo.cpp:1224-1228 call sequence
      dyn.force_distribution(&base[b * 3], &feet[b * 12], &F[b * 6], mode[b], y[b], &rf[b * 3],
                             &lf[b * 3], b);
      dyn.force_opt(&base[b * 3], &feet[b * 12], &feet[b * 12 + 3], &feet[b * 12 + 6],
                    &feet[b * 12 + 9], &F[b * 6], mode[b], rs[b], y[b], b);
      qo_force_distribution(&ref[b], &base[b * 3], &feet[b * 12], &F[b * 6], mode[b], y[b],
                            &rf[b * 3], &lf[b * 3]);
      const int ok = qo_force_opt(&ref[b], &prm, &base[b * 3], &feet[b * 12], &feet[b * 12 + 3],
                                  &feet[b * 12 + 6], &feet[b * 12 + 9], &F[b * 6], mode[b], rs[b],
                                  y[b], nullptr, nullptr);
      CHECK(dyn.qp_solution[b] == ok, "force qp_solution tick %d robot %d", tick, b);
    }
    for (int b = 0; b < B; ++b)
      for (int k = 0; k < 12; ++k) {
        CHECK(close(dyn.grf_opt[b * 12 + k], ref[b].grf_opt[k], 1e-9, 1e-8),
              "grf_opt tick %d robot %d [%d] %.12g vs %.12g", tick, b, k, dyn.grf_opt[b * 12 + k],
              ref[b].grf_opt[k]);
        CHECK(dyn.F_leg_guess[b * 12 + k] == ref[b].F_leg_guess[k], "F_leg_guess %d %d", b, k);
      }
  }
  // config 1: the four stance legs carry the robot's weight
  double fz = 0.0;
  for (int l = 0; l < 4; ++l) fz += dyn.grf_opt[3 * l + 2];
  CHECK(std::fabs(fz) > 50.0, "stand-balance total fz %.3f", fz);
  for (auto &s : ref) qo_dyn_free(&s);
  std::printf("force QP ok (config 1 total fz %.4f N)\n", fz);
}

static void test_qpsolver_size(int n, int p, int m, int trials, int zero_ce);
static void test_qpsolver() {
  test_qpsolver_size(12, 3, 24, 20, 0);
  // QPBaseClass's capacity (nVars <= 60, nIneq <= 300, QPBaseClass.h:49-51):
  // the one-QP-per-wavefront kernel, zero CE columns included
  test_qpsolver_size(60, 10, 300, 4, 3);
  test_qpsolver_size(30, 0, 120, 4, 0);
  std::printf("QPsolver ok\n");
}

static void test_qpsolver_size(int n, int p, int m, int trials, int zero_ce) {
  std::mt19937_64 rng(11 + n);
  std::normal_distribution<double> N01(0.0, 1.0);
  qloco::QPBaseClassGpu qp;
  qp.resizeQP(n, p, m);
  for (int trial = 0; trial < trials; ++trial) {
    std::vector<double> M(n * n);
    for (auto &v : M) v = N01(rng);
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c) {
        double a = 0.0;
        for (int k = 0; k < n; ++k) a += M[k * n + r] * M[k * n + c];
        qp.G[c * n + r] = a + (r == c ? n : 0.0);
      }
    for (auto &v : qp.g0) v = 3.0 * N01(rng);
    for (auto &v : qp.CE) v = N01(rng);
    for (int z = 0; z < zero_ce && p > 0; ++z) {  // EiQuadProg skips all-zero CE columns
      const int c = (int)(rng() % (uint64_t)p);
      for (int r = 0; r < n; ++r) qp.CE[c * n + r] = 0.0;
    }
    for (auto &v : qp.ce0) v = 0.3 * N01(rng);
    for (auto &v : qp.CI) v = N01(rng);
    for (auto &v : qp.ci0) v = N01(rng) + 0.5;
    std::vector<double> G = qp.G, x(n);
    qo_eqp_ws *ws = qo_eqp_create(n, p, m);
    int st = 0, it = 0;
    qo_eqp_solve(ws, G.data(), qp.g0.data(), qp.CE.data(), qp.ce0.data(), qp.CI.data(),
                 qp.ci0.data(), x.data(), &st, &it);
    qo_eqp_destroy(ws);
    const bool ok = qp.solveQP();
    bool ref_ok = true;  // QPBaseClass.cpp:137-150: success = no NaN in X
    for (double v : x) ref_ok = ref_ok && !std::isnan(v);
    CHECK(ok == ref_ok, "QPBaseClass success flag (%d,%d,%d) trial %d", n, p, m, trial);
    if (st == QO_OK)
      for (int k = 0; k < n; ++k)
        CHECK(close(qp.X[k], x[k], 1e-9, 1e-9), "QP (%d,%d,%d) x trial %d [%d] %.12g vs %.12g", n,
              p, m, trial, k, qp.X[k], x[k]);
  }
}

static void test_body_mpc() {
  qloco::PRMPCClass body(1);
  qo_body_state ref;
  qo_body_init(&ref);
  std::mt19937_64 rng(5);
  std::normal_distribution<double> N01(0.0, 1.0);
  for (int i = 96; i < 160; ++i) {
    double bs[4], zmp[10], ang[10], rf[10], lf[10], acc[15], gen[9] = {0};
    for (auto &v : bs) v = 0.05 * N01(rng);
    for (int k = 0; k < 10; ++k) {
      zmp[k] = 0.02 * N01(rng);
      ang[k] = 0.02 * N01(rng);
      rf[k] = 0.05 * N01(rng);
      lf[k] = 0.05 * N01(rng);
    }
    for (auto &v : acc) v = 0.5 * N01(rng);
    const std::array<double, 14> out = body.body_theta_mpc(i, bs, zmp, ang, rf, lf, acc, gen);
    double ct[14];
    int st = 0;
    qo_body_theta_mpc(&ref, i, bs, zmp, ang, rf, lf, acc, gen, ct, &st);
    for (int k = 0; k < 14; ++k)
      CHECK(close(out[k], ct[k], 1e-9, 1e-12), "body i=%d [%d] %.12g vs %.12g", i, k, out[k], ct[k]);
    if (i >= 100) {
      CHECK((int)body.state[26] == ref.bjx1 && (int)body.state[27] == ref.bjx2 &&
                (int)body.state[28] == ref.t_yu,
            "schedule ints at i=%d", i);
    }
  }
  for (double t = 0.0; t < 17.0; t += 0.37)
    CHECK(body.Indexfind(t) == qo_body_indexfind(&ref, t), "Indexfind(%.2f)", t);
  qo_body_free(&ref);
  std::printf("body MPC ok\n");
}

static void test_convex_mpc() {
  qloco_srbd_spec sp;
  qloco_srbd_spec_default(&sp);
  sp.mass = 15.0f;  // test_mpc.cpp:19-23
  const float I[9] = {0.0158533f, 0, 0, 0, 0.0377999f, 0, 0, 0, 0.0456542f};
  for (int k = 0; k < 9; ++k) sp.inertia[k] = I[k];
  const float q[13] = {1, 1, 1, 0, 0, 50, 0, 0, 1, 1, 1, 1, 0};  // :52-56
  for (int k = 0; k < 13; ++k) sp.q_weights[k] = q[k];
  for (int k = 0; k < 12; ++k) sp.r_weights[k] = 1e-6f;
  qloco::ConvexMpcBatch mpc(2, &sp);
  qloco::A1MpcState st[2] = {};
  for (auto &s : st) {
    s.root_pos[2] = 0.15;
    const double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 9; ++k) s.root_rot_mat[k] = R[k];
    const double feet[12] = {0.17, 0.15, -0.35, 0.17, -0.15, -0.35,
                             -0.17, 0.15, -0.35, -0.17, -0.15, -0.35};
    for (int k = 0; k < 12; ++k) s.foot_pos_abs[k] = feet[k];
    s.contacts[0] = true;   // FL
    s.contacts[1] = false;  // FR
    s.contacts[2] = true;   // RL
    s.contacts[3] = false;  // RR
  }
  // the harness's x_d sets z from root_pos + v_d,y * t (:83), = root_pos_d[2] at v_d = 0
  for (auto &s : st) s.root_pos_d[2] = 0.15;
  double forces[24] = {0};
  mpc.compute_grf(st, forces);
  // exact optimum of the same QP (tests/golden/srbd_test_mpc_kat.npz, u_exact[:12])
  const double ex[12] = {0.0, -12.8370297, 42.790099, 0.0, 0.0, 0.0,
                         0.0, -12.8370297, 42.790099, 0.0, 0.0, 0.0};
  for (int b = 0; b < 2; ++b) {
    CHECK(mpc.status[b] == QLOCO_OK, "compute_grf status %d", mpc.status[b]);
    for (int k = 0; k < 12; ++k)
      CHECK(std::fabs(forces[b * 12 + k] - ex[k]) < 0.5, "compute_grf robot %d [%d] %.4f vs %.4f",
            b, k, forces[b * 12 + k], ex[k]);
  }
  std::printf("compute_grf ok: FL (%.3f, %.3f, %.3f) iters %d\n", forces[0], forces[1], forces[2],
              mpc.iters[0]);
}

// The reference's member solver semantics: a default-constructed
// ConvexMpcBatch keeps each robot's OSQP solver across compute_grf calls
// (A1RobotControl.cpp:556-578); an identical second call resumes at the
// converged iterate and stops at the first termination check, reset()
// restores the cold solve.
static void test_convex_mpc_persistent() {
  qloco::ConvexMpcBatch mpc(2);
  CHECK(mpc.spec.warm_start == 2, "default ConvexMpcBatch is persistent");
  CHECK(mpc.spec.literal_full_qp == 1, "default ConvexMpcBatch solves the literal 12N QP");
  qloco::A1MpcState st[2] = {};
  for (auto &s : st) {
    s.root_pos[2] = 0.30;
    s.root_pos_d[2] = 0.30;
    s.root_euler[2] = 0.4;
    s.root_lin_vel[0] = 0.2;
    const double c = std::cos(0.4), sn = std::sin(0.4);
    const double R[9] = {c, sn, 0, -sn, c, 0, 0, 0, 1};
    for (int k = 0; k < 9; ++k) s.root_rot_mat[k] = R[k];
    const double feet[12] = {0.15, 0.127, -0.31, 0.15, -0.127, -0.31,
                             -0.225, 0.127, -0.31, -0.225, -0.127, -0.31};
    for (int k = 0; k < 12; ++k) s.foot_pos_abs[k] = feet[k];
    s.contacts[0] = s.contacts[3] = true;
  }
  st[1].contacts[0] = st[1].contacts[3] = false;
  st[1].contacts[1] = st[1].contacts[2] = true;
  double f1[24] = {0}, f2[24] = {0}, f3[24] = {0};
  mpc.compute_grf(st, f1);
  const int cold = mpc.iters[0];
  mpc.compute_grf(st, f2);
  for (int b = 0; b < 2; ++b) {
    CHECK(mpc.status[b] == QLOCO_OK, "persistent status %d", mpc.status[b]);
    CHECK(mpc.iters[b] == 25, "resumed solve iters %d (cold %d)", mpc.iters[b], cold);
  }
  mpc.reset();
  mpc.compute_grf(st, f3);
  CHECK(mpc.iters[0] == cold, "after reset: cold again (%d vs %d)", mpc.iters[0], cold);
  for (int k = 0; k < 24; ++k) CHECK(f3[k] == f1[k], "reset reproduces the cold solve [%d]", k);
  std::printf("persistent compute_grf ok: cold %d iters, resumed %d\n", cold, mpc.iters[1]);
}

// The multi-GPU form at world 1 (RCCL with one rank): a ConvexMpcBatch over
// a global batch of 5 robots, interleaved shard mode, gives the single-GPU
// object's forces, status and iterations exactly, in all_forces() and in its
// own shard's outputs.
static void test_convex_mpc_multi_gpu() {
  const int T = 5;
  std::vector<qloco::A1MpcState> st(T);
  for (int b = 0; b < T; ++b) {
    auto &s = st[b];
    s.root_pos[2] = 0.30;
    s.root_pos_d[2] = 0.30;
    s.root_euler[2] = 0.1 * b;
    s.root_lin_vel[0] = 0.05 * b;
    const double c = std::cos(0.1 * b), sn = std::sin(0.1 * b);
    const double R[9] = {c, sn, 0, -sn, c, 0, 0, 0, 1};
    for (int k = 0; k < 9; ++k) s.root_rot_mat[k] = R[k];
    const double feet[12] = {0.15, 0.127, -0.31, 0.15, -0.127, -0.31,
                             -0.225, 0.127, -0.31, -0.225, -0.127, -0.31};
    for (int k = 0; k < 12; ++k) s.foot_pos_abs[k] = feet[k];
    const bool ph = b & 1;
    s.contacts[0] = s.contacts[3] = ph;
    s.contacts[1] = s.contacts[2] = !ph;
  }
  qloco::ConvexMpcBatch one(T);
  std::vector<double> f1(T * 12, 0.0), f2(T * 12, 0.0);
  one.compute_grf(st.data(), f1.data());
  uint8_t id[QLOCO_MGPU_ID_BYTES];
  CHECK(qloco_mgpu_unique_id(id) == QLOCO_OK, "qloco_mgpu_unique_id: %s", qloco_last_error());
  qloco::ConvexMpcBatch mg(T, 1, 0, id, QLOCO_SHARD_INTERLEAVED);
  CHECK(mg.shard_first == 0 && mg.shard_count == T && mg.shard_stride == 1, "world-1 shard");
  for (int call = 0; call < 2; ++call) {  // the persistent update path too
    if (call == 1) one.compute_grf(st.data(), f1.data());
    mg.compute_grf(st.data(), f2.data());
    for (int k = 0; k < T * 12; ++k) {
      CHECK(f2[k] == f1[k], "call %d: shard forces [%d] %.6f vs %.6f", call, k, f2[k], f1[k]);
      CHECK(mg.all_forces()[k] == f1[k], "call %d: all_forces [%d]", call, k);
    }
    for (int b = 0; b < T; ++b)
      CHECK(mg.status[b] == one.status[b] && mg.iters[b] == one.iters[b], "call %d: stats %d", call, b);
  }
  std::printf("multi-GPU compute_grf ok (world 1): iters %d / %d\n", mg.iters[0], mg.iters[1]);
}

// A1RobotControl::compute_grf QP branch (A1QpBatch) vs oracle/a1_qp.c.
static void test_a1_qp() {
  const int B = 8;
  qloco::A1QpBatch qp(B);
  std::vector<qloco::A1QpState> st(B);
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  qo_a1_params prm;
  qo_a1_params_default(&prm);
  qo_admm_settings set;
  qo_admm_settings_default(&set);
  for (int b = 0; b < B; ++b) {
    qloco::A1QpState &s = st[b];
    s = qloco::A1QpState{};
    const double yaw = 3.0 * U(rng);
    const double c = std::cos(yaw), sn = std::sin(yaw);
    const double R[9] = {c, sn, 0, -sn, c, 0, 0, 0, 1};
    for (int k = 0; k < 9; ++k) s.root_rot_mat[k] = s.root_rot_mat_z[k] = R[k];
    s.root_euler[2] = yaw;
    s.root_euler_d[2] = yaw + 0.2 * U(rng);
    for (int k = 0; k < 3; ++k) {
      s.root_lin_vel[k] = 0.3 * U(rng);
      s.root_ang_vel[k] = 0.3 * U(rng);
    }
    s.root_pos[2] = 0.28;
    s.root_pos_d[2] = 0.30;
    const double fb[12] = {0.17, 0.15, -0.3, 0.17, -0.15, -0.3, -0.17, 0.15, -0.3, -0.17, -0.15, -0.3};
    for (int l = 0; l < 4; ++l)  // foot_pos_abs = R * foot_pos_rel
      for (int r = 0; r < 3; ++r)
        s.foot_pos_abs[3 * l + r] =
            R[r] * fb[3 * l] + R[3 + r] * fb[3 * l + 1] + R[6 + r] * fb[3 * l + 2];
    for (int l = 0; l < 4; ++l) s.contacts[l] = (b & 1) ? (l == 1 || l == 2) : (l == 0 || l == 3);
    if (b == 5) s.contacts[0] = s.contacts[1] = s.contacts[2] = s.contacts[3] = true;
  }
  std::vector<double> f(B * 12);
  qp.compute_grf(st.data(), f.data());
  for (int b = 0; b < B; ++b) {
    const qloco::A1QpState &s = st[b];
    double rec[QO_A1_STATE_LEN];
    const double *src[8] = {s.root_pos, s.root_pos_d, s.root_euler, s.root_euler_d,
                            s.root_lin_vel, s.root_lin_vel_d, s.root_ang_vel, s.root_ang_vel_d};
    for (int q = 0; q < 8; ++q)
      for (int k = 0; k < 3; ++k) rec[3 * q + k] = src[q][k];
    for (int k = 0; k < 9; ++k) {
      rec[24 + k] = s.root_rot_mat[k];
      rec[33 + k] = s.root_rot_mat_z[k];
    }
    for (int k = 0; k < 12; ++k) rec[42 + k] = s.foot_pos_abs[k];
    uint8_t ct[4];
    for (int l = 0; l < 4; ++l) ct[l] = s.contacts[l];
    double fo[12];
    qo_admm_info info;
    qo_a1_compute_grf(&prm, &set, rec, ct, fo, nullptr, &info);
    CHECK(qp.status[b] == info.status && qp.iters[b] == info.iters, "A1 QP robot %d status/iters",
          b);
    for (int k = 0; k < 12; ++k)
      CHECK(std::fabs(f[b * 12 + k] - fo[k]) < 1e-5, "A1 QP robot %d [%d] %.9f vs %.9f", b, k,
            f[b * 12 + k], fo[k]);
  }
  std::printf("A1 QP compute_grf ok\n");
}

// Kinematicclass: per-leg calls (servo.cpp:734-741 / :1038-1051 pattern)
// and a batch, against the C restatement (oracle/kinematics.c).
static void test_kinematics() {
  qloco::Kinematicclass kin(256);
  const double P[3] = {0.1, -0.2, 0.3}, E[3] = {0.05, -0.08, 1.2};
  const double home[3] = {0.0, 0.87, -1.5};
  for (int f = 0; f < 4; ++f) {
    double po[3], Jo[9];
    std::array<double, 3> p = kin.Forward_kinematics_g(P, E, home, f);
    qo_leg_fk_g(P, E, home, f, po, Jo);
    for (int r = 0; r < 3; ++r) CHECK(std::fabs(p[r] - po[r]) < 1e-12, "FK_g leg %d [%d]", f, r);
    for (int r = 0; r < 9; ++r)
      CHECK(std::fabs(kin.Jacobian_kin[r] - Jo[r]) < 1e-12, "Jacobian_kin leg %d [%d]", f, r);
    // IK_g back to a perturbed target from the homing pose
    const double qt[3] = {0.1, 0.8, -1.4};
    double target[3], Jt[9];
    qo_leg_fk_g(P, E, qt, f, target, Jt);
    std::array<double, 3> q = kin.Inverse_kinematics_g(P, E, target, home, f);
    double qo[3], pos_o[3], Jq[9];
    const int n = qo_leg_ik(P, E, target, home, f, qo, pos_o, Jq);
    CHECK(kin.last_updates == n, "IK_g updates %d vs %d", kin.last_updates, n);
    for (int r = 0; r < 3; ++r) CHECK(std::fabs(q[r] - qo[r]) < 1e-9, "IK_g leg %d q[%d]", f, r);
    // hip-frame IK (10 steps, signed-max stop)
    q = kin.Inverse_kinematics(target, home, f);
    const int nl = qo_leg_ik(nullptr, nullptr, target, home, f, qo, pos_o, Jq);
    CHECK(kin.last_updates == nl, "IK updates %d vs %d", kin.last_updates, nl);
    for (int r = 0; r < 3; ++r) CHECK(std::fabs(q[r] - qo[r]) < 1e-9, "IK leg %d q[%d]", f, r);
  }
  // batch of 256 legs, hip frame
  const int n = 256;
  std::vector<double> q(3 * n), pos(3 * n), J(9 * n);
  std::vector<int32_t> leg(n);
  for (int i = 0; i < n; ++i) {
    leg[i] = i % 4;
    q[3 * i] = 0.3 * std::sin(0.1 * i);
    q[3 * i + 1] = 0.9 + 0.3 * std::cos(0.07 * i);
    q[3 * i + 2] = -1.6 + 0.4 * std::sin(0.05 * i);
  }
  kin.forward_batch(n, q.data(), leg.data(), nullptr, nullptr, pos.data(), J.data());
  for (int i = 0; i < n; ++i) {
    double po[3], Jo[9];
    qo_leg_fk(&q[3 * i], leg[i], po, Jo);
    for (int r = 0; r < 3; ++r) CHECK(std::fabs(pos[3 * i + r] - po[r]) < 1e-12, "FK batch %d", i);
    for (int r = 0; r < 9; ++r) CHECK(std::fabs(J[9 * i + r] - Jo[r]) < 1e-12, "J batch %d", i);
  }
  std::printf("kinematics ok: FK/IK per leg + batch of %d\n", n);
}


static void test_rt_node() {
  const int B = 3, T = 400;
  qloco::RtMpcNode node(B);
  qo_rt *ref = qo_rt_create_n(B);
  std::vector<double> gait(B * 100, 0.0), ctrl(B * 25, 0.0), traj(B * 100), nrt(B * 25);
  std::vector<int32_t> sched(B * QO_RT_SCHED);
  for (int t = 0; t < T; ++t) {
    for (int b = 0; b < B; ++b) {  // a walking planner stream, started at tick b
      double *g = &gait[b * 100], *c = &ctrl[b * 25];
      const double tn = std::floor(t * 0.4) * 0.025;
      c[0] = t >= b ? 1.0 : 0.0;
      for (int k = 1; k < 25; ++k) c[k] = 0.03 * std::sin(0.2 * t + k + b);
      g[0] = 0.05 * tn;
      g[1] = 0.01 * std::sin(3.0 * tn);
      g[2] = 0.3;
      g[36] = 0.05;
      for (int k : {12, 13, 34, 35, 42, 43, 44, 45, 76, 77, 78, 79}) g[k] = 0.02 * std::cos(tn + k);
      for (int k : {39, 40, 41, 80, 81, 82, 83, 84, 85}) g[k] = 0.2 * std::sin(2 * tn + k);
      const double bj = std::fmin(std::floor(std::fmax(tn - 1.0, 0.0) / 0.7) + 1, 25);
      g[27] = g[86] = bj;
      g[87] = 0.04 * bj;
      g[88] = 0.04 * (bj + 1);
      g[89] = ((int)bj % 2) ? 0.12675 : -0.12675;
      g[90] = -g[89];
      g[93] = bj - 1;
      g[94] = b == 1 ? 0.65 : 0.0;
      g[99] = std::floor(t * 0.4) + 1;
      node.nrt_gait_sub_operation(g, b);
      node.control_gait_sub_operation(c, b);
    }
    node.loop_once();
    qo_rt_tick_n(ref, B, gait.data(), ctrl.data(), traj.data(), nrt.data(), nullptr, sched.data());
    for (int b = 0; b < B; ++b) {
      for (int k = 0; k < QO_RT_SCHED; ++k)
        CHECK(node.sched[b * QLOCO_RT_SCHED_LEN + k] == sched[b * QO_RT_SCHED + k],
              "rt sched t=%d robot %d [%d] %d vs %d\n", t, b, k, node.sched[b * 8 + k],
              sched[b * QO_RT_SCHED + k]);
      for (int k = 0; k < 25; ++k)
        CHECK(node.nrt[b * 25 + k] == nrt[b * 25 + k], "rt nrt t=%d robot %d [%d]\n", t, b, k);
      for (int k = 0; k < 100; ++k)
        CHECK(close(node.traj[b * 100 + k], traj[b * 100 + k], 1e-9, 1e-9),
              "rt traj t=%d robot %d [%d] %.12g vs %.12g\n", t, b, k, node.traj[b * 100 + k],
              traj[b * 100 + k]);
    }
  }
  qo_rt_destroy_n(ref, B);
  std::printf("rt node ok: %d robots x %d ticks\n", B, T);
}

static void test_servo_block() {
  const int B = 4, T = 40;
  qloco::ServoForceBlock blk(B);
  std::vector<qo_servo_state> ref(B);
  for (auto &r : ref) qo_servo_init(&r);
  qo_force_params prm;
  qo_force_params_default(&prm);
  const double homing[12] = {0.150786, -0.12675, 0, 0.150786, 0.12675, 0,
                             -0.225414, -0.12675, 0, -0.225414, 0.12675, 0};
  const int modes[B] = {101, 102, 103, 104};
  std::vector<double> coma(3 * B), com(3 * B), rf(3 * B), lf(3 * B), bp(3 * B), ft(12 * B), y(B),
      J(36 * B), rm(12 * B), ve(12 * B);
  std::vector<int32_t> rs(B), md(B), cnt(B);
  for (int t = 0; t < T; ++t) {
    for (int b = 0; b < B; ++b) {
      const double ph = 0.7 * b + 0.05 * t;
      for (int k = 0; k < 3; ++k) coma[3 * b + k] = 0.3 * std::sin(ph + k);
      bp[3 * b] = 0.01 * t;
      bp[3 * b + 1] = 0.01 * std::sin(ph);
      bp[3 * b + 2] = 0.3;
      for (int k = 0; k < 12; ++k)
        ft[12 * b + k] = homing[k] + (k % 3 == 2 ? 0.01 * std::fabs(std::sin(ph + k)) : bp[3 * b + k % 3]);
      for (int k = 0; k < 3; ++k) {
        com[3 * b + k] = bp[3 * b + k] + 0.002 * std::cos(ph + k);
        rf[3 * b + k] = 0.5 * (ft[12 * b + k] + ft[12 * b + 9 + k]);
        lf[3 * b + k] = 0.5 * (ft[12 * b + 3 + k] + ft[12 * b + 6 + k]);
      }
      for (int k = 0; k < 36; ++k) J[36 * b + k] = ((k % 4) == 0 ? 0.3 : 0.05 * std::sin(k + ph));
      for (int k = 0; k < 12; ++k) {
        rm[12 * b + k] = ft[12 * b + k] - bp[3 * b + k % 3] + 0.001 * std::cos(k + ph);
        ve[12 * b + k] = 0.02 * std::sin(2 * k + ph);
      }
      md[b] = modes[b];
      rs[b] = (t / 7 + b) % 3;
      y[b] = md[b] == 101 ? 0.75 : (md[b] == 102 ? 0.0 : 0.11);
      cnt[b] = t;
    }
    blk.step(coma.data(), com.data(), rf.data(), lf.data(), bp.data(), ft.data(), rs.data(),
             md.data(), y.data(), cnt.data(), J.data(), rm.data(), ve.data());
    for (int b = 0; b < B; ++b) {
      double Fs[6], Fl[6], g[12], tau[12];
      int sw[4], st = 0;
      const int ok = qo_servo_force_block(&ref[b], &prm, &coma[3 * b], &com[3 * b], &rf[3 * b],
                                          &lf[3 * b], &bp[3 * b], &ft[12 * b], rs[b], md[b], y[b],
                                          cnt[b], &J[36 * b], &rm[12 * b], &ve[12 * b], Fs, Fl,
                                          nullptr, g, tau, sw, &st);
      for (int k = 0; k < 6; ++k)
        CHECK(blk.F_sum[6 * b + k] == Fs[k] && blk.Force_L_R[6 * b + k] == Fl[k],
              "servo F t=%d robot %d [%d]\n", t, b, k);
      for (int k = 0; k < 4; ++k) CHECK(blk.swing[4 * b + k] == sw[k], "servo swing t=%d %d\n", t, b);
      CHECK(blk.qp_solution[b] == ok && blk.status[b] == st, "servo status t=%d %d\n", t, b);
      for (int k = 0; k < 12; ++k) {
        CHECK(close(blk.grf_opt[12 * b + k], g[k], 1e-9, 1e-8), "servo grf t=%d %d [%d]\n", t, b, k);
        CHECK(close(blk.Legs_torque[12 * b + k], tau[k], 1e-9, 1e-9), "servo tau t=%d %d [%d]\n", t, b, k);
      }
    }
  }
  for (auto &r : ref) qo_servo_free(&r);
  std::printf("servo force block ok: %d robots x %d ticks\n", B, T);
}

int main() {
  try {
    test_force_qp();
    test_qpsolver();
    test_body_mpc();
    test_convex_mpc();
    test_convex_mpc_persistent();
    test_convex_mpc_multi_gpu();
    test_a1_qp();
    test_kinematics();
    test_rt_node();
    test_servo_block();
  } catch (const qloco::Error &e) {
    std::printf("FAIL: qloco::Error %s (status %d)\n", e.what(), e.status);
    return 2;
  }
  if (g_fail) {
    std::printf("%d FAILURES\n", g_fail);
    return 1;
  }
  std::printf("ALL OK\n");
  return 0;
}
