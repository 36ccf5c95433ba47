/*
 * qloco.hpp -- C++ host shim with the reference's class / method signatures.
 *
 * Drop-in layer for the ROS control loops of jtdingx/quadrupedal_loco: the
 * classes keep the reference's names, argument meaning and result members,
 * and run the solves on the MI355X through the C ABI of qloco.h
 * (libqloco_host.so -> libqloco.so).  Eigen fixed-size matrices of the
 * reference become column-major `double` arrays of the same shape (Eigen's
 * default storage: pass `m.data()`); INTEGRATION.md shows the three-line
 * adapters for the Eigen call sites.
 *
 *   QPsolverGpu / QPBaseClassGpu  <- QPsolver / QPsolver_EiQuadProg /
 *                                    QPBaseClass (rt_mpc_qp/src/QP/QPBaseClass.h:19-73,
 *                                    QPBaseClass.cpp:20-152)
 *   Dynamiccclass                 <- go1_rt_control Dynamiccclass
 *                                    (dynmics_compute.h:59-76; servo.cpp:1224-1228)
 *   PRMPCClass                    <- rt_mpc_qp PRMPCClass::body_theta_mpc / Indexfind
 *                                    (PRMPCClass.h:69-71; gait_fast.cpp:620)
 *   ConvexMpcBatch                <- A1RobotControl::compute_grf MPC branch +
 *                                    ConvexMpc (A1RobotControl.cpp:452-600)
 *   Kinematicclass                <- go1_rt_control Kinematicclass
 *                                    (Kinematics.h:30-61; servo.cpp:734-741, :1038-1051)
 *   ServoForceBlock               <- the go1 servo loop's force block (servo.cpp:1052-1243)
 *   RtMpcNode                     <- the rt_mpc_qp node loop (gait_fast.cpp:79-735):
 *                                    subscriber callbacks + one 100 Hz iteration
 *
 * Every class is batched over B independent robots (B = 1 is the drop-in
 * case).  Host arrays are staged to the device on the object's HIP stream;
 * device-pointer entry points skip the staging.  Failures of the device
 * path throw qloco::Error (there is no CPU fallback); solver outcomes are
 * reported like the reference (NaN-free X / qp_solution flags).
 */
#pragma once

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "qloco.h"

namespace qloco {

class Error : public std::runtime_error {
 public:
  Error(const std::string &what, int status);
  int status;
};

// Owned device memory + one HIP stream (created on construction).
class DeviceArena {
 public:
  DeviceArena();
  ~DeviceArena();
  DeviceArena(const DeviceArena &) = delete;
  DeviceArena &operator=(const DeviceArena &) = delete;
  void *alloc(size_t bytes);        // persistent block, freed with the arena
  void release(void *p);            // free one block early (no-op on nullptr)
  void upload(void *dev, const void *host, size_t bytes);
  void download(void *host, const void *dev, size_t bytes);
  void sync();
  void *stream() const { return stream_; }

 private:
  void *stream_ = nullptr;
  std::vector<void *> blocks_;
};

// ------------------------------------------------------------------------
// QPsolver / QPsolver_EiQuadProg (QPBaseClass.cpp:20-56): min 0.5 x'Gx + g0'x
// s.t. CE'x + ce0 = 0, CI'x + ci0 >= 0 (EiQuadProg.hpp:15-36), quirk-compatible
// Goldfarb-Idnani in fp64 on the GPU.  Capacity n <= 64, p <= 64, m <= 320
// (qloco_gi_limits; the reference's QPBaseClass asserts nVars <= 60, nIneq <=
// 300, QPBaseClass.cpp:111-112): gi_kernel up to n, p <= 16 / m <= 64,
// gi_wide_kernel above that.
class QPsolverGpu {
 public:
  explicit QPsolverGpu(int max_batch = 1);
  ~QPsolverGpu();
  void resize(const int &nVar, const int &nEq, const int &nIneq);
  // One QP; matrices column-major (G n*n, CE n*p, CI n*m).  Returns the cost
  // (+inf when infeasible, as solve_quadprog).  G is left unchanged.
  double solve(const double *G, const double *g0, const double *CE, const double *ce0,
               const double *CI, const double *ci0, double *X);
  // B QPs of the current size; host arrays of B consecutive instances.
  void solve_batch(int batch, const double *G, const double *g0, const double *CE,
                   const double *ce0, const double *CI, const double *ci0, double *X,
                   double *f, int32_t *status);
  int last_status() const { return last_status_; }
  int last_iterations() const { return last_iters_; }

 private:
  int n_ = 0, p_ = 0, m_ = 0, cap_ = 0, max_batch_;
  int an_ = 0, ap_ = 0, am_ = 0;  // sizes the current device blocks were allocated for
  DeviceArena arena_;
  double *dG_ = nullptr, *dg0_ = nullptr, *dCE_ = nullptr, *dce0_ = nullptr, *dCI_ = nullptr,
         *dci0_ = nullptr, *dX_ = nullptr, *df_ = nullptr;
  int32_t *dst_ = nullptr, *dit_ = nullptr;
  int last_status_ = 0, last_iters_ = 0;
  void ensure(int batch);
};

// QPBaseClass (QPBaseClass.h:19-73): owns the QP buffers, solveQP() reports
// success as "no NaN in X" and ignores the cost (QPBaseClass.cpp:126-152).
class QPBaseClassGpu {
 public:
  std::vector<double> G, g0, CE, ce0, CI, ci0, X;
  int nVars = 0, nEq = 0, nIneq = 0;
  void resizeQP(const int &nVars, const int &nEq, const int &nIneq);
  bool solveQP();

 private:
  QPsolverGpu solver_{1};
};

// ------------------------------------------------------------------------
// Dynamiccclass (go1_rt_control/src/whole_body_dynamics/dynmics_compute.h:59-76).
// force_distribution + force_opt of robot r are staged; the batch runs on
// the GPU when force_opt is called for the last robot (robot == batch-1),
// or explicitly with run().  For batch == 1 this is exactly the reference's
// call sequence (servo.cpp:1224-1228).  Leg order FR, FL, RR, RL.
class Dynamiccclass {
 public:
  explicit Dynamiccclass(int batch = 1, const qloco_force_params *params = nullptr);
  void force_distribution(const double com_des[3], const double leg_des[12],
                          const double F_force_des[6], int mode, double y_coefficient,
                          const double rfoot_des[3], const double lfoot_des[3], int robot = 0);
  void force_opt(const double base_p[3], const double FR_p[3], const double FL_p[3],
                 const double RR_p[3], const double RL_p[3], const double FT_total_des[6],
                 int mode, int right_support, double y_coefficient, int robot = 0);
  void run();
  // compute_joint_torques for all legs of all robots (dynmics_compute.cpp:109-138)
  void compute_joint_torques(const double *Jaco /*B*4*9*/, const int32_t *swing /*B*4*/,
                             const double *p_des, const double *p_est, const double *pv_des,
                             const double *pv_est, double *tau /*B*12*/);
  // reference result members, B consecutive records
  std::vector<double> grf_opt;      // 12 per robot
  std::vector<double> F_leg_ref;    // 3x4 col-major per robot
  std::vector<double> F_leg_guess;  // 12 per robot
  std::vector<int32_t> qp_solution, status, iters;
  int batch() const { return batch_; }

 private:
  int batch_;
  qloco_force_params prm_;
  DeviceArena arena_;
  std::vector<double> h_com_, h_leg_, h_F_, h_rf_, h_lf_, h_base_, h_feet_, h_FT_, h_y_;
  std::vector<int32_t> h_mode_, h_rs_;
  double *d_com_, *d_leg_, *d_F_, *d_rf_, *d_lf_, *d_base_, *d_feet_, *d_FT_, *d_y_, *d_Fref_,
      *d_grf_, *d_guess_;
  int32_t *d_mode_, *d_rs_, *d_qps_, *d_st_, *d_it_;
  int32_t *d_ord_;           // grouped-launch workspace (qloco_force_order_ws_len)
  double *d_jt_ = nullptr;   // joint-torque staging (allocated on first use)
  int32_t *d_sw_ = nullptr;
};

// ------------------------------------------------------------------------
// PRMPCClass::body_theta_mpc (rt_mpc_qp/src/FastMPC/PRMPCClass.h:69-71): the
// 8-variable body-inclination QP with the reference's member state
// (thetaxk/thetayk, V_ini, bjx1/bjx2/t_yu), one record per robot.
class PRMPCClass {
 public:
  explicit PRMPCClass(int batch = 1);
  // Eigen 2x5 / 3x5 inputs as column-major arrays; returns the 14-vector
  // [thx0, thy0, taux0, tauy0, zmpx0, zmpy0, thx1, thy1, zmpx1, zmpy1, thx2, thy2,
  //  zmpx2, zmpy2] (PRMPCClass.cpp:696-709).  Nrtfoorpr_gen is unused by the
  // reference body and accepted for signature compatibility.
  std::array<double, 14> body_theta_mpc(int i, const double bodyangle_state[4],
                                        const double zmp_ref[10], const double angle_ref[10],
                                        const double rfoot_ref[10], const double lfoot_ref[10],
                                        const double comacc_ref[15],
                                        const double Nrtfoorpr_gen[9] = nullptr);
  // B robots at once (host arrays, B consecutive records each); com_traj B*14.
  void body_theta_mpc_batch(const int32_t *i, const double *bodyangle_state, const double *zmp_ref,
                            const double *angle_ref, const double *rfoot_ref,
                            const double *lfoot_ref, const double *comacc_ref, double *com_traj);
  int Indexfind(double goal_P);
  std::vector<double> state;  // QLOCO_BODY_STATE_LEN doubles per robot (host mirror)

 private:
  int batch_;
  DeviceArena arena_;
  double *d_state_, *d_in_, *d_traj_, *d_t_;
  int32_t *d_i_, *d_st_, *d_j_;
};

// ------------------------------------------------------------------------
// A1RobotControl::compute_grf, MPC branch (A1RobotControl.cpp:452-600) over B
// robots: x0 and the desired trajectory are built exactly as :459-497, the
// batched fused build + OSQP-algorithm ADMM runs on the GPU, and the forces
// come back in the body frame (root_rot_mat' u, :596-599).  A leg whose
// solution is NaN keeps its previous output (the reference's isnan guard).
// Like the reference's member OsqpEigen::Solver (A1RobotControl.h:67, set up
// once with warm start on, then update* + solve every tick, :556-578), each
// robot's solver persists across compute_grf calls (spec.warm_start = 2, the
// per-robot record on the device) and, by default, solves the reference's
// literal 12N-variable QP (spec.literal_full_qp = 1), so every call after
// the first takes OSQP's update path as the reference's does, contact
// changes included; reset() forgets it.  Pass a spec with warm_start = 0
// for independent cold solves, literal_full_qp = 0 for the faster
// stance-only reduction (same optimum; DESIGN.md §3c for its persistence).
struct A1MpcState {                // the A1CtrlStates fields compute_grf reads
  double root_euler[3], root_pos[3], root_ang_vel[3], root_lin_vel[3];
  double root_rot_mat[9];          // col-major; used for root_lin_vel_d_world
  double root_euler_d[3], root_pos_d[3], root_ang_vel_d[3], root_lin_vel_d[3];
  double foot_pos_abs[12];         // 3x4 col-major, legs FL, FR, RL, RR
  bool contacts[4];
};

class ConvexMpcBatch {
 public:
  ConvexMpcBatch(int batch, const qloco_srbd_spec *spec = nullptr);
  // Multi-GPU (include/qloco.h §10): this object is rank `rank` of `world`
  // (one process or thread per GPU, its device current) over a global batch
  // of `total` robots.  It owns the shard qloco_mgpu_shard assigns
  // (shard_first + k * shard_stride, k < shard_count): compute_grf takes and
  // returns that shard, and one RCCL all-gather per call leaves every
  // robot's forces (same frame, same NaN guard) in all_forces(), total * 12,
  // on every rank.  comm_id: qloco_mgpu_unique_id() on rank 0, shipped to
  // the other ranks by the caller (QLOCO_MGPU_ID_BYTES bytes).
  ConvexMpcBatch(int64_t total, int world, int rank, const uint8_t *comm_id,
                 int shard_mode = QLOCO_SHARD_CONTIGUOUS, const qloco_srbd_spec *spec = nullptr);
  ~ConvexMpcBatch();
  ConvexMpcBatch(const ConvexMpcBatch &) = delete;
  ConvexMpcBatch &operator=(const ConvexMpcBatch &) = delete;
  const std::vector<double> &all_forces() const { return all_forces_; }
  int64_t shard_first = 0, shard_count = 0, shard_stride = 1;
  // foot_forces_grf: B * 12 (3x4 col-major per robot), in/out
  void compute_grf(const A1MpcState *states, double *foot_forces_grf);
  // device-resident form (inputs already in HBM): thin wrapper of qloco_srbd_solve_ex
  void solve_device(const float *x0, const float *x_ref, const float *feet,
                    const uint8_t *contacts, float *u0, int32_t *status, int32_t *iters);
  void reset();  // fresh solvers (the next call sets each one up again)
  // settings / weights may be edited between calls; horizon and warm_start
  // size the device buffers and are fixed at construction (a changed value
  // throws qloco::Error on the next call)
  qloco_srbd_spec spec;
  std::vector<int32_t> status, iters;

 private:
  void check_spec() const;
  int batch_;
  int horizon_ = 0, warm_mode_ = 0;
  DeviceArena arena_;
  float *d_x0_, *d_xr_, *d_feet_, *d_u0_, *d_rec_ = nullptr;
  uint8_t *d_ct_;
  int32_t *d_st_, *d_it_;
  // multi-GPU form
  qloco_mgpu *mg_ = nullptr;
  int64_t total_ = 0;
  float *d_u0_all_ = nullptr;
  int32_t *d_st_all_ = nullptr, *d_it_all_ = nullptr;
  std::vector<double> all_forces_;
};

// ------------------------------------------------------------------------
// A1RobotControl::compute_grf, QP branch (stance_leg_control_type == 0,
// A1RobotControl.cpp:383-450) over B robots: the A1CtrlStates fields it
// reads, the weights / gains of qloco_a1_params, one cold OSQP solve per
// robot (fp64, qloco_a1_qp_solve), forces in the body frame.
struct A1QpState {
  double root_pos[3], root_pos_d[3], root_euler[3], root_euler_d[3];
  double root_lin_vel[3], root_lin_vel_d[3], root_ang_vel[3], root_ang_vel_d[3];
  double root_rot_mat[9], root_rot_mat_z[9];  // col-major
  double foot_pos_abs[12];                    // 3x4 col-major, legs FL, FR, RL, RR
  bool contacts[4];
};

class A1QpBatch {
 public:
  A1QpBatch(int batch, const qloco_a1_params *params = nullptr);
  // foot_forces_grf: B * 12 (3x4 col-major per robot)
  void compute_grf(const A1QpState *states, double *foot_forces_grf);
  qloco_a1_params params;
  std::vector<int32_t> status, iters;

 private:
  int batch_;
  DeviceArena arena_;
  double *d_state_, *d_forces_;
  uint8_t *d_ct_;
  int32_t *d_st_, *d_it_;
};


// ------------------------------------------------------------------------
// Kinematicclass (go1_rt_control/src/kinematics/Kinematics.h:30-61).  The
// per-leg methods keep the reference's signatures and leave the Jacobian of
// the last evaluation in Jacobian_kin (3x3 col-major), as the servo reads it
// (servo.cpp:735, :1039); the batch methods run n legs in one launch and are
// the intended use on the GPU (one leg per call is a host<->device round trip).
// feet_flag: 0 FR, 1 FL, 2 RR, 3 RL.  body_R = (roll, pitch, yaw).
class Kinematicclass {
 public:
  explicit Kinematicclass(int max_legs = 4);
  std::array<double, 3> Forward_kinematics(const double q_joint[3], int feet_flag);
  std::array<double, 3> Forward_kinematics_g(const double body_P[3], const double body_R[3],
                                             const double q_joint[3], int feet_flag);
  std::array<double, 3> Inverse_kinematics(const double pos_des[3], const double q_ini[3],
                                           int feet_flag);
  std::array<double, 3> Inverse_kinematics_g(const double body_P[3], const double body_R[3],
                                             const double pos_des[3], const double q_ini[3],
                                             int feet_flag);
  // n legs (host arrays, row layout of qloco_leg_fk / qloco_leg_ik); body_p /
  // body_r both NULL for the hip frame.  jac / pos_out / updates may be NULL.
  void forward_batch(int n, const double *q, const int32_t *leg, const double *body_p,
                     const double *body_r, double *pos, double *jac);
  void inverse_batch(int n, const double *pos_des, const double *q_ini, const int32_t *leg,
                     const double *body_p, const double *body_r, double *q_out, double *pos_out,
                     double *jac, int32_t *updates);
  std::array<double, 9> Jacobian_kin{};  // after the last per-leg call
  std::array<double, 3> pos_cal{};       // FK at the last IK result (the reference's pos_cal)
  int last_updates = 0;                  // Newton steps of the last per-leg IK

 private:
  int cap_;
  DeviceArena arena_;
  double *d_a_, *d_b_, *d_p_, *d_r_, *d_q_, *d_pos_, *d_jac_;
  int32_t *d_leg_, *d_upd_;
  void ensure(int n);
};

// ------------------------------------------------------------------------
// The rt_mpc_qp node (unitree_ros/rt_mpc_qp/src/gait_fast.cpp) for B robots:
// the two subscriber callbacks store the latest /MPC/Gait (100 doubles,
// :79-89) and /control2rtmpc/state (25 doubles, :92-110) message of a robot;
// loop_once() runs one iteration of the 100 Hz loop (:505-735) -- reference
// interpolation, PRMPCClass contact schedule / swing-foot / foot-rotation
// generators, body_theta_mpc -- for every robot on the GPU (qloco_rt_tick)
// and leaves the outgoing messages in `traj` (/rtMPC/traj, 100 per robot)
// and `nrt` (/rt2nrt/state, 25 per robot; valid when published(robot)).
class RtMpcNode {
 public:
  explicit RtMpcNode(int batch = 1);
  void nrt_gait_sub_operation(const double msg[QLOCO_GAIT_MSG_LEN], int robot = 0);
  void control_gait_sub_operation(const double msg[QLOCO_CTRL_MSG_LEN], int robot = 0);
  void loop_once();
  bool published(int robot = 0) const { return sched[robot * QLOCO_RT_SCHED_LEN + 6] != 0; }
  std::vector<double> traj;     // B * 100
  std::vector<double> nrt;      // B * 25
  std::vector<int32_t> sched;   // B * QLOCO_RT_SCHED_LEN (bjx1, bjxx, t_end, counters, ...)
  int batch() const { return batch_; }

 private:
  int batch_;
  DeviceArena arena_;
  std::vector<double> gait_, ctrl_;
  void *d_ws_;
  double *d_gait_, *d_ctrl_, *d_traj_, *d_nrt_;
  int32_t *d_sched_;
};

// ------------------------------------------------------------------------
// The go1 servo loop's force block (servo.cpp:1052-1243, :1318) for B robots:
// one call per servo tick replaces the F_sum / F_lr_predict / swing-flag
// glue, Dynam.force_distribution + force_opt and the four
// compute_joint_torques calls.  Host arrays of B consecutive records; legs
// FR, FL, RR, RL; Jaco = the four Jacobian_kin (3x3 col-major) per robot.
class ServoForceBlock {
 public:
  explicit ServoForceBlock(int batch = 1, const qloco_force_params *params = nullptr);
  void step(const double *coma_des, const double *com_des, const double *rfoot_des,
            const double *lfoot_des, const double *body_p_des, const double *foot_des,
            const int32_t *right_support, const int32_t *gait_mode, const double *y_offset,
            const int32_t *count_in_rt_loop, const double *Jaco, const double *foot_rel_mea,
            const double *v_est_rel);
  std::vector<double> F_sum, Force_L_R, grf_opt, Legs_torque;  // 6, 6, 12, 12 per robot
  std::vector<int32_t> swing, qp_solution, status;             // 4, 1, 1 per robot
  int batch() const { return batch_; }

 private:
  int batch_;
  qloco_force_params prm_;
  DeviceArena arena_;
  void *d_ws_;
  double *d_in_, *d_out_;
  int32_t *d_iin_, *d_iout_;
};

}  // namespace qloco
