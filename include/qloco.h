/*
 * qloco.h -- C ABI of the MI355X-native batched convex-MPC solver
 * (libqloco.so).  Plain pointers and sizes only; no torch / Eigen types.
 *
 * Every entry point below replaces one interface of the reference
 * (jtdingx/quadrupedal_loco, paths relative to its root) and is batched over
 * independent instances.  Device entry points take DEVICE pointers that are
 * already resident in HBM plus a hipStream_t (passed as void*; NULL = the
 * default stream); they only enqueue work and return immediately.  Host
 * entry points (suffix _host) take host pointers and block.
 *
 * Layout conventions
 *  - instance-major ("AoS per field"): field f of instance b lives at
 *    ptr[b * len(f) + k]; one instance's data is contiguous, so the one
 *    wavefront that owns the instance reads it with coalesced loads.
 *  - small matrices mirror Eigen's default column-major storage.
 *  - SRBD leg order is ConvexMpc's FL, FR, RL, RR (A1CtrlStates.h:44-46);
 *    force-QP leg order is the Go1 servo's FR, FL, RR, RL (servo.cpp:1054-1058).
 *
 * Errors: every function returns a qloco_status (0 = success).  Per-instance
 * solver outcomes go to the status[] arrays, mirroring QPBaseClass::solveQP
 * (QPBaseClass.cpp:126-152), which reports failure only through NaN in X.
 */
#ifndef QLOCO_H
#define QLOCO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QLOCO_ABI_VERSION 1

typedef enum qloco_status {
  QLOCO_OK = 0,
  QLOCO_MAX_ITER = 1,          /* ADMM hit max_iter (OSQP_MAX_ITER_REACHED)          */
  QLOCO_INFEASIBLE = 2,        /* EiQuadProg returned +inf (EiQuadProg.cpp:394-400)   */
  QLOCO_NAN = 3,               /* non-finite solution                                 */
  QLOCO_BAD_SIZE = 4,          /* sizes outside the compiled limits                   */
  QLOCO_NOT_PD = 5,            /* Cholesky failed (EiQuadProg.cpp:507-510)            */
  QLOCO_DEGENERATE = 6,        /* dependent equalities (EiQuadProg.cpp:270-275)       */
  QLOCO_UB_PATH = 7,           /* reference reads an uninitialised index (:105-110)   */
  QLOCO_SOLVED_INACCURATE = 8, /* OSQP_SOLVED_INACCURATE                              */
  QLOCO_ERR_ARG = 100,         /* invalid argument (call-level)                       */
  QLOCO_ERR_DEVICE = 101,      /* HIP runtime error (call-level)                      */
  QLOCO_ERR_NO_GPU = 102       /* no gfx950 device visible                            */
} qloco_status;

const char *qloco_status_string(int status);
int qloco_abi_version(void);
/* last HIP error string of the calling thread (empty if none) */
const char *qloco_last_error(void);

/* ====================================================================== */
/* 1. SRBD convex MPC (Go1, N-step horizon, 12 contact forces)             */
/*    replaces ConvexMpc (a1_cpp_open_source/src/ConvexMpc.h:22-94,        */
/*    ConvexMpc.cpp:8-264) + the OSQP solve in                             */
/*    A1RobotControl::compute_grf (A1RobotControl.cpp:452-600)             */
/* ====================================================================== */
typedef struct qloco_srbd_spec {
  int32_t horizon;           /* N = PLAN_HORIZON (A1Params.h:26)                   */
  int32_t feet_per_step;     /* 0: feet[12] per instance (compute_grf); 1: [12N]   */
  int32_t contacts_per_step; /* 0: contacts[4] (ConvexMpc.cpp:232-249); 1: [4N]    */
  int32_t output_frame;      /* 0: u0 = QP solution (world);                        */
                             /* 1: R^T u0 per leg (compute_grf return, :596-599)    */
  float dt;                  /* mpc_dt = 0.0025 (A1RobotControl.cpp:469)            */
  float mass;                /* robot_mass                                           */
  float inertia[9];          /* trunk inertia, col-major                             */
  float q_weights[13];       /* ConvexMpc ctor q_weights_ (Q = diag(2q))             */
  float r_weights[12];       /* r_weights_ (R = diag(2r))                            */
  float mu;                  /* 0.3 (ConvexMpc.cpp:9)                                */
  float fz_min, fz_max;      /* 0 / 180 (ConvexMpc.cpp:227-228)                      */
  /* ADMM settings: OSQP names and defaults */
  float rho, sigma, alpha, eps_abs, eps_rel;
  int32_t max_iter, check_termination, scaling, adaptive_rho, adaptive_rho_interval;
  float adaptive_rho_tolerance;
  int32_t warm_start;        /* 0: cold start every call                            */
                             /* 1: osqp_warm_start from the unscaled x|y in warm    */
                             /*    (B*32N floats, in/out)                           */
                             /* 2: persistent solver, the reference's member        */
                             /*    OsqpEigen::Solver (A1RobotControl.cpp:556-578):  */
                             /*    warm = B*QLOCO_SRBD_PERSIST_LEN(N) floats, zeroed */
                             /*    before the first call; see DESIGN.md §3          */
  int32_t polish;            /* must be 0: OSQP polishing is not implemented (the    */
                             /* reference leaves it off); 1 -> QLOCO_ERR_ARG         */
  int32_t literal_full_qp;   /* 0: the stance-only reduction (swing forces removed  */
                             /*    exactly; same optimum, fastest kernels)          */
                             /* 1: the reference's call as written: all 12N forces  */
                             /*    are ADMM variables, swing legs held by their     */
                             /*    fz in [fz_min*c, fz_max*c] = [0, 0] rows (OSQP   */
                             /*    equality rows, rho_eq = 1e3 rho), Ruiz over the  */
                             /*    full P and A (ConvexMpc.cpp:162-264,             */
                             /*    A1RobotControl.cpp:557-578); DESIGN.md §3e       */
  int32_t reserved[5];
} qloco_srbd_spec;

/* Per-instance record of the persistent solver (spec.warm_start == 2),
 * floats, full index (variable 12k+3i+c, constraint row 20k+5i+r):
 *   [0,12N) scaled x  [12N,32N) scaled z  [32N,52N) scaled y
 *   [52N,64N) unscaled x  [64N,84N) unscaled y  [84N,96N) unscaled q
 *   [96N,100N) contact flags  [100N] rho  [100N+1] 1 after the first call.
 * literal_full_qp = 1 (the reference's semantics): the first call sets the
 * solver up, EVERY later call takes OSQP's update path (osqp_update_P /
 * _lin_cost / _lower_bound / _upper_bound + solve: Ruiz on the new P with
 * the previous q in the cost scale, the rho vector re-typed from the new
 * bounds, the adapted rho kept, the scaled x, z, y carried) -- the
 * reference's Hessian pattern does not depend on the contacts, so OsqpEigen
 * never re-initialises.  literal_full_qp = 0 (stance-only reduction, whose
 * variable set follows the stance set): same stance set as the last call ->
 * the update path; a changed stance set re-initialises (settings rho),
 * warm-started from the last unscaled solution -- a documented deviation
 * from the reference. */
#define QLOCO_SRBD_PERSIST_LEN(N) (100 * (N) + 4)

/* Go1 SRBD constants + OSQP default settings. */
void qloco_srbd_spec_default(qloco_srbd_spec *spec);

/* Largest stance-variable count the compiled kernels accept (3 x 4 x 20). */
int qloco_srbd_max_stance_vars(void);

/* Batched build + ADMM solve (the hot path).  Device pointers:
 *   x0[B*13]        mpc_states: [rpy, p, omega, v, -9.8]   (A1RobotControl.cpp:459-463)
 *   x_ref[B*13N]    mpc_states_d                             (:480-497)
 *   feet[B*12] or [B*12N]  foot_pos_abs, 3 per leg (FL,FR,RL,RR)
 *   contacts[B*4] or [B*4N] uint8 0/1
 * Outputs (NULL = not wanted, except u0):
 *   u0[B*12]        first-step forces (frame per spec->output_frame)
 *   u[B*12N]        full solution (world frame)
 *   status[B], iters[B] (ADMM iterations), obj[B] (QP objective)
 *   warm[B*(12N+20N)] in/out x|y warm-start state when spec->warm_start. */
int qloco_srbd_solve(const qloco_srbd_spec *spec, int64_t batch, const float *x0,
                     const float *x_ref, const float *feet, const uint8_t *contacts,
                     float *u0, float *u, int32_t *status, int32_t *iters, float *obj,
                     float *warm, void *stream);

/* Extended form of qloco_srbd_solve: additionally returns rho_updates[B]
 * (number of adaptive-rho refactorisations) and takes max_stance_legs, the
 * largest number of stance (step, leg) pairs of any instance in the batch,
 * or 0 = unknown (assume 4N).  Instances run by class: <= 21 stance pairs
 * in one-wavefront workgroups, 22..42 in two-wavefront workgroups, 43..80
 * (up to N = 20 all-stance, 240 variables) in the wide 512-thread kernel --
 * one launch per class the maximum admits, on the stream.  Any N <= 20
 * schedule is accepted; an instance with more stance pairs than a
 * caller-supplied max_stance_legs admits gets status QLOCO_BAD_SIZE, NaN u0 /
 * u / obj and iters = 0. */
int qloco_srbd_solve_ex(const qloco_srbd_spec *spec, int64_t batch, const float *x0,
                        const float *x_ref, const float *feet, const uint8_t *contacts,
                        float *u0, float *u, int32_t *status, int32_t *iters,
                        int32_t *rho_updates, float *obj, float *warm,
                        int32_t max_stance_legs, void *stream);

/* The kernel family a qloco_srbd_solve[_ex] call with this spec runs
 * (host-only, no device work; the solve uses the same decision):
 *   QLOCO_ROUTE_LIT_ONE_WAVE  literal QP, N <= 10: srbd_lit_kernel (one wavefront
 *                             per instance, the OSQP solve through the wrench space)
 *   QLOCO_ROUTE_LIT_TWO_WAVE  literal QP, N = 11..20: srbd_lit2_kernel
 *   QLOCO_ROUTE_LIT_GENERIC   literal QP otherwise (a q_omega / q_v weight of 0,
 *                             a state weight above 1000, per-step feet, N > 20):
 *                             the 12N-variable kernels
 *   QLOCO_ROUTE_REDUCED       literal_full_qp = 0: the stance-only classes
 * The Go1 defaults and the reference's config/{gazebo,hardware}_a1_mpc.yaml
 * sets take the wrench-space kernels, and so would anisotropic omega
 * weights of that size; config/isaac_a1_mpc.yaml's (roll 8000) take the
 * generic ones, where float32 converges as float64 does (the wrench-space
 * solve's precision limit).  Returns QLOCO_ERR_ARG on a bad
 * spec. */
#define QLOCO_ROUTE_LIT_ONE_WAVE 1
#define QLOCO_ROUTE_LIT_TWO_WAVE 2
#define QLOCO_ROUTE_LIT_GENERIC 3
#define QLOCO_ROUTE_REDUCED 4
int qloco_srbd_route(const qloco_srbd_spec *spec);

/* Class-dispatch scratch of qloco_srbd_solve_ex (instance lists, counters,
 * side streams, events): one set per (device, caller stream), at most 8
 * live -- the least recently used set beyond that is released.  Returns the
 * live sets; *pinned (may be NULL) = allocations kept for the life of the
 * process because a stream capture baked them into a graph. */
int qloco_srbd_scratch_sets(int32_t *pinned);

/* Batched condensed-QP build only (ConvexMpc::calculate_qp_mats, dense,
 * as the reference materialises it).  Outputs per instance (NULL = skip):
 *   H[B*(12N)^2] col-major, g[B*12N], lb[B*20N], ub[B*20N] (+-1e30 = INFTY),
 *   Aqp[B*13N*13], Bqp[B*13N*12N] col-major. */
int qloco_srbd_build(const qloco_srbd_spec *spec, int64_t batch, const float *x0,
                     const float *x_ref, const float *feet, const uint8_t *contacts,
                     float *H, float *g, float *lb, float *ub, float *Aqp, float *Bqp,
                     void *stream);

/* Deterministic synthetic instances, host memory.
 * gait: 0 trot, 1 pace (reference gait_mode 101), 2 mixed per-step, 3 stance.
 * x_ref must hold count*13N floats, contacts count*4N bytes. */
int qloco_gen_srbd_host(uint64_t seed, int32_t horizon, float dt, int32_t gait,
                        int64_t first, int64_t count, float *x0, float *x_ref,
                        float *feet, uint8_t *contacts);
/* Same instances for the global ids first + k * stride, k < count (the
 * interleaved shard of a rank: first = rank, stride = world). */
int qloco_gen_srbd_host_strided(uint64_t seed, int32_t horizon, float dt, int32_t gait,
                                int64_t first, int64_t stride, int64_t count, float *x0,
                                float *x_ref, float *feet, uint8_t *contacts);

/* ====================================================================== */
/* 2. Dense small-QP active-set solver (Goldfarb-Idnani), batched.          */
/*    replaces QPsolver_EiQuadProg::solve -> Eigen::QP::solve_quadprog      */
/*    (rt_mpc_qp/src/QP/QPBaseClass.cpp:36-58; EiQuadProg.cpp:172-513),     */
/*    quirk-compatible.  Double precision.              */
/*    n <= 64, p <= 64, m <= 320 (covers QPBaseClass's nVars <= 60,         */
/*    nIneq <= 300, QPBaseClass.h:49-51): n, p <= 16 and m <= 64 run four   */
/*    QPs per wavefront (bit-exact with the restatement in the common       */
/*    case), larger ones one per wavefront (to rounding; qloco_gi_wide.hip). */
/*    Matrices col-major, per instance:                                      */
/*    G[n*n] (only the lower triangle is read), g0[n], CE[n*p], ce0[p],     */
/*    CI[n*m], ci0[m].  A NULL CE/ce0/CI/ci0 with stride 0 broadcasts one    */
/*    shared copy; *_stride = elements between instances (0 = shared).     */
/*    Outputs x[B*n], f[B] (cost, +inf when infeasible), status[B],         */
/*    iters[B].                                                             */
/* ====================================================================== */
int qloco_eiquadprog_solve(int32_t n, int32_t p, int32_t m, int64_t batch, const double *G,
                           int64_t G_stride, const double *g0, int64_t g0_stride,
                           const double *CE, int64_t CE_stride, const double *ce0,
                           int64_t ce0_stride, const double *CI, int64_t CI_stride,
                           const double *ci0, int64_t ci0_stride, double *x, double *f,
                           int32_t *status, int32_t *iters, void *stream);
/* the largest n of the fast path (four QPs per wavefront, bit-exact in the */
/* common case): 16 -- unchanged since round 1; sizes above it up to        */
/* qloco_gi_limits run one QP per wavefront                                 */
int qloco_max_gi_vars(void);
/* the fast path's limits n, p, m (16, 16, 64; any pointer may be NULL)    */
void qloco_gi_fast_limits(int32_t *n, int32_t *p, int32_t *m);
/* the size limits above (QPBaseClass's capacity rounded up): n, p, m      */
/* (64, 64, 320; any pointer may be NULL)                                   */
void qloco_gi_limits(int32_t *n, int32_t *p, int32_t *m);

/* ====================================================================== */
/* 3. Go1 force-distribution QP, batched                                    */
/*    replaces Dynamiccclass::force_distribution + force_opt               */
/*    (go1_rt_control/src/whole_body_dynamics/dynmics_compute.cpp:141-373, */
/*    called at servo.cpp:1224-1228 and torque_mode.cpp:1364-1367)          */
/* ====================================================================== */
typedef struct qloco_force_params {
  double mass;    /* 12    dynmics_compute.cpp:31 */
  double alpha;   /* 1e4   :61 */
  double beta;    /* 1e3   :62 */
  double gamma;   /* 10    :63 */
  double fz_max;  /* 160   :64 */
  double mu;      /* 0.25 sim (:65), 0.5 HW copy */
} qloco_force_params;
void qloco_force_params_default(qloco_force_params *p);

/* Per-instance inputs (device, double):
 *   com_des[B*3], leg_des[B*12], F_force_des[B*6], rfoot_des[B*3],
 *   lfoot_des[B*3]      -> force_distribution arguments
 *   base_p[B*3], feet_p[B*12] (FR,FL,RR,RL), FT_total_des[B*6] -> force_opt
 *   mode[B], right_support[B] (int32), y_coef[B]
 * Per-instance state (in/out, double): F_leg_ref[B*12] (3x4 col-major),
 *   grf_opt[B*12] (previous solution = F_prev of q_goal, :305).
 * Outputs: F_leg_guess[B*12], qp_solution[B] (int32, 1 = no NaN),
 *   status[B] (EiQuadProg outcome), iters[B]. */
int qloco_force_qp_solve(const qloco_force_params *prm, int64_t batch, const double *com_des,
                         const double *leg_des, const double *F_force_des,
                         const double *rfoot_des, const double *lfoot_des,
                         const double *base_p, const double *feet_p,
                         const double *FT_total_des, const int32_t *mode,
                         const int32_t *right_support, const double *y_coef,
                         double *F_leg_ref, double *grf_opt, double *F_leg_guess,
                         int32_t *qp_solution, int32_t *status, int32_t *iters,
                         void *stream);

/* The same solve with the robots grouped by control flow before the launch
 * (swing-leg pattern, then the robot's previous active-set iteration count):
 * the four robots that share a wavefront then take the same path.  Results
 * are bit-identical to qloco_force_qp_solve.  order_ws: device int32
 * workspace of qloco_force_order_ws_len(batch) entries, allocated and
 * zero-filled once by the caller and passed unchanged on every call -- like
 * F_leg_ref / grf_opt it carries per-robot state between calls (the
 * iteration counts that predict the next call's grouping); NULL = the
 * ungrouped launch.  No allocation happens inside, so the call can be
 * captured in a HIP graph. */
int64_t qloco_force_order_ws_len(int64_t batch);
int qloco_force_qp_solve_ordered(const qloco_force_params *prm, int64_t batch,
                                 const double *com_des, const double *leg_des,
                                 const double *F_force_des, const double *rfoot_des,
                                 const double *lfoot_des, const double *base_p,
                                 const double *feet_p, const double *FT_total_des,
                                 const int32_t *mode, const int32_t *right_support,
                                 const double *y_coef, double *F_leg_ref, double *grf_opt,
                                 double *F_leg_guess, int32_t *qp_solution, int32_t *status,
                                 int32_t *iters, int32_t *order_ws, void *stream);

/* The hardware servo's Dynamiccclass constants (unitree_legged_real copy of
 * dynmics_compute.cpp:31,65: mass = gait::mass = 14, robot_const_para_config
 * .cpp:28; mu = 0.5), the call at torque_mode.cpp:1364-1367; the other
 * fields as qloco_force_params_default (the sim copy: mass 12, mu 0.25). */
void qloco_force_params_hw(qloco_force_params *p);

/* Robots per wavefront of the force-QP kernel: 8 (eight 8-lane groups, the
 * default) or 16 (four 16-lane groups).  The outputs are bit-identical
 * either way; the knob exists for A/B measurements and the test that pins
 * that identity (QLOCO_FORCE_GW=16 in the environment sets the initial
 * value).  Returns the previous width, or QLOCO_ERR_ARG for other values.
 * Process-wide; set it while no force-QP launch is being enqueued. */
int qloco_force_set_group_width(int gw);

/* The hardware loop's feed-forward after force_opt (unitree_legged_real
 * torque_mode.cpp:1370-1384): rate = min((dynamic_count / 500)^2, 1),
 * F_opt = rate (grf_opt - grf_base) + grf_base per leg (grf_base: the
 * stand-up FR_GRF .. RL_GRF of :1057-1058), tau = -J^T F_opt -- no gravity
 * compensation.  Per instance: Jaco[4*9] (col-major per leg), grf_opt[12],
 * grf_base[12], dynamic_count (int32) -> tau[12]; legs FR, FL, RR, RL. */
int qloco_hw_torque_ff(int64_t batch, const double *Jaco, const double *grf_opt,
                       const double *grf_base, const int32_t *dynamic_count, double *tau,
                       void *stream);

/* Joint torques tau = -J^T F + g_comp (stance) or PD (swing),
 * Dynamiccclass::compute_joint_torques (dynmics_compute.cpp:109-138), for
 * all 4 legs of B instances.  Jaco[B*4*9] col-major per leg, swing[B*4],
 * p_des/p_est/pv_des/pv_est[B*12], F_leg_ref[B*12] -> tau[B*12]. */
int qloco_joint_torques(int64_t batch, const double *Jaco, const int32_t *swing,
                        const double *p_des, const double *p_est, const double *pv_des,
                        const double *pv_est, const double *F_leg_ref, double *tau,
                        void *stream);

/* ====================================================================== */
/* 4. rt body-inclination MPC step, batched                                 */
/*    replaces PRMPCClass::body_theta_mpc (rt_mpc_qp/src/FastMPC/          */
/*    PRMPCClass.cpp:379-714) called at gait_fast.cpp:620                  */
/* ====================================================================== */
/* Per-instance state record (double[32]), created by qloco_body_state_init:
 *   [0:2] thetaxk  [2:4] thetayk  [4:12] V_ini  [12:26] last com_traj
 *   [26] bjx1 [27] bjx2 [28] t_yu [29] qp_solution [30:32] reserved        */
#define QLOCO_BODY_STATE_LEN 32
int qloco_body_state_init_host(int64_t batch, double *state);
/* i[B] (loop counter, int32), bodyangle_state[B*4], zmp_ref/angle_ref/
 * rfoot_ref/lfoot_ref[B*10] (Eigen 2x5 col-major), comacc_ref[B*15] (3x5)
 * -> com_traj[B*14]; state in/out; status[B] EiQuadProg outcome. */
int qloco_body_mpc_step(int64_t batch, const int32_t *i, const double *bodyangle_state,
                        const double *zmp_ref, const double *angle_ref,
                        const double *rfoot_ref, const double *lfoot_ref,
                        const double *comacc_ref, double *state, double *com_traj,
                        int32_t *status, void *stream);
/* PRMPCClass::Indexfind (PRMPCClass.cpp:716-738) on B fp64 times -> int32 */
int qloco_body_indexfind(int64_t batch, const double *t, int32_t *j_period, void *stream);

/* ====================================================================== */
/* 5. Go1 leg kinematics, batched (fp64, one leg per lane)                  */
/*    replaces Kinematicclass (go1_rt_control/src/kinematics/Kinematics.cpp) */
/*    called per leg at servo.cpp:734-741 (FK_g + Jacobian_kin) and         */
/*    servo.cpp:1038-1051 (IK_g + Jacobian_kin)                             */
/* ====================================================================== */
/* Forward_kinematics (:63-142, body_p = body_r = NULL: hip frame) or
 * Forward_kinematics_g (:145-229; body_p[n*3], body_r[n*3] = roll, pitch,
 * yaw).  q[n*3] (hip, thigh, calf), leg[n] (0 FR, 1 FL, 2 RR, 3 RL)
 * -> pos[n*3], jac[n*9] (Jacobian_kin, 3x3 column-major; may be NULL). */
int qloco_leg_fk(int64_t n, const double *q, const int32_t *leg, const double *body_p,
                 const double *body_r, double *pos, double *jac, void *stream);
/* Inverse_kinematics (:233-267, 10 damped Newton steps, lamda 0.5) or
 * Inverse_kinematics_g (:270-304, 15 steps) from q_ini[n*3] toward
 * pos_des[n*3] -> q_out[n*3]; optional pos[n*3] / jac[n*9] at q_out (the
 * reference's pos_cal / Jacobian_kin after the call) and updates[n] (Newton
 * steps applied).  Reference stop tests reproduced as written. */
int qloco_leg_ik(int64_t n, const double *pos_des, const double *q_ini, const int32_t *leg,
                 const double *body_p, const double *body_r, double *q_out, double *pos,
                 double *jac, int32_t *updates, void *stream);

/* ====================================================================== */
/* 6. rt_mpc_qp node tick, batched                 */
/*    replaces one iteration of the rt node loop, unitree_ros/rt_mpc_qp/   */
/*    src/gait_fast.cpp:505-735: callbacks (:79-110), counters and         */
/*    /rt2nrt/state (:512-527), xget_position_interpolation (:113-372 ->   */
/*    PRMPCClass::XGetSolution_position_mod3, PRMPCClass.cpp:1170-1261),   */
/*    Foot_trajectory_solve_mod2 (:1756-2195) + Indexfind (:716-738),      */
/*    XGetSolution_Foot_rotation (:2255-2380), body_theta_mpc (:379-714)   */
/*    and the /rtMPC/traj message (gait_fast.cpp:633-729)                  */
/* ====================================================================== */
/* Wire formats, one message per robot, row-major [B][len], double:
 *   /MPC/Gait            gait_msg[B*100]  (NLPRTControlClass.cpp:284-392;
 *                        [86..94] = Nrtfoorpr_gen, [99] = mpc_gait_flag)
 *   /control2rtmpc/state ctrl_msg[B*25]   ([0] > 0 starts the loop; [10],
 *                        [11], [13], [14] = bodyangle_state, gait_fast.cpp:105-108)
 *   /rtMPC/traj          traj_msg[B*100]  ([0..35] = gait_msg[0..35],
 *                        [36..86] = low_mpc_gait_inte, [86] = 0 (the node's
 *                        wall-clock duration), [98] = (int)_tx_total/0.001,
 *                        [99] = count_in_rt_loop)
 *   /rt2nrt/state        nrt_msg[B*25]    (last published state_to_MPC)  */
#define QLOCO_GAIT_MSG_LEN 100
#define QLOCO_CTRL_MSG_LEN 25
#define QLOCO_TRAJ_MSG_LEN 100
#define QLOCO_NRT_MSG_LEN 25
/* sched[B*8] (optional): bjx1, bjxx, t_end_footstep, count_in_rt_mpc, t_int,
 * body EiQuadProg status (-1 = body_theta_mpc not called this tick),
 * /rt2nrt/state published this tick (0/1), bjx2 */
#define QLOCO_RT_SCHED_LEN 8
/* Bytes of the device workspace holding B robots' node + PRMPCClass state. */
int64_t qloco_rt_workspace_bytes(int64_t batch);
/* PRMPCClass() + Initialize() + gait_fast.cpp main() init (:384-502) for B
 * robots, on device. */
int qloco_rt_init(int64_t batch, void *workspace, void *stream);
/* One loop iteration for B robots, given each robot's latest /MPC/Gait and
 * /control2rtmpc/state (device pointers).  gen[B*60] (optional) =
 * foorpr_gen (30) | foortheta_gen (30). */
int qloco_rt_tick(int64_t batch, void *workspace, const double *gait_msg,
                  const double *ctrl_msg, double *traj_msg, double *nrt_msg, double *gen,
                  int32_t *sched, void *stream);

/* ====================================================================== */
/* 7. go1 servo force block, batched                */
/*    replaces servo.cpp:1052-1243 (+ :1318) of go1_rt_control: leg        */
/*    positions, body-relative desired feet and their velocity, F_sum,      */
/*    rleg_com / F_lr_predict, swing flags, then Dynamiccclass::            */
/*    force_distribution + force_opt and compute_joint_torques x 4          */
/* ====================================================================== */
/* Per-robot inputs (device, double unless noted), legs FR, FL, RR, RL:
 *   coma_des[B*3], com_des[B*3], rfoot_des[B*3], lfoot_des[B*3],
 *   body_p_des[B*3], foot_des[B*12] (desired feet, world frame),
 *   right_support[B], gait_mode[B], loop_count[B] (int32; count_in_rt_loop),
 *   y_offset[B], Jaco[B*4*9] (each leg's 3x3 Jacobian_kin, col-major),
 *   foot_rel_mea[B*12] (measured foot - body), v_est_rel[B*12].
 * Outputs: grf_opt[B*12] and tau[B*12] (Legs_torque) required; F_sum[B*6],
 *   Force_L_R[B*6] (F_lr_predict), swing[B*4], qp_solution[B], status[B]
 *   optional.  Member / loop state (F_leg_ref, grf_opt, swing flags,
 *   relative_des_old, v_relative) lives in the workspace. */
int64_t qloco_servo_workspace_bytes(int64_t batch);
int qloco_servo_init(int64_t batch, void *workspace, void *stream);
int qloco_servo_force_block(const qloco_force_params *prm, int64_t batch, void *workspace,
                            const double *coma_des, const double *com_des,
                            const double *rfoot_des, const double *lfoot_des,
                            const double *body_p_des, const double *foot_des,
                            const int32_t *right_support, const int32_t *gait_mode,
                            const double *y_offset, const int32_t *loop_count,
                            const double *Jaco, const double *foot_rel_mea,
                            const double *v_est_rel, double *F_sum, double *Force_L_R,
                            double *grf_opt, double *tau, int32_t *swing,
                            int32_t *qp_solution, int32_t *status, void *stream);

/* ====================================================================== */
/* 8. slow planner's contact-phase flag, batched     */
/*    replaces the schedule indices of NLPClass::step_timing_opti_loop     */
/*    (mosek_nlp_kmp NLPClass_sqp.cpp:1029-1039) and the right_support     */
/*    branch of NLPClass::Foot_trajectory_solve_mod2 (:2076-2090,          */
/*    :2187-2202, :2311-2313) -- the /MPC/Gait[99] flag servo.cpp:673 reads */
/* ====================================================================== */
/* ts[B*27], tx[B*27] (device, double): each robot's _ts / _tx after the
 * planner's step-timing update (row per robot); t_int[B] (_t_int, the slow
 * loop index) and t_end_footstep[B] (int32).  Outputs (int32): bjxx[B] and
 * bjx1[B] (optional), right_support[B] (0 left, 1 right, 2 double
 * support).  Integer results are bit-exact with the restatement. */
#define QLOCO_NLP_STEPS 27
int qloco_support_phase(int64_t batch, const double *ts, const double *tx, const int32_t *t_int,
                        const int32_t *t_end_footstep, int32_t *bjxx, int32_t *bjx1,
                        int32_t *right_support, void *stream);

/* ====================================================================== */
/* 9. A1 single-step force QP, batched (fp64)                               */
/*    replaces the stance_leg_control_type == 0 branch of                  */
/*    A1RobotControl::compute_grf (unitree_ros/a1_cpp_open_source/src/     */
/*    A1RobotControl.cpp:383-450; constructor :8-49): root_acc from PD      */
/*    gains, H = R I + inv' Q inv, g = -inv' Q root_acc, 20-row friction    */
/*    pyramid / normal-force block, cold OSQP solve with default settings,  */
/*    forces rotated into the body frame.                                   */
/* ====================================================================== */
typedef struct qloco_a1_params {
  double kp_linear[3], kd_linear[3], kp_angular[3], kd_angular[3]; /* A1CtrlStates.h:123-126 */
  double robot_mass;                                                /* A1CtrlStates.h:39 */
  double q_diag[6];  /* Q (A1RobotControl.cpp:12) */
  double r;          /* R = 1e-3 (:13) */
  double mu;         /* 0.7 (:14) */
  double f_min, f_max; /* 0 / 180 (:15-16) */
  /* OSQP settings (defaults = OsqpEigen's, i.e. OSQP v0.6 defaults) */
  double rho, sigma, alpha, eps_abs, eps_rel, adaptive_rho_tolerance;
  int32_t max_iter, check_termination, scaling, adaptive_rho, adaptive_rho_interval;
  int32_t reserved[3];
} qloco_a1_params;
void qloco_a1_params_default(qloco_a1_params *p);
/* Per-robot state record, double[QLOCO_A1_STATE_LEN] (A1CtrlStates fields):
 *   [0:3] root_pos  [3:6] root_pos_d  [6:9] root_euler  [9:12] root_euler_d
 *   [12:15] root_lin_vel (world)  [15:18] root_lin_vel_d (body)
 *   [18:21] root_ang_vel (world)  [21:24] root_ang_vel_d (body)
 *   [24:33] root_rot_mat  [33:42] root_rot_mat_z  (3x3 col-major)
 *   [42:54] foot_pos_abs (3x4 col-major, legs FL, FR, RL, RR)
 * contacts[B*4] uint8.  Outputs: forces_body[B*12] (foot_forces_grf, 3x4
 * col-major) required; qp_solution[B*12] (world frame), status[B],
 * iters[B], rho_updates[B], obj[B] optional (NULL). */
#define QLOCO_A1_STATE_LEN 54
int qloco_a1_qp_solve(const qloco_a1_params *prm, int64_t batch, const double *state,
                      const uint8_t *contacts, double *forces_body, double *qp_solution,
                      int32_t *status, int32_t *iters, int32_t *rho_updates, double *obj,
                      void *stream);

/* ====================================================================== */
/* 10. Multi-GPU handles                         */
/*    The instances are independent: each rank (one process or thread per */
/*    GPU) solves its own shard of the global batch with                   */
/*    qloco_srbd_solve_ex and ONE RCCL all-gather over xGMI, on the        */
/*    caller's stream, leaves every rank with u0 of the whole batch in     */
/*    global instance order.  Replaces nothing in the reference (its       */
/*    controllers are one process each, A1RobotControl.cpp:553-578); it is */
/*    the C++ caller's way to shard.  RCCL (librccl.so.1) is loaded on     */
/*    first use.                                                           */
/* ====================================================================== */
#define QLOCO_MGPU_ID_BYTES 128
enum {
  QLOCO_SHARD_CONTIGUOUS = 0,  /* balanced contiguous ranges                        */
  QLOCO_SHARD_INTERLEAVED = 1  /* ids rank, rank + world, ... (divergent schedules) */
};
typedef struct qloco_mgpu qloco_mgpu;
/* Global ids owned by `rank`: first + k * stride, k < count.  Contiguous:
 * first = rank * (total / world) + min(rank, total % world), count = total /
 * world (+1 for rank < total % world), stride 1.  Interleaved: first = rank,
 * stride = world, count = ceil((total - rank) / world).  Host only. */
int qloco_mgpu_shard(int64_t total, int32_t world, int32_t rank, int32_t mode, int64_t *first,
                     int64_t *count, int64_t *stride);
/* Row of global id g in the gathered (world x P) buffer, P = ceil(total /
 * world) the padded shard: rows[g] = owner * P + position.  Host only (the
 * device reorder uses the same map). */
int qloco_mgpu_gather_rows(int64_t total, int32_t world, int32_t mode, int64_t *rows);
/* The device half of qloco_mgpu_solve's step 3, for a caller that runs its
 * own all-gather (e.g. torch.distributed): `stage` holds the gathered
 * (world x P x width) shard rows, P = ceil(total / world), width 12 (u0) or
 * 14 (u0, then status and iterations as raw int32 bits); writes u0_all
 * [total*12] and, for width 14, status_all / iters_all [total] (optional) in
 * global id order -- the map of qloco_mgpu_gather_rows.  Device pointers,
 * stream-ordered on `stream`. */
int qloco_mgpu_reorder(int64_t total, int32_t world, int32_t mode, int32_t width, const float *stage,
                       float *u0_all, int32_t *status_all, int32_t *iters_all, void *stream);
/* Rank 0: a new communicator id; the caller ships the bytes to every rank. */
int qloco_mgpu_unique_id(uint8_t *id /* [QLOCO_MGPU_ID_BYTES] */);
/* Collective: every rank, with its device current, the same id / world /
 * total / mode.  Allocates the rank's padded shard buffers on that device. */
int qloco_mgpu_init(qloco_mgpu **h, const uint8_t *id, int32_t world, int32_t rank, int64_t total,
                    int32_t mode);
/* This rank's shard (first, count, stride) and the padded shard size P. */
int qloco_mgpu_info(const qloco_mgpu *h, int64_t *first, int64_t *count, int64_t *stride,
                    int64_t *padded);
/* Solve this rank's shard -- x0 / x_ref / feet / contacts / warm hold ITS
 * `count` instances, laid out as for qloco_srbd_solve_ex -- then all-gather:
 * u0_all[total*12] (required), status_all[total], iters_all[total]
 * (optional) in global id order on every rank.  Collective and stream-
 * ordered on `stream` (the handle's device must be current). */
int qloco_mgpu_solve(qloco_mgpu *h, const qloco_srbd_spec *spec, const float *x0,
                     const float *x_ref, const float *feet, const uint8_t *contacts, float *warm,
                     float *u0_all, int32_t *status_all, int32_t *iters_all,
                     int32_t max_stance_legs, void *stream);
/* Releases the communicator and the buffers (NULL is a no-op). */
int qloco_mgpu_destroy(qloco_mgpu *h);

#ifdef __cplusplus
}
#endif
#endif /* QLOCO_H */
