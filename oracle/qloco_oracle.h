/*
 * qloco_oracle.h -- CPU restatement of the reference's hot-path algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the *checker*: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product (quadrupedal_loco_amd/, libqloco.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned".  The reference (jtdingx/quadrupedal_loco)
 * holds no golden vectors or known-answer tests for this path (SURVEY.md §4,
 * §8c), and its sources cannot be compiled here: EiQuadProg.cpp needs Eigen,
 * ConvexMpc needs OsqpEigen/OSQP, dynmics_compute.cpp needs ROS -- none of
 * them is present in the image.  The restatement below follows the cited
 * reference lines; the committed fixtures under tests/golden/ were generated
 * from this restatement (tests/golden/make_golden.py) and are self-checked
 * against analytic KKT certificates, not against reference outputs.
 *
 * Conventions: all matrices are column-major (Eigen's default storage), i.e.
 * M(r,c) = M[c*rows + r], so an Eigen `.data()` pointer maps 1:1.
 * Everything is double precision, like the reference.
 */
#ifndef QLOCO_ORACLE_H
#define QLOCO_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  QO_OK = 0,
  QO_MAX_ITER = 1,
  QO_INFEASIBLE = 2,   /* EiQuadProg returned +inf (t >= inf) */
  QO_NAN = 3,
  QO_BAD_SIZE = 4,
  QO_NOT_PD = 5,       /* LLT failed (EiQuadProg.cpp:507-510) */
  QO_DEGENERATE = 6,   /* dependent equalities: early return (EiQuadProg.cpp:270-275) */
  QO_UB_PATH = 7,      /* reference would read an uninitialised index (EiQuadProg.cpp:105-110) */
  QO_SOLVED_INACCURATE = 8
};

/* ------------------------------------------------------------------ */
/* EiQuadProg (Goldfarb-Idnani dual active set), quirk-compatible.     */
/* utils/EiQuadProg/EiQuadProg.cpp:4-513                              */
/* ------------------------------------------------------------------ */
typedef struct qo_eqp_ws qo_eqp_ws;
qo_eqp_ws *qo_eqp_create(int n, int p, int m);
void qo_eqp_destroy(qo_eqp_ws *ws);
/* min 0.5 x'Gx + g0'x  s.t.  CE'x + ce0 = 0,  CI'x + ci0 >= 0.
 * G (n*n) is overwritten by its Cholesky factor, like the reference.
 * CE is n*p, CI is n*m (column = one constraint).  Returns f_value or +inf.
 * status: QO_OK / QO_INFEASIBLE / QO_NOT_PD / QO_DEGENERATE / QO_UB_PATH.
 * iters: number of passes through label l1 (the reference's `iter`).      */
double qo_eqp_solve(qo_eqp_ws *ws, double *G, const double *g0,
                    const double *CE, const double *ce0,
                    const double *CI, const double *ci0,
                    double *x, int *status, int *iters);

/* ------------------------------------------------------------------ */
/* Go1 force QP: Dynamiccclass (go1_rt_control/.../dynmics_compute.cpp) */
/* ------------------------------------------------------------------ */
typedef struct {
  double mass;       /* 12      dynmics_compute.cpp:31  */
  double alpha;      /* 1e4     :61 */
  double beta;       /* 1e3     :62 */
  double gamma;      /* 10      :63 */
  double fz_max;     /* 160     :64 */
  double mu;         /* 0.25 (sim) / 0.5 (HW copy)  :65 */
} qo_force_params;
void qo_force_params_default(qo_force_params *p);

typedef struct {
  double F_leg_ref[12];   /* 3x4 col-major, columns FR,FL,RR,RL */
  double F_leg_guess[12];
  double grf_opt[12];     /* solution; also F_prev for the next call (:305) */
  int qp_solution;
  qo_eqp_ws *ws;          /* persistent Eigen::QP object (n=12,p=12,m=24) */
} qo_dyn_state;
void qo_dyn_init(qo_dyn_state *s);
void qo_dyn_free(qo_dyn_state *s);
/* dynmics_compute.cpp:141-261 */
void qo_force_distribution(qo_dyn_state *s, const double com_des[3],
                           const double leg_des[12], const double F_force_des[6],
                           int mode, double y_coefficient,
                           const double rfoot_des[3], const double lfoot_des[3]);
/* dynmics_compute.cpp:265-373 (+ solve_grf_opt :387-427, Solve :432-445).
 * Returns qp_solution.  eqp_status/iters are optional (may be NULL).      */
int qo_force_opt(qo_dyn_state *s, const qo_force_params *prm,
                 const double base_p[3], const double FR_p[3], const double FL_p[3],
                 const double RR_p[3], const double RL_p[3],
                 const double FT_total_des[6], int mode, int right_support,
                 double y_coefficient, int *eqp_status, int *iters);
/* batch driver (CPU baseline): force_distribution + force_opt for n robots,
 * row layout of qloco_force_qp_solve; states = n initialised records */
void qo_force_batch(int64_t n, qo_dyn_state *states, const qo_force_params *prm,
                    const double *com_des, const double *leg_des, const double *F_force_des,
                    const double *rfoot_des, const double *lfoot_des, const double *base_p,
                    const double *feet_p, const double *FT_total_des, const int32_t *mode,
                    const int32_t *right_support, const double *y_coef, double *grf_opt);
/* unitree_legged_real torque_mode.cpp:1370-1384 (hardware feed-forward):
 * ramp-blended grf_opt, tau = -J' F per leg, legs FR, FL, RR, RL */
void qo_hw_torque_ff(const double Jaco[36], const double grf_opt[12], const double grf_base[12],
                     int32_t dynamic_count, double tau[12]);
/* dynmics_compute.cpp:109-138; Jaco 3x3 col-major; swing_flag = `support_flag` */
void qo_compute_joint_torques(const qo_dyn_state *s, const double Jaco[9],
                              int swing_flag, const double p_des[3],
                              const double p_est[3], const double pv_des[3],
                              const double pv_est[3], int leg_number,
                              double tau_out[3]);

/* ------------------------------------------------------------------ */
/* Body-inclination MPC QP part: PRMPCClass (rt_mpc_qp/src/FastMPC)    */
/* ------------------------------------------------------------------ */
#define QO_FOOTSTEPS 27
#define QO_NH 4
typedef struct {
  /* schedule / constants fixed by Initialize() (PRMPCClass.cpp:157-374) */
  double tx[QO_FOOTSTEPS];
  int nsum_mpc, nstepx;
  double dt_mpc, j_ini, mass, g;
  double a[4], b[2];                        /* 2x2 col-major, 2x1 */
  double pps[QO_NH * 2], pvs[QO_NH * 2];    /* nh x 2 col-major */
  double ppu[QO_NH * QO_NH], pvu[QO_NH * QO_NH];
  double ppu_2[QO_NH * QO_NH], pvu_2[QO_NH * QO_NH];
  double thetax_max, thetax_min, thetay_max, thetay_min;
  double torque_max, torque_min;
  double zmpx_max, zmpx_min, zmpy_max, zmpy_min;
  double Rthetax, Rthetay, alphathetax, alphathetay, beltathetax, beltathetay,
         gama_zmpx, gama_zmpy;
  /* member state carried between calls */
  double thetaxk[2], thetayk[2];
  double V_ini[2 * QO_NH];
  double thetax[QO_NH], thetay[QO_NH], torquex_real[QO_NH], torquey_real[QO_NH],
         zmpx_real[QO_NH], zmpy_real[QO_NH];
  int bjx1, bjx2, t_yu;
  int qp_solution;
  qo_eqp_ws *ws;    /* n=8, p=0, m=48 (columns 32..47 inert, see below) */
} qo_body_state;
void qo_body_init(qo_body_state *s);
void qo_body_free(qo_body_state *s);
/* PRMPCClass::Indexfind, PRMPCClass.cpp:716-738 (xyz=0 branch) */
int qo_body_indexfind(const qo_body_state *s, double goal);
/* PRMPCClass::body_theta_mpc, PRMPCClass.cpp:379-714.  Reference refs are
 * Eigen 2x5 / 3x5 col-major.  Only columns 0..nh-1 are read (:384-388).  */
int qo_body_theta_mpc(qo_body_state *s, int i, const double bodyangle_state[4],
                      const double zmp_ref[10], const double angle_ref[10],
                      const double rfoot_ref[10], const double lfoot_ref[10],
                      const double comacc_ref[15], const double Nrtfoorpr_gen[9],
                      double com_traj[14], int *eqp_status);

/* ------------------------------------------------------------------ */
/* rt_mpc_qp node tick: gait_fast.cpp:505-735 + PRMPCClass reference     */
/* generators (rt_tick.c).  One opaque record per robot.                */
/* ------------------------------------------------------------------ */
#define QO_RT_SCHED 8
typedef struct qo_rt qo_rt;
/* PRMPCClass() + Initialize() + gait_fast.cpp main() init, n robots */
qo_rt *qo_rt_create_n(int64_t n);
void qo_rt_destroy_n(qo_rt *arr, int64_t n);
/* One loop iteration per robot with the latest /MPC/Gait gait[n*100] and
 * /control2rtmpc/state ctrl[n*25] -> /rtMPC/traj traj[n*100] and the last
 * /rt2nrt/state nrt[n*25].  Optional: gen[n*60] = foorpr_gen | foortheta_gen,
 * sched[n*QO_RT_SCHED] = bjx1, bjxx, t_end_footstep, count_in_rt_mpc, t_int,
 * body EiQuadProg status (-1: body_theta_mpc not called), flags (bit 0:
 * /rt2nrt/state published), bjx2. */
void qo_rt_tick_n(qo_rt *arr, int64_t n, const double *gait, const double *ctrl, double *traj,
                  double *nrt, double *gen, int32_t *sched);
/* row-major 4x4 inverse used for solve_AAA_inv* (Gauss-Jordan, partial pivoting) */
void qo_inv4(const double A[16], double Ainv[16]);

/* ------------------------------------------------------------------ */
/* go1 servo force block: servo.cpp:1052-1243, :1318 (servo_block.c)    */
/* ------------------------------------------------------------------ */
typedef struct {
  qo_dyn_state dyn;      /* Dynamiccclass members (F_leg_ref, grf_opt, QP object) */
  int swing[4];          /* FR_swing, FL_swing, RR_swing, RL_swing */
  double rel_des_old[12];/* *_foot_relative_des_old */
  double v_rel[12];      /* *_v_relative */
} qo_servo_state;
void qo_servo_init(qo_servo_state *s);
void qo_servo_free(qo_servo_state *s);
/* One servo tick's force block for one robot; legs FR, FL, RR, RL; Jaco 4 x
 * (3x3 col-major).  Outputs F_sum, Force_L_R (F_lr_predict), rleg_com
 * (optional), grf_opt (force_opt result), tau (12), swing flags (optional).
 * Returns qp_solution. */
int qo_servo_force_block(qo_servo_state *s, const qo_force_params *prm, const double coma_des[3],
                         const double com_des[3], const double rfoot_des[3],
                         const double lfoot_des[3], const double body_p_des[3],
                         const double foot_des[12], int right_support, int gait_mode,
                         double y_offset, int loop_count, const double Jaco[36],
                         const double rel_mea[12], const double v_est[12], double F_sum[6],
                         double Force_L_R[6], double *rleg_com_out, double grf_opt[12],
                         double tau[12], int swing_out[4], int *eqp_status);
void qo_servo_batch(int64_t n, qo_servo_state *states, const qo_force_params *prm,
                    const double *coma, const double *com, const double *rfoot,
                    const double *lfoot, const double *body_p, const double *foot,
                    const int32_t *rs, const int32_t *mode, const double *y,
                    const int32_t *loop, const double *Jaco, const double *rel_mea,
                    const double *v_est, double *grf_opt, double *tau);

/* ------------------------------------------------------------------ */
/* SRBD convex MPC: ConvexMpc + A1RobotControl::compute_grf            */
/* ------------------------------------------------------------------ */
#define QO_NX 13
#define QO_NU 12
#define QO_NC 20
typedef struct {
  int N;
  double dt, mass, inertia[9]; /* inertia col-major (symmetric) */
  double q_w[13], r_w[12];
  double mu, fz_min, fz_max;
} qo_srbd_spec;
/* ConvexMpc.cpp:111-133 */
void qo_srbd_A_c(double yaw, double A_c[169]);
/* ConvexMpc.cpp:135-147 with Utils::skew (utils/Utils.cpp:35-41).
 * R col-major 3x3; feet 3x4 col-major (leg i = column i). */
void qo_srbd_B_c(double mass, const double inertia[9], const double R[9],
                 const double feet[12], double B_c[156]);
/* ConvexMpc.cpp:149-160 (forward Euler) */
void qo_srbd_discretize(const double A_c[169], const double B_c[156], double dt,
                        double A_d[169], double B_d[156]);
/* ConvexMpc.cpp:162-264, literal dense restatement.
 * B_d_list: N blocks of 13x12 (block k at B_d_list + 156k).
 * contacts: 4 flags (constant over horizon, like the reference) or 4N flags
 * (per-step generalisation) selected by contacts_per_step.
 * Outputs (any may be NULL): Aqp (13N x 13), Bqp (13N x 12N), H (12N x 12N),
 * g (12N), lb/ub (20N).  +-1e30 stands for OsqpEigen::INFTY.              */
void qo_srbd_qp_mats(const qo_srbd_spec *sp, const double A_d[169],
                     const double *B_d_list, const double x0[13],
                     const double *x_ref, const uint8_t *contacts,
                     int contacts_per_step, double *Aqp, double *Bqp, double *H,
                     double *g, double *lb, double *ub);
/* Linear constraint matrix C (20N x 12N dense col-major), ConvexMpc.cpp:47-59 */
void qo_srbd_constraints(const qo_srbd_spec *sp, double *C);
/* compute_grf MPC branch (A1RobotControl.cpp:452-600) on one instance:
 * x0 (13), x_ref (13N), feet (12 = constant, or 12N per step), contacts
 * (4 or 4N).  Builds A_c from x0 yaw, the yaw matrix R (:502-510), B_c per
 * step, discretises, builds the QP and writes H/g/lb/ub (sizes as above). */
void qo_srbd_build_instance(const qo_srbd_spec *sp, const double x0[13],
                            const double *x_ref, const double *feet,
                            int feet_per_step, const uint8_t *contacts,
                            int contacts_per_step, double *H, double *g,
                            double *lb, double *ub);

/* ------------------------------------------------------------------ */
/* OSQP ADMM restatement (OSQP v0.6.x algorithm, default settings)      */
/* ------------------------------------------------------------------ */
typedef struct {
  double rho, sigma, alpha, eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
  int max_iter, check_termination, scaling, adaptive_rho,
      adaptive_rho_interval; /* 0 -> 4*check_termination (non-PROFILING build) */
  double adaptive_rho_tolerance;
  int warm_start;
} qo_admm_settings;
void qo_admm_settings_default(qo_admm_settings *s);
typedef struct {
  int iters, rho_updates, status;
  double obj, pri_res, dua_res, rho_final;
} qo_admm_info;
/* min 0.5x'Px + q'x  s.t.  l <= A x <= u.  P n*n dense (full symmetric),
 * A m*n dense col-major.  x (n) and y (m) are in/out (warm start if set). */
int qo_admm_solve(const qo_admm_settings *st, int n, int m, const double *P,
                  const double *q, const double *A, const double *l,
                  const double *u, double *x, double *y, qo_admm_info *info);
/* Extended entry: how the iterates start and what survives the solve.
 *   QO_ADMM_COLD   x = z = y = 0, rho = settings rho (osqp_setup + solve)
 *   QO_ADMM_WARM   osqp_warm_start from UNSCALED x, y (z = A x)
 *   QO_ADMM_RESUME OsqpEigen's update*() + solve() on a live solver with
 *                  warm start on (A1RobotControl.cpp:556-575): scaled x, z, y
 *                  carried as they are, rho = the adapted rho of the last
 *                  solve, Ruiz's cost scale computed with q_scale (the
 *                  previous, unscaled q) before the new q is scaled in.
 * out (may be NULL): scaled final x (n), z (m), y (m) and rho.            */
enum { QO_ADMM_COLD = 0, QO_ADMM_WARM = 1, QO_ADMM_RESUME = 2 };
typedef struct {
  int mode;
  const double *x, *z, *y; /* WARM: unscaled x, y; RESUME: scaled x, z, y */
  double rho;              /* RESUME */
  const double *q_scale;   /* RESUME: previous unscaled q (NULL = new q) */
} qo_admm_init;
typedef struct {
  double *x, *z, *y;
  double rho;
} qo_admm_state;
int qo_admm_solve_ex(const qo_admm_settings *st, int n, int m, const double *P,
                     const double *q, const double *A, const double *l, const double *u,
                     const qo_admm_init *in, qo_admm_state *out, double *x, double *y,
                     qo_admm_info *info);

/* Persistent SRBD MPC solver: the reference's member OsqpEigen::Solver
 * (A1RobotControl.h:67) called every control tick (A1RobotControl.cpp:556-
 * 578) -- restated on the stance-only QP the GPU kernel solves.  Same stance
 * set as the last call: QO_ADMM_RESUME.  Stance set changed (the reduced
 * problem's dimensions change): a fresh setup warm-started from the last
 * unscaled solution, as OsqpEigen's re-initialisation path does
 * (clearSolver + initSolver + setPrimal/DualVariable).  First call: cold.
 * The record is full-index (12N variables, 20N rows) like the GPU's:
 * QO_SRBD_PERSIST_LEN(N) doubles, layout in qloco.h (qloco_srbd_spec). */
#define QO_SRBD_PERSIST_LEN(N) (100 * (N) + 4)
int qo_srbd_persist_step(double *rec, const qo_srbd_spec *sp, const qo_admm_settings *st,
                         const float *x0, const float *x_ref, const float *feet,
                         int feet_per_step, const uint8_t *contacts, int contacts_per_step,
                         double *u, qo_admm_info *info);
/* literal = 1: the reference's semantics on its literal 12N-variable QP
 * (every (step, leg) pair a variable, swing pairs held by fz in [0, 0]):
 * the first call is a cold setup, EVERY later call takes QO_ADMM_RESUME --
 * OsqpEigen's updateHessianMatrix finds the (contact-independent, dense)
 * Hessian pattern unchanged and calls osqp_update_P, then
 * osqp_update_lin_cost and osqp_update_{lower,upper}_bound, whose
 * update_rho_vec re-types the fz rows whose contact flag changed
 * (equality <-> inequality, rho_vec from the adapted rho); osqp_solve then
 * starts from the scaled x, z, y of the last solve.  literal = 0: as
 * qo_srbd_persist_step. */
int qo_srbd_persist_step_ex(double *rec, const qo_srbd_spec *sp, const qo_admm_settings *st,
                            const float *x0, const float *x_ref, const float *feet,
                            int feet_per_step, const uint8_t *contacts, int contacts_per_step,
                            int literal, double *u, qo_admm_info *info);

/* Exact optimum of the same box/row-bounded QP via the EiQuadProg
 * restatement (p = 0, so none of the equality quirks apply).             */
int qo_exact_solve(int n, int m, const double *P, const double *q, const double *A,
                   const double *l, const double *u, double *x, int *iters);

/* ------------------------------------------------------------------ */
/* A1 single-step force QP: A1RobotControl::compute_grf with            */
/* stance_leg_control_type == 0 (A1RobotControl.cpp:383-450, ctor :8-49) */
/* (a1_qp.c).  12 variables (legs FL, FR, RL, RR), 20 rows, OSQP.        */
/* ------------------------------------------------------------------ */
#define QO_A1_STATE_LEN 54
typedef struct {
  double kp_linear[3], kd_linear[3], kp_angular[3], kd_angular[3];
  double robot_mass;
  double q_diag[6], r, mu, f_min, f_max;
} qo_a1_params;
void qo_a1_params_default(qo_a1_params *p);
/* the QP the branch hands to OSQP: H (12x12), g, linearMatrix A (20x12,
 * col-major), bounds; root_acc (6) as computed at :384-397 */
void qo_a1_qp_build(const qo_a1_params *p, const double *state, const uint8_t contacts[4],
                    double root_acc[6], double H[144], double g[12], double A[240],
                    double l[20], double u[20]);
/* build + cold OSQP-algorithm solve + rotation into the body frame
 * (:445-449).  x (world-frame QPSolution, 12) and info may be NULL. */
int qo_a1_compute_grf(const qo_a1_params *p, const qo_admm_settings *st, const double *state,
                      const uint8_t contacts[4], double forces_body[12], double x[12],
                      qo_admm_info *info);

/* ------------------------------------------------------------------ */
/* Deterministic synthetic instances.                   */
/* Restated independently from the product's generator; tests compare. */
/* ------------------------------------------------------------------ */
uint64_t qo_splitmix64(uint64_t x);
/* gait: 0 = trot, 1 = pace/biped (reference gait_mode 101), 2 = mixed
 * per-step schedule (config 5), 3 = all stance.  Outputs fp32 arrays for
 * instances [first, first+count): x0 (13), x_ref (13N), feet (12),
 * contacts (4N, uint8).  Leg order FL,FR,RL,RR (ConvexMpc / A1).           */
void qo_gen_srbd(uint64_t seed, int N, double dt, int gait, int64_t first,
                 int64_t count, float *x0, float *x_ref, float *feet,
                 uint8_t *contacts);

/* Batch driver (baseline.c): build + solve `count` instances with
 * solver 0 = ADMM restatement (CPU-A), 1 = exact EiQuadProg (CPU-B), using
 * nthreads pthreads.  u: count x 12N (may be NULL).  seconds: wall time.  */
int qo_srbd_batch(const qo_srbd_spec *sp, const qo_admm_settings *st, int solver,
                  int64_t count, const float *x0, const float *x_ref, const float *feet,
                  int feet_per_step, const uint8_t *contacts, int contacts_per_step,
                  double *u, int *iters, int *status, double *obj, int nthreads,
                  double *seconds);


/* ------------------------------------------------------------------ */
/* Go1 leg kinematics: go1_rt_control/src/kinematics/Kinematics.cpp     */
/* (kinematics.c).  flag 0 FR, 1 FL, 2 RR, 3 RL; J 3x3 col-major.        */
/* ------------------------------------------------------------------ */
/* Forward_kinematics :63-142 (hip frame) */
void qo_leg_fk(const double q[3], int flag, double pos[3], double J[9]);
/* Forward_kinematics_g :145-229 (world frame; body_R = roll, pitch, yaw) */
void qo_leg_fk_g(const double body_P[3], const double body_R[3], const double q[3], int flag,
                 double pos[3], double J[9]);
/* Inverse_kinematics :233-267 (body_P = body_R = NULL) or
 * Inverse_kinematics_g :270-304.  Returns the number of Newton updates. */
int qo_leg_ik(const double *body_P, const double *body_R, const double pos_des[3],
              const double q_ini[3], int flag, double q_des[3], double pos[3], double J[9]);
/* batch drivers (CPU baseline), row layout of qloco_leg_fk / qloco_leg_ik */
void qo_leg_fk_batch(int64_t n, const double *q, const int32_t *leg, const double *body_p,
                     const double *body_r, double *pos, double *J);
void qo_leg_ik_batch(int64_t n, const double *pos_des, const double *q_ini, const int32_t *leg,
                     const double *body_p, const double *body_r, double *q, double *pos, double *J,
                     int32_t *updates);

/* ------------------------------------------------------------------ */
/* Slow planner's contact-phase flag (support_phase.c): NLPClass_sqp.cpp */
/* :1029-1039 schedule indices + Foot_trajectory_solve_mod2 right_support */
/* ------------------------------------------------------------------ */
/* ts, tx: n x 27 (row per robot); t_int, t_end_footstep: n.  Outputs n. */
void qo_support_phase(int64_t n, const double *ts, const double *tx, const int32_t *t_int,
                      const int32_t *t_end_footstep, int32_t *bjxx, int32_t *bjx1,
                      int32_t *right_support);

#ifdef __cplusplus
}
#endif
#endif
