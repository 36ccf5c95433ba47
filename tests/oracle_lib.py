"""ctypes binding of the CPU oracle (oracle/_build/libqloco_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "libqloco_oracle.so")
if os.environ.get("QLOCO_ORACLE_UBSAN") == "1":  # tests/test_sanitizers.py
    LIB_PATH = os.path.join(ORACLE_DIR, "_build_ubsan", "libqloco_oracle.so")

_lib = None

dp = C.POINTER(C.c_double)
fp = C.POINTER(C.c_float)
ip = C.POINTER(C.c_int)
u8p = C.POINTER(C.c_uint8)


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR] +
                   (["asan"] if "_build_ubsan" in LIB_PATH else []), check=True)


class SrbdSpec(C.Structure):
    _fields_ = [("N", C.c_int), ("dt", C.c_double), ("mass", C.c_double),
                ("inertia", C.c_double * 9), ("q_w", C.c_double * 13),
                ("r_w", C.c_double * 12), ("mu", C.c_double),
                ("fz_min", C.c_double), ("fz_max", C.c_double)]


class AdmmSettings(C.Structure):
    _fields_ = [("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double),
                ("eps_abs", C.c_double), ("eps_rel", C.c_double),
                ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
                ("max_iter", C.c_int), ("check_termination", C.c_int),
                ("scaling", C.c_int), ("adaptive_rho", C.c_int),
                ("adaptive_rho_interval", C.c_int),
                ("adaptive_rho_tolerance", C.c_double), ("warm_start", C.c_int)]


class AdmmInfo(C.Structure):
    _fields_ = [("iters", C.c_int), ("rho_updates", C.c_int), ("status", C.c_int),
                ("obj", C.c_double), ("pri_res", C.c_double), ("dua_res", C.c_double),
                ("rho_final", C.c_double)]


class A1Params(C.Structure):
    _fields_ = [("kp_linear", C.c_double * 3), ("kd_linear", C.c_double * 3),
                ("kp_angular", C.c_double * 3), ("kd_angular", C.c_double * 3),
                ("robot_mass", C.c_double), ("q_diag", C.c_double * 6), ("r", C.c_double),
                ("mu", C.c_double), ("f_min", C.c_double), ("f_max", C.c_double)]


class ForceParams(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("mass", "alpha", "beta", "gamma", "fz_max", "mu")]


class DynState(C.Structure):
    _fields_ = [("F_leg_ref", C.c_double * 12), ("F_leg_guess", C.c_double * 12),
                ("grf_opt", C.c_double * 12), ("qp_solution", C.c_int),
                ("ws", C.c_void_p)]


NH = 4


class BodyState(C.Structure):
    _fields_ = [("tx", C.c_double * 27), ("nsum_mpc", C.c_int), ("nstepx", C.c_int),
                ("dt_mpc", C.c_double), ("j_ini", C.c_double), ("mass", C.c_double),
                ("g", C.c_double), ("a", C.c_double * 4), ("b", C.c_double * 2),
                ("pps", C.c_double * (NH * 2)), ("pvs", C.c_double * (NH * 2)),
                ("ppu", C.c_double * (NH * NH)), ("pvu", C.c_double * (NH * NH)),
                ("ppu_2", C.c_double * (NH * NH)), ("pvu_2", C.c_double * (NH * NH)),
                ("thetax_max", C.c_double), ("thetax_min", C.c_double),
                ("thetay_max", C.c_double), ("thetay_min", C.c_double),
                ("torque_max", C.c_double), ("torque_min", C.c_double),
                ("zmpx_max", C.c_double), ("zmpx_min", C.c_double),
                ("zmpy_max", C.c_double), ("zmpy_min", C.c_double),
                ("Rthetax", C.c_double), ("Rthetay", C.c_double),
                ("alphathetax", C.c_double), ("alphathetay", C.c_double),
                ("beltathetax", C.c_double), ("beltathetay", C.c_double),
                ("gama_zmpx", C.c_double), ("gama_zmpy", C.c_double),
                ("thetaxk", C.c_double * 2), ("thetayk", C.c_double * 2),
                ("V_ini", C.c_double * (2 * NH)),
                ("thetax", C.c_double * NH), ("thetay", C.c_double * NH),
                ("torquex_real", C.c_double * NH), ("torquey_real", C.c_double * NH),
                ("zmpx_real", C.c_double * NH), ("zmpy_real", C.c_double * NH),
                ("bjx1", C.c_int), ("bjx2", C.c_int), ("t_yu", C.c_int),
                ("qp_solution", C.c_int), ("ws", C.c_void_p)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.qo_eqp_create.restype = C.c_void_p
        L.qo_eqp_create.argtypes = [C.c_int] * 3
        L.qo_eqp_destroy.argtypes = [C.c_void_p]
        L.qo_eqp_solve.restype = C.c_double
        L.qo_eqp_solve.argtypes = [C.c_void_p, dp, dp, dp, dp, dp, dp, dp, ip, ip]
        L.qo_splitmix64.restype = C.c_uint64
        L.qo_splitmix64.argtypes = [C.c_uint64]
        L.qo_gen_srbd.argtypes = [C.c_uint64, C.c_int, C.c_double, C.c_int, C.c_int64,
                                  C.c_int64, fp, fp, fp, u8p]
        L.qo_srbd_build_instance.argtypes = [C.POINTER(SrbdSpec), dp, dp, dp, C.c_int, u8p,
                                             C.c_int, dp, dp, dp, dp]
        L.qo_srbd_qp_mats.argtypes = [C.POINTER(SrbdSpec), dp, dp, dp, dp, u8p, C.c_int,
                                      dp, dp, dp, dp, dp, dp]
        L.qo_srbd_constraints.argtypes = [C.POINTER(SrbdSpec), dp]
        L.qo_srbd_A_c.argtypes = [C.c_double, dp]
        L.qo_srbd_B_c.argtypes = [C.c_double, dp, dp, dp, dp]
        L.qo_srbd_discretize.argtypes = [dp, dp, C.c_double, dp, dp]
        L.qo_admm_settings_default.argtypes = [C.POINTER(AdmmSettings)]
        L.qo_admm_solve.restype = C.c_int
        L.qo_admm_solve.argtypes = [C.POINTER(AdmmSettings), C.c_int, C.c_int, dp, dp, dp, dp,
                                    dp, dp, dp, C.POINTER(AdmmInfo)]
        L.qo_exact_solve.restype = C.c_int
        L.qo_exact_solve.argtypes = [C.c_int, C.c_int, dp, dp, dp, dp, dp, dp, ip]
        L.qo_srbd_batch.restype = C.c_int
        L.qo_srbd_batch.argtypes = [C.POINTER(SrbdSpec), C.POINTER(AdmmSettings), C.c_int,
                                    C.c_int64, fp, fp, fp, C.c_int, u8p, C.c_int, dp, ip, ip,
                                    dp, C.c_int, dp]
        L.qo_force_params_default.argtypes = [C.POINTER(ForceParams)]
        L.qo_dyn_init.argtypes = [C.POINTER(DynState)]
        L.qo_dyn_free.argtypes = [C.POINTER(DynState)]
        L.qo_force_distribution.argtypes = [C.POINTER(DynState), dp, dp, dp, C.c_int,
                                            C.c_double, dp, dp]
        L.qo_force_opt.restype = C.c_int
        L.qo_force_opt.argtypes = [C.POINTER(DynState), C.POINTER(ForceParams), dp, dp, dp,
                                   dp, dp, dp, C.c_int, C.c_int, C.c_double, ip, ip]
        L.qo_compute_joint_torques.argtypes = [C.POINTER(DynState), dp, C.c_int, dp, dp, dp,
                                               dp, C.c_int, dp]
        L.qo_hw_torque_ff.argtypes = [dp, dp, dp, C.c_int32, dp]
        L.qo_body_init.argtypes = [C.POINTER(BodyState)]
        L.qo_body_free.argtypes = [C.POINTER(BodyState)]
        L.qo_body_indexfind.restype = C.c_int
        L.qo_body_indexfind.argtypes = [C.POINTER(BodyState), C.c_double]
        L.qo_leg_fk.argtypes = [dp, C.c_int, dp, dp]
        L.qo_leg_fk_g.argtypes = [dp, dp, dp, C.c_int, dp, dp]
        L.qo_leg_ik.restype = C.c_int
        L.qo_leg_ik.argtypes = [dp, dp, dp, dp, C.c_int, dp, dp, dp]
        L.qo_leg_fk_batch.argtypes = [C.c_int64] + [C.c_void_p] * 6
        L.qo_leg_ik_batch.argtypes = [C.c_int64] + [C.c_void_p] * 9
        L.qo_body_theta_mpc.restype = C.c_int
        L.qo_body_theta_mpc.argtypes = [C.POINTER(BodyState), C.c_int, dp, dp, dp, dp, dp,
                                        dp, dp, dp, ip]
        L.qo_rt_create_n.restype = C.c_void_p
        L.qo_rt_create_n.argtypes = [C.c_int64]
        L.qo_rt_destroy_n.argtypes = [C.c_void_p, C.c_int64]
        L.qo_rt_tick_n.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 6
        L.qo_inv4.argtypes = [dp, dp]
        L.qo_support_phase.argtypes = [C.c_int64] + [C.c_void_p] * 7
        L.qo_srbd_persist_step.restype = C.c_int
        L.qo_srbd_persist_step.argtypes = [dp, C.POINTER(SrbdSpec), C.POINTER(AdmmSettings),
                                           fp, fp, fp, C.c_int, u8p, C.c_int, dp,
                                           C.POINTER(AdmmInfo)]
        L.qo_srbd_persist_step_ex.restype = C.c_int
        L.qo_srbd_persist_step_ex.argtypes = [dp, C.POINTER(SrbdSpec), C.POINTER(AdmmSettings),
                                              fp, fp, fp, C.c_int, u8p, C.c_int, C.c_int, dp,
                                              C.POINTER(AdmmInfo)]
        L.qo_a1_params_default.argtypes = [C.POINTER(A1Params)]
        L.qo_a1_qp_build.argtypes = [C.POINTER(A1Params), dp, u8p, dp, dp, dp, dp, dp, dp]
        L.qo_a1_compute_grf.restype = C.c_int
        L.qo_a1_compute_grf.argtypes = [C.POINTER(A1Params), C.POINTER(AdmmSettings), dp, u8p,
                                        dp, dp, C.POINTER(AdmmInfo)]
        _lib = L
    return _lib


class ServoState(C.Structure):
    _fields_ = [("dyn", DynState), ("swing", C.c_int * 4), ("rel_des_old", C.c_double * 12),
                ("v_rel", C.c_double * 12)]


class ServoOracle:
    """B go1 servo force blocks in the C restatement (oracle/servo_block.c)."""

    def __init__(self, batch):
        L = lib()
        L.qo_servo_init.argtypes = [C.POINTER(ServoState)]
        L.qo_servo_free.argtypes = [C.POINTER(ServoState)]
        L.qo_servo_force_block.restype = C.c_int
        L.qo_servo_force_block.argtypes = ([C.POINTER(ServoState), C.POINTER(ForceParams)] +
                                           [dp] * 6 + [C.c_int, C.c_int, C.c_double, C.c_int] +
                                           [dp] * 3 + [dp, dp, dp, dp, dp, ip, ip])
        self.batch = batch
        self.states = (ServoState * batch)()
        for s in self.states:
            L.qo_servo_init(C.byref(s))
        self.prm = ForceParams()
        L.qo_force_params_default(C.byref(self.prm))

    def step(self, d):
        B = self.batch
        out = {"F_sum": np.zeros((B, 6)), "Force_L_R": np.zeros((B, 6)),
               "grf_opt": np.zeros((B, 12)), "tau": np.zeros((B, 12)),
               "swing": np.zeros((B, 4), np.int32), "qp_solution": np.zeros(B, np.int32),
               "status": np.zeros(B, np.int32)}
        row = lambda k, b: np.ascontiguousarray(d[k][b], np.float64)
        for b in range(B):
            sw = np.zeros(4, np.int32)
            st = C.c_int(0)
            ins = [row(k, b) for k in ("coma_des", "com_des", "rfoot_des", "lfoot_des",
                                       "body_p_des", "foot_des")]
            J, rm, ve = row("Jaco", b), row("foot_rel_mea", b), row("v_est_rel", b)
            o = [np.zeros(6), np.zeros(6), np.zeros(12), np.zeros(12)]
            ok = lib().qo_servo_force_block(
                C.byref(self.states[b]), C.byref(self.prm), *[P(a) for a in ins],
                int(d["right_support"][b]), int(d["gait_mode"][b]), float(d["y_offset"][b]),
                int(d["loop_count"][b]), P(J), P(rm), P(ve), P(o[0]), P(o[1]), None, P(o[2]),
                P(o[3]), sw.ctypes.data_as(ip), C.byref(st))
            out["F_sum"][b], out["Force_L_R"][b], out["grf_opt"][b], out["tau"][b] = o
            out["swing"][b], out["qp_solution"][b], out["status"][b] = sw, ok, st.value
        return out

    def __del__(self):
        if getattr(self, "states", None) is not None and _lib is not None:
            try:
                for s in self.states:
                    _lib.qo_servo_free(C.byref(s))
            except Exception:
                pass
            self.states = None


class RtOracle:
    """B rt_mpc_qp nodes in the C restatement (oracle/rt_tick.c)."""
    SCHED = 8

    def __init__(self, batch):
        self.batch = batch
        self.h = lib().qo_rt_create_n(batch)

    def tick(self, gait, ctrl):
        B = self.batch
        gait = np.ascontiguousarray(gait, np.float64)
        ctrl = np.ascontiguousarray(ctrl, np.float64)
        traj, nrt = np.zeros((B, 100)), np.zeros((B, 25))
        gen, sched = np.zeros((B, 60)), np.zeros((B, self.SCHED), np.int32)
        lib().qo_rt_tick_n(self.h, B, gait.ctypes.data, ctrl.ctypes.data, traj.ctypes.data,
                           nrt.ctypes.data, gen.ctypes.data, sched.ctypes.data)
        return traj, nrt, gen, sched

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            try:
                _lib.qo_rt_destroy_n(self.h, self.batch)
            except Exception:  # interpreter teardown
                pass
            self.h = None


class BodyStep:
    """body_theta_mpc of the C restatement on a caller-supplied _tx / _bjx1
    (the per-robot members the rt generators rewrite) -- for tests/rt_ref.py."""

    def __init__(self):
        self.s = BodyState()
        lib().qo_body_init(C.byref(self.s))

    def __call__(self, i, bodyangle_state, zmp, ang, rfoot, lfoot, acc, tx, bjx1):
        for j in range(27):
            self.s.tx[j] = float(tx[j])
        self.s.bjx1 = int(bjx1)
        col = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).T.reshape(-1))
        out = np.zeros(14)
        st = C.c_int(0)
        bs = np.ascontiguousarray(bodyangle_state, np.float64)
        args = [col(zmp), col(ang), col(rfoot), col(lfoot), col(acc)]
        nrt = np.zeros(9)
        lib().qo_body_theta_mpc(C.byref(self.s), int(i), P(bs), *[P(a) for a in args], P(nrt),
                                P(out), C.byref(st))
        return out, self.s.bjx1, st.value


def P(a, t=C.c_double):
    return a.ctypes.data_as(C.POINTER(t))


GO1_INERTIA = 2.0 * np.array([[0.0168352186, 0.0004636141, 0.0002367952],
                              [0.0004636141, 0.0656071082, 3.6671e-05],
                              [0.0002367952, 3.6671e-05, 0.0742720659]])
Q_W = [20.0, 10.0, 1.0, 0.0, 0.0, 420.0, 0.05, 0.05, 0.05, 30.0, 30.0, 10.0, 0.0]
R_W = [1e-7] * 12


def srbd_spec(N=10, dt=0.0025, mass=12.0, inertia=GO1_INERTIA, q_w=Q_W, r_w=R_W, mu=0.3,
              fz_min=0.0, fz_max=180.0):
    s = SrbdSpec()
    s.N = N
    s.dt = dt
    s.mass = mass
    for i, v in enumerate(np.asarray(inertia, dtype=np.float64).T.ravel()):
        s.inertia[i] = v
    for i, v in enumerate(q_w):
        s.q_w[i] = v
    for i, v in enumerate(r_w):
        s.r_w[i] = v
    s.mu, s.fz_min, s.fz_max = mu, fz_min, fz_max
    return s


def admm_settings(**kw):
    s = AdmmSettings()
    lib().qo_admm_settings_default(C.byref(s))
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def gen_srbd(seed, N, count, gait=0, first=0, dt=0.0025):
    x0 = np.zeros((count, 13), np.float32)
    xr = np.zeros((count, 13 * N), np.float32)
    ft = np.zeros((count, 12), np.float32)
    ct = np.zeros((count, 4 * N), np.uint8)
    lib().qo_gen_srbd(seed, N, float(np.float32(dt)), gait, first, count, P(x0, C.c_float), P(xr, C.c_float),
                      P(ft, C.c_float), P(ct, C.c_uint8))
    return x0, xr, ft, ct


def build_instance(spec, x0, xr, feet, contacts, contacts_per_step=1, feet_per_step=0):
    N = spec.N
    n, m = 12 * N, 20 * N
    H = np.zeros((n, n))
    g = np.zeros(n)
    lb = np.zeros(m)
    ub = np.zeros(m)
    x0d = np.ascontiguousarray(x0, np.float64)
    xrd = np.ascontiguousarray(xr, np.float64)
    ftd = np.ascontiguousarray(feet, np.float64)
    ct = np.ascontiguousarray(contacts, np.uint8)
    lib().qo_srbd_build_instance(C.byref(spec), P(x0d), P(xrd), P(ftd), feet_per_step,
                                 P(ct, C.c_uint8), contacts_per_step, P(H), P(g), P(lb), P(ub))
    return H.T.copy(), g, lb, ub  # H is symmetric; .T converts col-major view


def constraints(spec):
    N = spec.N
    Cm = np.zeros((12 * N, 20 * N))  # col-major storage of a 20N x 12N matrix
    lib().qo_srbd_constraints(C.byref(spec), P(Cm))
    return Cm.T.copy()  # (20N, 12N) row-major numpy


def admm_solve(H, g, A, l, u, settings=None, x=None, y=None):
    n, m = H.shape[0], A.shape[0]
    settings = settings or admm_settings()
    Hc = np.asfortranarray(H).ravel(order="F").copy()
    Ac = np.asfortranarray(A).ravel(order="F").copy()
    x = np.zeros(n) if x is None else x.astype(np.float64).copy()
    y = np.zeros(m) if y is None else y.astype(np.float64).copy()
    info = AdmmInfo()
    g = np.ascontiguousarray(g, np.float64)
    l = np.ascontiguousarray(l, np.float64)
    u = np.ascontiguousarray(u, np.float64)
    st = lib().qo_admm_solve(C.byref(settings), n, m, P(Hc), P(g), P(Ac), P(l), P(u), P(x),
                             P(y), C.byref(info))
    return x, y, info


def exact_solve(H, g, A, l, u):
    n, m = H.shape[0], A.shape[0]
    Hc = np.asfortranarray(H).ravel(order="F").copy()
    Ac = np.asfortranarray(A).ravel(order="F").copy()
    x = np.zeros(n)
    it = C.c_int(0)
    g = np.ascontiguousarray(g, np.float64)
    l = np.ascontiguousarray(l, np.float64)
    u = np.ascontiguousarray(u, np.float64)
    st = lib().qo_exact_solve(n, m, P(Hc), P(g), P(Ac), P(l), P(u), P(x), C.byref(it))
    return x, st, it.value


def leg_fk(q, flag, body_p=None, body_r=None):
    """Kinematics.cpp Forward_kinematics(_g) restatement: (pos[3], J[9] col-major)."""
    q = np.ascontiguousarray(q, np.float64)
    pos = np.zeros(3)
    J = np.zeros(9)
    if body_p is None:
        lib().qo_leg_fk(P(q), int(flag), P(pos), P(J))
    else:
        lib().qo_leg_fk_g(P(np.ascontiguousarray(body_p, np.float64)),
                          P(np.ascontiguousarray(body_r, np.float64)), P(q), int(flag), P(pos), P(J))
    return pos, J


def leg_ik(pos_des, q_ini, flag, body_p=None, body_r=None):
    """Inverse_kinematics(_g) restatement: (q[3], pos[3], J[9], newton updates)."""
    q = np.zeros(3)
    pos = np.zeros(3)
    J = np.zeros(9)
    bp = None if body_p is None else P(np.ascontiguousarray(body_p, np.float64))
    br = None if body_r is None else P(np.ascontiguousarray(body_r, np.float64))
    n = lib().qo_leg_ik(bp, br, P(np.ascontiguousarray(pos_des, np.float64)),
                        P(np.ascontiguousarray(q_ini, np.float64)), int(flag), P(q), P(pos), P(J))
    return q, pos, J, n


def support_phase(ts, tx, t_int, t_end):
    """oracle/support_phase.c over numpy arrays -> (bjxx, bjx1, right_support)"""
    ts = np.ascontiguousarray(ts, np.float64)
    tx = np.ascontiguousarray(tx, np.float64)
    t_int = np.ascontiguousarray(t_int, np.int32)
    t_end = np.ascontiguousarray(t_end, np.int32)
    n = t_int.shape[0]
    out = np.zeros((3, n), np.int32)
    lib().qo_support_phase(n, ts.ctypes.data, tx.ctypes.data, t_int.ctypes.data,
                           t_end.ctypes.data, out[0].ctypes.data, out[1].ctypes.data,
                           out[2].ctypes.data)
    return out[0], out[1], out[2]


# ---- A1 single-step QP (oracle/a1_qp.c)
def a1_params():
    p = A1Params()
    lib().qo_a1_params_default(C.byref(p))
    return p


def a1_build(state, contacts, params=None):
    """(root_acc, H, g, A, l, u) of the A1 QP branch, column-major A (20x12)."""
    p = params or a1_params()
    s = np.ascontiguousarray(state, np.float64)
    c = np.ascontiguousarray(contacts, np.uint8)
    acc, H, g = np.zeros(6), np.zeros(144), np.zeros(12)
    A, l, u = np.zeros(240), np.zeros(20), np.zeros(20)
    lib().qo_a1_qp_build(C.byref(p), P(s), P(c, C.c_uint8), P(acc), P(H), P(g), P(A), P(l), P(u))
    return acc, H.reshape(12, 12).T.copy(), g, A.reshape(12, 20).T.copy(), l, u


def a1_compute_grf(state, contacts, params=None, **admm):
    """qo_a1_compute_grf: (forces_body (12,), x (12,), AdmmInfo)."""
    p = params or a1_params()
    st = admm_settings(**admm)
    s = np.ascontiguousarray(state, np.float64)
    c = np.ascontiguousarray(contacts, np.uint8)
    f, x, info = np.zeros(12), np.zeros(12), AdmmInfo()
    lib().qo_a1_compute_grf(C.byref(p), C.byref(st), P(s), P(c, C.c_uint8), P(f), P(x),
                            C.byref(info))
    return f, x, info


# ---- persistent SRBD solver (oracle/persist.c)
def persist_len(N):
    return 100 * N + 4


class PersistentMpc:
    """The reference's member OSQP solver, one record per controller: on the
    literal 12N-variable QP (literal=True: every call after the first is
    OSQP's update path) or on the stance-only reduction (literal=False:
    re-initialised when the stance set changes)."""

    def __init__(self, N, literal=False, **admm):
        self.N = N
        self.literal = int(bool(literal))
        self.sp = srbd_spec(N=N)
        self.st = admm_settings(**admm)
        self.rec = np.zeros(persist_len(N))

    def step(self, x0, xr, ft, ct):
        u = np.zeros(12 * self.N)
        info = AdmmInfo()
        x0 = np.ascontiguousarray(x0, np.float32)
        xr = np.ascontiguousarray(xr, np.float32)
        ft = np.ascontiguousarray(ft, np.float32)
        ct = np.ascontiguousarray(ct, np.uint8)
        fps = int(ft.size == 12 * self.N and self.N > 1)
        cps = int(ct.size == 4 * self.N and self.N > 1)
        lib().qo_srbd_persist_step_ex(P(self.rec), C.byref(self.sp), C.byref(self.st),
                                      P(x0, C.c_float), P(xr, C.c_float), P(ft, C.c_float), fps,
                                      P(ct, C.c_uint8), cps, self.literal, P(u), C.byref(info))
        return u, info
