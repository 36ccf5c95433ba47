"""Reference computations for the SRBD parity tests (test infrastructure).

Builds each instance's literal QP with the oracle (oracle/srbd.c), solves it
exactly (EiQuadProg restatement) and with the OSQP-algorithm ADMM
restatement, on the full 12N-variable problem and on the stance-only
reduction that the GPU kernel solves.
"""
import numpy as np

import oracle_lib as O


def stance_index(contacts, N):
    """Variable / row indices of stance (step, leg) pairs, ConvexMpc order."""
    idx, rows = [], []
    for k in range(N):
        for i in range(4):
            if contacts[4 * k + i]:
                idx += [12 * k + 3 * i + j for j in range(3)]
                rows += [20 * k + 5 * i + j for j in range(5)]
    return np.array(idx, dtype=np.int64), np.array(rows, dtype=np.int64)


class Instance:
    def __init__(self, spec, x0, xr, ft, ct, feet_per_step=0):
        self.N = N = spec.N
        self.ct = np.asarray(ct, np.uint8)
        self.H, self.g, self.lb, self.ub = O.build_instance(spec, x0, xr, ft, ct,
                                                            contacts_per_step=1,
                                                            feet_per_step=feet_per_step)
        self.A = O.constraints(spec)
        self.idx, self.rows = stance_index(self.ct, N)

    def obj(self, u):
        u = np.asarray(u, np.float64)
        return 0.5 * u @ self.H @ u + self.g @ u

    def exact(self):
        x, st, it = O.exact_solve(self.H, self.g, self.A, self.lb, self.ub)
        return x, st, it

    def exact_obj(self):
        x, st, _ = self.exact()
        assert st == 0, st
        return self.obj(x)

    def admm_full(self, **kw):
        x, y, info = O.admm_solve(self.H, self.g, self.A, self.lb, self.ub,
                                  O.admm_settings(**kw))
        return x, info

    def admm_reduced(self, **kw):
        i, r = self.idx, self.rows
        H = self.H[np.ix_(i, i)]
        A = self.A[np.ix_(r, i)]
        xr, y, info = O.admm_solve(H, self.g[i], A, self.lb[r], self.ub[r], O.admm_settings(**kw))
        x = np.zeros(12 * self.N)
        x[i] = xr
        return x, info

    def violation(self, u):
        Au = self.A @ np.asarray(u, np.float64)
        return max(0.0, float(np.max(self.lb - Au)), float(np.max(Au - self.ub)))


# ---- independent numpy restatement of the reference build (test_oracle.py checks it
#      against the C oracle; test_srbd_gpu.py checks qloco_srbd_build against it)
def np_A_c(yaw):
    """ConvexMpc::calculate_A_mat_c (ConvexMpc.cpp:111-133)."""
    A = np.zeros((13, 13))
    c, s = np.cos(yaw), np.sin(yaw)
    A[0:3, 6:9] = [[c, s, 0], [-s, c, 0], [0, 0, 1]]
    A[3:6, 9:12] = np.eye(3)
    A[11, 12] = 1.0
    return A


def np_skew(v):
    """Utils::skew (utils/Utils.cpp:35-41)."""
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def np_B_c(mass, I, R, feet):
    """ConvexMpc::calculate_B_mat_c (ConvexMpc.cpp:135-147)."""
    Iw_inv = np.linalg.inv(R @ I @ R.T)
    B = np.zeros((13, 12))
    for i in range(4):
        B[6:9, 3 * i:3 * i + 3] = Iw_inv @ np_skew(feet[3 * i:3 * i + 3])
        B[9:12, 3 * i:3 * i + 3] = np.eye(3) / mass
    return B


def np_build(x0, xr, feet, ct, N, dt=0.0025, mass=12.0, I=O.GO1_INERTIA, q_w=O.Q_W, r_w=O.R_W,
             mu=0.3, fz_max=180.0, feet_per_step=False):
    """compute_grf MPC branch + ConvexMpc::calculate_qp_mats (:162-264)."""
    x0 = np.asarray(x0, np.float64)
    yaw = x0[2]
    c, s = np.cos(yaw), np.sin(yaw)
    R = np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]])  # A1RobotControl.cpp:506-508
    A_d = np.eye(13) + np_A_c(yaw) * dt                # state_space_discretization :149-160
    Bd = [np_B_c(mass, I, R, feet[12 * k:12 * k + 12] if feet_per_step else feet) * dt
          for k in range(N)]
    Aqp = np.vstack([np.linalg.matrix_power(A_d, i + 1) for i in range(N)])
    Bqp = np.zeros((13 * N, 12 * N))
    for i in range(N):
        for j in range(i + 1):
            Bqp[13 * i:13 * i + 13, 12 * j:12 * j + 12] = np.linalg.matrix_power(A_d, i - j) @ Bd[j]
    Q = np.diag(np.tile(2.0 * np.asarray(q_w), N))
    Rm = np.diag(np.tile(2.0 * np.asarray(r_w), N))
    H = Bqp.T @ Q @ Bqp + Rm
    g = Bqp.T @ Q @ (Aqp @ x0 - np.asarray(xr, np.float64))
    lb, ub = np.zeros(20 * N), np.zeros(20 * N)
    for k in range(N):
        for i in range(4):
            cc = float(ct[4 * k + i])
            lb[20 * k + 5 * i:20 * k + 5 * i + 5] = [0, -1e30, 0, -1e30, 0]
            ub[20 * k + 5 * i:20 * k + 5 * i + 5] = [1e30, 0, 1e30, 0, fz_max * cc]
    Cm = np.zeros((20 * N, 12 * N))
    for i in range(4 * N):
        Cm[5 * i:5 * i + 5, 3 * i:3 * i + 3] = [[1, 0, mu], [1, 0, -mu], [0, 1, mu], [0, 1, -mu],
                                                [0, 0, 1]]
    return H, g, lb, ub, Cm, Aqp, Bqp
