"""Second, independent transcription of the rt_mpc_qp node tick (pure Python).

TEST INFRASTRUCTURE ONLY.  Written straight from the reference text, keeping
its structure (both support sides spelled out, Eigen members as numpy
arrays), to hold the C oracle (oracle/rt_tick.c) to the reference: the two
transcriptions must agree bit-for-bit on every schedule integer and to
rounding on every double -- bit-for-bit in practice: the numeric primitives
that the reference leaves to Eigen / libm are shared definitions (the 4x4
Gauss-Jordan inverse `inv4`, the compensated cube `cube`, dot products summed
in index order), because the cubic swing fits of solve_AAA_inv2 become
ill-conditioned where the swing time crosses its knots and amplify any
rounding difference.  The body-inclination QP (body_theta_mpc) is taken
from the C oracle through `body_step` -- it is pinned separately
(tests/test_oracle.py).  Small cases only (a few robots, a few thousand ticks).

Reference: unitree_ros/rt_mpc_qp/src/gait_fast.cpp:79-735 and
unitree_ros/rt_mpc_qp/src/FastMPC/PRMPCClass.cpp (line numbers per method).
"""
import math
from fractions import Fraction

import numpy as np

NSTEPS = 27          # _footstepsnumber, PRMPCClass.h:30
DT = 0.025           # _dt = gait::dt_mpc_slow
DT_MPC = 0.01        # _dt_mpc = gait::dt_mpc_fast
NH = 4               # _nh
TSTEP = 0.7          # gait::t_period
HALF_HIP = 0.12675


def cround(x):
    """C/C++ round(): half away from zero."""
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def fma(a, b, c):
    """exactly rounded a*b + c (Python 3.10 has no math.fma)"""
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def cube(x):
    """pow(x, 3) as the compensated cube of oracle/rt_tick.c"""
    p = x * x
    e = fma(x, x, -p)
    hi = p * x
    lo = fma(p, x, -hi)
    return hi + (lo + e * x)


def inv4(A):
    """Gauss-Jordan with partial pivoting, row-major 4x4 (oracle/rt_tick.c:qo_inv4)"""
    M = [[float(A[r][c]) for c in range(4)] + [1.0 if r == c else 0.0 for c in range(4)]
         for r in range(4)]
    for k in range(4):
        p = k
        for r in range(k + 1, 4):
            if abs(M[r][k]) > abs(M[p][k]):
                p = r
        if p != k:
            M[k], M[p] = M[p], M[k]
        piv = M[k][k]
        M[k] = [v / piv for v in M[k]]
        for r in range(4):
            if r != k:
                f = M[r][k]
                M[r] = [M[r][c] - f * M[k][c] for c in range(8)]
    return [[M[r][4 + c] for c in range(4)] for r in range(4)]


def dot(a, b):
    s = 0.0
    for x, y in zip(a, b):
        s += x * y
    return s


class PRMPCGen:
    """PRMPCClass members used by the reference generators."""

    def __init__(self):
        # Initialize(): FootStepInputs(2*half_hip, 0, 0, 0.015) (:48-53, :2198-2222)
        stepwidth, steplengthx, stepheight, lift = 2 * HALF_HIP, 0.0, 0.0, 0.015
        self.steplength = np.full(NSTEPS, steplengthx)
        self.steplength[[-1, -2, -3, -4, -5, 0, 1, 2]] = 0
        self.steplength[3] = steplengthx / 2
        self.stepwidth = np.full(NSTEPS, stepwidth)
        self.stepwidth[0] = self.stepwidth[0] / 2
        self.stepheight = np.full(NSTEPS, stepheight)
        self.lift_height_ref = np.full(NSTEPS, lift)
        self.lift_height_ref[-1] = 0
        self.lift_height_ref[-2] = 0
        self.lift_height_ref[-3] = lift / 2
        self.lift_height_ref[-4] = lift
        fx, fy, fz = np.zeros(NSTEPS), np.zeros(NSTEPS), np.zeros(NSTEPS)
        for i in range(1, NSTEPS):  # :111-116
            fx[i] = fx[i - 1] + self.steplength[i - 1]
            fy[i] = fy[i - 1] + int(math.pow(-1, i - 1)) * self.stepwidth[i - 1]
            fz[i] = fz[i - 1] + self.stepheight[i - 1]
        self.footxyz_real = np.vstack([fx, fy, fz])
        self.bjxx = 0
        self.Lfoot = {k: np.zeros(10) for k in ("x", "y", "z", "vx", "vy", "vz", "ax", "ay", "az")}
        self.Rfoot = {k: np.zeros(10) for k in ("x", "y", "z", "vx", "vy", "vz", "ax", "ay", "az")}
        self.Lfoot["y"][:] = self.stepwidth[0]
        self.Rfoot["y"][:] = -self.stepwidth[0]
        self.ry_left_right = 0.0
        self.Lfoot_r = np.zeros((3, 5))
        self.Rfoot_r = np.zeros((3, 5))
        self.footx_max = 0.15
        self.tdsp_ratio = 0.1
        self.ts = np.full(NSTEPS, TSTEP)
        self.td = self.tdsp_ratio * self.ts
        self.tx = np.zeros(NSTEPS)
        for i in range(1, NSTEPS):  # :174-178
            self.tx[i] = self.tx[i - 1] + self.ts[i - 1]
            self.tx[i] = cround(self.tx[i] / DT) * DT - 0.00001
        self.t_end_footstep = int(cround((self.tx[NSTEPS - 1] - 3 * TSTEP) / DT_MPC))
        self.tx_total = self.tx[NSTEPS - 1]
        self.bjx1 = 0
        self.j_period = 0
        # solve_AAA_inv_mod1 (:1344-1362)
        t = [-DT, 0, DT, 2 * DT]
        self.AAA_inv_mod = inv4([[cube(t[r]), t[r] * t[r], t[r], 1.0] for r in range(4)])

    def indexfind(self, goal):  # :716-738, xyz = 0
        self.j_period = 0
        while self.j_period < NSTEPS and goal >= self.tx[self.j_period]:
            self.j_period += 1
        self.j_period -= 1

    def position_mod3(self, walktime, dt_sample, in1, in2, ref, ref2):  # :1170-1261
        out = np.zeros(21)
        if walktime <= self.t_end_footstep:
            for jx in range(NH):
                t = walktime * dt_sample + jx * dt_sample
                tp = [cube(t), t * t, t, 1.0]
                tv = [3 * (t * t), 2 * t, 1.0, 0.0]
                ta = [6 * t, 2.0, 0.0, 0.0]
                Ai = self.AAA_inv_mod
                col = lambda c: [Ai[k][c] for k in range(4)]
                rp = [dot(tp, col(c)) for c in range(4)]   # (t_a_plan * _AAA_inv_mod)
                rv = [dot(tv, col(c)) for c in range(4)]
                ra = [dot(ta, col(c)) for c in range(4)]
                for ax in range(3):
                    temp = [in1[ax], in2[ax], ref[ax], ref2[ax]]
                    if jx == 0:
                        out[ax] = dot(rp, temp)
                        out[3 + ax] = dot(rv, temp)
                        out[6 + ax] = dot(ra, temp)
                    else:
                        out[8 + 3 * jx - 2 + ax] = dot(rp, temp)
        return out

    @staticmethod
    def aaa_inv2(tp):  # :2225-2237
        return inv4([[cube(tp[0]), tp[0] * tp[0], tp[0], 1.0],
                     [cube(tp[1]), tp[1] * tp[1], tp[1], 1.0],
                     [cube(tp[2]), tp[2] * tp[2], tp[2], 1.0],
                     [3 * (tp[2] * tp[2]), 2 * tp[2], 1.0, 0.0]])

    def _swing(self, F, k, j_index, bjxx, bjx1):
        """the swing-leg block of :1878-1951 (right) / :2044-2118 (left)"""
        fr = self.footxyz_real
        bm = bjxx - 2 if bjxx >= 2 else 0   # reference reads out of bounds below 0
        t_des = (j_index + 1 - cround(self.tx[bjx1 - 1] / DT_MPC) + 1) * DT_MPC
        t_plan = [t_des - DT_MPC, (self.td[bjx1 - 1] + self.ts[bjx1 - 1]) / 2 + 0.0001,
                  self.ts[bjx1 - 1] - (2 * DT_MPC + 0.001)]
        if abs(t_des - self.ts[bjx1 - 1]) <= DT_MPC:
            for ax in "xyz":
                i = "xyz".index(ax)
                F[ax][k] = fr[i, bjxx]
                F[ax][k + 1] = fr[i, bjxx]
            return
        AAA_inv = self.aaa_inv2(t_plan)
        tp = [cube(t_des), t_des * t_des, t_des, 1.0]
        tv = [3 * (t_des * t_des), 2 * t_des, 1.0, 0.0]
        ta = [6 * t_des, 2.0, 0.0, 0.0]
        fit = lambda plan: [dot(AAA_inv[r], plan) for r in range(4)]
        co = fit([F["x"][k - 1], (fr[0, bm] + fr[0, bjxx]) / 2, fr[0, bjxx], 0.0])
        F["x"][k], F["vx"][k], F["ax"][k] = dot(tp, co), dot(tv, co), dot(ta, co)
        if (j_index + 1 - cround(self.tx[bjx1 - 1] / DT_MPC)) * DT_MPC < self.td[bjx1 - 1] + DT_MPC:
            self.ry_left_right = (fr[1, bjxx] + fr[1, bm]) / 2
        co = fit([F["y"][k - 1], self.ry_left_right, fr[1, bjxx], 0.0])
        F["y"][k], F["vy"][k], F["ay"][k] = dot(tp, co), dot(tv, co), dot(ta, co)
        zmid = max(fr[2, bm], fr[2, bjxx]) + self.lift_height_ref[bjx1 - 1]
        co = fit([F["z"][k - 1], zmid, fr[2, bjxx], 0.0])
        F["z"][k], F["vz"][k], F["az"][k] = dot(tp, co), dot(tv, co), dot(ta, co)
        for a in "xyz":
            F[a][k + 1] = F[a][k] + DT_MPC * F["v" + a][k]

    def foot_trajectory_solve_mod2(self, j_indexx, stopwalking, nrt):  # :1756-2195
        b = int(nrt[0])
        if 0 <= b and b + 1 < NSTEPS:
            self.footxyz_real[0, b], self.footxyz_real[0, b + 1] = nrt[1], nrt[2]
            self.footxyz_real[1, b], self.footxyz_real[1, b + 1] = nrt[3], nrt[4]
            self.footxyz_real[2, b], self.footxyz_real[2, b + 1] = nrt[5], nrt[6]
        p = int(nrt[7])
        if nrt[8] > 0 and 0 <= p < NSTEPS:
            self.ts[p] = nrt[8]
        self.td = self.tdsp_ratio * self.ts
        self.tx = np.zeros(NSTEPS)
        for i in range(1, NSTEPS):
            self.tx[i] = self.tx[i - 1] + self.ts[i - 1]
            self.tx[i] = cround(self.tx[i] / DT) * DT - 0.00001
        self.t_end_footstep = int(cround((self.tx[NSTEPS - 1] - 2 * TSTEP) / DT_MPC))
        self.tx_total = self.tx[NSTEPS - 1]
        L, R = self.Lfoot, self.Rfoot
        for j_index in range(j_indexx, j_indexx + NH):
            k = j_index - j_indexx + 1
            if j_index <= self.t_end_footstep:
                self.indexfind(j_index * DT_MPC)
                self.bjxx = self.j_period + 1
                self.j_period = 0
                self.indexfind((j_index + 1) * DT_MPC)
                self.bjx1 = self.j_period + 1
                self.j_period = 0
            if stopwalking or j_index > self.t_end_footstep:
                for i_t in range(self.bjx1 + 1, NSTEPS):
                    self.lift_height_ref[i_t] = 0
            for i_t in range(24, NSTEPS):
                self.lift_height_ref[i_t] = 0
            self.footxyz_real[1, 0] = -self.stepwidth[0]
            if self.bjx1 >= 2 and j_index <= self.t_end_footstep:
                ds = (j_index + 1 - cround(self.tx[self.bjx1 - 1] / DT_MPC)) * DT_MPC < self.td[self.bjx1 - 1]
                if self.bjx1 % 2 == 0:  # left support, right swing
                    for a in "xyz":
                        L[a][k] = L[a][k - 1]
                        L[a][k + 1] = L[a][k - 1]
                    if ds:
                        for a in "xyz":
                            R[a][k] = R[a][k - 1]
                            R[a][k + 1] = R[a][k - 1]
                    else:
                        self._swing(R, k, j_index, self.bjxx, self.bjx1)
                else:  # right support, left swing
                    for a in "xyz":
                        R[a][k] = R[a][k - 1]
                        R[a][k + 1] = R[a][k - 1]
                    if ds:
                        for a in "xyz":
                            L[a][k] = L[a][k - 1]
                            L[a][k + 1] = L[a][k - 1]
                    else:
                        self._swing(L, k, j_index, self.bjxx, self.bjx1)
            else:
                if j_index > self.t_end_footstep:
                    for a in "xyz":
                        R[a][k] = R[a][k - 1]
                        L[a][k] = L[a][k - 1]
                else:
                    R["y"][k] = -self.stepwidth[0]
                    L["y"][k] = self.stepwidth[0]
        out = np.zeros(30)
        for j in range(5):
            out[6 * j:6 * j + 6] = [R["x"][j + 1], R["y"][j + 1], R["z"][j + 1],
                                    L["x"][j + 1], L["y"][j + 1], L["z"][j + 1]]
        for F in (R, L):
            for key in F:
                F[key][0] = F[key][1]
        return out

    def foot_rotation(self, walktimex, dt_sample):  # :2255-2380
        out = np.zeros(30)
        fr = self.footxyz_real
        for walktime in range(walktimex, walktimex + NH):
            c = walktime - walktimex
            if walktime <= self.t_end_footstep:
                self.indexfind(walktime * DT_MPC)
                self.bjxx = self.j_period + 1
                self.j_period = 0
                self.indexfind((walktime + 1) * DT_MPC)
                self.bjx1 = self.j_period + 1
                self.j_period = 0
            b1 = self.bjx1
            if b1 >= 2 and walktime <= self.t_end_footstep:
                t_desxx = (walktime + 1) * dt_sample - (self.tx[b1 - 1] + 2 * self.td[b1 - 1] / 4)
                ts, ph = self.ts[b1 - 1], t_desxx + 2 * self.td[b1 - 1] / 4
                if b1 % 2 == 0:
                    self.Rfoot_r[0, c] = -0.065 * (1 - math.cos(2 * math.pi / ts * ph))
                    if ph >= ts / 2:
                        if fr[0, b1] - fr[0, b1 - 1] > 0:
                            self.Rfoot_r[1, c] = 0.075 * (fr[0, b1] - fr[0, b1 - 1]) / self.footx_max * (
                                math.cos(4 * math.pi / ts * ph) - 1)
                    else:
                        self.Rfoot_r[1, c] = 0
                else:
                    self.Lfoot_r[0, c] = 0.075 * (1 - math.cos(2 * math.pi / ts * ph))
                    if ph >= ts / 2:
                        if fr[0, b1] - fr[0, b1 - 1] > 0:
                            self.Lfoot_r[1, c] = 0.075 * (fr[0, b1] - fr[0, b1 - 1]) / self.footx_max * (
                                math.cos(4 * math.pi / ts * ph) - 1)
                    else:
                        self.Lfoot_r[1, c] = 0
            out[6 * c:6 * c + 6] = [self.Rfoot_r[0, c], self.Rfoot_r[1, c], self.Rfoot_r[2, 0],
                                    self.Lfoot_r[0, c], self.Lfoot_r[1, c], self.Lfoot_r[2, 0]]
        return out


class RtNode:
    """gait_fast.cpp globals + one PRMPCClass; `tick` = one loop iteration."""

    def __init__(self, body_step):
        self.g = PRMPCGen()
        self.body_step = body_step   # (i, bodyangle_state, refs..., tx, bjx1) -> (com_traj, bjx1, bjx2, status)
        z = lambda: np.zeros(3)
        self.COM = {k: z() for k in ("in1", "in2", "ref", "v", "ref2")}
        for k in ("in1", "in2", "ref", "ref2"):
            self.COM[k][2] = 0.309458
        self.ACC = {k: z() for k in ("in1", "in2", "ref", "ref2")}
        self.ZMP = {k: z() for k in ("in1", "in2", "ref", "ref2")}
        self.DCM = {k: z() for k in ("in1", "in2", "ref", "ref2")}
        self.rpy_mpc_body = np.zeros(21)
        self.rpy_mpc_body[2] = 0.309458
        self.comacc_inter, self.zmp_inter, self.dcm_inter = np.zeros(21), np.zeros(21), np.zeros(21)
        self.foorpr_gen = np.zeros(30)
        for j in range(5):
            self.foorpr_gen[1 + 6 * j] = -HALF_HIP
            self.foorpr_gen[4 + 6 * j] = HALF_HIP
        self.foortheta_gen = np.zeros(30)
        self.body_thetax = np.zeros(3)
        self.bodyangle_mpc = np.zeros(14)
        self.state_feedback = np.zeros(25)
        self.state_to_MPC = np.zeros(25)
        self.count_in_rt_loop = self.count_in_rt_mpc = self.count_inteplotation = 0
        self.t_int = 0
        self.mpc_gait_flag_old = 0

    def _interp(self, low, flag):  # xget_position_interpolation, :113-372
        self.count_inteplotation += 1
        g = self.g
        if self.t_int > 2:
            args = (self.count_inteplotation, DT_MPC)
            self.rpy_mpc_body = g.position_mod3(*args, self.COM["in1"], self.COM["in2"], self.COM["ref"], self.COM["ref2"])
            self.comacc_inter = g.position_mod3(*args, self.ACC["in1"], self.ACC["in2"], self.ACC["ref"], self.ACC["ref2"])
            self.zmp_inter = g.position_mod3(*args, self.ZMP["in1"], self.ZMP["in2"], self.ZMP["ref"], self.ZMP["ref2"])
            self.dcm_inter = g.position_mod3(*args, self.DCM["in1"], self.DCM["in2"], self.DCM["ref"], self.DCM["ref2"])
        if self.count_inteplotation % 2 == 0:
            for V in (self.COM, self.ZMP, self.DCM, self.ACC):
                V["in1"] = V["in2"].copy()
                V["in2"] = V["ref"].copy()
            C, A, Z, D = self.COM, self.ACC, self.ZMP, self.DCM
            if flag > self.mpc_gait_flag_old:
                C["ref"] = low[0:3].copy()
                C["v"] = low[36:39].copy()
                C["ref2"] = C["ref"] + C["v"] * DT
                A["ref"] = low[39:42].copy()
                A["ref2"] = low[80:83].copy()
                Z["ref"][0:2] = low[12:14]
                Z["ref2"][0:2] = low[42:44]
                D["ref"][0:2] = low[34:36]
                D["ref2"][0:2] = low[44:46]
            else:
                C["ref"] = low[0:3].copy()
                C["v"] = low[36:39].copy()
                C["ref"] = C["ref"] + C["v"] * DT
                C["v"] = C["v"] + low[39:42] * DT
                C["ref2"] = C["ref"] + C["v"] * DT
                A["ref"] = low[80:83].copy()
                A["ref2"] = low[83:86].copy()
                Z["ref"][0:2] = low[42:44]
                Z["ref2"][0:2] = low[76:78]
                D["ref"][0:2] = low[44:46]
                D["ref2"][0:2] = low[78:80]
            self.count_inteplotation = 0
            self.mpc_gait_flag_old = flag

    def tick(self, low, ctrl):
        low = np.asarray(low, np.float64)
        flag = int(low[99])
        nrt = low[86:95]
        self.state_feedback[1:25] = ctrl[1:25]
        bodyangle_state = self.state_feedback[[10, 11, 13, 14]].copy()
        status, published = -1, 0
        if ctrl[0] > 0:
            self.count_in_rt_loop += 1
            self.t_int = int(np.int32(np.int64(self.t_int) + self.count_in_rt_loop // 2))
            self.state_feedback[0] = self.t_int
            self.state_to_MPC = self.state_feedback.copy()
            published = 1
            if flag > 0:
                self.count_in_rt_mpc += 1
                self._interp(low, flag)
                if self.count_in_rt_mpc * DT_MPC > 1.0:
                    fi = int(self.count_in_rt_mpc - 1 / DT_MPC)
                    self.foorpr_gen = self.g.foot_trajectory_solve_mod2(fi, False, nrt)
                    self.foortheta_gen = self.g.foot_rotation(fi, DT_MPC)
                self.ZMP["ref"][2] = 0.0
                zmp = np.zeros((2, 5)); rfoot = np.zeros((2, 5)); lfoot = np.zeros((2, 5))
                ang = np.zeros((2, 5)); acc = np.zeros((3, 5))
                for j in range(5):
                    if j == 0:
                        zmp[:, 0] = self.zmp_inter[0:2]
                        acc[2, 0] = self.comacc_inter[2]
                    else:
                        zmp[0, j] = self.zmp_inter[8 + 3 * j - 2]
                        zmp[1, j] = self.zmp_inter[8 + 3 * j - 1]
                        acc[2, j] = self.comacc_inter[8 + 3 * j]
                    rfoot[0, j] = self.foorpr_gen[j * 6]
                    rfoot[0, j] = self.foorpr_gen[j * 6 + 1]
                    lfoot[0, j] = self.foorpr_gen[j * 6 + 3]
                    lfoot[1, j] = self.foorpr_gen[j * 6 + 4]
                    ang[0, j] = (self.foortheta_gen[j * 6] + self.foortheta_gen[j * 6 + 3]) / 5
                    ang[1, j] = (self.foortheta_gen[j * 6 + 1] + self.foortheta_gen[j * 6 + 4]) / 5
                self.body_thetax[0:2] = ang[:, 0]
                self.bodyangle_mpc, self.g.bjx1, status = self.body_step(
                    self.count_in_rt_mpc, bodyangle_state, zmp, ang, rfoot, lfoot, acc,
                    self.g.tx.copy(), self.g.bjx1)
        inte = np.zeros(51)
        inte[0:3] = self.rpy_mpc_body[0:3]
        inte[3:6] = self.body_thetax
        inte[6:12] = [self.foorpr_gen[3], self.foorpr_gen[4], self.foorpr_gen[5],
                      self.foorpr_gen[0], self.foorpr_gen[1], self.foorpr_gen[2]]
        inte[12:14] = self.zmp_inter[0:2]
        inte[14] = self.ZMP["ref"][2]
        inte[27] = low[27]
        inte[28:34] = [self.foortheta_gen[3], self.foortheta_gen[4], self.foortheta_gen[5],
                       self.foortheta_gen[0], self.foortheta_gen[1], self.foortheta_gen[2]]
        inte[34:36] = self.dcm_inter[0:2]
        inte[36:50] = self.bodyangle_mpc
        traj = np.zeros(100)
        traj[0:36] = low[0:36]
        traj[36:87] = inte
        traj[98] = int(self.g.tx_total) / 0.001
        traj[99] = self.count_in_rt_loop
        sched = [self.g.bjx1, self.g.bjxx, self.g.t_end_footstep, self.count_in_rt_mpc,
                 self.t_int, status, published]
        gen = np.concatenate([self.foorpr_gen, self.foortheta_gen])
        return traj, self.state_to_MPC.copy(), gen, sched
