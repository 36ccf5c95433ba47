"""Batched small-QP paths of the reference, on gfx950.

* `eiquadprog_solve`  -- QPsolver_EiQuadProg::solve / Eigen::QP::solve_quadprog
  (rt_mpc_qp/src/QP/QPBaseClass.cpp:36-58, utils/EiQuadProg/EiQuadProg.cpp),
  batched, quirk-compatible, fp64.
* `ForceQP`           -- Dynamiccclass::force_distribution + force_opt
  (go1_rt_control/src/whole_body_dynamics/dynmics_compute.cpp:141-445), with
  the per-instance member state (F_leg_ref, grf_opt) kept on the device.
* `BodyMPC`           -- PRMPCClass::body_theta_mpc
  (rt_mpc_qp/src/FastMPC/PRMPCClass.cpp:379-714) with its member state.
* `indexfind`         -- PRMPCClass::Indexfind (:716-738).

All tensors are device tensors (torch is the allocator); the compute is in
libqloco.so and there is no host fallback.
"""
import ctypes as C

from ._lib import ForceParams, check, lib, ptr

STATE_LEN = 32  # QLOCO_BODY_STATE_LEN


def _stream(t):
    import torch
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def eiquadprog_solve(G, g0, CE, ce0, CI, ci0, n, p, m):
    """Batched solve of min 0.5x'Gx + g0'x s.t. CE'x + ce0 = 0, CI'x + ci0 >= 0.

    Each argument is (B, k) float64 with column-major matrices flattened per
    instance (Eigen storage), or a 1-D tensor shared by all instances.
    Returns dict(x, f, status, iters)."""
    import torch
    B = G.shape[0]
    dev = G.device
    out = {"x": torch.empty((B, n), dtype=torch.float64, device=dev),
           "f": torch.empty(B, dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev),
           "iters": torch.empty(B, dtype=torch.int32, device=dev)}

    def sd(t, k):
        if t is None:
            return None, 0
        t = t.contiguous()
        if t.dtype != torch.float64:
            raise ValueError("float64 expected")
        return t, (0 if t.dim() == 1 else k)

    Gt, sG = sd(G, n * n)
    gt, sg = sd(g0, n)
    CEt, sCE = sd(CE if p else None, n * p)
    ce0t, sce0 = sd(ce0 if p else None, p)
    CIt, sCI = sd(CI if m else None, n * m)
    ci0t, sci0 = sd(ci0 if m else None, m)
    check(lib().qloco_eiquadprog_solve(n, p, m, B, ptr(Gt), sG, ptr(gt), sg, ptr(CEt), sCE,
                                       ptr(ce0t), sce0, ptr(CIt), sCI, ptr(ci0t), sci0,
                                       ptr(out["x"]), ptr(out["f"]), ptr(out["status"]),
                                       ptr(out["iters"]), _stream(G)), "qloco_eiquadprog_solve")
    return out


def force_params(hw=False, **kw):
    """Dynamiccclass constants: the sim copy (go1_rt_control
    dynmics_compute.cpp:29-100, mass 12, mu 0.25) or, hw=True, the hardware
    copy the torque-mode loop uses (unitree_legged_real: mass = gait::mass
    = 14, mu = 0.5; qloco_force_params_hw)."""
    p = ForceParams()
    (lib().qloco_force_params_hw if hw else lib().qloco_force_params_default)(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def hw_torque_ff(Jaco, grf_opt, grf_base, dynamic_count, stream=None):
    """The hardware loop's joint feed-forward after force_opt
    (unitree_legged_real torque_mode.cpp:1370-1384): stand-up ramp
    rate = min((dynamic_count / 500)^2, 1), F = rate (grf_opt - grf_base) +
    grf_base per leg, tau = -J^T F (no gravity compensation).  Jaco (B, 4, 9)
    col-major per leg, grf_opt / grf_base (B, 12) float64, dynamic_count (B,)
    int32; legs FR, FL, RR, RL.  Returns tau (B, 12) float64."""
    import torch
    B = grf_opt.shape[0]
    for name, t, dt, n in (("Jaco", Jaco, torch.float64, 36), ("grf_opt", grf_opt, torch.float64, 12),
                           ("grf_base", grf_base, torch.float64, 12),
                           ("dynamic_count", dynamic_count, torch.int32, 1)):
        if t.dtype != dt or not t.is_contiguous() or not t.is_cuda or t.numel() != B * n:
            raise ValueError("%s: need a contiguous %s device tensor with %d entries per instance"
                             % (name, dt, n))
    tau = torch.empty((B, 12), dtype=torch.float64, device=grf_opt.device)
    check(lib().qloco_hw_torque_ff(B, ptr(Jaco), ptr(grf_opt), ptr(grf_base), ptr(dynamic_count),
                                   ptr(tau), C.c_void_p(stream) if stream is not None else _stream(grf_opt)),
          "qloco_hw_torque_ff")
    return tau


class ForceQP:
    """Batched Dynamiccclass (force distribution QP) with device-resident state."""

    def __init__(self, batch, device="cuda:0", grouped=True, **params):
        import torch
        self.batch = batch
        self.params = force_params(**params)
        z = lambda *s: torch.zeros(s, dtype=torch.float64, device=device)
        self.F_leg_ref = z(batch, 12)  # member F_leg_ref (3x4 col-major), :43
        self.grf_opt = z(batch, 12)    # member grf_opt, F_prev of q_goal, :53
        self.F_leg_guess = z(batch, 12)
        self.qp_solution = torch.ones(batch, dtype=torch.int32, device=device)
        self.status = torch.zeros(batch, dtype=torch.int32, device=device)
        self.iters = torch.zeros(batch, dtype=torch.int32, device=device)
        # grouping workspace (qloco_force_qp_solve_ordered): zero-filled once,
        # carried between calls like the member state; None = ungrouped launch
        self.order_ws = (torch.zeros(int(lib().qloco_force_order_ws_len(batch)), dtype=torch.int32,
                                     device=device) if grouped else None)

    def step(self, com_des, leg_des, F_force_des, rfoot_des, lfoot_des, base_p, feet_p,
             FT_total_des, mode, right_support, y_coef):
        """servo.cpp:1224-1228: force_distribution(...) then force_opt(...)."""
        check(lib().qloco_force_qp_solve_ordered(
            C.byref(self.params), self.batch, ptr(com_des), ptr(leg_des), ptr(F_force_des),
            ptr(rfoot_des), ptr(lfoot_des), ptr(base_p), ptr(feet_p), ptr(FT_total_des),
            ptr(mode), ptr(right_support), ptr(y_coef), ptr(self.F_leg_ref), ptr(self.grf_opt),
            ptr(self.F_leg_guess), ptr(self.qp_solution), ptr(self.status), ptr(self.iters),
            ptr(self.order_ws), _stream(com_des)), "qloco_force_qp_solve_ordered")
        return {"grf_opt": self.grf_opt, "F_leg_guess": self.F_leg_guess,
                "F_leg_ref": self.F_leg_ref, "qp_solution": self.qp_solution,
                "status": self.status, "iters": self.iters}

    def joint_torques(self, Jaco, swing, p_des, p_est, pv_des, pv_est):
        """compute_joint_torques for all four legs (dynmics_compute.cpp:109-138)."""
        import torch
        tau = torch.empty((self.batch, 12), dtype=torch.float64, device=Jaco.device)
        check(lib().qloco_joint_torques(self.batch, ptr(Jaco), ptr(swing), ptr(p_des), ptr(p_est),
                                        ptr(pv_des), ptr(pv_est), ptr(self.F_leg_ref), ptr(tau),
                                        _stream(Jaco)), "qloco_joint_torques")
        return tau


class BodyMPC:
    """Batched PRMPCClass body-inclination MPC with device-resident state."""

    def __init__(self, batch, device="cuda:0"):
        import numpy as np
        import torch
        self.batch = batch
        st = np.zeros((batch, STATE_LEN), np.float64)
        check(lib().qloco_body_state_init_host(batch, ptr(st)), "qloco_body_state_init_host")
        self.state = torch.from_numpy(st).to(device)
        self.com_traj = torch.zeros((batch, 14), dtype=torch.float64, device=device)
        self.status = torch.zeros(batch, dtype=torch.int32, device=device)

    def step(self, i, bodyangle_state, zmp_ref, angle_ref, rfoot_ref, lfoot_ref, comacc_ref):
        """gait_fast.cpp:620 body_theta_mpc(i, ...) for every instance."""
        check(lib().qloco_body_mpc_step(self.batch, ptr(i), ptr(bodyangle_state), ptr(zmp_ref),
                                        ptr(angle_ref), ptr(rfoot_ref), ptr(lfoot_ref),
                                        ptr(comacc_ref), ptr(self.state), ptr(self.com_traj),
                                        ptr(self.status), _stream(i)), "qloco_body_mpc_step")
        return {"com_traj": self.com_traj, "status": self.status}


def indexfind(t):
    """PRMPCClass::Indexfind on a float64 device tensor of times -> int32."""
    import torch
    j = torch.empty(t.shape[0], dtype=torch.int32, device=t.device)
    check(lib().qloco_body_indexfind(t.shape[0], ptr(t.contiguous()), ptr(j), _stream(t)),
          "qloco_body_indexfind")
    return j


class ServoForceBlock:
    """The go1 servo loop's force block (servo.cpp:1052-1243, :1318) for B
    robots: F_sum, rleg_com / F_lr_predict and the swing flags from the
    desired motion, then force_distribution + force_opt and the four legs'
    compute_joint_torques.  Member / loop state stays on the device."""

    IN_F64 = ("coma_des", "com_des", "rfoot_des", "lfoot_des", "body_p_des", "foot_des")

    def __init__(self, batch, device="cuda:0", **params):
        import torch
        self.batch = int(batch)
        self.params = force_params(**params)
        n = int(lib().qloco_servo_workspace_bytes(self.batch))
        self.ws = torch.empty(max(n, 1), dtype=torch.uint8, device=device)
        f64 = dict(dtype=torch.float64, device=device)
        i32 = dict(dtype=torch.int32, device=device)
        self.out = {"F_sum": torch.zeros((batch, 6), **f64),
                    "Force_L_R": torch.zeros((batch, 6), **f64),
                    "grf_opt": torch.zeros((batch, 12), **f64),
                    "tau": torch.zeros((batch, 12), **f64),
                    "swing": torch.zeros((batch, 4), **i32),
                    "qp_solution": torch.zeros(batch, **i32),
                    "status": torch.zeros(batch, **i32)}
        check(lib().qloco_servo_init(self.batch, ptr(self.ws), _stream(self.ws)), "qloco_servo_init")

    def step(self, coma_des, com_des, rfoot_des, lfoot_des, body_p_des, foot_des, right_support,
             gait_mode, y_offset, loop_count, Jaco, foot_rel_mea, v_est_rel):
        o = self.out
        check(lib().qloco_servo_force_block(
            C.byref(self.params), self.batch, ptr(self.ws), ptr(coma_des), ptr(com_des),
            ptr(rfoot_des), ptr(lfoot_des), ptr(body_p_des), ptr(foot_des), ptr(right_support),
            ptr(gait_mode), ptr(y_offset), ptr(loop_count), ptr(Jaco), ptr(foot_rel_mea),
            ptr(v_est_rel), ptr(o["F_sum"]), ptr(o["Force_L_R"]), ptr(o["grf_opt"]), ptr(o["tau"]),
            ptr(o["swing"]), ptr(o["qp_solution"]), ptr(o["status"]), _stream(self.ws)),
            "qloco_servo_force_block")
        return o


def synth_servo_inputs(seed, batch, tick):
    """Deterministic servo-loop inputs for tick `tick` (numpy, legs FR, FL,
    RR, RL): Go1 homing feet (servo.cpp:799-802) stepping with the body,
    small desired COM accelerations, gait modes 101/102/103 and one outside
    them (104, which keeps the swing flags), right_support cycling 0/1/2 on a
    per-robot phase, FK-like Jacobians and measured feet near the desired."""
    import numpy as np
    rng = np.random.default_rng([seed, batch])
    ph = rng.uniform(0, 2 * np.pi, batch)
    mode = rng.choice([101, 102, 103, 104], batch, p=[0.3, 0.4, 0.2, 0.1]).astype(np.int32)
    J0 = rng.normal(0, 0.15, (batch, 4, 3, 3)) + 0.3 * np.eye(3)
    trng = np.random.default_rng([seed, batch, tick])
    t = tick * 0.005
    body = np.stack([0.05 * t + 0.01 * np.sin(ph), 0.02 * np.sin(3 * t + ph),
                     0.30 + 0.005 * np.cos(5 * t + ph)], 1)
    homing = np.array([[0.150786, -0.12675, 0.0], [0.150786, 0.12675, 0.0],
                       [-0.225414, -0.12675, 0.0], [-0.225414, 0.12675, 0.0]])
    feet = homing[None] + body[:, None, :] * np.array([1.0, 1.0, 0.0])
    feet[:, :, 2] += 0.02 * np.maximum(np.sin(8 * t + ph[:, None] + np.arange(4)[None] * np.pi / 2), 0)
    rs = ((np.floor(t / 0.35 + ph) % 3)).astype(np.int32)
    rfoot = (feet[:, 0] + feet[:, 3]) / 2
    lfoot = (feet[:, 1] + feet[:, 2]) / 2
    com = body + trng.normal(0, 0.003, (batch, 3))
    coma = trng.normal(0, 0.4, (batch, 3))
    y = np.where(mode == 101, 0.75, np.where(mode == 102, 0.0, 0.11))
    Jaco = J0 + 0.02 * np.sin(t + ph)[:, None, None, None]
    rel_mea = (feet - body[:, None, :]) + trng.normal(0, 0.002, (batch, 4, 3))
    v_est = trng.normal(0, 0.05, (batch, 4, 3))
    return dict(coma_des=coma, com_des=com, rfoot_des=rfoot, lfoot_des=lfoot, body_p_des=body,
                foot_des=feet.reshape(batch, 12), right_support=rs, gait_mode=mode, y_offset=y,
                loop_count=np.full(batch, tick, np.int32),
                Jaco=np.ascontiguousarray(np.transpose(Jaco, (0, 1, 3, 2))).reshape(batch, 36),
                foot_rel_mea=rel_mea.reshape(batch, 12), v_est_rel=v_est.reshape(batch, 12))
