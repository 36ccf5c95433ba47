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


def force_params(**kw):
    p = ForceParams()
    lib().qloco_force_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class ForceQP:
    """Batched Dynamiccclass (force distribution QP) with device-resident state."""

    def __init__(self, batch, device="cuda:0", **params):
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

    def step(self, com_des, leg_des, F_force_des, rfoot_des, lfoot_des, base_p, feet_p,
             FT_total_des, mode, right_support, y_coef):
        """servo.cpp:1224-1228: force_distribution(...) then force_opt(...)."""
        check(lib().qloco_force_qp_solve(
            C.byref(self.params), self.batch, ptr(com_des), ptr(leg_des), ptr(F_force_des),
            ptr(rfoot_des), ptr(lfoot_des), ptr(base_p), ptr(feet_p), ptr(FT_total_des),
            ptr(mode), ptr(right_support), ptr(y_coef), ptr(self.F_leg_ref), ptr(self.grf_opt),
            ptr(self.F_leg_guess), ptr(self.qp_solution), ptr(self.status), ptr(self.iters),
            _stream(com_des)), "qloco_force_qp_solve")
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
