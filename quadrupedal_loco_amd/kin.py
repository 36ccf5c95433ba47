"""Batched Go1 leg kinematics on gfx950.

* `leg_fk` -- Kinematicclass::Forward_kinematics / Forward_kinematics_g
  (go1_rt_control/src/kinematics/Kinematics.cpp:63-229): foot position and
  Jacobian_kin for every leg row.
* `leg_ik` -- Kinematicclass::Inverse_kinematics / Inverse_kinematics_g
  (:233-304): the reference's damped Newton loop (lamda 0.5, 10 / 15 steps,
  its stop tests as written).

Rows are legs: q / pos (n, 3) float64, leg (n,) int32 with 0 FR, 1 FL, 2 RR,
3 RL (the servo's order), body_p / body_r (n, 3) for the world-frame forms
(body_r = roll, pitch, yaw) or None for the hip frame.  Jacobians are (n, 9)
column-major 3x3 (Eigen storage).  Device tensors only; the compute is in
libqloco.so (qloco_leg_fk / qloco_leg_ik) and there is no host fallback.
"""
from ._lib import check, lib, ptr
from .qp import _stream

LEGS = {"FR": 0, "FL": 1, "RR": 2, "RL": 3}


def _rows(t, name, cols, dtype):
    import torch
    if t.dtype != dtype or not t.is_cuda:
        raise ValueError("%s: need a %s device tensor" % (name, dtype))
    t = t.contiguous()
    if cols and (t.dim() != 2 or t.shape[1] != cols):
        raise ValueError("%s: need shape (n, %d)" % (name, cols))
    return t


def _body(body_p, body_r, n):
    import torch
    if (body_p is None) != (body_r is None):
        raise ValueError("body_p and body_r go together (world frame) or are both None")
    if body_p is None:
        return None, None
    bp = _rows(body_p, "body_p", 3, torch.float64)
    br = _rows(body_r, "body_r", 3, torch.float64)
    if bp.shape[0] != n or br.shape[0] != n:
        raise ValueError("body_p / body_r need one row per leg")
    return bp, br


def leg_fk(q, leg, body_p=None, body_r=None, jacobian=True):
    """Foot positions (n, 3) and, if requested, Jacobians (n, 9)."""
    import torch
    q = _rows(q, "q", 3, torch.float64)
    n = q.shape[0]
    leg = _rows(leg, "leg", 0, torch.int32)
    if leg.numel() != n:
        raise ValueError("leg: one flag per row")
    bp, br = _body(body_p, body_r, n)
    pos = torch.empty((n, 3), dtype=torch.float64, device=q.device)
    jac = torch.empty((n, 9), dtype=torch.float64, device=q.device) if jacobian else None
    check(lib().qloco_leg_fk(n, ptr(q), ptr(leg), ptr(bp), ptr(br), ptr(pos), ptr(jac), _stream(q)),
          "qloco_leg_fk")
    return pos, jac


def leg_ik(pos_des, q_ini, leg, body_p=None, body_r=None):
    """Joint angles (n, 3) reaching pos_des from q_ini; also returns the FK
    position and Jacobian at the result and the Newton steps applied."""
    import torch
    pos_des = _rows(pos_des, "pos_des", 3, torch.float64)
    n = pos_des.shape[0]
    q_ini = _rows(q_ini, "q_ini", 3, torch.float64)
    leg = _rows(leg, "leg", 0, torch.int32)
    if q_ini.shape[0] != n or leg.numel() != n:
        raise ValueError("pos_des, q_ini and leg need the same number of rows")
    bp, br = _body(body_p, body_r, n)
    dev = pos_des.device
    q = torch.empty((n, 3), dtype=torch.float64, device=dev)
    pos = torch.empty((n, 3), dtype=torch.float64, device=dev)
    jac = torch.empty((n, 9), dtype=torch.float64, device=dev)
    upd = torch.empty(n, dtype=torch.int32, device=dev)
    check(lib().qloco_leg_ik(n, ptr(pos_des), ptr(q_ini), ptr(leg), ptr(bp), ptr(br), ptr(q),
                             ptr(pos), ptr(jac), ptr(upd), _stream(pos_des)), "qloco_leg_ik")
    return q, pos, jac, upd
