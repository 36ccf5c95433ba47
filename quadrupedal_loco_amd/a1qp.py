"""Batched A1 single-step force QP (fp64) on gfx950.

Python mirror of the `stance_leg_control_type == 0` branch of
A1RobotControl::compute_grf (unitree_ros/a1_cpp_open_source/src/
A1RobotControl.cpp:383-450; weights, friction pyramid and bounds from the
constructor :8-49): one cold OSQP solve of a 12-variable, 20-row QP per
robot, forces returned in the body frame.  The compute is the
`a1_qp_kernel` behind `qloco_a1_qp_solve` (csrc/qloco_a1qp.hip); there is no
host fallback.

Per-robot state record (STATE_LEN doubles, A1CtrlStates fields):
  [0:3] root_pos  [3:6] root_pos_d  [6:9] root_euler  [9:12] root_euler_d
  [12:15] root_lin_vel (world)  [15:18] root_lin_vel_d (body)
  [18:21] root_ang_vel (world)  [21:24] root_ang_vel_d (body)
  [24:33] root_rot_mat  [33:42] root_rot_mat_z  (3x3 column-major)
  [42:54] foot_pos_abs (3x4 column-major, legs FL, FR, RL, RR)
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import A1Params, check, lib, ptr

STATE_LEN = 54  # QLOCO_A1_STATE_LEN


def default_params(**overrides):
    """A1CtrlStates::reset() gains, the A1RobotControl ctor weights and OSQP's
    default settings; keyword overrides by field name."""
    p = A1Params()
    lib().qloco_a1_params_default(C.byref(p))
    for k, v in overrides.items():
        f = getattr(p, k)
        if hasattr(f, "__len__"):
            for i, x in enumerate(np.asarray(v, dtype=np.float64).ravel()):
                f[i] = float(x)
        else:
            setattr(p, k, v)
    return p


def _rot_zyx(roll, pitch, yaw):
    """root_rot_mat from Euler angles (Eigen AngleAxis Z * Y * X)."""
    cr, sr, cp, sp, cy, sy = (np.cos(roll), np.sin(roll), np.cos(pitch), np.sin(pitch),
                              np.cos(yaw), np.sin(yaw))
    R = np.empty(roll.shape + (3, 3))
    R[..., 0, 0] = cy * cp
    R[..., 0, 1] = cy * sp * sr - sy * cr
    R[..., 0, 2] = cy * sp * cr + sy * sr
    R[..., 1, 0] = sy * cp
    R[..., 1, 1] = sy * sp * sr + cy * cr
    R[..., 1, 2] = sy * sp * cr - cy * sr
    R[..., 2, 0] = -sp
    R[..., 2, 1] = cp * sr
    R[..., 2, 2] = cp * cr
    return R


def synth_states(seed, batch):
    """Deterministic synthetic A1 states (numpy, host) and contact flags:
    trunk around the standing height, small roll/pitch, any yaw (a quarter of
    the targets across the +-pi seam, so the yaw-error wrap of :333-337 is
    exercised), body-frame velocity targets, feet near the A1 default stance
    rotated into the world frame, trot / stand / random contact patterns."""
    rng = np.random.default_rng(seed)
    B = batch
    s = np.zeros((B, STATE_LEN))
    pos = np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), rng.uniform(0.26, 0.32, B)], 1)
    eul = np.stack([rng.uniform(-0.1, 0.1, B), rng.uniform(-0.1, 0.1, B),
                    rng.uniform(-np.pi, np.pi, B)], 1)
    eul_d = np.stack([np.zeros(B), np.zeros(B), eul[:, 2] + rng.uniform(-0.3, 0.3, B)], 1)
    wrap = rng.random(B) < 0.25
    eul_d[wrap, 2] += np.where(eul[wrap, 2] > 0, 2 * np.pi, -2 * np.pi)
    s[:, 0:3] = pos
    s[:, 3:6] = pos + np.stack([rng.uniform(-0.02, 0.02, B), rng.uniform(-0.02, 0.02, B),
                                rng.uniform(-0.02, 0.02, B)], 1)
    s[:, 6:9] = eul
    s[:, 9:12] = eul_d
    s[:, 12:15] = rng.normal(0, 0.3, (B, 3))
    s[:, 15:18] = np.stack([rng.uniform(-0.5, 0.5, B), rng.uniform(-0.3, 0.3, B), np.zeros(B)], 1)
    s[:, 18:21] = rng.normal(0, 0.3, (B, 3))
    s[:, 21:24] = np.stack([np.zeros(B), np.zeros(B), rng.uniform(-0.5, 0.5, B)], 1)
    R = _rot_zyx(eul[:, 0], eul[:, 1], eul[:, 2])
    Rz = _rot_zyx(np.zeros(B), np.zeros(B), eul[:, 2])
    s[:, 24:33] = R.transpose(0, 2, 1).reshape(B, 9)   # column-major
    s[:, 33:42] = Rz.transpose(0, 2, 1).reshape(B, 9)
    # A1CtrlStates default_foot_pos (FL, FR, RL, RR), body frame, at -0.3 m
    feet_b = np.array([[0.17, 0.15, -0.3], [0.17, -0.15, -0.3], [-0.17, 0.15, -0.3],
                       [-0.17, -0.15, -0.3]])
    fb = feet_b[None] + rng.uniform(-0.03, 0.03, (B, 4, 3))
    fw = np.einsum("bij,blj->bli", R, fb)            # foot_pos_abs = R * foot_pos_rel
    s[:, 42:54] = fw.reshape(B, 12)                   # columns = legs -> legwise 3-vectors
    pats = np.array([[1, 0, 0, 1], [0, 1, 1, 0], [1, 1, 1, 1]], np.uint8)
    kind = rng.integers(0, 4, B)
    ct = np.where(kind[:, None] < 3, pats[np.minimum(kind, 2)],
                  (rng.random((B, 4)) < 0.6).astype(np.uint8)).astype(np.uint8)
    return s, ct


@dataclass
class A1QpResult:
    forces: object              # (B, 12) foot_forces_grf, body frame, 3x4 col-major
    qp_solution: object = None  # (B, 12) world-frame QP solution
    status: object = None
    iters: object = None
    rho_updates: object = None
    obj: object = None


class A1QpBatch:
    """Batched drop-in for the QP branch of A1RobotControl::compute_grf."""

    def __init__(self, params=None, **overrides):
        self.params = params if params is not None else default_params(**overrides)

    def solve(self, state, contacts, out=None, stats=True, stream=None):
        import torch
        B = state.shape[0]
        if (state.dtype != torch.float64 or not state.is_contiguous() or not state.is_cuda
                or tuple(state.shape) != (B, STATE_LEN)):
            raise ValueError("state: contiguous float64 (B, %d) device tensor expected" % STATE_LEN)
        if (contacts.dtype != torch.uint8 or not contacts.is_contiguous() or not contacts.is_cuda
                or tuple(contacts.shape) != (B, 4)):
            raise ValueError("contacts: contiguous uint8 (B, 4) device tensor expected")
        dev = state.device
        if out is None:
            f64 = dict(dtype=torch.float64, device=dev)
            i32 = dict(dtype=torch.int32, device=dev)
            out = A1QpResult(forces=torch.empty((B, 12), **f64))
            if stats:
                out.qp_solution = torch.empty((B, 12), **f64)
                out.status = torch.empty(B, **i32)
                out.iters = torch.empty(B, **i32)
                out.rho_updates = torch.empty(B, **i32)
                out.obj = torch.empty(B, **f64)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        check(lib().qloco_a1_qp_solve(C.byref(self.params), B, ptr(state), ptr(contacts),
                                      ptr(out.forces), ptr(out.qp_solution), ptr(out.status),
                                      ptr(out.iters), ptr(out.rho_updates), ptr(out.obj),
                                      C.c_void_p(stream)), "qloco_a1_qp_solve")
        return out
