"""Batched rt_mpc_qp node tick on gfx950.

`RtNodeBatch.tick(gait_msg, ctrl_msg)` runs one iteration of the rt node's
100 Hz loop (unitree_ros/rt_mpc_qp/src/gait_fast.cpp:505-735) for B robots:
the subscriber callbacks on the latest /MPC/Gait (100 doubles) and
/control2rtmpc/state (25 doubles) messages, the reference interpolation,
the contact-schedule / swing-foot / foot-rotation generators of PRMPCClass
and body_theta_mpc, and returns the /rtMPC/traj (100) and /rt2nrt/state (25)
messages.  Member state stays on the device (one workspace per batch).

`synth_messages` produces deterministic wire-format traffic for tests and
the benchmark (there is no recorded ROS traffic in the reference): a slow
planner publishing at 40 Hz with the layout of NLPRTControlClass.cpp:284-392
(Nrtfoorpr_gen from NLPClass_sqp.cpp:1079-1087) and a servo state stream.
"""
import numpy as np

from ._lib import check, lib, ptr

GAIT_LEN, CTRL_LEN, TRAJ_LEN, NRT_LEN, SCHED_LEN = 100, 25, 100, 25, 8


def _stream(t):
    import ctypes as C

    import torch
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check_rows(rows, device):
    """The tick kernels read shape[1] doubles per robot row straight from the
    device pointer: anything but a contiguous float64 tensor of exactly that
    shape on the node's device would be read out of bounds (or a host address
    dereferenced on the GPU), so it is rejected here, before any launch.
    rows: (name, tensor, shape) triples; every layout is checked before any
    device, so a malformed message is named even when both sit on the host."""
    import torch
    for name, t, shape in rows:
        if not isinstance(t, torch.Tensor):
            raise ValueError("%s: expected a torch tensor, got %s" % (name, type(t).__name__))
        if tuple(t.shape) != tuple(shape) or t.dtype != torch.float64 or not t.is_contiguous():
            raise ValueError("%s: expected contiguous float64 %s, got %s %s%s" % (
                name, tuple(shape), t.dtype, tuple(t.shape),
                "" if t.is_contiguous() else " (non-contiguous)"))
    for name, t, _ in rows:
        if t.device != torch.device(device):
            raise ValueError("%s: on %s, the node batch lives on %s" % (name, t.device, device))


class RtNodeBatch:
    """B rt_mpc_qp nodes (PRMPCClass + gait_fast.cpp globals) on one device."""

    def __init__(self, batch, device="cuda:0"):
        import torch
        self.batch = int(batch)
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        nbytes = int(lib().qloco_rt_workspace_bytes(self.batch))
        if nbytes < 0:
            raise ValueError("bad batch %d" % batch)
        self.ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        f64 = dict(dtype=torch.float64, device=self.device)
        self.traj = torch.zeros((self.batch, TRAJ_LEN), **f64)
        self.nrt = torch.zeros((self.batch, NRT_LEN), **f64)
        self.gen = torch.zeros((self.batch, 60), **f64)
        self.sched = torch.zeros((self.batch, SCHED_LEN), dtype=torch.int32, device=self.device)
        check(lib().qloco_rt_init(self.batch, ptr(self.ws), _stream(self.ws)), "qloco_rt_init")

    def tick(self, gait_msg, ctrl_msg, with_debug=True, stream=None):
        """One loop iteration; gait_msg (B,100), ctrl_msg (B,25) float64 device
        tensors.  Returns (traj, nrt, gen, sched) device tensors (reused)."""
        _check_rows((("gait_msg", gait_msg, (self.batch, GAIT_LEN)),
                     ("ctrl_msg", ctrl_msg, (self.batch, CTRL_LEN))), self.device)
        s = _stream(self.ws) if stream is None else stream
        check(lib().qloco_rt_tick(self.batch, ptr(self.ws), ptr(gait_msg), ptr(ctrl_msg),
                                  ptr(self.traj), ptr(self.nrt),
                                  ptr(self.gen) if with_debug else None,
                                  ptr(self.sched) if with_debug else None, s), "qloco_rt_tick")
        return self.traj, self.nrt, self.gen, self.sched


def _u(seed, b, field):
    """counter-based uniform [0,1) per (seed, robot, field), vectorised over b"""
    with np.errstate(over="ignore"):  # mod-2^64 arithmetic (splitmix64 finaliser)
        x = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
             + b.astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9)
             + np.uint64(field) * np.uint64(0x94D049BB133111EB))
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return (x >> np.uint64(11)).astype(np.float64) / float(1 << 53)


_CONSTS = {}


def _robot_consts(seed, first, batch):
    """memoised per-robot uniforms U(field) for one (seed, first, batch)"""
    key = (seed, first, batch)
    if key not in _CONSTS:
        if len(_CONSTS) > 64:
            _CONSTS.clear()
        b = np.arange(first, first + batch, dtype=np.int64)
        cache = {}

        def U(f):
            if f not in cache:
                if isinstance(f, tuple):  # ("c"|"s", field): cos / sin of 2*pi*U(field)
                    ph = 6.28 * U(f[1])
                    cache[f] = np.cos(ph) if f[0] == "c" else np.sin(ph)
                else:
                    cache[f] = _u(seed, b, f)
            return cache[f]
        _CONSTS[key] = U
    return _CONSTS[key]


def synth_messages(seed, batch, tick, first=0):
    """(gait_msg, ctrl_msg) float64 arrays (B,100), (B,25) for loop tick `tick`.

    Per robot: start delay 0..3 ticks on /control2rtmpc/state[0]; a planner
    message index m = floor(tick * 0.01 / 0.025) (40 Hz vs 100 Hz); step
    index bjxx = floor(t_nlp / T) + 1 with a per-robot step period T (half
    the robots also send it as ts, Nrtfoorpr_gen[8]); footholds advance by
    a per-robot step length with the reference's alternating y pattern;
    /MPC/Gait[99] is a per-message counter for 3/4 of the robots (new-data
    branch of xget_position_interpolation) and the planner's right_support
    (0/1/2) for the rest.  COM/ZMP/DCM references are smooth functions of
    the planner time plus per-robot offsets.
    """
    U = _robot_consts(int(seed), int(first), int(batch))
    start = np.floor(U(1) * 4)
    period = 0.6 + 0.2 * U(2)                # step period T
    send_ts = U(3) < 0.5
    steplen = 0.08 * U(4)
    counter_flag = U(5) < 0.75
    vx = steplen / period
    m = np.floor(tick * 0.01 / 0.025)        # planner message index
    t_nlp = m * 0.025
    gait = np.zeros((GAIT_LEN, batch))  # field-major while filling
    ctrl = np.zeros((CTRL_LEN, batch))
    ctrl[0] = (tick >= start).astype(np.float64)
    # sin(a + c) = sin(a) cos(c) + cos(a) sin(c): per-tick scalars a, cached
    # per-robot phases c -- no per-robot transcendental per column
    for k in range(1, CTRL_LEN):
        a = 0.37 * tick + 1.3 * k
        ctrl[k] = 0.05 * (np.sin(a) * U(("c", 100 + k)) + np.cos(a) * U(("s", 100 + k)))
    ph = 2 * np.pi * t_nlp / period
    sph, cph = np.sin(ph), np.cos(ph)
    sh, ch = np.sin(ph / 2), np.cos(ph / 2)
    gait[0] = vx * t_nlp + 0.01 * U(10)
    gait[1] = 0.02 * sh
    gait[2] = 0.309458 + 0.005 * sph
    gait[36] = vx
    gait[37] = 0.02 * np.pi / period * ch
    gait[38] = 0.005 * 2 * np.pi / period * cph
    for k in (39, 40, 41, 80, 81, 82, 83, 84, 85):
        gait[k] = 0.3 * (sph * np.cos(k) + cph * np.sin(k))
    for k in (12, 13, 34, 35, 42, 43, 44, 45, 76, 77, 78, 79):
        gait[k] = 0.03 * (sph * np.cos(0.5 * k) + cph * np.sin(0.5 * k)) + (
            0.0 if k % 2 else vx * t_nlp)
    for k in list(range(3, 12)) + list(range(14, 27)) + list(range(28, 34)) + list(range(46, 76)):
        a = 0.1 * m + k
        gait[k] = 0.01 * (np.sin(a) * U(("c", 200 + k)) + np.cos(a) * U(("s", 200 + k)))
    bjxx = np.minimum(np.floor(np.maximum(t_nlp - 1.0, 0.0) / period) + 1, 25)
    gait[27] = bjxx
    fy = lambda i: np.where(i % 2 == 1, 0.12675, -0.12675)
    gait[86] = bjxx
    gait[87] = bjxx * steplen
    gait[88] = (bjxx + 1) * steplen
    gait[89] = fy(bjxx) + 0.01 * (U(6) - 0.5)
    gait[90] = fy(bjxx + 1) + 0.01 * (U(7) - 0.5)
    gait[91] = 0.005 * U(8)
    gait[92] = 0.005 * U(9)
    gait[93] = bjxx - 1
    gait[94] = np.where(send_ts, period, 0.0)
    gait[97] = 0.0
    gait[98] = 1e-4
    right_support = np.where(bjxx < 2, 2, bjxx % 2)
    gait[99] = np.where(counter_flag, m + 1, right_support)
    return np.ascontiguousarray(gait.T), np.ascontiguousarray(ctrl.T)


NLP_STEPS, NLP_DT = 27, 0.025  # NLPClass _footstepsnumber, _dt (NLPClass.h:32)


def support_phase(ts, tx, t_int, t_end_footstep, stream=None):
    """Slow planner's contact-phase flag for B robots (qloco_support_phase):
    ts, tx (B, 27) float64, t_int, t_end_footstep (B,) int32 device tensors
    -> (bjxx, bjx1, right_support) int32 device tensors.  Restates
    NLPClass_sqp.cpp:1029-1039 + Foot_trajectory_solve_mod2's right_support
    (mosek_nlp_kmp); right_support is what /MPC/Gait[99] carries to servo.cpp:673."""
    import torch
    B = int(t_int.shape[0])
    for name, t, shape, dt in (("ts", ts, (B, NLP_STEPS), torch.float64),
                               ("tx", tx, (B, NLP_STEPS), torch.float64),
                               ("t_int", t_int, (B,), torch.int32),
                               ("t_end_footstep", t_end_footstep, (B,), torch.int32)):
        if tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous() or not t.is_cuda:
            raise ValueError("%s: expected contiguous %s %s on the GPU" % (name, shape, dt))
    out = torch.empty((3, B), dtype=torch.int32, device=t_int.device)
    s = _stream(t_int) if stream is None else stream
    check(lib().qloco_support_phase(B, ptr(ts), ptr(tx), ptr(t_int), ptr(t_end_footstep),
                                    ptr(out[0]), ptr(out[1]), ptr(out[2]), s),
          "qloco_support_phase")
    return out[0], out[1], out[2]


def synth_schedules(seed, batch):
    """Deterministic planner schedules (numpy): per robot a current step k,
    _ts = 0.7 s (Initialize) up to k and SQP-updated durations in [0.45, 1.0]
    after it; _tx rounded to the 0.025 s grid minus 1e-6 up to k
    (NLPClass_sqp.cpp:204-205) and accumulated unrounded after it (:908);
    t_int inside or around step k (a quarter exactly on the grid points of
    _tx), t_end_footstep = round((_tx(26) - 2 * 0.7) / dt) (:593) with some
    robots past it.  Returns ts, tx (B, 27) f64 and t_int, t_end (B,) i32."""
    rng = np.random.default_rng(seed)
    B, S, dt = batch, NLP_STEPS, NLP_DT
    k = rng.integers(1, S - 1, size=B)
    ts = np.full((B, S), 0.7)
    upd = np.arange(S)[None, :] >= k[:, None]
    ts = np.where(upd, rng.uniform(0.45, 1.0, size=(B, S)), ts)
    tx = np.zeros((B, S))
    for i in range(1, S):
        rounded = np.round((tx[:, i - 1] + ts[:, i - 1]) / dt) * dt - 0.000001
        tx[:, i] = np.where(i <= k, rounded, tx[:, i - 1] + ts[:, i - 1])
    lo = np.round(tx[np.arange(B), k - 1] / dt).astype(np.int64)
    hi = np.round(tx[np.arange(B), k] / dt).astype(np.int64)
    t_int = lo + (rng.uniform(size=B) * (hi - lo + 6)).astype(np.int64) - 3
    on_grid = rng.uniform(size=B) < 0.25
    t_int = np.where(on_grid, lo, t_int)
    t_int = np.maximum(t_int, 0)
    t_end = np.round((tx[:, S - 1] - 2 * 0.7) / dt).astype(np.int64)
    late = rng.uniform(size=B) < 0.1
    t_end = np.where(late, t_int - 1 - rng.integers(0, 5, size=B), t_end)
    return ts, tx, t_int.astype(np.int32), t_end.astype(np.int32)
