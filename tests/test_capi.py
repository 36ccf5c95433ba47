"""CPU tests of the C ABI (include/qloco.h) -- no compute calls, no GPU.

* libqloco.so loads and exports exactly the functions the header declares;
  the ctypes table in quadrupedal_loco_amd/_lib.py covers all of them.
* Host-only entry points: defaults carry the reference's constants, the
  synthetic-instance generator is bit-identical to the oracle's, status
  strings are defined.
* Argument validation returns before any device work (empty batch OK,
  bad sizes / NULL pointers rejected).
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle_lib as O
from quadrupedal_loco_amd import _lib, qp, srbd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "qloco.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(qloco_\w+)\s*\(", txt, flags=re.M)))


def test_header_symbols_exported():
    fns = header_functions()
    assert len(fns) >= 17, fns
    L = _lib.lib()
    missing = [f for f in fns if not hasattr(L, f)]
    assert not missing, missing
    assert sorted(_lib.SIGNATURES) == fns, set(_lib.SIGNATURES) ^ set(fns)
    assert _lib.missing_symbols() == []


def test_abi_version_and_status_strings():
    L = _lib.lib()
    assert L.qloco_abi_version() == 1
    for code in (0, 1, 2, 3, 4, 5, 6, 7, 8, 100, 101, 102):
        s = L.qloco_status_string(code).decode()
        assert s and "unknown" not in s.lower(), (code, s)


def test_srbd_spec_defaults_are_reference_constants():
    s = srbd.default_spec()
    assert s.horizon == 10 and abs(s.dt - 0.0025) < 1e-9 and s.mass == 12.0
    assert np.allclose(np.array(s.inertia[:]).reshape(3, 3), O.GO1_INERTIA, rtol=1e-6)
    assert np.allclose(s.q_weights[:], O.Q_W) and np.allclose(s.r_weights[:], O.R_W)
    assert abs(s.mu - 0.3) < 1e-7 and s.fz_min == 0.0 and s.fz_max == 180.0
    # OSQP v0.6 defaults
    assert abs(s.rho - 0.1) < 1e-8 and abs(s.sigma - 1e-6) < 1e-12 and abs(s.alpha - 1.6) < 1e-7
    assert abs(s.eps_abs - 1e-3) < 1e-9 and abs(s.eps_rel - 1e-3) < 1e-9
    assert s.max_iter == 4000 and s.check_termination == 25 and s.scaling == 10
    assert s.adaptive_rho == 1 and s.adaptive_rho_interval == 0
    assert s.adaptive_rho_tolerance == 5.0 and s.warm_start == 0 and s.polish == 0
    # up to N = 20 all-stance: 80 stance legs, 240 variables (the wide kernel)
    assert _lib.lib().qloco_srbd_max_stance_vars() == 240


def test_force_params_defaults():
    p = qp.force_params()
    # Dynamiccclass ctor constants (dynmics_compute.cpp:29-100)
    assert (p.alpha, p.beta, p.gamma, p.fz_max) == (1e4, 1e3, 10.0, 160.0)
    assert p.mass == 12.0
    o = O.ForceParams()
    O.lib().qo_force_params_default(C.byref(o))
    for k in ("mass", "alpha", "beta", "gamma", "fz_max", "mu"):
        assert getattr(p, k) == getattr(o, k), k


@pytest.mark.parametrize("weights", ["default", "gazebo", "hardware", "isaac"])
def test_srbd_route_keeps_reference_weights_on_the_wrench_space_kernels(weights):
    """qloco_srbd_route (host-only): the literal QP with the Go1 defaults and
    the reference's gazebo / hardware weight sets runs the wrench-space
    kernels -- one wave at N <= 10, two at 11..20; isaac's (state weights
    above 1000: the wrench-space solve's float32 limit), a
    zero omega / v weight or per-step feet take the generic literal kernels;
    literal_full_qp = 0 the reduced classes; an anisotropic omega weight of
    moderate size stays on the wrench-space kernels."""
    kw = {} if weights == "default" else dict(zip(("q_weights", "r_weights"), srbd.REFERENCE_WEIGHTS[weights]))
    stiff = weights == "isaac"  # state weights above the wrench-space kernels' 1000
    for N, want in ((1, 1), (10, 1), (11, 2), (16, 2), (20, 2)):
        want = 3 if stiff else want
        assert srbd.route(srbd.default_spec(horizon=N, literal_full_qp=1, **kw)) == want, (N, weights)
    assert srbd.route(srbd.default_spec(horizon=10, literal_full_qp=0, **kw)) == 4
    assert srbd.route(srbd.default_spec(horizon=10, literal_full_qp=1, feet_per_step=1, **kw)) == 3
    q = list(srbd.default_spec(**kw).q_weights)
    if not stiff:
        q2 = list(q)
        q2[7] = 2.0 * q2[6] + 0.3  # anisotropic omega weights
        assert srbd.route(srbd.default_spec(horizon=16, literal_full_qp=1, q_weights=q2)) == 2
    q[9] = 0.0
    assert srbd.route(srbd.default_spec(horizon=10, literal_full_qp=1, q_weights=q)) == 3
    bad = srbd.default_spec(horizon=0)
    assert _lib.lib().qloco_srbd_route(C.byref(bad)) == 100


@pytest.mark.parametrize("gait", ["trot", "pace", "mixed", "stance"])
@pytest.mark.parametrize("N", [1, 10, 20])
def test_generator_bit_identical_to_oracle(gait, N):
    g = srbd.GAITS[gait]
    a = srbd.generate(20261015, N, 37, gait, first=1000)
    b = O.gen_srbd(20261015, N, 37, gait=g, first=1000)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_generator_shards_concatenate():
    """Counter-based generator: rank shards regenerate the same global batch."""
    full = srbd.generate(7, 10, 64, "mixed")
    parts = [srbd.generate(7, 10, 16, "mixed", first=16 * r) for r in range(4)]
    for k in range(4):
        assert np.array_equal(full[k], np.concatenate([p[k] for p in parts]))


def test_generator_gait_structure():
    x0, xr, ft, ct = srbd.generate(1, 10, 64, "trot")
    c = ct.reshape(64, 10, 4)
    # trot: diagonal pairs {FL,RR} / {FR,RL} (FL, FR, RL, RR order), constant over the horizon
    assert np.all(c == c[:, :1])
    assert np.all((c[:, 0] == [1, 0, 0, 1]).all(1) | (c[:, 0] == [0, 1, 1, 0]).all(1))
    assert np.all(x0[:, 12] == np.float32(-9.8))
    _, _, _, ctp = srbd.generate(1, 10, 64, "pace")
    cp = ctp.reshape(64, 10, 4)[:, 0]
    assert np.all((cp == [1, 0, 1, 0]).all(1) | (cp == [0, 1, 0, 1]).all(1))


def test_body_state_init_host_matches_oracle():
    st = np.zeros((3, 32))
    assert _lib.lib().qloco_body_state_init_host(3, _lib.ptr(st)) == 0
    assert np.all(st[:, :26] == 0.0) and np.all(st[:, 29] == 1.0)  # qp_solution starts true
    s = O.BodyState()
    O.lib().qo_body_init(C.byref(s))
    assert np.all(st[:, 26] == s.bjx1) and np.all(st[:, 27] == s.bjx2)
    O.lib().qo_body_free(C.byref(s))


def test_argument_validation_without_device_work():
    L = _lib.lib()
    sp = srbd.default_spec()
    # empty batch: nothing to do, OK without touching the device
    assert L.qloco_srbd_solve(C.byref(sp), 0, *([None] * 10), None) == 0
    assert L.qloco_srbd_build(C.byref(sp), 0, *([None] * 10), None) == 0
    # NULL spec / negative batch / bad horizon
    assert L.qloco_srbd_solve(None, 4, *([None] * 10), None) == 100
    assert L.qloco_srbd_solve(C.byref(sp), -1, *([None] * 10), None) == 100
    bad = srbd.default_spec(horizon=21)
    assert L.qloco_srbd_solve(C.byref(bad), 4, *([None] * 10), None) == 4
    assert L.qloco_srbd_build(C.byref(bad), 4, *([None] * 10), None) == 4
    # missing required pointers
    assert L.qloco_srbd_solve(C.byref(sp), 4, *([None] * 10), None) == 100
    # EiQuadProg limits: QPBaseClass's capacity (nVars <= 60, nIneq <= 300,
    # QPBaseClass.h:49-51) rounded up -- n, p <= 64, m <= 320
    lim = (C.c_int32 * 3)()
    L.qloco_gi_limits(C.byref(lim, 0), C.byref(lim, 4), C.byref(lim, 8))
    assert list(lim) == [64, 64, 320]
    # the fast path (four QPs per wavefront): qloco_max_gi_vars keeps its
    # round-1 meaning, qloco_gi_fast_limits gives all three
    assert L.qloco_max_gi_vars() == 16
    L.qloco_gi_fast_limits(C.byref(lim, 0), C.byref(lim, 4), C.byref(lim, 8))
    assert list(lim) == [16, 16, 64]
    args = [None, 0] * 6 + [None] * 4 + [None]
    assert L.qloco_eiquadprog_solve(65, 0, 8, 1, *args) == 4
    assert L.qloco_eiquadprog_solve(8, 65, 8, 1, *args) == 4
    assert L.qloco_eiquadprog_solve(8, 0, 321, 1, *args) == 4
    assert L.qloco_eiquadprog_solve(60, 10, 300, 1, *args) == 100  # in range: NULL pointers refused
    assert L.qloco_eiquadprog_solve(8, 0, 8, 0, *args) == 100  # NULL G even when empty


def test_cpp_shim_exports_reference_classes():
    """libqloco_host.so carries the reference-shaped C++ classes."""
    import subprocess
    lib = os.path.join(ROOT, "quadrupedal_loco_amd", "lib", "libqloco_host.so")
    if not os.path.exists(lib):
        from quadrupedal_loco_amd import build as qb
        qb.build()
    out = subprocess.run(["nm", "-DC", "--defined-only", lib], capture_output=True, text=True).stdout
    for sym in ("qloco::Dynamiccclass::force_distribution", "qloco::Dynamiccclass::force_opt",
                "qloco::PRMPCClass::body_theta_mpc", "qloco::PRMPCClass::Indexfind",
                "qloco::QPsolverGpu::resize", "qloco::QPsolverGpu::solve",
                "qloco::QPBaseClassGpu::solveQP", "qloco::ConvexMpcBatch::compute_grf",
                "qloco::Kinematicclass::Forward_kinematics_g",
                "qloco::Kinematicclass::Inverse_kinematics_g"):
        assert sym in out, sym


def test_rt_servo_support_argument_validation_without_device_work():
    """the rt tick, servo block and contact-phase entry points reject bad
    calls (and accept empty batches) before any device work"""
    L = _lib.lib()
    assert L.qloco_rt_workspace_bytes(-1) == -1
    assert L.qloco_servo_workspace_bytes(-1) == -1
    # the rt node state is allocated in whole 64-robot tiles (551 doubles each)
    assert L.qloco_rt_workspace_bytes(1) >= 8 * 551 * 64
    assert L.qloco_rt_workspace_bytes(65) > L.qloco_rt_workspace_bytes(64)
    assert L.qloco_rt_init(-1, None, None) == 100
    assert L.qloco_rt_init(0, None, None) == 0
    assert L.qloco_rt_tick(-1, *([None] * 8)) == 100
    assert L.qloco_rt_tick(0, *([None] * 8)) == 0
    assert L.qloco_rt_tick(4, *([None] * 8)) == 100
    assert L.qloco_support_phase(-1, *([None] * 8)) == 100
    assert L.qloco_support_phase(0, *([None] * 8)) == 0
    assert L.qloco_support_phase(4, *([None] * 8)) == 100
    # servo force block (servo.cpp:1052-1243 replacement)
    fp = qp.force_params()
    assert L.qloco_servo_init(-1, None, None) == 100
    assert L.qloco_servo_init(0, None, None) == 0
    assert L.qloco_servo_init(4, None, None) == 100          # NULL workspace
    assert L.qloco_servo_force_block(None, 1, *([None] * 22)) == 100
    assert L.qloco_servo_force_block(C.byref(fp), -1, *([None] * 22)) == 100
    assert L.qloco_servo_force_block(C.byref(fp), 0, *([None] * 22)) == 0
    assert L.qloco_servo_force_block(C.byref(fp), 4, *([None] * 22)) == 100
    # the grouped force-QP launch: workspace length, argument checks
    assert L.qloco_force_order_ws_len(-1) == -1
    assert L.qloco_force_order_ws_len(1000) == 2 * 1000 + 160
    assert L.qloco_force_qp_solve_ordered(None, 1, *([None] * 19)) == 100
    assert L.qloco_force_qp_solve_ordered(C.byref(fp), -1, *([None] * 19)) == 100
    assert L.qloco_force_qp_solve_ordered(C.byref(fp), 0, *([None] * 19)) == 0
    assert L.qloco_force_qp_solve_ordered(C.byref(fp), 4, *([None] * 19)) == 100


def test_srbd_polish_rejected_until_implemented():
    """OSQP polishing is not implemented: a spec asking for it is refused
    (QLOCO_ERR_ARG) instead of silently returning unpolished iterates."""
    L = _lib.lib()
    sp = srbd.default_spec(polish=1)
    dummy = [C.c_void_p(16)] * 5  # never dereferenced: rejected before any device work
    assert L.qloco_srbd_solve(C.byref(sp), 4, *dummy, None, None, None, None, None, None) == 100
    assert L.qloco_srbd_solve_ex(C.byref(sp), 4, *dummy, None, None, None, None, None, None,
                                 0, None) == 100


def test_force_group_width_setter():
    """qloco_force_set_group_width (host-only, no GPU call): 8 / 16 accepted
    and the previous width returned, anything else QLOCO_ERR_ARG with the
    width unchanged."""
    from quadrupedal_loco_amd._lib import lib
    L = lib()
    prev = L.qloco_force_set_group_width(16)
    try:
        assert prev in (8, 16)
        assert L.qloco_force_set_group_width(8) == 16
        assert L.qloco_force_set_group_width(0) == 100
        assert L.qloco_force_set_group_width(32) == 100
        assert L.qloco_force_set_group_width(8) == 8
    finally:
        L.qloco_force_set_group_width(prev)
