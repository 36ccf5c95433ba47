#!/usr/bin/env python3
"""Generate the committed golden fixtures from the CPU oracle.

The reference holds no fixtures for this path, so the goldens
are the oracle's outputs (oracle/, double precision) on deterministic inputs,
plus one known-answer case whose INPUTS come from the reference's own
harness (a1_cpp_open_source/src/test/test_mpc.cpp:18-91; that harness only
prints its result).  Parity status: unpinned.

    python tests/golden/make_golden.py      # rewrites tests/golden/*.npz
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402
from srbd_ref import Instance  # noqa: E402

SEED = 20261015


def srbd_case(name, N, count, gait):
    x0, xr, ft, ct = O.gen_srbd(SEED, N, count, gait=gait)
    sp = O.srbd_spec(N=N)
    u_exact, f_exact, u_admm, it_admm, u_red, it_red, H0, g0 = [], [], [], [], [], [], [], []
    for b in range(count):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xe, st, _ = inst.exact()
        assert st == 0
        xa, info = inst.admm_full()
        xrd, infr = inst.admm_reduced()
        u_exact.append(xe)
        f_exact.append(inst.obj(xe))
        u_admm.append(xa)
        it_admm.append(info.iters)
        u_red.append(xrd)
        it_red.append(infr.iters)
        if b == 0:
            H0, g0 = inst.H, inst.g
    np.savez_compressed(os.path.join(HERE, name), x0=x0, x_ref=xr, feet=ft, contacts=ct,
                        horizon=N, gait=gait, u_exact=np.array(u_exact), f_exact=np.array(f_exact),
                        u_admm=np.array(u_admm), iters_admm=np.array(it_admm),
                        u_admm_reduced=np.array(u_red), iters_admm_reduced=np.array(it_red),
                        H0=H0, g0=g0)


def test_mpc_kat():
    """Inputs of a1_cpp_open_source/src/test/test_mpc.cpp (A1, mass 15,
    contacts FL,RL), with the harness's own x_d quirk (z uses the y velocity,
    :83) and constant feet (v_d = 0 makes its foot update a no-op)."""
    N = 10
    sp = O.srbd_spec(N=N, mass=15.0, inertia=np.diag([0.0158533, 0.0377999, 0.0456542]),
                     q_w=[1, 1, 1, 0, 0, 50, 0, 0, 1, 1, 1, 1, 0], r_w=[1e-6] * 12)
    x0 = np.array([0, 0, 0, 0, 0, 0.15, 0, 0, 0, 0, 0, 0, -9.8], np.float32)
    xr = np.tile(np.array([0, 0, 0, 0, 0, 0.15, 0, 0, 0, 0, 0, 0, -9.8], np.float32), N)
    feet = np.array([0.17, 0.15, -0.35, 0.17, -0.15, -0.35, -0.17, 0.15, -0.35,
                     -0.17, -0.15, -0.35], np.float32)
    ct = np.tile(np.array([1, 0, 1, 0], np.uint8), N)
    inst = Instance(sp, x0, xr, feet, ct)
    xe, st, _ = inst.exact()
    xa, info = inst.admm_full()
    np.savez_compressed(os.path.join(HERE, "srbd_test_mpc_kat.npz"), x0=x0, x_ref=xr, feet=feet,
                        contacts=ct, mass=15.0, inertia=np.diag([0.0158533, 0.0377999, 0.0456542]),
                        q_w=np.array([1, 1, 1, 0, 0, 50, 0, 0, 1, 1, 1, 1, 0], float),
                        r_w=np.full(12, 1e-6), u_exact=xe, f_exact=inst.obj(xe), u_admm=xa,
                        iters_admm=info.iters)


def force_case(ticks=3, B=32):
    from cases import force_inputs
    rng = np.random.default_rng(7)
    prm = O.ForceParams()
    O.lib().qo_force_params_default(C.byref(prm))
    states = []
    for b in range(B):
        s = O.DynState()
        O.lib().qo_dyn_init(C.byref(s))
        states.append(s)
    rec = {k: [] for k in ("com_des", "leg_des", "F_force_des", "rfoot_des", "lfoot_des", "base_p",
                           "feet_p", "FT_total_des", "mode", "right_support", "y_coef", "grf_opt",
                           "F_leg_guess", "qp_solution", "status", "iters")}
    for t in range(ticks):
        inp = force_inputs(rng, B)
        outs = {"grf_opt": [], "F_leg_guess": [], "qp_solution": [], "status": [], "iters": []}
        for b in range(B):
            d = lambda k, b=b: np.ascontiguousarray(inp[k][b], dtype=np.float64)
            O.lib().qo_force_distribution(C.byref(states[b]), O.P(d("com_des")), O.P(d("leg_des")),
                                          O.P(d("F_force_des")), int(inp["mode"][b]),
                                          float(inp["y_coef"][b]), O.P(d("rfoot_des")),
                                          O.P(d("lfoot_des")))
            fe = np.ascontiguousarray(inp["feet_p"][b].reshape(4, 3))
            st, it = C.c_int(0), C.c_int(0)
            ok = O.lib().qo_force_opt(C.byref(states[b]), C.byref(prm), O.P(d("base_p")),
                                      O.P(fe[0].copy()), O.P(fe[1].copy()), O.P(fe[2].copy()),
                                      O.P(fe[3].copy()), O.P(d("FT_total_des")), int(inp["mode"][b]),
                                      int(inp["right_support"][b]), float(inp["y_coef"][b]),
                                      C.byref(st), C.byref(it))
            outs["grf_opt"].append(np.array(states[b].grf_opt[:]))
            outs["F_leg_guess"].append(np.array(states[b].F_leg_guess[:]))
            outs["qp_solution"].append(ok)
            outs["status"].append(st.value)
            outs["iters"].append(it.value)
        for k in inp:
            rec[k].append(inp[k])
        for k in outs:
            rec[k].append(np.array(outs[k]))
    np.savez_compressed(os.path.join(HERE, "force_qp.npz"), **{k: np.array(v) for k, v in rec.items()})
    for s in states:
        O.lib().qo_dyn_free(C.byref(s))


def body_case(B=4):
    rng = np.random.default_rng(11)
    ostates = []
    for b in range(B):
        s = O.BodyState()
        O.lib().qo_body_init(C.byref(s))
        ostates.append(s)
    steps = list(range(96, 140)) + list(range(1905, 1925))
    rec = {k: [] for k in ("i", "bodyangle_state", "zmp_ref", "angle_ref", "rfoot_ref",
                           "lfoot_ref", "comacc_ref", "com_traj", "bjx")}
    cm = lambda a: np.ascontiguousarray(a.transpose(0, 2, 1).reshape(a.shape[0], -1))
    for i in steps:
        ins = dict(bodyangle_state=rng.normal(0, 0.05, (B, 4)), zmp_ref=cm(rng.normal(0, 0.02, (B, 2, 5))),
                   angle_ref=cm(rng.normal(0, 0.02, (B, 2, 5))), rfoot_ref=cm(rng.normal(0, 0.05, (B, 2, 5))),
                   lfoot_ref=cm(rng.normal(0, 0.05, (B, 2, 5))), comacc_ref=cm(rng.normal(0, 0.5, (B, 3, 5))))
        trajs, bjx = [], []
        for b in range(B):
            ct = np.zeros(14)
            O.lib().qo_body_theta_mpc(C.byref(ostates[b]), i, O.P(ins["bodyangle_state"][b].copy()),
                                      O.P(ins["zmp_ref"][b].copy()), O.P(ins["angle_ref"][b].copy()),
                                      O.P(ins["rfoot_ref"][b].copy()), O.P(ins["lfoot_ref"][b].copy()),
                                      O.P(ins["comacc_ref"][b].copy()), O.P(np.zeros(9)), O.P(ct), None)
            trajs.append(ct)
            bjx.append([ostates[b].bjx1, ostates[b].bjx2, ostates[b].t_yu])
        rec["i"].append(i)
        for k, v in ins.items():
            rec[k].append(v)
        rec["com_traj"].append(np.array(trajs))
        rec["bjx"].append(np.array(bjx))
    np.savez_compressed(os.path.join(HERE, "body_mpc.npz"), **{k: np.array(v) for k, v in rec.items()})
    s = ostates[0]
    np.savez_compressed(os.path.join(HERE, "body_schedule.npz"), tx=np.array(s.tx[:]),
                        nsum_mpc=s.nsum_mpc, nstepx=s.nstepx)
    for s in ostates:
        O.lib().qo_body_free(C.byref(s))


if __name__ == "__main__":
    O.build()
    srbd_case("srbd_trot_n10.npz", 10, 16, 0)
    srbd_case("srbd_mixed_n10.npz", 10, 8, 2)
    srbd_case("srbd_pace_n20.npz", 20, 4, 1)
    test_mpc_kat()
    force_case()
    body_case()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
