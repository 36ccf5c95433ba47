"""GPU parity tests for the small-QP paths (EiQuadProg / force QP / body MPC).

Checker: the oracle's double-precision restatement (oracle/eiquadprog.c,
force_qp.c, body_mpc.c).  The GPU kernels run the same fp64 operation
sequence (no FMA contraction, one lane per dot product in index order), so
the stated tolerance is tight: status and iteration count equal, results
within 1e-9 relative (bit-identical in the common case -- the fraction is
asserted >= 90 %); schedule integers (Indexfind, bjx1/bjx2/t_yu) bit-exact.
"""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import oracle_lib as O  # noqa: E402
from cases import force_inputs  # noqa: E402

from quadrupedal_loco_amd import qp  # noqa: E402


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def random_qp(rng, n, p, m, zero_ce=0):
    M = rng.standard_normal((n, n))
    G = M @ M.T + n * np.eye(n)
    g0 = rng.standard_normal(n) * 3
    CE = rng.standard_normal((n, p))
    for k in range(min(zero_ce, p)):
        CE[:, rng.integers(p)] = 0.0
    ce0 = rng.standard_normal(p) * 0.3
    CI = rng.standard_normal((n, m))
    ci0 = rng.standard_normal(m) + 0.5
    return G, g0, CE, ce0, CI, ci0


def random_feasible_qp(rng, n, p, m, zero_ce=0):
    """Random QP feasible by construction: equalities and inequalities hold
    at a random point x_f (inequalities strictly), so the solve ends OK and
    exercises the active set (the unconstrained minimum violates many rows)."""
    G, g0, CE, ce0, CI, ci0 = random_qp(rng, n, p, m, zero_ce)
    x_f = rng.standard_normal(n) * 0.3
    ce0 = -CE.T @ x_f
    ci0 = -CI.T @ x_f + np.abs(rng.standard_normal(m)) + 0.1
    return G, g0 * 10, CE, ce0, CI, ci0


def oracle_eqp(G, g0, CE, ce0, CI, ci0):
    n, p, m = G.shape[0], CE.shape[1], CI.shape[1]
    ws = O.lib().qo_eqp_create(n, p, m)
    Gc = np.asfortranarray(G).ravel(order="F").copy()
    CEc = np.asfortranarray(CE).ravel(order="F").copy() if p else np.zeros(1)
    CIc = np.asfortranarray(CI).ravel(order="F").copy() if m else np.zeros(1)
    x = np.zeros(n)
    st, it = C.c_int(0), C.c_int(0)
    ce0c = np.ascontiguousarray(ce0) if p else np.zeros(1)
    ci0c = np.ascontiguousarray(ci0) if m else np.zeros(1)
    f = O.lib().qo_eqp_solve(ws, O.P(Gc), O.P(np.ascontiguousarray(g0)), O.P(CEc), O.P(ce0c),
                             O.P(CIc), O.P(ci0c), O.P(x), C.byref(st), C.byref(it))
    O.lib().qo_eqp_destroy(ws)
    return x, f, st.value, it.value


@pytest.mark.parametrize("n,p,m,zero_ce", [(4, 0, 8, 0), (8, 0, 48, 0), (12, 12, 24, 6),
                                           (12, 3, 24, 0), (16, 4, 64, 2)])
def test_eiquadprog_matches_restatement(n, p, m, zero_ce):
    dev = _dev()
    rng = np.random.default_rng(n * 100 + p * 10 + m)
    B = 64
    probs = [random_qp(rng, n, p, m, zero_ce) for _ in range(B)]
    stack = lambda k: np.stack([np.asfortranarray(pr[k]).ravel(order="F") for pr in probs])
    res = qp.eiquadprog_solve(*(torch.from_numpy(stack(k)).to(dev) for k in range(6)),
                              n=n, p=p, m=m)
    torch.cuda.synchronize()
    x = res["x"].cpu().numpy()
    f = res["f"].cpu().numpy()
    st = res["status"].cpu().numpy()
    it = res["iters"].cpu().numpy()
    exact = 0
    for b in range(B):
        xo, fo, sto, ito = oracle_eqp(*probs[b])
        assert st[b] == sto, (b, st[b], sto)
        assert it[b] == ito, (b, it[b], ito)
        if sto == 0:
            assert np.allclose(x[b], xo, rtol=1e-9, atol=1e-9), (b, x[b], xo)
            assert np.isclose(f[b], fo, rtol=1e-9, atol=1e-9)
            exact += int(np.array_equal(x[b], xo))
    ok = int(np.sum(st == 0))
    assert exact >= 0.9 * ok, (exact, ok)


@pytest.mark.parametrize("n,p,m,zero_ce", [(60, 10, 300, 3), (30, 0, 120, 0), (17, 17, 65, 4),
                                           (64, 64, 320, 8), (40, 6, 200, 0)])
def test_eiquadprog_wide_matches_restatement(n, p, m, zero_ce):
    """The reference's QPBaseClass capacity (nVars <= 60, nIneq <= 300,
    QPBaseClass.h:49-51) through qloco_eiquadprog_solve's size dispatch: one
    QP per wavefront (qloco_gi_wide.hip), zero CE columns included (the
    me = p / A(i) quirks).  Status and active-set iterations equal to the
    restatement; x within 1e-9 relative (the triangular solves are column
    sweeps, so results agree to rounding, not bit for bit), f within 1e-9."""
    dev = _dev()
    rng = np.random.default_rng(n * 1000 + p * 10 + m)
    B = 24
    probs = [random_feasible_qp(rng, n, p, m, zero_ce) for _ in range(B)]
    stack = lambda k: np.stack([np.asfortranarray(pr[k]).ravel(order="F") for pr in probs])
    res = qp.eiquadprog_solve(*(torch.from_numpy(stack(k)).to(dev) for k in range(6)),
                              n=n, p=p, m=m)
    torch.cuda.synchronize()
    x = res["x"].cpu().numpy()
    f = res["f"].cpu().numpy()
    st = res["status"].cpu().numpy()
    it = res["iters"].cpu().numpy()
    solved = 0
    for b in range(B):
        xo, fo, sto, ito = oracle_eqp(*probs[b])
        assert st[b] == sto, (b, st[b], sto)
        assert it[b] == ito, (b, it[b], ito)
        if sto == 0:
            solved += 1
            sc = max(1.0, np.abs(xo).max())
            assert np.abs(x[b] - xo).max() <= 1e-9 * sc, (b, np.abs(x[b] - xo).max())
            assert abs(f[b] - fo) <= 1e-9 * max(1.0, abs(fo)), (b, f[b], fo)
    # p = n with skipped zero CE columns drives EiQuadProg's index quirks into
    # infeasible reports on some instances (the restatement does the same)
    assert solved >= (4 if p >= n else B // 2), solved
    assert np.mean(it) > 2  # the active set did work


@pytest.mark.parametrize("hw,grouped", [(False, False), (True, True), (True, False)])
def test_force_qp_matches_restatement_over_ticks(hw, grouped):
    """force_distribution + force_opt over three ticks of member state against
    the oracle (dynmics_compute.cpp:141-445), bit-exact in >= 90 % of
    instances and within 1e-9 otherwise -- with the sim's constants (mass 12,
    mu 0.25) and with the hardware copy's (unitree_legged_real: mass =
    gait::mass = 14, mu = 0.5, called at torque_mode.cpp:1364-1367), through
    the plain and the grouped launch."""
    dev = _dev()
    rng = np.random.default_rng(7)
    B, ticks = 96, 3
    prm = O.ForceParams()
    O.lib().qo_force_params_default(C.byref(prm))
    if hw:
        prm.mass, prm.mu = 14.0, 0.5
    states = []
    for b in range(B):
        s = O.DynState()
        O.lib().qo_dyn_init(C.byref(s))
        states.append(s)
    solver = qp.ForceQP(batch=B, device=dev, grouped=grouped, hw=hw)
    assert (solver.params.mass, solver.params.mu) == ((14.0, 0.5) if hw else (12.0, 0.25))
    exact, total = 0, 0
    for tick in range(ticks):
        inp = force_inputs(rng, B)
        out = solver.step(**{k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
                             for k, v in inp.items()})
        torch.cuda.synchronize()
        g = out["grf_opt"].cpu().numpy()
        guess = out["F_leg_guess"].cpu().numpy()
        qps = out["qp_solution"].cpu().numpy()
        st = out["status"].cpu().numpy()
        for b in range(B):
            d = lambda k, b=b: np.ascontiguousarray(inp[k][b], dtype=np.float64)
            O.lib().qo_force_distribution(C.byref(states[b]), O.P(d("com_des")), O.P(d("leg_des")),
                                          O.P(d("F_force_des")), int(inp["mode"][b]),
                                          float(inp["y_coef"][b]), O.P(d("rfoot_des")),
                                          O.P(d("lfoot_des")))
            fe = inp["feet_p"][b].reshape(4, 3)
            est, eit = C.c_int(0), C.c_int(0)
            ok = O.lib().qo_force_opt(C.byref(states[b]), C.byref(prm), O.P(d("base_p")),
                                      O.P(np.ascontiguousarray(fe[0])), O.P(np.ascontiguousarray(fe[1])),
                                      O.P(np.ascontiguousarray(fe[2])), O.P(np.ascontiguousarray(fe[3])),
                                      O.P(d("FT_total_des")), int(inp["mode"][b]),
                                      int(inp["right_support"][b]), float(inp["y_coef"][b]),
                                      C.byref(est), C.byref(eit))
            ref = np.array(states[b].grf_opt[:])
            assert np.array_equal(guess[b], np.array(states[b].F_leg_guess[:])), b
            assert qps[b] == ok and st[b] == est.value, (b, qps[b], ok, st[b], est.value)
            assert np.allclose(g[b], ref, rtol=1e-9, atol=1e-8), (tick, b, g[b], ref)
            exact += int(np.array_equal(g[b], ref))
            total += 1
    assert exact >= 0.9 * total, (exact, total)
    for s in states:
        O.lib().qo_dyn_free(C.byref(s))


@pytest.mark.parametrize("grouped", [True, False])
def test_force_qp_group_width_is_bit_identical(grouped):
    """Eight 8-lane groups per wave (the default) and four 16-lane groups run
    the same per-element operations in the same order (qloco_gi_core.hpp):
    every output equal bit for bit over four ticks, member state carried,
    B = 1001 (a partial last wavefront at both widths)."""
    from quadrupedal_loco_amd._lib import lib
    dev = _dev()
    L = lib()
    rng = np.random.default_rng(12)
    B, ticks = 1001, 4
    a = qp.ForceQP(batch=B, device=dev, grouped=grouped)
    b = qp.ForceQP(batch=B, device=dev, grouped=grouped)
    prev = L.qloco_force_set_group_width(8)
    try:
        for tick in range(ticks):
            inp = force_inputs(rng, B)
            d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in inp.items()}
            assert L.qloco_force_set_group_width(8) in (8, 16)
            oa = a.step(**d)
            torch.cuda.synchronize()
            assert L.qloco_force_set_group_width(16) == 8
            ob = b.step(**d)
            torch.cuda.synchronize()
            for k in ("grf_opt", "F_leg_guess", "F_leg_ref", "qp_solution", "status", "iters"):
                assert torch.equal(oa[k], ob[k]), (tick, k)
        assert L.qloco_force_set_group_width(4) == 100  # QLOCO_ERR_ARG, width unchanged
        assert L.qloco_force_set_group_width(16) == 16
    finally:
        L.qloco_force_set_group_width(prev)


def test_force_qp_grouped_launch_replays_from_a_hip_graph():
    """The grouped force-QP call (memset + count + scatter + force kernel,
    INTEGRATION.md §2) allocates nothing and keeps its state in caller
    buffers, so it can be captured once and replayed every servo tick: a
    captured ForceQP.step fed new inputs through static tensors gives the
    eager call's outputs bit for bit over four ticks, member state and
    grouping state carried by both."""
    dev = _dev()
    rng = np.random.default_rng(13)
    B, ticks = 1001, 4
    ticks_in = [{k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in force_inputs(rng, B).items()}
                for _ in range(ticks)]
    static = {k: v.clone() for k, v in ticks_in[0].items()}
    eager = qp.ForceQP(batch=B, device=dev)
    graphed = qp.ForceQP(batch=B, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):  # warm-up on a throw-away instance: constants uploaded
        qp.ForceQP(batch=B, device=dev).step(**static)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        og = graphed.step(**static)
    for tick in range(ticks):
        for k, v in ticks_in[tick].items():
            static[k].copy_(v)
        g.replay()
        oe = eager.step(**ticks_in[tick])
        torch.cuda.synchronize()
        for k in ("grf_opt", "F_leg_guess", "F_leg_ref", "qp_solution", "status", "iters"):
            assert torch.equal(og[k], oe[k]), (tick, k)
        # the carried iteration counts (the list's order inside a class is immaterial)
        assert torch.equal(graphed.order_ws[:B], eager.order_ws[:B]), tick


def test_force_qp_grouped_launch_is_bit_identical():
    """qloco_force_qp_solve_ordered groups the robots by swing-leg pattern and
    previous iteration count before the launch; every robot's
    arithmetic is unchanged, so grf_opt / F_leg_ref / status / iterations equal
    the ungrouped launch's bit for bit, tick after tick (the member state and
    the grouping state both carried).  B = 1001: a partial last wavefront.
    The workspace's list is a permutation in (pattern, previous iterations)
    order."""
    dev = _dev()
    rng = np.random.default_rng(11)
    B, ticks = 1001, 4
    grouped = qp.ForceQP(batch=B, device=dev)
    plain = qp.ForceQP(batch=B, device=dev, grouped=False)
    assert grouped.order_ws.numel() == 2 * B + 160
    for tick in range(ticks):
        inp = force_inputs(rng, B)
        d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in inp.items()}
        prev = grouped.order_ws[:B].clone()
        og = grouped.step(**d)
        op = plain.step(**d)
        torch.cuda.synchronize()
        for k in ("grf_opt", "F_leg_guess", "F_leg_ref", "qp_solution", "status", "iters"):
            assert torch.equal(og[k], op[k]), (tick, k)
        assert torch.equal(grouped.order_ws[:B], op["iters"]), tick  # carried for the next call
        lst = grouped.order_ws[B:2 * B].cpu().numpy()
        assert np.array_equal(np.sort(lst), np.arange(B)), tick
        m, rs = inp["mode"][lst], inp["right_support"][lst]
        pat = np.where(m == 102, np.where(rs == 0, 1, np.where(rs == 1, 2, 0)),
                       np.where(m == 101, np.where(rs == 0, 3, np.where(rs == 1, 4, 0)), 0))
        key = pat * 16 + np.minimum(prev.cpu().numpy()[lst], 15)
        assert np.all(np.diff(key) >= 0), tick


def test_hw_torque_ff_bit_exact():
    """The hardware loop's feed-forward after force_opt (unitree_legged_real
    torque_mode.cpp:1370-1384: stand-up ramp blend of grf_opt with the
    stand-up GRF, tau = -J^T F, no gravity compensation) against the oracle's
    restatement, bit for bit, over the ramp (dynamic_count 0 .. 700: rate 0,
    partial, 1, clamped)."""
    dev = _dev()
    rng = np.random.default_rng(5)
    B = 1003
    J = rng.normal(0, 0.3, (B, 4, 9))
    g = rng.normal(0, 40, (B, 12))
    base = rng.normal(0, 30, (B, 12))
    cnt = rng.integers(0, 700, B).astype(np.int32)
    cnt[:4] = [0, 1, 500, 501]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    tau = qp.hw_torque_ff(d(J), d(g), d(base), d(cnt)).cpu().numpy()
    for b in range(B):
        ref = np.zeros(12)
        O.lib().qo_hw_torque_ff(O.P(np.ascontiguousarray(J[b])), O.P(g[b].copy()), O.P(base[b].copy()),
                                int(cnt[b]), O.P(ref))
        assert np.array_equal(tau[b], ref), (b, tau[b], ref)
    with pytest.raises(ValueError):
        qp.hw_torque_ff(d(J), d(g), d(base), d(cnt.astype(np.int64)))


def test_body_mpc_matches_restatement_over_a_gait():
    dev = _dev()
    rng = np.random.default_rng(11)
    B = 16
    solver = qp.BodyMPC(batch=B, device=dev)
    ostates = []
    for b in range(B):
        s = O.BodyState()
        O.lib().qo_body_init(C.byref(s))
        ostates.append(s)
    for i in list(range(96, 180)) + list(range(1905, 1925)):
        zmp = rng.normal(0, 0.02, (B, 2, 5))
        ang = rng.normal(0, 0.02, (B, 2, 5))
        rf = rng.normal(0, 0.05, (B, 2, 5))
        lf = rng.normal(0, 0.05, (B, 2, 5))
        acc = rng.normal(0, 0.5, (B, 3, 5))
        bs = rng.normal(0, 0.05, (B, 4))
        cm = lambda a: np.ascontiguousarray(a.transpose(0, 2, 1).reshape(a.shape[0], -1))
        ins = dict(i=np.full(B, i, np.int32), bodyangle_state=bs, zmp_ref=cm(zmp),
                   angle_ref=cm(ang), rfoot_ref=cm(rf), lfoot_ref=cm(lf), comacc_ref=cm(acc))
        out = solver.step(**{k: torch.from_numpy(v).to(dev) for k, v in ins.items()})
        torch.cuda.synchronize()
        traj = out["com_traj"].cpu().numpy()
        state = solver.state.cpu().numpy()
        for b in range(B):
            ct = np.zeros(14)
            est = C.c_int(0)
            O.lib().qo_body_theta_mpc(C.byref(ostates[b]), i, O.P(np.ascontiguousarray(bs[b])),
                                      O.P(ins["zmp_ref"][b].copy()), O.P(ins["angle_ref"][b].copy()),
                                      O.P(ins["rfoot_ref"][b].copy()), O.P(ins["lfoot_ref"][b].copy()),
                                      O.P(ins["comacc_ref"][b].copy()), O.P(np.zeros(9)), O.P(ct),
                                      C.byref(est))
            assert np.allclose(traj[b], ct, rtol=1e-9, atol=1e-12), (i, b, traj[b], ct)
            if i >= 100:
                o = ostates[b]
                assert (int(state[b, 26]), int(state[b, 27]), int(state[b, 28])) == \
                    (o.bjx1, o.bjx2, o.t_yu), (i, b)
    for s in ostates:
        O.lib().qo_body_free(C.byref(s))


def test_indexfind_bit_exact():
    dev = _dev()
    s = O.BodyState()
    O.lib().qo_body_init(C.byref(s))
    tx = np.array(s.tx[:])
    t = np.concatenate([np.linspace(0, tx[-1] - 1e-9, 2001), tx[:-1], np.nextafter(tx[:-1], -1),
                        np.arange(0, 1880) * 0.01])
    j = qp.indexfind(torch.from_numpy(t).to(dev)).cpu().numpy()
    ref = np.array([O.lib().qo_body_indexfind(C.byref(s), float(v)) for v in t])
    assert np.array_equal(j, ref)
    O.lib().qo_body_free(C.byref(s))
