"""GPU parity tests for the fused SRBD convex-MPC kernel (qloco_srbd_solve).

Checker: the oracle (oracle/, CPU restatement of ConvexMpc + OSQP ADMM +
EiQuadProg, double).  Stated fp32 tolerances:
  * vs the OSQP-algorithm ADMM restatement on the same (stance-reduced) QP:
      ADMM iteration count within one check interval (25) and equal for
      >= 90 % of instances, objective within 1e-3 * max(1, |f|),
      |u0_gpu - u0_ref|_inf <= 0.5 N for >= 90 % of instances and <= 5 N
      for all (an ADMM iterate is only defined up to the termination
      tolerance: in the QP's near-flat directions -- internal forces between
      stance feet, curvature = R = 2e-7 -- fp32 and fp64 runs of the same
      algorithm land at different eps-optimal points);
  * the quantities the cost sees (per-step net wrench, predicted state
    trajectory in the Q-norm) vs that restatement, vs the exact optimum at
    eps 1e-6 and vs the literal full 12N-variable OSQP restatement, with the
    bounds stated in each test (the fp64 envelopes they come from are in
    DESIGN.md §6);
  * vs the exact optimum of the reference's literal 12N-variable QP
    (EiQuadProg restatement): objective gap within 1e-3 of the fp64
    restatement's own gap and violation <= 0.25 N;
  * integer structure (stance enumeration -> variable count) bit-exact,
    checked through the exactly-zero swing forces.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import oracle_lib as O  # noqa: E402
from srbd_ref import Instance, np_build  # noqa: E402

from quadrupedal_loco_amd import _lib, srbd  # noqa: E402
import ctypes as C  # noqa: E402

SEED = 20261015


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _traj_metrics(u, ref, x0, xr, ft, ct, N):
    """Differences between two solutions that the QP's cost actually sees:
    the per-step net contact wrench (sum f, sum r x f -- the SRBD dynamics
    depend on the forces only through it, ConvexMpc.cpp:135-147) and the
    predicted state trajectory X = Aqp x0 + Bqp u in the Q-norm
    sqrt(sum q_i dX_i^2) (ConvexMpc.cpp:162-221).  Returns (|du0|_inf,
    max step |dF|, max step |dM|, |dX|_Q)."""
    u = np.asarray(u, np.float64)
    ref = np.asarray(ref, np.float64)
    du = (u - ref).reshape(N, 4, 3)
    r = np.asarray(ft, np.float64).reshape(4, 3)
    dF = np.abs(du.sum(1)).max()
    dM = np.abs(np.cross(np.broadcast_to(r, (N, 4, 3)), du).sum(1)).max()
    Bqp = np_build(x0, xr, ft, ct, N)[6]
    d = Bqp @ (u - ref)
    q = np.tile(2.0 * np.asarray(O.Q_W), N)
    return np.abs(u[:12] - ref[:12]).max(), dF, dM, float(np.sqrt((q * d * d).sum()))


# u0 -- the forces compute_grf returns (A1RobotControl.cpp:593-599) -- of the
# literal QP against the fp64 restatement of the same OSQP call (DESIGN.md
# §6): where both runs stop at the same termination check (equal iteration
# counts) |du0|_inf <= 0.5 N for >= 99 % of instances and <= 2 N for every
# one (measured max 0.20 N, p99 0.05-0.17 N over 2,765 such instances at
# N = 10 / 16 / 20, profiles/r5c_literal_parity_scan.txt); where fp32 passes
# a check one interval earlier or later the runs stop at two eps-optimal
# points and |du0|_inf <= 30 N (measured max 22.8 N over 19 such instances;
# round 6: 40 -> 30 N, ADVICE r5 -- at the GPU's own iteration count the
# restatement is no closer, profiles/r6v_u0_at_gpu_stop_probe.txt, so the
# certificate for these points is OSQP's termination test,
# test_srbd_literal_iterate_passes_osqp_termination).
U0_SAME_NEAR, U0_SAME_ALL, U0_APART = 0.5, 2.0, 30.0


class U0Bound:
    """Accumulates the literal-mode u0 bound over a test's instances."""

    def __init__(self):
        self.same = self.far = 0

    def add(self, du0, same_check, where=None):
        if same_check:
            self.same += 1
            self.far += int(du0 > U0_SAME_NEAR)
            assert du0 <= U0_SAME_ALL, ("u0, same check", where, du0)
        else:
            assert du0 <= U0_APART, ("u0, one check apart", where, du0)

    def check(self):
        # >= 99 % within 0.5 N, or one instance at most in a small batch (N = 20
        # mixed schedules: one of 30 same-check instances at 0.5 .. 2 N)
        assert self.far <= max(1, int(0.01 * self.same)), ("u0 > 0.5 N at the same check", self.far, self.same)


def _solve(N, B, gait, first=0, **spec):
    dev = _dev()
    x0, xr, ft, ct = srbd.generate(SEED, N, B, gait, first=first)
    solver = srbd.BatchedConvexMpc(horizon=N, **spec)
    out = solver.solve(*(torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)), full=True)
    torch.cuda.synchronize()
    res = {k: getattr(out, k).cpu().numpy() for k in ("u0", "u", "status", "iters", "obj")}
    return (x0, xr, ft, ct), res


@pytest.mark.parametrize("N,B,gait", [(10, 48, "trot"), (10, 24, "pace"), (10, 32, "mixed"),
                                      (16, 12, "trot"), (20, 16, "pace"), (4, 16, "stance")])
def test_srbd_matches_admm_restatement(N, B, gait):
    (x0, xr, ft, ct), r = _solve(N, B, gait)
    sp = O.srbd_spec(N=N)
    iters_equal = 0
    u0_close = 0
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xref, info = inst.admm_reduced()
        assert r["status"][b] == 0, (b, r["status"][b])
        assert abs(int(r["iters"][b]) - info.iters) <= 25, (b, r["iters"][b], info.iters)
        iters_equal += int(r["iters"][b]) == info.iters
        u = r["u"][b].astype(np.float64)
        du = np.abs(u[:12] - xref[:12]).max()
        assert du <= 5.0, (b, u[:12], xref[:12])
        u0_close += int(du <= 0.5)
        fr = inst.obj(xref)
        assert abs(inst.obj(u) - fr) <= 1e-3 * max(1.0, abs(fr)), (b, inst.obj(u), fr)
        # swing forces exactly zero (integer schedule reproduced bit-exactly)
        swing = np.repeat(ct[b] == 0, 3)
        assert np.all(u[swing] == 0.0)
        # u0 is the first 12 entries of u
        assert np.array_equal(r["u0"][b], r["u"][b][:12])
    assert iters_equal >= 0.9 * B
    assert u0_close >= 0.9 * B


@pytest.mark.parametrize("N,B,gait", [(10, 24, "trot"), (10, 16, "mixed")])
def test_srbd_vs_exact_optimum(N, B, gait):
    """Objective gap to the exact optimum f* of the literal 12N-variable QP:
    within 1e-3 of the gap the fp64 OSQP-algorithm restatement itself lands
    at (OSQP's default eps stops anywhere in an eps-ball; measured fp64 gaps
    on configs 2-5 shapes span [-2.1e-3, 0.137] of max(1, |f*|), measured
    GPU - fp64 differences <= 3.6e-4), inside that envelope with margin, and
    constraint violation <= 0.25 N.  (The former eps-1e-6 check is
    test_srbd_tight_eps_wrench_vs_exact.)"""
    (x0, xr, ft, ct), r = _solve(N, B, gait)
    sp = O.srbd_spec(N=N)
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xe, st, _ = inst.exact()
        assert st == 0
        fe = inst.obj(xe)
        sc = max(1.0, abs(fe))
        u = r["u"][b].astype(np.float64)
        gap = (inst.obj(u) - fe) / sc
        gap64 = (inst.obj(inst.admm_reduced()[0]) - fe) / sc
        assert abs(gap - gap64) <= 1e-3, (b, gap, gap64)
        assert -2.5e-3 <= gap <= 0.15, (b, gap)
        assert inst.violation(u) <= 0.25, (b, inst.violation(u))
        assert abs(r["obj"][b] - inst.obj(u)) <= 1e-3 * max(1.0, abs(inst.obj(u)))


def test_srbd_body_frame_output_and_determinism():
    N, B = 10, 32
    dev = _dev()
    x0, xr, ft, ct = srbd.generate(SEED, N, B, "trot")
    args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
    w = srbd.BatchedConvexMpc(horizon=N).solve(*args)
    w2 = srbd.BatchedConvexMpc(horizon=N).solve(*args)
    body = srbd.BatchedConvexMpc(horizon=N, output_frame=1).solve(*args)
    torch.cuda.synchronize()
    u0w = w.u0.cpu().numpy().astype(np.float64)
    assert np.array_equal(u0w, w2.u0.cpu().numpy())  # bit-identical reruns
    u0b = body.u0.cpu().numpy().astype(np.float64)
    for b in range(B):  # compute_grf: F_i = R' u_i, R = [[c,s,0],[-s,c,0],[0,0,1]]
        c, s = np.cos(x0[b, 2]), np.sin(x0[b, 2])
        R = np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]])
        ref = (R.T @ u0w[b].reshape(4, 3).T).T.ravel()
        assert np.abs(ref - u0b[b]).max() <= 1e-3 * max(1.0, np.abs(ref).max())


def test_srbd_edge_cases():
    dev = _dev()
    N, B = 10, 4
    x0, xr, ft, ct = srbd.generate(SEED, N, B, "trot")
    ct[0, :] = 0          # all legs in swing: no variables, u = 0
    ct[1, :] = 1          # all stance: 120 variables (two-wave kernel)
    ct[2, 4:] = 0         # stance only at step 0
    solver = srbd.BatchedConvexMpc(horizon=N)
    out = solver.solve(*(torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)), full=True)
    torch.cuda.synchronize()
    u = out.u.cpu().numpy()
    st = out.status.cpu().numpy()
    assert np.all(u[0] == 0.0) and st[0] == 0
    sp = O.srbd_spec(N=N)
    for b in (1, 2, 3):
        assert st[b] == 0
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xref, info = inst.admm_reduced()
        assert np.abs(u[b, :12] - xref[:12]).max() <= 5.0
        assert abs(inst.obj(u[b].astype(np.float64)) - inst.obj(xref)) <= \
            1e-3 * max(1.0, abs(inst.obj(xref)))
    # empty batch is a no-op
    e = [torch.empty((0, k), dtype=t, device=dev) for k, t in
         ((13, torch.float32), (13 * N, torch.float32), (12, torch.float32), (4 * N, torch.uint8))]
    solver.solve(*e, max_legs=0)


def test_srbd_warm_start_resumes_at_solution():
    dev = _dev()
    N, B = 10, 16
    x0, xr, ft, ct = srbd.generate(SEED, N, B, "trot")
    args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
    warm = torch.zeros((B, 32 * N), dtype=torch.float32, device=dev)
    s = srbd.BatchedConvexMpc(horizon=N, warm_start=1)
    first = s.solve(*args, warm=warm)
    torch.cuda.synchronize()
    first.obj = first.obj.clone()
    second = s.solve(*args, warm=warm)
    torch.cuda.synchronize()
    it2 = second.iters.cpu().numpy()
    assert np.all(it2 <= 50), it2
    o1, o2 = first.obj.cpu().numpy(), second.obj.cpu().numpy()
    # both solves sit in the eps-optimal band around the exact optimum f*, and
    # resuming from the warm state does not make the objective worse
    sp = O.srbd_spec(N=N)
    for b in range(B):
        fs = Instance(sp, x0[b], xr[b], ft[b], ct[b]).exact_obj()
        sc = max(1.0, abs(fs))
        for o in (o1[b], o2[b]):
            assert -1e-3 * sc <= o - fs <= 0.1 * sc, (b, o, fs)
        assert o2[b] - fs <= max(o1[b] - fs, 0.0) + 1e-3 * sc, (b, o1[b], o2[b], fs)


def test_srbd_full_size_properties():
    """BASELINE configs[1] full size (4096, N=10 trot): every instance solves,
    all forces finite and within the friction pyramid to ADMM tolerance,
    spot-check against the oracle."""
    N, B = 10, 4096
    (x0, xr, ft, ct), r = _solve(N, B, "trot")
    assert np.all(r["status"] == 0)
    assert np.all(np.isfinite(r["u"]))
    u = r["u"].reshape(B, N, 4, 3)
    mu = 0.3
    tol = 0.25
    assert np.all(u[..., 2] >= -tol) and np.all(u[..., 2] <= 180 + tol)
    assert np.all(np.abs(u[..., 0]) <= mu * u[..., 2] + tol)
    assert np.all(np.abs(u[..., 1]) <= mu * u[..., 2] + tol)
    sp = O.srbd_spec(N=N)
    for b in (0, 1, 1234, 4095):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xref, info = inst.admm_reduced()
        assert np.abs(r["u"][b, :12] - xref[:12]).max() <= 5.0
        fr = inst.obj(xref)
        assert abs(inst.obj(r["u"][b].astype(np.float64)) - fr) <= 1e-3 * max(1.0, abs(fr))


@pytest.mark.parametrize("N,gait,fps", [(10, "trot", False), (20, "pace", False), (10, "mixed", True)])
def test_srbd_dense_build_matches_restatement(N, gait, fps):
    """qloco_srbd_build (literal A_qp, B_qp, H, g, lb, ub) vs the oracle's
    dense build and the independent numpy restatement; fp32 vs fp64."""
    dev = _dev()
    B = 6
    x0, xr, ft, ct = srbd.generate(SEED, N, B, gait)
    if fps:
        rng = np.random.default_rng(9)
        ft = (np.tile(ft, (1, N)) + rng.uniform(-0.02, 0.02, (B, 12 * N))).astype(np.float32)
    solver = srbd.BatchedConvexMpc(horizon=N)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = solver.build(d(x0), d(xr), d(ft), d(ct), want=("H", "g", "lb", "ub", "Aqp", "Bqp"))
    torch.cuda.synchronize()
    r = {k: v.cpu().numpy().astype(np.float64) for k, v in out.items()}
    sp = O.srbd_spec(N=N)
    for b in range(B):
        H, g, lb, ub = O.build_instance(sp, x0[b], xr[b], ft[b], ct[b], feet_per_step=int(fps))
        Hn, gn, lbn, ubn, _, Aqp, Bqp = np_build(x0[b], xr[b], ft[b], ct[b], N, feet_per_step=fps)
        Hg = r["H"][b].T  # stored col-major
        assert np.allclose(Hg, H, rtol=2e-5, atol=2e-6 * np.abs(H).max()), b
        assert np.allclose(r["g"][b], g, rtol=2e-4, atol=2e-5 * np.abs(g).max()), b
        assert np.array_equal(r["lb"][b].astype(np.float32), lb.astype(np.float32))
        assert np.array_equal(r["ub"][b].astype(np.float32), ub.astype(np.float32))
        assert np.allclose(r["Aqp"][b].T, Aqp, rtol=1e-5, atol=1e-7)
        assert np.allclose(r["Bqp"][b].T, Bqp, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("N,B,gait", [(16, 65536, "trot"), (20, 32768, "pace"), (10, 65536, "mixed")])
def test_srbd_two_wave_large_batches(N, B, gait):
    """BASELINE configs 3-5 shapes (two-wavefront workgroups; the mixed batch
    also exercises the one/two-wave split): at full occupancy every instance
    converges with finite forces inside the friction pyramid -- a regression
    guard for the inverse's LDS buffer hand-over between the two waves, a
    race that only showed under load (NaN in ~1e-4 of 65536 instances) --
    and the run is deterministic."""
    (x0, xr, ft, ct), r = _solve(N, B, gait)
    assert np.all(r["status"] == 0), np.unique(r["status"], return_counts=True)
    assert np.all(r["iters"] < 4000)
    u = r["u"].reshape(B, N, 4, 3)
    assert np.all(np.isfinite(u))
    tol = 0.25
    assert np.all(u[..., 2] >= -tol) and np.all(u[..., 2] <= 180 + tol)
    assert np.all(np.abs(u[..., 0]) <= 0.3 * u[..., 2] + tol)
    _, r2 = _solve(N, B, gait)
    assert np.array_equal(r["u"], r2["u"])


# --- trajectory / wrench parity.  Individual leg forces are
# only defined up to the termination tolerance along the internal-force
# directions (curvature R = 2e-7); the cost sees the forces through the
# per-step net wrench and the predicted state trajectory, so those are the
# quantities pinned here.  Measured envelopes (tools/srbd_parity_scan.py,
# gpurun_out/r2b/scan.txt) set the bounds, each with ~2x margin.

# Per-step net wrench envelopes of the reduced mode against the fp64
# restatement (round 6, tools/srbd_parity_scan.py over 1,056 instances:
# N = 10 trot 512 / mixed 256, N = 16 trot 128, N = 20 pace 96 / mixed 64;
# profiles/r6u_reduced_parity_envelope.txt): where both runs stop at the same
# check max |dF| 18.2 N, |dM| 1.52 N m, |dX|_Q 0.029; one check apart 60.0 N,
# 7.3 N m, 0.17.  The bounds are about twice that, so a compiler-level change
# of the residual rounding (17.3 N on an unshipped build) cannot
# turn the suite red by itself; OSQP's own termination test on every iterate
# (test_srbd_reduced_iterate_passes_osqp_termination) is the certificate.
RED_SAME_DF, RED_SAME_DM, RED_APART_DF, RED_APART_DM, RED_DX = 40.0, 3.0, 120.0, 15.0, 0.3


@pytest.mark.parametrize("N,B,gait", [(10, 64, "trot"), (16, 24, "trot"), (20, 16, "pace"),
                                      (10, 48, "mixed")])
def test_srbd_trajectory_parity_vs_restatement(N, B, gait):
    """BASELINE configs 2-5 shapes at OSQP's default eps: GPU fp32 vs the
    oracle's fp64 OSQP-algorithm ADMM on the same stance-only QP.  Per
    instance: predicted-trajectory difference |dX|_Q <= 0.1 where both stop
    at the same check, <= 0.3 otherwise; per-step net force <= 1 N and
    moment <= 0.1 N m for >= 90 % of instances (measured 0.94-0.99 over
    1,056 instances), within the RED_* envelopes above for all; objective
    gap to the exact optimum within 1e-3 of the fp64 restatement's own gap
    (measured |diff| <= 3.6e-4)."""
    (x0, xr, ft, ct), r = _solve(N, B, gait)
    sp = O.srbd_spec(N=N)
    near = 0
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xa, info = inst.admm_reduced()
        fe = inst.exact_obj()
        sc = max(1.0, abs(fe))
        assert r["status"][b] == 0
        du0, dF, dM, dX = _traj_metrics(r["u"][b], xa, x0[b], xr[b], ft[b], ct[b], N)
        same = int(r["iters"][b]) == info.iters
        assert dX <= (0.1 if same else RED_DX), (b, dX)
        assert dF <= (RED_SAME_DF if same else RED_APART_DF), (b, same, dF)
        assert dM <= (RED_SAME_DM if same else RED_APART_DM), (b, same, dM)
        near += int(dF <= 1.0 and dM <= 0.1)
        g_gpu = (inst.obj(r["u"][b]) - fe) / sc
        g_64 = (inst.obj(xa) - fe) / sc
        assert abs(g_gpu - g_64) <= 1e-3, (b, g_gpu, g_64)
    assert near >= 0.9 * B, near


@pytest.mark.parametrize("N,B,gait", [(10, 32, "trot"), (10, 24, "mixed"), (20, 12, "pace"),
                                      (20, 8, "mixed"), (16, 4, "stance")])
def test_srbd_tight_eps_wrench_vs_exact(N, B, gait):
    """eps_abs = eps_rel = 1e-6: the GPU iterate against the exact optimum of
    the literal 12N-variable QP (EiQuadProg restatement).  The bound is the
    envelope the reference algorithm itself reaches in double at that eps
    (fp64 OSQP-algorithm ADMM, same instances: per-step net force 1.67 N,
    moment 0.25 N m, |dX|_Q 0.0018, measured) with margin: per-step
    |dF| <= 2.5 N, |dM| <= 0.5 N m, |dX|_Q <= 0.005, objective gap <= 2e-5
    relative.  fp32 cannot always certify eps 1e-6 (a few mixed / N = 20
    instances end SOLVED_INACCURATE or MAX_ITER at 20000 iterations); their
    iterates are held to the same bounds."""
    (x0, xr, ft, ct), r = _solve(N, B, gait, eps_abs=1e-6, eps_rel=1e-6, max_iter=20000)
    sp = O.srbd_spec(N=N)
    assert np.all(np.isin(r["status"], [0, 1, 8])), r["status"]
    assert np.mean(r["status"] == 0) >= 0.5
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xe, st, _ = inst.exact()
        assert st == 0
        fe = inst.obj(xe)
        _, dF, dM, dX = _traj_metrics(r["u"][b], xe, x0[b], xr[b], ft[b], ct[b], N)
        assert dF <= 2.5 and dM <= 0.5 and dX <= 0.005, (b, dF, dM, dX)
        assert abs(inst.obj(r["u"][b]) - fe) <= 2e-5 * max(1.0, abs(fe)), b


@pytest.mark.parametrize("N,B,gait", [(10, 32, "trot"), (10, 24, "mixed")])
def test_srbd_vs_literal_full_qp_restatement(N, B, gait):
    """Against the reference's literal call: OSQP on the full 12N-variable
    QP (swing forces kept as variables with fz in [0, 0], the oracle's fp64
    restatement).  Eliminating the swing variables leaves the optimum
    unchanged but changes Ruiz's scaling and so the ADMM trajectory; the
    same elimination in fp64 (reduced vs full restatement, measured on these
    shapes) moves u0 by up to 15 N, the Q-norm trajectory by up to 0.17,
    the iteration count by up to 75 and the objective by up to 2.2 % of
    |f*|.  Bounds: iterations within 100, |dX|_Q <= 0.3, |du0| <= 25 N,
    objective within 0.03 |f*| of the full restatement's, and equal
    iteration counts for >= 60 % of instances."""
    (x0, xr, ft, ct), r = _solve(N, B, gait)
    sp = O.srbd_spec(N=N)
    same = 0
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xf, info = inst.admm_full()
        assert abs(int(r["iters"][b]) - info.iters) <= 100, (b, r["iters"][b], info.iters)
        same += int(r["iters"][b]) == info.iters
        du0, dF, dM, dX = _traj_metrics(r["u"][b], xf, x0[b], xr[b], ft[b], ct[b], N)
        assert dX <= 0.3 and du0 <= 25.0, (b, dX, du0)
        sc = max(1.0, abs(inst.exact_obj()))
        assert abs(inst.obj(r["u"][b]) - inst.obj(xf)) <= 0.03 * sc, b
    assert same >= 0.6 * B, same


def test_srbd_two_wave_c6_bucket_regression():
    """Round-3 divergence regression: the
    26-29-leg instances of mixed N = 10 schedules run in the C2 = 6 two-wave
    bucket.  48 such instances against the fp64 restatement (status,
    iterations within one check and equal for >= 90 %, u0 / objective bounds
    of test_srbd_matches_admm_restatement), then the same 48 replicated to
    6,144 instances in one launch -- every SIMD holding several of them, so
    the two waves' LDS hand-offs run under full load -- must give each
    replica bit-identical results."""
    dev = _dev()
    N = 10
    x0, xr, ft, ct = srbd.generate(SEED, N, 4096, "mixed")
    legs = ct.reshape(len(ct), -1).astype(bool).sum(axis=1)
    pick = np.nonzero((legs >= 26) & (legs <= 29))[0][:48]
    assert len(pick) == 48 and set(np.unique(legs[pick])) >= {26, 28}
    a = [np.ascontiguousarray(v[pick]) for v in (x0, xr, ft, ct)]
    solver = srbd.BatchedConvexMpc(horizon=N)
    out = solver.solve(*(torch.from_numpy(v).to(dev) for v in a), full=True)
    torch.cuda.synchronize()
    u = out.u.cpu().numpy().astype(np.float64)
    st, it = out.status.cpu().numpy(), out.iters.cpu().numpy()
    sp = O.srbd_spec(N=N)
    same = 0
    for b in range(len(pick)):
        inst = Instance(sp, a[0][b], a[1][b], a[2][b], a[3][b])
        xref, info = inst.admm_reduced()
        assert st[b] == 0 and info.status == 0, (b, st[b], info.status)
        assert abs(int(it[b]) - info.iters) <= 25, (b, it[b], info.iters)
        same += int(it[b]) == info.iters
        assert np.abs(u[b, :12] - xref[:12]).max() <= 5.0, b
        fr = inst.obj(xref)
        assert abs(inst.obj(u[b]) - fr) <= 1e-3 * max(1.0, abs(fr)), b
    assert same >= 0.9 * len(pick), same
    R = 128
    big = [torch.from_numpy(np.ascontiguousarray(np.tile(v, (R, 1)))).to(dev) for v in a]
    ob = solver.solve(*big, full=True)
    torch.cuda.synchronize()
    ub = ob.u.cpu().numpy().reshape(R, len(pick), -1)
    ib = ob.iters.cpu().numpy().reshape(R, len(pick))
    assert np.array_equal(ib, np.tile(it, (R, 1)))
    assert np.array_equal(ub, np.tile(out.u.cpu().numpy(), (R, 1, 1)))


def test_srbd_config4_share_sampled_against_oracle():
    """BASELINE configs[3] per-GPU share at full size: Go1 pace N = 20,
    65,536 instances in one launch.  Whole batch: every instance converges,
    forces finite and inside the friction pyramid; 16 instances spread over
    the batch (both ends, both pace phases) against the fp64 restatement
    with the trajectory-parity bounds above."""
    N, B = 20, 65536
    (x0, xr, ft, ct), r = _solve(N, B, "pace")
    assert np.all(r["status"] == 0), np.unique(r["status"], return_counts=True)
    u = r["u"].reshape(B, N, 4, 3)
    assert np.all(np.isfinite(u))
    tol = 0.25
    assert np.all(u[..., 2] >= -tol) and np.all(u[..., 2] <= 180 + tol)
    assert np.all(np.abs(u[..., 0]) <= 0.3 * u[..., 2] + tol)
    assert np.all(np.abs(u[..., 1]) <= 0.3 * u[..., 2] + tol)
    sp = O.srbd_spec(N=N)
    for b in np.linspace(0, B - 1, 16).astype(int):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xa, info = inst.admm_reduced()
        assert abs(int(r["iters"][b]) - info.iters) <= 25, (b, r["iters"][b], info.iters)
        du0, dF, dM, dX = _traj_metrics(r["u"][b], xa, x0[b], xr[b], ft[b], ct[b], N)
        same = int(r["iters"][b]) == info.iters
        assert dX <= (0.1 if same else RED_DX) and du0 <= (5.0 if same else 40.0), (b, du0, dX)
        assert dF <= (RED_SAME_DF if same else RED_APART_DF) and dM <= (RED_SAME_DM if same else RED_APART_DM), \
            (b, du0, dF, dM, dX)


def test_srbd_config5_share_sampled_against_oracle():
    """BASELINE configs[4] per-GPU share at full size: mixed trot + bipedal
    per-instance schedules, N = 10, 131,072 instances in one call (through
    the device classification and the class lists).  Whole batch: every instance converges, forces finite and inside
    the friction pyramid; 16 instances spread over the batch against the
    fp64 restatement with the trajectory-parity bounds above."""
    N, B = 10, 131072
    (x0, xr, ft, ct), r = _solve(N, B, "mixed")
    assert np.all(r["status"] == 0), np.unique(r["status"], return_counts=True)
    u = r["u"].reshape(B, N, 4, 3)
    assert np.all(np.isfinite(u))
    tol = 0.25
    assert np.all(u[..., 2] >= -tol) and np.all(u[..., 2] <= 180 + tol)
    assert np.all(np.abs(u[..., 0]) <= 0.3 * u[..., 2] + tol)
    assert np.all(np.abs(u[..., 1]) <= 0.3 * u[..., 2] + tol)
    legs = ct.reshape(B, -1).astype(bool).sum(axis=1)
    assert legs.max() > 21  # the two-wave class, through the device class lists
    sp = O.srbd_spec(N=N)
    for b in np.linspace(0, B - 1, 16).astype(int):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xa, info = inst.admm_reduced()
        assert abs(int(r["iters"][b]) - info.iters) <= 25, (b, r["iters"][b], info.iters)
        du0, dF, dM, dX = _traj_metrics(r["u"][b], xa, x0[b], xr[b], ft[b], ct[b], N)
        same = int(r["iters"][b]) == info.iters
        assert dX <= (0.1 if same else RED_DX) and du0 <= (5.0 if same else 40.0), (b, du0, dX)
        assert dF <= (RED_SAME_DF if same else RED_APART_DF) and dM <= (RED_SAME_DM if same else RED_APART_DM), \
            (b, du0, dF, dM, dX)


def test_srbd_persistent_closed_loop_matches_restatement():
    """The reference's member OSQP solver over a control loop
    (A1RobotControl.cpp:556-578: update* + solve with warm start on): 32
    controllers x 24 MPC ticks, the inputs drifting between ticks and half the
    controllers switching trot phase at tick 12 (re-initialisation path).
    Per tick, GPU (spec.warm_start = 2, record on the device) vs the oracle's
    restatement (oracle/persist.c): status, iteration counts within one check
    interval and equal for >= 85 % of (tick, controller) pairs, the adapted
    rho carried in the record within 10 % for >= 95 % (an adaptation step
    changes rho by >= 5x, rho_tol; the fp32 residual ratios it is computed
    from differ from fp64 at the 1e-3 level, compounding over ticks), and the
    trajectory-parity bounds of test_srbd_trajectory_parity_vs_restatement
    on every solution.  The resumed solves need fewer iterations than the
    cold first tick."""
    from cases import closed_loop_srbd
    dev = _dev()
    N, B, T = 10, 32, 24
    seq = closed_loop_srbd(N, B, T, switch_at=12)
    gpu = srbd.PersistentConvexMpc(B, dev, horizon=N)
    orc = [O.PersistentMpc(N) for _ in range(B)]
    same = rho_ok = total = 0
    it_first, it_later = [], []
    for t, (x0, xr, ft, ct) in enumerate(seq):
        out = gpu.solve(*(torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)), full=True)
        torch.cuda.synchronize()
        u = out.u.cpu().numpy()
        st = out.status.cpu().numpy()
        its = out.iters.cpu().numpy()
        rec = gpu.record.cpu().numpy()
        for b in range(B):
            ub, info = orc[b].step(x0[b], xr[b], ft[b], ct[b])
            assert st[b] == info.status == 0, (t, b, st[b], info.status)
            assert abs(int(its[b]) - info.iters) <= 25, (t, b, its[b], info.iters)
            same += int(its[b]) == info.iters
            r64 = orc[b].rec[100 * N]
            rho_ok += int(abs(rec[b, 100 * N] - r64) <= 0.1 * r64)
            total += 1
            _, dF, dM, dX = _traj_metrics(u[b], ub, x0[b], xr[b], ft[b], ct[b], N)
            eq = int(its[b]) == info.iters  # the reduced-mode envelopes (RED_*)
            assert dX <= (0.1 if eq else RED_DX), (t, b, dX)
            assert dF <= (RED_SAME_DF if eq else RED_APART_DF) and dM <= (RED_SAME_DM if eq else RED_APART_DM), \
                (t, b, dF, dM, dX)
            (it_first if t == 0 else it_later).append(int(its[b]))
    assert same >= 0.85 * total, (same, total)
    assert rho_ok >= 0.95 * total, (rho_ok, total)
    assert np.mean(it_later) < np.mean(it_first)


# --- the wide kernel (43..80 stance legs, 129..240 variables; srbd_admm_big_kernel)

@pytest.mark.parametrize("N,B,gait", [(12, 6, "stance"), (16, 6, "stance"), (20, 4, "stance"),
                                      (20, 12, "mixed")])
def test_srbd_wide_instances_match_restatement(N, B, gait):
    """Instances above 42 stance legs -- every N >= 11 stand-balance, N = 20
    mixed schedules with double-support windows -- solve through the wide
    kernel: status OK, iterations within one check interval of the fp64
    OSQP-algorithm restatement on the same stance-only QP within two check
    intervals (240 fp32 residual terms: measured one instance in 12 at two) and
    equal for >= 75 %,
    objective gap to the exact optimum within 1e-3 of the restatement's own.
    Where both stop at the same check, the trajectory-parity bounds of
    test_srbd_trajectory_parity_vs_restatement hold (|dX|_Q <= 0.1, per-step
    net force <= 15 N / moment <= 3 N m).  Where fp32 residuals pass one check
    earlier or later, the two runs stop at different eps-optimal points
    (measured on N = 20 mixed: |dX|_Q 0.17, step force 40 N, with the GPU's
    objective gap 7.7e-4 vs 1.4e-3 in fp64; at eps 1e-6 the same instances
    agree to |dX|_Q 1e-3, test_srbd_tight_eps_wrench_vs_exact): |dX|_Q <= 0.3."""
    (x0, xr, ft, ct), r = _solve(N, B, gait)
    assert (ct.reshape(B, -1).sum(1) > 42).all()
    sp = O.srbd_spec(N=N)
    same = 0
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xa, info = inst.admm_reduced()
        assert r["status"][b] == 0, (b, r["status"][b])
        assert abs(int(r["iters"][b]) - info.iters) <= 50, (b, r["iters"][b], info.iters)
        u = r["u"][b].astype(np.float64)
        assert np.all(u[np.repeat(ct[b] == 0, 3)] == 0.0)
        assert np.array_equal(r["u0"][b], r["u"][b][:12])
        du0, dF, dM, dX = _traj_metrics(u, xa, x0[b], xr[b], ft[b], ct[b], N)
        if int(r["iters"][b]) == info.iters:
            same += 1
            assert dX <= 0.1 and dF <= 15.0 and dM <= 3.0, (b, du0, dF, dM, dX)
        assert dX <= 0.3, (b, du0, dF, dM, dX)
        fe = inst.exact_obj()
        sc = max(1.0, abs(fe))
        assert abs((inst.obj(u) - fe) / sc - (inst.obj(xa) - fe) / sc) <= 1e-3, b
        assert abs(r["obj"][b] - inst.obj(u)) <= 1e-3 * max(1.0, abs(inst.obj(u)))
    assert same >= 0.75 * B, same


def test_srbd_three_kernel_classes_in_one_batch():
    """One N = 20 batch holding all three kernel families (<= 20 legs:
    one-wave, 21..41: the two-wave column buckets, >= 42: wide) -- one launch
    per populated class,
    each instance solved exactly once and matching the restatement; then the
    same batch with a too-small caller max_stance_legs: the instances above it
    report QLOCO_BAD_SIZE with NaN outputs instead of stale memory."""
    dev = _dev()
    N = 20
    parts = [srbd.generate(SEED, N, 4, g) for g in ("trot", "mixed", "stance")]
    x0, xr, ft, ct = (np.concatenate([p[k] for p in parts]) for k in range(4))
    ct[0:2, 4 * 5:] = 0  # 2 legs x 5 steps = 10 legs: one-wave class
    legs = ct.reshape(len(ct), -1).sum(1)
    assert legs.min() <= 20 and ((legs > 20) & (legs <= 41)).any() and legs.max() > 41
    solver = srbd.BatchedConvexMpc(horizon=N)
    args = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x0, xr, ft, ct)]
    out = solver.solve(*args, full=True)
    torch.cuda.synchronize()
    u = out.u.cpu().numpy()
    st = out.status.cpu().numpy()
    it = out.iters.cpu().numpy()
    sp = O.srbd_spec(N=N)
    for b in range(len(ct)):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xa, info = inst.admm_reduced()
        assert st[b] == 0 and abs(int(it[b]) - info.iters) <= (50 if legs[b] > 41 else 25), \
            (b, legs[b], st[b], it[b], info.iters)
        _, dF, dM, dX = _traj_metrics(u[b], xa, x0[b], xr[b], ft[b], ct[b], N)
        if int(it[b]) == info.iters:  # else: another eps-optimal point (wide test)
            assert dX <= 0.1 and dF <= 15.0 and dM <= 3.0, (b, legs[b], dF, dM, dX)
        assert dX <= 0.3, (b, legs[b], dF, dM, dX)
    small = solver.solve(*args, full=True, max_legs=41)  # the two-wave capacity
    torch.cuda.synchronize()
    st2 = small.status.cpu().numpy()
    big = legs > 41
    assert np.all(st2[big] == 4) and np.all(st2[~big] == 0)  # QLOCO_BAD_SIZE
    assert np.all(np.isnan(small.u.cpu().numpy()[big])) and np.all(np.isnan(small.u0.cpu().numpy()[big]))
    assert np.all(np.isnan(small.obj.cpu().numpy()[big])) and np.all(small.iters.cpu().numpy()[big] == 0)
    assert np.array_equal(small.u.cpu().numpy()[~big], u[~big])


def test_srbd_wide_warm_and_persistent():
    """The wide kernel's warm-start modes: warm_start = 1 resumes at the
    solution (<= 50 iterations, objective not worse); the persistent solver
    (warm_start = 2) over 12 ticks of N = 20 mixed schedules, half the
    controllers flipping their contacts at tick 6 (their stance set drops to
    the two-wave class and back: re-initialisation across kernels), each tick
    against the oracle's restatement (oracle/persist.c) resumed from the GPU's
    own record of the previous tick (so that two eps-optimal stopping points
    do not compound over the ticks): iterations within two check
    intervals and equal for >= 70 % of (tick, controller) pairs, the
    trajectory-parity bounds where they are equal, |dX|_Q <= 0.3 elsewhere
    (test_srbd_wide_instances_match_restatement)."""
    from cases import closed_loop_srbd
    dev = _dev()
    N, B = 20, 6
    x0, xr, ft, ct = srbd.generate(SEED, N, B, "mixed")
    args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
    warm = torch.zeros((B, 32 * N), dtype=torch.float32, device=dev)
    s = srbd.BatchedConvexMpc(horizon=N, warm_start=1)
    o1 = s.solve(*args, warm=warm).obj.cpu().numpy()
    second = s.solve(*args, warm=warm)
    torch.cuda.synchronize()
    assert np.all(second.iters.cpu().numpy() <= 50), second.iters.cpu().numpy()
    o2 = second.obj.cpu().numpy()
    sp = O.srbd_spec(N=N)
    for b in range(B):
        sc = max(1.0, abs(Instance(sp, x0[b], xr[b], ft[b], ct[b]).exact_obj()))
        assert o2[b] <= o1[b] + 1e-3 * sc, (b, o1[b], o2[b])
    T = 12
    seq = closed_loop_srbd(N, B, T, switch_at=6, gait="mixed")
    gpu = srbd.PersistentConvexMpc(B, dev, horizon=N)
    orc = [O.PersistentMpc(N) for _ in range(B)]
    same = total = 0
    for t, (x0, xr, ft, ct) in enumerate(seq):
        prev = gpu.record.cpu().numpy().astype(np.float64)
        out = gpu.solve(*(torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)), full=True)
        torch.cuda.synchronize()
        u = out.u.cpu().numpy()
        st = out.status.cpu().numpy()
        its = out.iters.cpu().numpy()
        for b in range(B):
            orc[b].rec[:] = prev[b]  # resume from the GPU's own record: one-step parity
            ub, info = orc[b].step(x0[b], xr[b], ft[b], ct[b])
            assert st[b] == info.status == 0, (t, b, st[b], info.status)
            assert abs(int(its[b]) - info.iters) <= 50, (t, b, its[b], info.iters)
            _, dF, dM, dX = _traj_metrics(u[b], ub, x0[b], xr[b], ft[b], ct[b], N)
            if int(its[b]) == info.iters:
                same += 1
                assert dX <= 0.1 and dF <= 15.0 and dM <= 3.0, (t, b, dF, dM, dX)
            assert dX <= 0.3, (t, b, dF, dM, dX)
            total += 1
    assert same >= 0.7 * total, (same, total)


# --- the literal full QP (spec.literal_full_qp = 1): the reference's call as
# written -- all 12N forces are ADMM variables, swing legs held by their
# fz in [0, 0] rows (OSQP equality rows, rho_eq = 1e3 rho), Ruiz over the
# full P and A (ConvexMpc.cpp:162-264, A1RobotControl.cpp:557-578).  Checked
# against the oracle's fp64 OSQP-algorithm restatement of the SAME problem
# (Instance.admm_full), at the reduced mode's bounds.

@pytest.mark.parametrize("N,B,gait", [(10, 48, "trot"), (10, 24, "pace"), (10, 32, "mixed"),
                                      (16, 12, "trot"), (20, 8, "pace"), (4, 16, "trot"),
                                      (1, 16, "trot"), (2, 16, "mixed"), (7, 16, "pace"),
                                      # two waves, odd N (unequal wave halves H = ceil(N / 2))
                                      (11, 16, "trot"), (13, 16, "pace"), (15, 16, "mixed"),
                                      (17, 16, "trot"), (19, 16, "pace"),
                                      # two waves, mixed per-step schedules (128: the
                                      # rates below are fractions of a batch)
                                      (16, 128, "mixed"), (20, 128, "mixed")])
def test_srbd_literal_matches_full_restatement(N, B, gait):
    """Literal mode vs Instance.admm_full (the reference's full 12N-variable
    OSQP call, fp64): status OK, iterations within one check interval and
    equal for >= 90 % (measured 0.97-1.0, tools/srbd_parity_scan.py
    --literal, profiles/r3_literal_parity_scan.txt); where both stop at the
    same check, predicted trajectory |dX|_Q <= 0.1 (measured max 0.031) and
    per-step net wrench <= 15 N / 3 N m; where fp32 residuals pass one check
    earlier or later the runs stop at different eps-optimal points (measured
    |dX|_Q 0.1005, 77 N on one N = 10 pace instance of 48): |dX|_Q <= 0.3;
    per-step net wrench <= 1 N / 0.1 N m for >= 90 % of instances at
    N <= 10 (measured 0.94-0.98) and >= 85 % at N = 16 / 20 (192 / 240
    fp32 variables: measured 0.875 / 0.917); objective within
    5e-3 * max(1, |f*|) of the restatement's (measured p90 1.1e-5, max
    2.9e-3 on the instance that stops a check early); swing forces within
    the ADMM tolerance of zero (|f| <= 0.25 N); u0 = u[:12] and within the
    U0Bound tolerance of the restatement's u0 (the forces the reference
    returns)."""
    (x0, xr, ft, ct), r = _solve(N, B, gait, literal_full_qp=1)
    sp = O.srbd_spec(N=N)
    same = near = 0
    u0b = U0Bound()
    # two waves (N > 10): within two checks (N = 20 mixed: one instance in 64
    # stops at 175 against the restatement's 125, the round-5 kernel too,
    # gpurun_out r6b; its iterate passes OSQP's own termination test,
    # test_srbd_literal_iterate_passes_osqp_termination)
    it_tol = 25 if N <= 10 else 50
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xf, info = inst.admm_full()
        assert r["status"][b] == 0 and info.status == 0, (b, r["status"][b], info.status)
        assert abs(int(r["iters"][b]) - info.iters) <= it_tol, (b, r["iters"][b], info.iters)
        u = r["u"][b].astype(np.float64)
        du0, dF, dM, dX = _traj_metrics(u, xf, x0[b], xr[b], ft[b], ct[b], N)
        u0b.add(du0, int(r["iters"][b]) == info.iters, b)
        if int(r["iters"][b]) == info.iters:
            same += 1
            assert dX <= 0.1, (b, dX)
            assert dF <= 15.0 and dM <= 3.0, (b, dF, dM)
        assert dX <= 0.3, (b, dX)
        near += int(dF <= 1.0 and dM <= 0.1)
        # objective scale: the exact optimum (EiQuadProg restatement); at N = 1 the
        # active-set restatement can report its equality rows degenerate, then
        # the fp64 OSQP restatement's objective is the scale
        xe, st_e, _ = inst.exact()
        sc = max(1.0, abs(inst.obj(xe) if st_e == 0 else inst.obj(xf)))
        assert abs(inst.obj(u) - inst.obj(xf)) <= 5e-3 * sc, (b, inst.obj(u), inst.obj(xf))
        swing = np.repeat(ct[b] == 0, 3)
        assert np.all(np.abs(u[swing]) <= 0.25), (b, np.abs(u[swing]).max())
        assert np.array_equal(r["u0"][b], r["u"][b][:12])
    # equal iteration counts: >= 90 % at N <= 10, >= 85 % on two waves
    # (measured 0.977 / 0.938 on N = 16 / 20 mixed, 128 instances each;
    # wrench <= 1 N / 0.1 N m 0.953 / 0.914, tools/srbd_parity_scan.py)
    assert same >= (0.9 if N <= 10 else 0.85) * B, same
    assert near >= (0.9 if N <= 10 else 0.85) * B, near
    u0b.check()


@pytest.mark.parametrize("interval", [25, 50])
def test_srbd_literal_rho_interval_matches_restatement(interval):
    """OSQP v0.6 built with PROFILING (its default) turns adaptive_rho_interval
    = 0 into a timing-derived interval on the first solve (DESIGN.md §6:
    25-75 iterations on a typical host for this problem, not the
    deterministic 100).  A caller reproducing a given host sets
    spec.adaptive_rho_interval; here 25 / 50 against the restatement run with
    the same interval: status, iterations within one check and equal for
    >= 90 %, and the literal-mode trajectory / objective bounds."""
    N, B, gait = 10, 32, "trot"
    (x0, xr, ft, ct), r = _solve(N, B, gait, literal_full_qp=1, adaptive_rho_interval=interval)
    sp = O.srbd_spec(N=N)
    same = 0
    u0b = U0Bound()
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xf, info = inst.admm_full(adaptive_rho_interval=interval)
        assert r["status"][b] == 0 and info.status == 0, (b, r["status"][b], info.status)
        assert abs(int(r["iters"][b]) - info.iters) <= 25, (b, r["iters"][b], info.iters)
        u = r["u"][b].astype(np.float64)
        du0, dF, dM, dX = _traj_metrics(u, xf, x0[b], xr[b], ft[b], ct[b], N)
        u0b.add(du0, int(r["iters"][b]) == info.iters, b)
        if int(r["iters"][b]) == info.iters:
            same += 1
            assert dX <= 0.1, (b, dX)
        assert dX <= 0.3, (b, dX)
        sc = max(1.0, abs(inst.exact_obj()))
        assert abs(inst.obj(u) - inst.obj(xf)) <= 5e-3 * sc, (b, inst.obj(u), inst.obj(xf))
    assert same >= 0.9 * B, same
    u0b.check()


@pytest.mark.parametrize("N,B,gait,samples", [(10, 4096, "trot", 16), (16, 65536, "trot", 8),
                                              (20, 65536, "pace", 6), (10, 131072, "mixed", 8),
                                              (20, 524288, "pace", 4), (10, 1048576, "mixed", 4)])
def test_srbd_literal_full_size_sampled(N, B, gait, samples):
    """The literal QP at full size, one launch each: BASELINE configs[1]
    (N = 10 trot, 4096), configs[2] (N = 16 trot, 65,536), the per-GPU
    shares of configs[3] / [4] (N = 20 pace 65,536, N = 10 mixed 131,072)
    and configs[3] / [4] whole on one GPU (N = 20 pace 524,288 through the
    two-wave wrench-space kernel, N = 10 mixed 1,048,576 through the
    one-wave one: what the 8-GPU runs shard).  Whole
    batch: every instance converges, forces finite and inside the friction
    pyramid, swing forces within the ADMM tolerance of zero, u0 = u[:12], and
    a second launch is bit-identical.  Instances spread over the batch (both
    ends, both phases) against the fp64 restatement of the same 12N-variable
    OSQP call (Instance.admm_full) at test_srbd_literal_matches_full_
    restatement's per-instance bounds."""
    (x0, xr, ft, ct), r = _solve(N, B, gait, literal_full_qp=1)
    assert np.all(r["status"] == 0), np.unique(r["status"], return_counts=True)
    u = r["u"].reshape(B, N, 4, 3)
    assert np.all(np.isfinite(u))
    tol = 0.25
    assert np.all(u[..., 2] >= -tol) and np.all(u[..., 2] <= 180 + tol)
    assert np.all(np.abs(u[..., 0]) <= 0.3 * u[..., 2] + tol)
    assert np.all(np.abs(u[..., 1]) <= 0.3 * u[..., 2] + tol)
    swing = ct.reshape(B, N, 4) == 0
    assert np.abs(u[swing]).max() <= tol
    assert np.array_equal(r["u0"], r["u"][:, :12])
    _, r2 = _solve(N, B, gait, literal_full_qp=1)
    assert np.array_equal(r["u"], r2["u"]) and np.array_equal(r["iters"], r2["iters"])
    sp = O.srbd_spec(N=N)
    u0b = U0Bound()
    for b in np.linspace(0, B - 1, samples).astype(int):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xf, info = inst.admm_full()
        assert info.status == 0
        assert abs(int(r["iters"][b]) - info.iters) <= 25, (b, r["iters"][b], info.iters)
        ub = r["u"][b].astype(np.float64)
        du0, dF, dM, dX = _traj_metrics(ub, xf, x0[b], xr[b], ft[b], ct[b], N)
        u0b.add(du0, int(r["iters"][b]) == info.iters, b)
        if int(r["iters"][b]) == info.iters:
            assert dX <= 0.1 and dF <= 15.0 and dM <= 3.0, (b, dX, dF, dM)
        assert dX <= 0.3, (b, dX)
        sc = max(1.0, abs(inst.exact_obj()))
        assert abs(inst.obj(ub) - inst.obj(xf)) <= 5e-3 * sc, b
    u0b.check()


@pytest.mark.parametrize("N,B,gait,wset,qpatch,route", [
    (10, 24, "trot", "isaac", {}, 3), (16, 6, "trot", "isaac", {}, 3),
    (10, 16, "trot", "hardware", {}, 1), (16, 16, "trot", "hardware", {}, 2),
    (10, 24, "trot", "gazebo", {7: 0.2}, 1), (10, 16, "mixed", "gazebo", {6: 0.4, 7: 0.1}, 1),
    (16, 16, "trot", "gazebo", {7: 0.2}, 2), (20, 8, "pace", "gazebo", {}, 2),
    (10, 12, "trot", None, {6: 0.0}, 3), (16, 6, "trot", None, {10: 0.0}, 3)])
def test_srbd_literal_reference_weight_sets(N, B, gait, wset, qpatch, route):
    """The MPC weight sets the reference ships (config/{isaac,hardware,
    gazebo}_a1_mpc.yaml).  hardware and gazebo run the wrench-space kernels
    at N = 10 / 16 / 20 (one and two waves), and so do anisotropic omega
    weights on the gazebo set (omega x != y couples the two axes through
    the yaw rotation: the eigen-axis pair of the G^-1 tables, DESIGN.md
    §3j); isaac's state weights (roll 8000: the wrench-space solve's float32
    limit) and a zero omega / v weight (G singular) take the generic literal
    kernels (two-wave column bucket / wide kernel).  qloco_srbd_route says
    which.  Same bounds against the restatement of the same QP as
    test_srbd_literal_matches_full_restatement (status, iterations within
    one check, objective, swing forces, u0)."""
    q, rw = (list(O.Q_W), list(O.R_W)) if wset is None else map(list, srbd.REFERENCE_WEIGHTS[wset])
    for k, v in qpatch.items():
        q[k] = v
    assert srbd.route(srbd.default_spec(horizon=N, literal_full_qp=1, q_weights=q, r_weights=rw)) == route
    (x0, xr, ft, ct), r = _solve(N, B, gait, literal_full_qp=1, q_weights=q, r_weights=rw)
    sp = O.srbd_spec(N=N, q_w=q, r_w=rw)
    u0b = U0Bound()
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xf, info = inst.admm_full()
        assert r["status"][b] == 0 and info.status == 0, (b, r["status"][b], info.status)
        assert abs(int(r["iters"][b]) - info.iters) <= 25, (b, r["iters"][b], info.iters)
        u = r["u"][b].astype(np.float64)
        du0, dF, dM, dX = _traj_metrics(u, xf, x0[b], xr[b], ft[b], ct[b], N)
        u0b.add(du0, int(r["iters"][b]) == info.iters, b)
        sc = max(1.0, abs(inst.obj(xf)))
        assert abs(inst.obj(u) - inst.obj(xf)) <= 5e-3 * sc, (b, inst.obj(u), inst.obj(xf))
        swing = np.repeat(ct[b] == 0, 3)
        assert np.all(np.abs(u[swing]) <= 0.25), (b, np.abs(u[swing]).max())
    u0b.check()


@pytest.mark.parametrize("N", [10, 16, 20, 13])
def test_srbd_literal_edge_cases_and_modes(N):
    """Literal mode corner cases: an all-swing instance (every fz row an
    equality [0, 0]: the optimum is u = 0), an all-stance one, a
    single-stance-step one and (two waves) one whose stance steps all sit in
    the second wave's half, in one batch -- at N = 10 (one wave) and
    N = 13 / 16 / 20 (two waves); the caller's max_stance_legs is ignored
    (the literal problem always has 4N leg triples); warm_start = 1 resumes
    at the solution in <= 50 iterations."""
    dev = _dev()
    B = 5
    x0, xr, ft, ct = srbd.generate(SEED, N, B, "trot")
    ct[0, :] = 0
    ct[1, :] = 1
    ct[2, 4:] = 0
    ct[4, :4 * ((N + 1) // 2)] = 0  # stance only in the second wave's steps
    args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
    solver = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=1)
    out = solver.solve(*args, full=True, max_legs=1)
    torch.cuda.synchronize()
    u = out.u.cpu().numpy().astype(np.float64)
    st = out.status.cpu().numpy()
    assert np.all(st == 0), st
    assert np.abs(u[0]).max() <= 0.25, np.abs(u[0]).max()
    sp = O.srbd_spec(N=N)
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        xf, info = inst.admm_full()
        assert abs(int(out.iters[b]) - info.iters) <= 25
        sc = max(1.0, abs(inst.exact_obj()))
        assert abs(inst.obj(u[b]) - inst.obj(xf)) <= 1e-3 * sc, b
    warm = torch.zeros((B, 32 * N), dtype=torch.float32, device=dev)
    s = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=1, warm_start=1)
    s.solve(*args, warm=warm)
    second = s.solve(*args, warm=warm)
    torch.cuda.synchronize()
    assert np.all(second.iters.cpu().numpy() <= 50), second.iters.cpu().numpy()


def _osqp_termination(inst, x, y, eps_abs=1e-3, eps_rel=1e-3):
    """OSQP v0.6's unscaled termination test (auxil.c compute_prim_res /
    compute_dual_res / compute_prim_tol / compute_dual_tol, scaled_termination
    off: the reference's settings, A1RobotControl.cpp:558-559) in float64 on an
    iterate (x, y) of the reference's QP (H, g, A, l, u of ConvexMpc.cpp:
    162-264).  OSQP's z is the projection of its iterate onto [l, u]; the
    returned pair does not carry it, so z = Pi_[l,u](A x): ||A x - z|| is then
    the distance of A x to the box, never above the solver's own primal
    residual.  Returns (prim_res / prim_tol, dual_res / dual_tol)."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    Ax = inst.A @ x
    z = np.clip(Ax, inst.lb, inst.ub)
    prim = np.abs(Ax - z).max()
    prim_tol = eps_abs + eps_rel * max(np.abs(Ax).max(), np.abs(z).max())
    Px = inst.H @ x
    Aty = inst.A.T @ y
    dual = np.abs(Px + inst.g + Aty).max()
    dual_tol = eps_abs + eps_rel * max(np.abs(Px).max(), np.abs(Aty).max(), np.abs(inst.g).max())
    return prim / prim_tol, dual / dual_tol


# The float64 re-evaluation must pass outright: measured max residual /
# tolerance 0.998 over 560 instances of eight shapes (gpurun_out r6l; the
# kernels are deterministic, so a rerun reproduces the same ratios).
OSQP_TOL_SLACK = 1.0


@pytest.mark.parametrize("N,B,gait,wset", [(10, 256, "trot", None), (10, 96, "mixed", None),
                                           (16, 48, "trot", None), (20, 32, "pace", None),
                                           (20, 16, "mixed", None), (13, 32, "trot", None),
                                           (19, 24, "mixed", None), (10, 64, "trot", "isaac"),
                                           (16, 16, "trot", "isaac")])
def test_srbd_literal_iterate_passes_osqp_termination(N, B, gait, wset):
    """Every GPU iterate that the kernel reports SOLVED passes OSQP's own
    termination test re-evaluated in float64 on the reference's unscaled QP
    (_osqp_termination), whether or not it stops at the same check as the
    fp64 restatement -- the criterion, not a u0 distance, is what certifies
    the instances that stop one check apart (U0Bound's 30 N).  The unscaled
    y comes from the warm_start = 1 form of the same call started from zeros
    (x = y = z = 0 is the cold start): its iterations equal the cold
    launch's and its u0 agrees to rounding.  Reports the instances one check
    apart and asserts the test on those too."""
    dev = _dev()
    x0, xr, ft, ct = srbd.generate(SEED, N, B, gait)
    args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
    q, rw = (list(O.Q_W), list(O.R_W)) if wset is None else map(list, srbd.REFERENCE_WEIGHTS[wset])
    kw = dict(literal_full_qp=1, q_weights=q, r_weights=rw)
    cold = srbd.BatchedConvexMpc(horizon=N, **kw).solve(*args, full=True)
    warm = torch.zeros((B, 32 * N), dtype=torch.float32, device=dev)
    ws = srbd.BatchedConvexMpc(horizon=N, warm_start=1, **kw).solve(*args, full=True, warm=warm)
    torch.cuda.synchronize()
    st = ws.status.cpu().numpy()
    it, it_cold = ws.iters.cpu().numpy(), cold.iters.cpu().numpy()
    assert np.all(st == 0) and np.all(cold.status.cpu().numpy() == 0)
    u, u_cold = ws.u.cpu().numpy().astype(np.float64), cold.u.cpu().numpy().astype(np.float64)
    if srbd.route(srbd.default_spec(horizon=N, **kw)) in (1, 2):  # the same wrench-space kernel
        assert np.array_equal(it, it_cold)
        assert np.abs(u - u_cold).max() <= 1e-3 * max(1.0, np.abs(u_cold).max())
    else:  # generic literal kernels: the warm form runs another column bucket (another iterate)
        assert np.abs(it.astype(int) - it_cold).max() <= 25
    wy = warm.cpu().numpy().astype(np.float64)[:, 12 * N:]
    sp = O.srbd_spec(N=N, q_w=q, r_w=rw)
    apart, worst = [], (0.0, 0.0)
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        rp, rd = _osqp_termination(inst, u[b], wy[b])
        worst = (max(worst[0], rp), max(worst[1], rd))
        assert rp <= OSQP_TOL_SLACK and rd <= OSQP_TOL_SLACK, (b, rp, rd)
        _, info = inst.admm_full()
        if info.iters != int(it[b]):
            apart.append((b, int(it[b]), info.iters, rp, rd))
    print("N=%d %s B=%d: max prim_res/tol %.3f dual_res/tol %.3f; one check apart: %s" % (
        N, gait, B, worst[0], worst[1], apart))


@pytest.mark.parametrize("N,B,gait", [(10, 128, "trot"), (10, 64, "mixed"), (16, 32, "trot"),
                                      (20, 24, "pace"), (20, 16, "mixed")])
def test_srbd_reduced_iterate_passes_osqp_termination(N, B, gait):
    """The stance-only reduction (literal_full_qp = 0, the bench's reduced_qp
    line) certified the same way as the literal mode: every SOLVED iterate
    passes OSQP's unscaled termination test in float64 on the reduced QP
    (the stance variables and their friction / bound rows of the reference's
    H, g, A, l, u), with y from the warm_start = 1 form of the call started
    from zeros (the kernels write it in the full row indexing).  This is the
    certificate behind the wrench bounds of test_srbd_trajectory_parity_vs_
    restatement, whose per-instance values move with the compiler's
    contraction of the residual expressions (17.3 N against the
    15 N bound on an unshipped build) while the criterion holds."""
    dev = _dev()
    x0, xr, ft, ct = srbd.generate(SEED, N, B, gait)
    args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
    warm = torch.zeros((B, 32 * N), dtype=torch.float32, device=dev)
    ws = srbd.BatchedConvexMpc(horizon=N, warm_start=1).solve(*args, full=True, warm=warm)
    torch.cuda.synchronize()
    assert np.all(ws.status.cpu().numpy() == 0)
    u = ws.u.cpu().numpy().astype(np.float64)
    wy = warm.cpu().numpy().astype(np.float64)[:, 12 * N:]
    sp = O.srbd_spec(N=N)
    worst = (0.0, 0.0)
    for b in range(B):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        i, r = inst.idx, inst.rows
        red = type("Red", (), {})()
        red.H, red.g, red.A = inst.H[np.ix_(i, i)], inst.g[i], inst.A[np.ix_(r, i)]
        red.lb, red.ub = inst.lb[r], inst.ub[r]
        assert np.all(u[b][np.setdiff1d(np.arange(12 * N), i)] == 0.0)  # swing forces exactly 0
        rp, rd = _osqp_termination(red, u[b][i], wy[b][r])
        worst = (max(worst[0], rp), max(worst[1], rd))
        assert rp <= OSQP_TOL_SLACK and rd <= OSQP_TOL_SLACK, (b, rp, rd)
    print("reduced N=%d %s B=%d: max prim_res/tol %.3f dual_res/tol %.3f" % (N, gait, B, worst[0], worst[1]))


@pytest.mark.parametrize("N,B,T,every", [(10, 32, 24, 6), (16, 8, 12, 4)])
def test_srbd_literal_persistent_closed_loop_matches_restatement(N, B, T, every):
    """The reference's member OSQP solver over a trotting control loop
    (A1RobotControl.cpp:556-578), on its literal QP: every controller flips
    its trot phase each `every` MPC ticks (odd controllers half a period
    later), and -- as in the reference, whose Hessian pattern never depends
    on the contacts -- every call after the first takes OSQP's update path
    (osqp_update_P / _lin_cost / _bounds: the fz rows re-typed, the adapted
    rho and the scaled x, z, y carried).  Per tick, GPU (warm_start = 2,
    literal_full_qp = 1) vs oracle/persist.c (qo_srbd_persist_step_ex,
    literal = 1): status, iterations within one check interval and equal for
    >= 85 % of (tick, controller) pairs, the carried rho within 10 % for
    >= 90 % (an adaptation step changes rho by >= 5x; fp32 residual ratios
    differ from fp64 at the 1e-3 level and compound over ticks: measured
    0.92 at N = 16), and the trajectory-parity bounds: |dX|_Q <= 0.1, per-step
    wrench <= 15 N / 3 N m where both stop at the same check, |dX|_Q <= 0.3
    where fp32 stops one check apart (N = 10 one-wave literal kernel,
    tools/lit_closed_loop.py: iterations equal for 767 / 768, same-check
    wrench max 6.9 N; the one early stop 28 N at |dX|_Q 0.086), and u0 --
    the forces each tick returns -- within U0Bound.  Phase
    switches resume rather than restart: the ticks after a switch need fewer
    iterations than the cold first tick."""
    from cases import closed_loop_srbd
    dev = _dev()
    seq = closed_loop_srbd(N, B, T, switch_every=every)
    gpu = srbd.PersistentConvexMpc(B, dev, horizon=N, literal_full_qp=1)
    orc = [O.PersistentMpc(N, literal=True) for _ in range(B)]
    same = rho_ok = total = 0
    u0b = U0Bound()
    it_first, it_switch = [], []
    prev_ct = None
    for t, (x0, xr, ft, ct) in enumerate(seq):
        out = gpu.solve(*(torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)), full=True)
        torch.cuda.synchronize()
        u = out.u.cpu().numpy()
        st = out.status.cpu().numpy()
        its = out.iters.cpu().numpy()
        rec = gpu.record.cpu().numpy()
        for b in range(B):
            ub, info = orc[b].step(x0[b], xr[b], ft[b], ct[b])
            assert st[b] == info.status == 0, (t, b, st[b], info.status)
            assert abs(int(its[b]) - info.iters) <= 25, (t, b, its[b], info.iters)
            same += int(its[b]) == info.iters
            r64 = orc[b].rec[100 * N]
            rho_ok += int(abs(rec[b, 100 * N] - r64) <= 0.1 * r64)
            total += 1
            du0, dF, dM, dX = _traj_metrics(u[b], ub, x0[b], xr[b], ft[b], ct[b], N)
            u0b.add(du0, int(its[b]) == info.iters, (t, b))
            if int(its[b]) == info.iters:
                assert dX <= 0.1 and dF <= 15.0 and dM <= 3.0, (t, b, dF, dM, dX)
            # a check passed one interval earlier / later in fp32: a different
            # eps-optimal point (test_srbd_literal_matches_full_restatement's rule)
            assert dX <= 0.3, (t, b, dF, dM, dX)
            if t == 0:
                it_first.append(int(its[b]))
            elif not np.array_equal(ct[b], prev_ct[b]):
                it_switch.append(int(its[b]))
        prev_ct = ct
    assert it_switch, "the sequence holds phase switches"
    assert same >= 0.85 * total, (same, total)
    assert rho_ok >= 0.9 * total, (rho_ok, total)
    u0b.check()
    assert np.mean(it_switch) < np.mean(it_first)


# --- stream / graph behaviour of the class dispatch (its scratch is one set
# per (device, caller stream), never freed while the process lives)

def _three_class_batch(N=20):
    parts = [srbd.generate(SEED, N, 6, g) for g in ("trot", "mixed", "stance")]
    x0, xr, ft, ct = (np.concatenate([p[k] for p in parts]) for k in range(4))
    ct[0:2, 4 * 5:] = 0  # one-wave class instances
    return x0, xr, ft, ct


def test_srbd_two_streams_mixed_classes():
    """Two multi-class batches solved concurrently on two caller streams
    (different batch sizes, so each stream's scratch is sized separately)
    give bit-for-bit the results of one-at-a-time solves on the default
    stream: no shared lists, counters or fork / join events."""
    dev = _dev()
    N = 20
    a = _three_class_batch(N)
    b = tuple(np.ascontiguousarray(np.concatenate([v, v[:5]])) for v in a)  # 23 instances
    solver = srbd.BatchedConvexMpc(horizon=N)
    ta = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in a]
    tb = [torch.from_numpy(v).to(dev) for v in b]
    ref_a = solver.solve(*ta, full=True)
    ref_b = solver.solve(*tb, full=True)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    outs = []
    for rep in range(3):
        with torch.cuda.stream(s1):
            oa = solver.solve(*ta, full=True, stream=s1.cuda_stream)
        with torch.cuda.stream(s2):
            ob = solver.solve(*tb, full=True, stream=s2.cuda_stream)
        outs.append((oa, ob))
    torch.cuda.synchronize()
    for oa, ob in outs:
        assert torch.equal(oa.u, ref_a.u) and torch.equal(oa.status, ref_a.status)
        assert torch.equal(ob.u, ref_b.u) and torch.equal(ob.iters, ref_b.iters)


def test_srbd_graph_capture_replay():
    """The multi-class call captured into a HIP graph (after a warm-up call
    on the capture stream sized its scratch) replays to the eager results;
    a later, larger eager batch on that stream grows the scratch without
    freeing the lists the graph reads, so a replay afterwards still matches."""
    dev = _dev()
    N = 20
    x0, xr, ft, ct = _three_class_batch(N)
    args = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (x0, xr, ft, ct)]
    solver = srbd.BatchedConvexMpc(horizon=N)
    ref = solver.solve(*args, full=True)
    torch.cuda.synchronize()
    B = x0.shape[0]
    out = solver.alloc_outputs(B, dev, full=True)
    s = torch.cuda.Stream(dev)
    legs = srbd.max_stance_legs(ct, N)
    with torch.cuda.stream(s):
        solver.solve(*args, out=out, max_legs=legs, stream=s.cuda_stream)  # warm-up: sizes the scratch
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        solver.solve(*args, out=out, max_legs=legs, stream=s.cuda_stream)
    for k in range(2):
        out.u.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out.u, ref.u) and torch.equal(out.status, ref.status)
    big = [torch.cat([t] * 300) for t in args]  # 5400 instances: the scratch grows
    with torch.cuda.stream(s):
        solver.solve(*big, max_legs=legs, stream=s.cuda_stream)
    torch.cuda.synchronize()
    out.u.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out.u, ref.u)


def test_srbd_scratch_bounded_over_short_lived_streams():
    """A caller that makes a new stream per call: the class-dispatch
    scratch stays bounded -- at most 8 live sets, the least recently used one
    released once its last launch is done -- and every call still gives the
    default stream's results bit for bit.  The set of the captured stream of
    test_srbd_graph_capture_replay (same process) may be pinned, never freed."""
    dev = _dev()
    N = 20
    a = _three_class_batch(N)
    ta = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in a]
    solver = srbd.BatchedConvexMpc(horizon=N)
    ref = solver.solve(*ta, full=True)
    torch.cuda.synchronize()
    L = _lib.lib()
    pinned = C.c_int32(0)
    for k in range(24):
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            o = solver.solve(*ta, full=True, stream=s.cuda_stream)
        s.synchronize()
        assert torch.equal(o.u, ref.u) and torch.equal(o.iters, ref.iters)
        del s
        live = L.qloco_srbd_scratch_sets(C.byref(pinned))
        assert live <= 8, (k, live)
    assert L.qloco_srbd_scratch_sets(None) == 8
    before = pinned.value
    for k in range(8):  # more churn: nothing new gets pinned by eager calls
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            solver.solve(*ta, full=True, stream=s.cuda_stream)
        s.synchronize()
    L.qloco_srbd_scratch_sets(C.byref(pinned))
    assert pinned.value == before
