"""Distribution of the SRBD parity quantities (GPU fp32 vs the oracle's fp64
OSQP-algorithm ADMM restatement and vs the exact optimum of the literal QP),
used to set the tolerances written in tests/test_srbd_gpu.py.
    python tools/srbd_parity_scan.py [--literal] [N B gait eps] ...   (GPU)
--literal: the literal 12N-variable mode (spec.literal_full_qp = 1) against
the restatement of the same full QP (Instance.admm_full).
Quantities per instance: |du0|, per-step net wrench (sum f, sum r x f),
the predicted state trajectory X = Aqp x0 + Bqp u in the Q-norm, objective
gap (f - f*) / max(1, |f*|), iterations."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import torch  # noqa: E402

import oracle_lib as O  # noqa: E402
from srbd_ref import Instance, np_build  # noqa: E402
from quadrupedal_loco_amd import _lib, srbd  # noqa: E402

if os.environ.get("QLOCO_LIB"):  # experimental variant (tools/variant_lib.py)
    _lib.LIB_PATH = os.environ["QLOCO_LIB"]


def metrics(inst, u, ref, x0, xr, ft, N, Bqp, q):
    u = np.asarray(u, np.float64)
    ur = u.reshape(N, 4, 3) - ref.reshape(N, 4, 3)
    r = np.asarray(ft, np.float64).reshape(4, 3)
    dF = np.abs(ur.sum(1)).max()
    dM = np.abs(np.cross(np.broadcast_to(r, (N, 4, 3)), ur).sum(1)).max()
    d = Bqp @ (u - ref)
    dX = np.sqrt((q * d * d).sum())
    return np.abs(u[:12] - ref[:12]).max(), dF, dM, dX


def main(cases, literal=False):
    dev = torch.device("cuda:0")
    for N, B, gait, eps in cases:
        x0, xr, ft, ct = srbd.generate(20261015, N, B, gait)
        kw = dict(eps_abs=eps, eps_rel=eps, max_iter=20000) if eps != 1e-3 else {}
        s = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=int(literal), **kw)
        out = s.solve(*(torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)), full=True)
        torch.cuda.synchronize()
        u = out.u.cpu().numpy()
        st = out.status.cpu().numpy()
        it = out.iters.cpu().numpy()
        sp = O.srbd_spec(N=N)
        q = np.tile(2.0 * np.asarray(O.Q_W), N)
        rows = []
        for b in range(B):
            inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
            Bqp = np_build(x0[b], xr[b], ft[b], ct[b], N)[6]
            ref = inst.admm_full if literal else inst.admm_reduced
            xa, info = ref(eps_abs=eps, eps_rel=eps, max_iter=20000)
            xe, _, _ = inst.exact()
            fe = inst.obj(xe)
            sc = max(1.0, abs(fe))
            ga = (inst.obj(u[b]) - fe) / sc
            g64 = (inst.obj(xa) - fe) / sc
            m_a = metrics(inst, u[b], xa, x0[b], xr[b], ft[b], N, Bqp, q)
            m_e = metrics(inst, u[b], xe, x0[b], xr[b], ft[b], N, Bqp, q)
            m_64 = metrics(inst, xa, xe, x0[b], xr[b], ft[b], N, Bqp, q)
            rows.append(m_a + m_e + m_64 + (ga, g64, ga - g64, int(it[b]) - info.iters,
                                            int(st[b])))
        R = np.array(rows)
        names = ["du0_adm", "dF_adm", "dM_adm", "dX_adm", "du0_ex", "dF_ex", "dM_ex", "dX_ex",
                 "du0_64ex", "dF_64ex", "dM_64ex", "dX_64ex", "gap_gpu", "gap_64", "gap_diff",
                 "dit", "status"]
        print("== [%s] N=%d B=%d %s eps=%g%s  status counts %s  iters equal %.3f" % (
            os.path.basename(os.path.dirname(os.environ.get("QLOCO_LIB", "/prod/x"))),
            N, B, gait, eps, " literal" if literal else "",
            dict(zip(*np.unique(st, return_counts=True))), float(np.mean(R[:, 15] == 0))))
        near = np.mean((R[:, 1] <= 1.0) & (R[:, 2] <= 0.1))
        print("  wrench <= 1 N / 0.1 N m: %.3f of instances" % near)
        for k, nm in enumerate(names[:-1]):
            v = R[:, k]
            print("  %-9s p50 %10.4g p90 %10.4g max %10.4g min %10.4g" % (
                nm, np.percentile(v, 50), np.percentile(v, 90), v.max(), v.min()))
        # u0 (the forces compute_grf returns, A1RobotControl.cpp:593-599) split by
        # whether both runs stopped at the same termination check
        for nm, sel in (("same-check", R[:, 15] == 0), ("check-apart", R[:, 15] != 0)):
            v = R[sel, 0]
            if v.size:
                print("  du0 %-11s n %5d  p50 %9.4g p95 %9.4g p99 %9.4g max %9.4g  <=0.5N %.4f  <=2N %.4f" % (
                    nm, v.size, *np.percentile(v, [50, 95, 99]), v.max(), np.mean(v <= 0.5),
                    np.mean(v <= 2.0)))
                print("  wrench %-11s max dF %9.4g N  max dM %9.4g N m  max dX_Q %9.4g" % (
                    nm, R[sel, 1].max(), R[sel, 2].max(), R[sel, 3].max()))
        sys.stdout.flush()


if __name__ == "__main__":
    a = sys.argv[1:]
    lit = bool(a) and a[0] == "--literal"
    if lit:
        a = a[1:]
    if a:
        cases = [(int(a[i]), int(a[i + 1]), a[i + 2], float(a[i + 3])) for i in range(0, len(a), 4)]
    else:
        cases = [(10, 64, "trot", 1e-3), (10, 48, "mixed", 1e-3), (16, 24, "trot", 1e-3),
                 (20, 16, "pace", 1e-3), (10, 32, "trot", 1e-5), (10, 32, "trot", 1e-6),
                 (10, 24, "mixed", 1e-6), (20, 12, "pace", 1e-6)]
    main(cases, lit)
