"""Float32 numerics of the literal wrench-space factorisations:
the KKT solve of OSQP's reduced system through (a) the S form of §3i with the
pivot-free Gauss-Jordan in several pivot orders, (b) the M = U + (cG)^-1 form
of the two-wave kernel, (c) the dense K Gauss-Jordan, all emulated in float32
(numpy), against float64.  Development aid, not product code; the table in
DESIGN.md §3j is SERR=1 on instance 47547.

    N=16 [GAIT=trot] SERR=1 RHOS= python tools/lit_numerics.py ID ...   backward error per form / rho
    N=16 FS=nat,rev,small RHOS= python tools/lit_numerics.py ID ...     full ADMM (adaptive rho), iterations
    N=16 IV=lapack32,plain,fusedNS1 python tools/lit_numerics.py ID ... fixed-rho ADMM per inverse kind
    N=16 T64=1 python tools/lit_numerics.py ID ...                      float64 T vs float64 iteration
"""
import os, sys
import numpy as np
_H = os.path.dirname(os.path.abspath(__file__)); sys.path.insert(0, _H); sys.path.insert(0, os.path.join(os.path.dirname(_H), "tests")); sys.path.insert(0, os.path.dirname(_H))
import proto_lit as P, proto_lit_fused as F
import oracle_lib as O
from srbd_ref import Instance
from quadrupedal_loco_amd import srbd
f = np.float32
N = int(os.environ.get("N", 16)); gait = os.environ.get("GAIT", "trot")
ids = [int(a) for a in sys.argv[1:]]
x0, xr, ft, ct = srbd.generate(20261015, N, max(ids) + 1, gait)
sp = O.srbd_spec(N=N)
base_factor_admm = P.admm

class DenseGJ:
    def __init__(self, K):
        self.Ki = F.gj_fused(K.astype(f)).astype(f)
    def __call__(self, b):
        return (self.Ki @ b.astype(f)).astype(np.float64)

class WrenchRefined(P.WrenchSolve):
    """wrench-space solve + one step of fixed-precision refinement with the
    structured K product (fp32)"""
    def __init__(self, G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, f32):
        super().__init__(G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, True)
        AE = Araw * E[:, None]
        self.K = (D[:, None] * (c * (Vu.T @ G @ Vu + np.diag(Rdiag)) + np.diag(sigma / D ** 2)
                  + AE.T @ (rho_vec[:, None] * AE)) * D[None, :]).astype(f)
    def __call__(self, b):
        x = super().__call__(b)
        r = (b.astype(f) - self.K @ x.astype(f)).astype(f)
        return x + super().__call__(r.astype(np.float64))

def run(mode, inst, G, Vu, rho):
    st = dict(rho=rho, sigma=1e-6, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, ctm=25, tol=1e30)
    if mode == "dense32":
        # patch factor: dense K fp32 GJ
        orig = P.WrenchSolve
        class DS:
            def __init__(s, G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, f32):
                AE = Araw * E[:, None]
                K = D[:, None] * (c * (Vu.T @ G @ Vu + np.diag(Rdiag)) + np.diag(sigma / D ** 2) + AE.T @ (rho_vec[:, None] * AE)) * D[None, :]
                s.d = DenseGJ(K)
            def __call__(s, b): return s.d(b)
        P.WrenchSolve = DS
        r = P.admm(inst, G, Vu, "wrench32", st=st, max_iter=600)
        P.WrenchSolve = orig
        return r
    if mode == "scaled":
        orig = P.WrenchSolve; P.WrenchSolve = F.solver(True)
        r = P.admm(inst, G, Vu, "wrench32", st=st, max_iter=600); P.WrenchSolve = orig; return r
    if mode == "refined":
        orig = P.WrenchSolve; P.WrenchSolve = WrenchRefined
        r = P.admm(inst, G, Vu, "wrench32", st=st, max_iter=600); P.WrenchSolve = orig; return r

for b in ids:
    inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
    G, Vu = P.wrench_model(x0[b], ft[b], N)
    for rho in [float(x) for x in os.environ.get("RHOS", "3e-4,1e-4").split(",") if x]:
        xo, info = inst.admm_full(rho=rho, adaptive_rho=0, max_iter=600)
        out = ["b=%d rho %.0e restatement it %d st %d" % (b, rho, info.iters, info.status)]
        for mode in os.environ.get("MODES", "scaled,dense32,refined").split(","):
            xm, it, stt, _, _ = run(mode, inst, G, Vu, rho)
            out.append("%s it %d st %d |du| %.3g" % (mode, it, stt, np.abs(xm - xo).max()))
        print("  ".join(out), flush=True)

class T64(P.WrenchSolve):
    """T from a float64 factorisation, rounded to fp32; fp32 iteration"""
    def __init__(self, G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, f32):
        super().__init__(G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, False)
        self.t = f
        self.T = self.T.astype(f); self.W0i = self.W0i.astype(f); self.Vu = self.Vu.astype(f); self.Dinv = self.Dinv.astype(f)
class It64(F.solver(True)):
    """fp32 scaled factorisation, fp64 iteration"""
    def __call__(self, b):
        T = self.T.astype(np.float64); W0i = self.W0i.astype(np.float64); Vu = self.Vu.astype(np.float64); Dinv = self.Dinv.astype(np.float64)
        a = W0i @ (Dinv * b); v = Vu @ a; s = T @ v
        return Dinv * (a - W0i @ (Vu.T @ s))
def run2(cls, inst, G, Vu, rho):
    st = dict(rho=rho, sigma=1e-6, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, ctm=25, tol=1e30)
    orig = P.WrenchSolve; P.WrenchSolve = cls
    r = P.admm(inst, G, Vu, "wrench32", st=st, max_iter=600); P.WrenchSolve = orig; return r
if os.environ.get("T64"):
    for b in ids:
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        G, Vu = P.wrench_model(x0[b], ft[b], N)
        for rho in (3e-4, 1e-4):
            xo, info = inst.admm_full(rho=rho, adaptive_rho=0, max_iter=600)
            out = ["b=%d rho %.0e restatement it %d" % (b, rho, info.iters)]
            for nm, cls in (("T64", T64), ("it64", It64)):
                xm, it, stt, _, _ = run2(cls, inst, G, Vu, rho)
                out.append("%s it %d st %d |du| %.3g" % (nm, it, stt, np.abs(xm - xo).max()))
            print("  ".join(out), flush=True)

def make_variant(s_round, gj):
    """factorisation pieces: S rounded to fp32 or not; inverse by fused fp32 GJ or exact fp64"""
    class V(P.WrenchSolve):
        def __init__(self, G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, f32):
            super().__init__(G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, False)
            N6 = G.shape[0]
            AE = Araw * E[:, None]
            W0 = np.diag(c * Rdiag + sigma / D ** 2) + AE.T @ (rho_vec[:, None] * AE)
            W0i = np.zeros_like(W0)
            for bb in range(Vu.shape[1] // 3):
                sl = slice(3 * bb, 3 * bb + 3); W0i[sl, sl] = np.linalg.inv(W0[sl, sl])
            U = Vu @ W0i @ Vu.T
            L = np.zeros_like(U); Li = np.zeros_like(U)
            for j in range(N6 // 6):
                sl = slice(6 * j, 6 * j + 6); L[sl, sl] = np.linalg.cholesky(U[sl, sl]); Li[sl, sl] = np.linalg.inv(L[sl, sl])
            Gc = c * G
            S = np.eye(N6) + L.T @ Gc @ L
            s = 1.0 / np.diag(S).max()
            Ss = S * s
            if s_round: Ss = Ss.astype(f)
            Si = (F.gj_fused(Ss.astype(f)).astype(np.float64) if gj else np.linalg.inv(Ss.astype(np.float64))) * s
            T = Gc @ L @ Si @ Li
            self.T = T.astype(f); self.W0i = W0i.astype(f); self.Vu = Vu.astype(f); self.Dinv = (1.0 / D).astype(f); self.t = f
    return V
if os.environ.get("SV"):
    for b in ids:
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        G, Vu = P.wrench_model(x0[b], ft[b], N)
        for rho in (3e-4, 1e-4):
            xo, info = inst.admm_full(rho=rho, adaptive_rho=0, max_iter=600)
            out = ["b=%d rho %.0e restatement it %d" % (b, rho, info.iters)]
            for nm, cls in (("S32exact", make_variant(True, False)), ("S64gj32", make_variant(False, True)), ("S32gj32", make_variant(True, True))):
                xm, it, stt, _, _ = run2(cls, inst, G, Vu, rho)
                out.append("%s it %d st %d |du| %.3g" % (nm, it, stt, np.abs(xm - xo).max()))
            print("  ".join(out), flush=True)

def gj_plain(S):
    A = S.astype(f).copy(); n = A.shape[0]
    for k in range(n):
        p = A[k, k]; pinv = f(1) / p
        row = (A[k, :] * pinv).astype(f); row[k] = pinv
        col = A[:, k].copy()
        A = (A - np.outer(col, row).astype(f)).astype(f)
        A[k, :] = row
        A[:, k] = (-col * pinv).astype(f); A[k, k] = pinv
    return A
def inv_variant(kind):
    class V(P.WrenchSolve):
        def __init__(self, G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, f32):
            super().__init__(G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, False)
            N6 = G.shape[0]
            AE = Araw * E[:, None]
            W0 = np.diag(c * Rdiag + sigma / D ** 2) + AE.T @ (rho_vec[:, None] * AE)
            W0i = np.zeros_like(W0)
            for bb in range(Vu.shape[1] // 3):
                sl = slice(3 * bb, 3 * bb + 3); W0i[sl, sl] = np.linalg.inv(W0[sl, sl])
            U = Vu @ W0i @ Vu.T
            L = np.zeros_like(U); Li = np.zeros_like(U)
            for j in range(N6 // 6):
                sl = slice(6 * j, 6 * j + 6); L[sl, sl] = np.linalg.cholesky(U[sl, sl]); Li[sl, sl] = np.linalg.inv(L[sl, sl])
            Gc = c * G
            S = np.eye(N6) + L.T @ Gc @ L
            s = 1.0 / np.diag(S).max()
            Ss = (S * s).astype(f)
            if kind in ("rev", "bigfirst", "smallfirst", "cmaj", "cmajf"):
                dg = np.diag(S)
                jj, ss = np.arange(N6) // 6, np.arange(N6) % 6
                perm = {"rev": np.arange(N6)[::-1], "bigfirst": np.argsort(-dg), "smallfirst": np.argsort(dg),
                        "cmaj": np.lexsort((-jj, ss)), "cmajf": np.lexsort((jj, ss))}[kind]
                Sp = Ss[np.ix_(perm, perm)]
                Xp = F.gj_fused(Sp).astype(f)
                X = np.empty_like(Xp); X[np.ix_(perm, perm)] = Xp
            elif kind == "jacobi":
                d = (1.0 / np.sqrt(np.diag(S))).astype(f)
                Sj = (d[:, None] * S * d[None, :]).astype(f)
                Xj = F.gj_fused(Sj).astype(np.float64)
                X = (d[:, None] * Xj * d[None, :] / s).astype(f)
            elif kind == "jacobiNS1":
                d = (1.0 / np.sqrt(np.diag(S))).astype(f)
                Sj = (d[:, None] * S * d[None, :]).astype(f)
                Xj = F.gj_fused(Sj).astype(f)
                R = (np.eye(N6, dtype=f) - (Sj @ Xj).astype(f)).astype(f)
                Xj = (Xj + (Xj @ R).astype(f)).astype(np.float64)
                X = (d[:, None] * Xj * d[None, :] / s).astype(f)
            elif kind == "lapack32": X = np.linalg.inv(Ss).astype(f)
            elif kind == "plain": X = gj_plain(Ss)
            elif kind.startswith("fusedNS"):
                X = F.gj_fused(Ss).astype(f)
                for _ in range(int(kind[-1])):
                    R = (np.eye(N6, dtype=f) - (Ss @ X).astype(f)).astype(f)
                    X = (X + (X @ R).astype(f)).astype(f)
            Si = X.astype(np.float64) * s
            T = Gc @ L @ Si @ Li
            self.T = T.astype(f); self.W0i = W0i.astype(f); self.Vu = Vu.astype(f); self.Dinv = (1.0 / D).astype(f); self.t = f
    return V
if os.environ.get("IV"):
    for b in ids:
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        G, Vu = P.wrench_model(x0[b], ft[b], N)
        for rho in (3e-4, 1e-4):
            xo, info = inst.admm_full(rho=rho, adaptive_rho=0, max_iter=600)
            out = ["b=%d rho %.0e restatement it %d" % (b, rho, info.iters)]
            for nm in os.environ["IV"].split(","):
                xm, it, stt, _, _ = run2(inv_variant(nm), inst, G, Vu, rho)
                out.append("%s it %d st %d |du| %.3g" % (nm, it, stt, np.abs(xm - xo).max()))
            print("  ".join(out), flush=True)

def fused_solver(order):
    class Fused(P.WrenchSolve):
        def __init__(self, G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, f32):
            super().__init__(G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, True)
            N6, n = G.shape[0], Vu.shape[1]
            AE = Araw * E[:, None]
            W0 = (np.diag(c * Rdiag + sigma / D ** 2) + AE.T @ (rho_vec[:, None] * AE)).astype(f)
            W0i = np.zeros_like(W0)
            for bb in range(n // 3):
                sl = slice(3 * bb, 3 * bb + 3); W0i[sl, sl] = np.linalg.inv(W0[sl, sl])
            Vu32 = Vu.astype(f)
            U = (Vu32 @ W0i @ Vu32.T).astype(f)
            L = np.zeros_like(U); Li = np.zeros_like(U)
            for j in range(N6 // 6):
                sl = slice(6 * j, 6 * j + 6); L[sl, sl] = np.linalg.cholesky(U[sl, sl]); Li[sl, sl] = np.linalg.inv(L[sl, sl])
            Gc = (c * G).astype(f)
            S = (np.eye(N6, dtype=f) + L.T @ Gc @ L).astype(f)
            s = f(1.0 / np.diag(S).max())
            Ss = (S * s).astype(f)
            jj, ss = np.arange(N6) // 6, np.arange(N6) % 6
            perm = {"nat": np.arange(N6), "rev": np.arange(N6)[::-1], "small": np.argsort(np.diag(S))}[order]
            Xp = F.gj_fused(Ss[np.ix_(perm, perm)]).astype(f)
            X = np.empty_like(Xp); X[np.ix_(perm, perm)] = Xp
            Si = (X * s).astype(f)
            self.T = (Gc @ (L @ (Si @ Li).astype(f)).astype(f)).astype(f)
    return Fused
if os.environ.get("FS"):
    agree = {}
    for b in ids:
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        G, Vu = P.wrench_model(x0[b], ft[b], N)
        xo, info = inst.admm_full()
        out = ["b=%5d oracle it %4d ru %d" % (b, info.iters, info.rho_updates)]
        for k in os.environ["FS"].split(","):
            orig = P.WrenchSolve; P.WrenchSolve = fused_solver(k)
            xm, it, stt, ru, _ = P.admm(inst, G, Vu, "wrench32", max_iter=1000)
            P.WrenchSolve = orig
            agree[k] = agree.get(k, 0) + int(it == info.iters)
            out.append("%s it %4d st %d ru %d du0 %.3g" % (k, it, stt, ru, np.abs(xm[:12] - xo[:12]).max()))
        print("  ".join(out), flush=True)
    print(agree)

def gj_order(A, order):
    n = A.shape[0]
    perm = np.arange(n)[::-1] if order == "rev" else np.arange(n)
    Xp = F.gj_fused(A[np.ix_(perm, perm)]).astype(f)
    X = np.empty_like(Xp); X[np.ix_(perm, perm)] = Xp
    return X
def minv_solver(ginv32, gord="nat", mord="nat"):
    class MS(P.WrenchSolve):
        def __init__(self, G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, f32):
            super().__init__(G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, True)
            N6, n = G.shape[0], Vu.shape[1]
            AE = Araw * E[:, None]
            W0 = (np.diag(c * Rdiag + sigma / D ** 2) + AE.T @ (rho_vec[:, None] * AE)).astype(f)
            W0i = np.zeros_like(W0)
            for bb in range(n // 3):
                sl = slice(3 * bb, 3 * bb + 3); W0i[sl, sl] = np.linalg.inv(W0[sl, sl])
            Vu32 = Vu.astype(f)
            U = (Vu32 @ W0i @ Vu32.T).astype(f)
            if ginv32:
                sg = f(1.0 / np.diag(G).max())
                Gi = (gj_order((G * sg).astype(f), gord) * sg).astype(f)
            else:
                Gi = np.linalg.inv(G).astype(f)
            M = (U + (Gi / f(c)).astype(f)).astype(f)
            sm = f(1.0 / np.diag(M).max())
            self.T = (gj_order((M * sm).astype(f), mord) * sm).astype(f)
    return MS
if os.environ.get("MS"):
    for b in ids:
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        G, Vu = P.wrench_model(x0[b], ft[b], N)
        print("cond(G) %.3g" % np.linalg.cond(G))
        xo, info = inst.admm_full()
        out = ["b=%5d oracle it %4d ru %d" % (b, info.iters, info.rho_updates)]
        for nm, g32 in (("M_G64", False), ("M_G32", True)):
            orig = P.WrenchSolve; P.WrenchSolve = minv_solver(g32)
            xm, it, stt, ru, _ = P.admm(inst, G, Vu, "wrench32", max_iter=1000)
            P.WrenchSolve = orig
            out.append("%s it %4d st %d ru %d du0 %.3g" % (nm, it, stt, ru, np.abs(xm[:12] - xo[:12]).max()))
        print("  ".join(out), flush=True)
if os.environ.get("TERR"):
    for b in ids:
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        G, Vu = P.wrench_model(x0[b], ft[b], N)
        Pm, q, A, D, E, c = P.ruiz(inst.H, inst.g, inst.A)
        l, u = inst.lb * E, inst.ub * E
        Rdiag = np.diag(inst.H - Vu.T @ G @ Vu)
        for rho in (0.1, 1e-2, 1e-3, 3e-4, 1e-4):
            rv = np.where(u - l < 1e-4, 1e3 * rho, rho)
            ref = P.WrenchSolve(G, Vu, D, E, c, 1e-6, inst.A, rv, Rdiag, False).T
            out = ["b=%d rho %.0e |T64| %.3g" % (b, rho, np.abs(ref).max())]
            for k in ("nat", "rev", "small"):
                Tk = fused_solver(k)(G, Vu, D, E, c, 1e-6, inst.A, rv, Rdiag, True).T.astype(np.float64)
                out.append("%s %.3g" % (k, np.abs(Tk - ref).max() / np.abs(ref).max()))
            Tm = minv_solver(True)(G, Vu, D, E, c, 1e-6, inst.A, rv, Rdiag, True).T.astype(np.float64)
            out.append("M %.3g" % (np.abs(Tm - ref).max() / np.abs(ref).max()))
            print("  ".join(out), flush=True)
if os.environ.get("SERR"):
    for b in ids:
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        G, Vu = P.wrench_model(x0[b], ft[b], N)
        Pm, q, A, D, E, c = P.ruiz(inst.H, inst.g, inst.A)
        l, u = inst.lb * E, inst.ub * E
        Rdiag = np.diag(inst.H - Vu.T @ G @ Vu)
        rng = np.random.default_rng(0)
        for rho in (0.1, 1e-2, 1e-3, 3e-4, 1e-4):
            rv = np.where(u - l < 1e-4, 1e3 * rho, rho)
            K = Pm + 1e-6 * np.eye(Pm.shape[0]) + A.T @ (rv[:, None] * A)
            bs = [rng.standard_normal(K.shape[0]) for _ in range(4)]
            out = ["b=%d rho %.0e" % (b, rho)]
            sols = {k: fused_solver(k)(G, Vu, D, E, c, 1e-6, inst.A, rv, Rdiag, True) for k in ("nat", "rev", "small")}
            for go in ("nat", "rev"):
                for mo in ("nat", "rev"):
                    sols["M" + go[0] + mo[0]] = minv_solver(True, go, mo)(G, Vu, D, E, c, 1e-6, inst.A, rv, Rdiag, True)
            class DG:
                def __init__(s): s.Ki = F.gj_fused(K.astype(f)).astype(f)
                def __call__(s, bb): return (s.Ki @ bb.astype(f)).astype(np.float64)
            sols["dense"] = DG()
            for k, slv in sols.items():
                be = max(np.linalg.norm(K @ slv(bb) - bb) / np.linalg.norm(bb) for bb in bs)
                out.append("%s %.2g" % (k, be))
            print("  ".join(out), flush=True)

