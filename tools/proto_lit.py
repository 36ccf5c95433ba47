"""Numpy prototype of the literal-QP linear solve through the per-step wrench
space -- an experiment / derivation check, not product code.

OSQP's reduced KKT matrix for the literal 12N-variable SRBD QP is
    K = P~ + sigma I + A~' diag(rho) A~ = D [c (Vu' G Vu + R) + sigma D^-2 + A' E rho E A] D
with Vu = I_N (x) Bb (Bb: rows omega, v of B_d, 6 x 12; the forces enter the
dynamics only through the per-step wrench increment w_j = Bb u_j) and
G = K0 (x) Qb + K2 (x) Te (6N x 6N).  With W0 = c R + sigma D^-2 + A'E rho E A
(block-diagonal, 3 x 3 per (step, leg)), U = Vu W0^-1 Vu' (6 x 6 per step),
U = L L' and S = I + L' (cG) L:
    K^-1 b = D^-1 (a - W0^-1 Vu' T Vu a),  a = W0^-1 D^-1 b,
    T = (I + cG U)^-1 cG = (cG) L S^-1 L^-1           (symmetric).
This script runs OSQP's algorithm (the oracle's restatement, oracle/admm.c)
with that solve, in float64 and with every solve-side quantity rounded to
float32, against oracle_lib.admm_solve on the same instances.

    python tools/proto_lit.py [count] [N] [gait]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402
from srbd_ref import Instance, np_build  # noqa: E402

from quadrupedal_loco_amd import srbd  # noqa: E402


def k0k2(N):
    K0 = np.zeros((N, N))
    K2 = np.zeros((N, N))
    for j in range(N):
        for k in range(N):
            m = max(j, k)
            K0[j, k] = N - m
            K2[j, k] = sum((i - j) * (i - k) for i in range(m, N))
    return K0, K2


def wrench_model(x0, ft, N, dt=0.0025, mass=12.0, inertia=O.GO1_INERTIA, q_w=O.Q_W):
    yaw = float(x0[2])
    c, s = np.cos(yaw), np.sin(yaw)
    R = np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]])
    I = np.asarray(inertia, np.float64).reshape(3, 3)
    Iw_inv = np.linalg.inv(R @ I @ R.T)
    Bb = np.zeros((6, 12))
    for l in range(4):
        r = np.asarray(ft[3 * l:3 * l + 3], np.float64)
        sk = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
        Bb[0:3, 3 * l:3 * l + 3] = dt * Iw_inv @ sk
        Bb[3:6, 3 * l:3 * l + 3] = dt * np.eye(3) / mass
    q2 = 2.0 * np.asarray(q_w, np.float64)
    Qb = np.diag(q2[6:12])
    Te = np.zeros((6, 6))
    Te[0:3, 0:3] = dt * dt * R.T @ np.diag(q2[0:3]) @ R
    Te[3:6, 3:6] = dt * dt * np.diag(q2[3:6])
    K0, K2 = k0k2(N)
    G = np.kron(K0, Qb) + np.kron(K2, Te)
    Vu = np.kron(np.eye(N), Bb)
    return G, Vu


def ruiz(P, q, A, iters=10):
    n, m = P.shape[0], A.shape[0]
    P, q, A = P.copy(), q.copy(), A.copy()
    D, E, c = np.ones(n), np.ones(m), 1.0

    def lim(v):
        v = np.where(v < 1e-4, 1.0, v)
        return np.minimum(v, 1e4)
    for _ in range(iters):
        Dt = lim(np.maximum(np.abs(P).max(0), np.abs(A).max(0)))
        Et = lim(np.abs(A).max(1))
        Dt, Et = 1 / np.sqrt(Dt), 1 / np.sqrt(Et)
        P = P * Dt[:, None] * Dt[None, :]
        A = A * Et[:, None] * Dt[None, :]
        q = q * Dt
        D, E = D * Dt, E * Et
        mean = np.abs(P).max(0).mean()
        qn = lim(np.array([np.abs(q).max()]))[0]
        ct = 1.0 / lim(np.array([max(mean, qn)]))[0]
        P, q, c = P * ct, q * ct, c * ct
    return P, q, A, D, E, c


class WrenchSolve:
    """K^-1 through the wrench space; f32=True rounds every stored quantity
    and every step of the solve to float32 (the kernel's arithmetic)."""

    def __init__(self, G, Vu, D, E, c, sigma, Araw, rho_vec, Rdiag, f32):
        t = np.float32 if f32 else np.float64
        self.t = t
        N6 = G.shape[0]
        n = Vu.shape[1]
        # W0 = c R + sigma D^-2 + A' E rho E A (block diagonal 3 x 3)
        AE = Araw * E[:, None]
        W0 = np.diag(c * Rdiag + sigma / D ** 2) + AE.T @ (rho_vec[:, None] * AE)
        W0i = np.zeros_like(W0)
        for b in range(n // 3):
            sl = slice(3 * b, 3 * b + 3)
            W0i[sl, sl] = np.linalg.inv(W0[sl, sl].astype(t)).astype(np.float64)
        U = Vu @ W0i @ Vu.T
        L = np.zeros_like(U)
        for j in range(N6 // 6):
            sl = slice(6 * j, 6 * j + 6)
            L[sl, sl] = np.linalg.cholesky(U[sl, sl].astype(t)).astype(np.float64)
        Gc = (c * G).astype(t)
        S = np.eye(N6) + L.T @ Gc @ L
        Si = np.linalg.inv(S.astype(t))              # the kernel's Gauss-Jordan
        Li = np.zeros_like(L)
        for j in range(N6 // 6):
            sl = slice(6 * j, 6 * j + 6)
            Li[sl, sl] = np.linalg.inv(L[sl, sl].astype(t))
        T = ((Gc @ L).astype(t) @ Si).astype(t) @ Li.astype(t)
        self.T = T.astype(t)
        self.W0i = W0i.astype(t)
        self.Vu = Vu.astype(t)
        self.Dinv = (1.0 / D).astype(t)
        self.dense = np.linalg.inv(D[:, None] * (c * (Vu.T @ G @ Vu + np.diag(Rdiag)) + np.diag(sigma / D ** 2)
                                                 + AE.T @ (rho_vec[:, None] * AE)) * D[None, :])

    def __call__(self, b):
        t = self.t
        a = self.W0i @ (self.Dinv * b.astype(t))
        v = self.Vu @ a
        s = self.T @ v
        return (self.Dinv * (a - self.W0i @ (self.Vu.T @ s))).astype(np.float64)


def admm(inst, G, Vu, mode, st=None, max_iter=4000):
    """OSQP v0.6 algorithm (oracle/admm.c) with the chosen linear solve."""
    st = st or dict(rho=0.1, sigma=1e-6, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, ctm=25, tol=5.0)
    H, q0, A0, l0, u0 = inst.H, inst.g, inst.A, inst.lb, inst.ub
    n, m = H.shape[0], A0.shape[0]
    P, q, A, D, E, c = ruiz(H, q0, A0)
    l, u = l0 * E, u0 * E
    Rdiag = np.diag(H - Vu.T @ G @ Vu)
    rho, sigma, alpha = st["rho"], st["sigma"], st["alpha"]

    def rho_vec_of(rho):
        rv = np.where(u - l < 1e-4, 1e3 * rho, rho)
        return rv

    def factor(rho):
        rv = rho_vec_of(rho)
        if mode == "dense64":
            K = P + sigma * np.eye(n) + A.T @ (rv[:, None] * A)
            Ki = np.linalg.inv(K)
            return rv, (lambda b: Ki @ b)
        return rv, WrenchSolve(G, Vu, D, E, c, sigma, A0, rv, Rdiag, mode == "wrench32")

    rv, solve = factor(rho)
    x, z, y = np.zeros(n), np.zeros(m), np.zeros(m)
    status, rho_up = 1, 0
    it = 0
    for it in range(1, max_iter + 1):
        xt = solve(sigma * x - q + A.T @ (rv * z - y))
        zt = A @ xt
        xn = alpha * xt + (1 - alpha) * x
        zr = alpha * zt + (1 - alpha) * z
        zn = np.clip(zr + y / rv, l, u)
        y = y + rv * (zr - zn)
        x, z = xn, zn
        chk = it % st["ctm"] == 0
        rh = it % 100 == 0
        if chk or rh:
            Ax = A @ x
            Px = P @ x
            Aty = A.T @ y
            rp = Ax - z
            rd = q + Px + Aty
            pri = np.abs(rp / E).max()
            dua = np.abs(rd / D).max() / c
            if chk:
                ep = st["eps_abs"] + st["eps_rel"] * max(np.abs(z / E).max(), np.abs(Ax / E).max())
                ed = st["eps_abs"] + st["eps_rel"] / c * max(np.abs(q / D).max(), np.abs(Aty / D).max(),
                                                             np.abs(Px / D).max())
                if pri < ep and dua < ed:
                    status = 0
                    break
            if rh:
                pn = np.abs(rp).max() / (max(np.abs(z).max(), np.abs(Ax).max()) + 1e-30)
                dn = np.abs(rd).max() / (max(np.abs(q).max(), np.abs(Aty).max(), np.abs(Px).max()) + 1e-30)
                rn = min(max(rho * np.sqrt(pn / (dn + 1e-30)), 1e-6), 1e6)
                if rn > rho * st["tol"] or rn < rho / st["tol"]:
                    rho = rn
                    rho_up += 1
                    rv, solve = factor(rho)
    return D * x, it, status, rho_up, solve


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    gait = sys.argv[3] if len(sys.argv) > 3 else "trot"
    x0, xr, ft, ct = srbd.generate(20261015, N, count, gait)
    sp = O.srbd_spec(N=N)
    worst = {}
    same = {}
    for b in range(count):
        inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
        G, Vu = wrench_model(x0[b], ft[b], N)
        Hn = np_build(x0[b], xr[b], ft[b], ct[b], N)[0]
        rel = np.abs(Vu.T @ G @ Vu + np.diag(np.diag(Hn - Vu.T @ G @ Vu)) - Hn).max() / np.abs(Hn).max()
        assert rel < 1e-10, rel  # H = Vu' G Vu + R exactly
        xo, info = inst.admm_full()
        res = [f"b={b:3d} oracle it {info.iters:4d} st {info.status}"]
        for mode in ("dense64", "wrench64", "wrench32"):
            xm, it, stt, ru, solve = admm(inst, G, Vu, mode)
            if mode != "dense64":
                # the solve itself against the dense inverse on a random rhs
                rb = np.random.default_rng(b).standard_normal(Vu.shape[1])
                ref = solve.dense @ rb
                err = np.abs(solve(rb) - ref).max() / np.abs(ref).max()
                worst[mode] = max(worst.get(mode, 0.0), err)
            du = np.abs(xm - xo).max()
            same[mode] = same.get(mode, 0) + int(it == info.iters)
            res.append(f"{mode} it {it:4d} st {stt} ru {ru} |du| {du:8.3g}")
        print("  ".join(res), flush=True)
    print("solve rel err (max over instances):", {k: "%.3g" % v for k, v in worst.items()})
    print("iterations equal to the oracle:", same, "of", count)


if __name__ == "__main__":
    main()
