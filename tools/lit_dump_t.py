"""Check the literal wrench-space kernels' T = (I + cG U)^-1 cG against a
float64 computation (development aid).

    python tools/lit_dump_t.py build        (CPU: the variant library
                                             tools/_var/dumpt, product source
                                             + one write-out of T's rows)
    python tools/lit_dump_t.py run N gait id [rho ...]   (GPU)

The variant writes each lane's row of T after the first factorisation into
the caller's `warm` buffer (warm_start = 0, so the product never reads it);
a fixed rho (adaptive rho off, max_iter 0) picks the factorisation.  The
reference is tools/proto_lit.py's float64 WrenchSolve on the same instance
with numpy's Ruiz scaling (float32 vs float64 scaling: ~1e-6 relative), so
an indexing or sign bug shows up as O(1) and precision loss as the size of
the relative error."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "tests"))

PATCH = ("qloco_srbd_lit.hip:    bool refactor = false;\n=>"
         "    bool refactor = false;\n"
         "    if (a.warm && a.warm_start == 0 && S.sc[wv].rho_updates == 0) {\n"
         "      float *dst = a.warm + ((int64_t)b * (64 * W) + threadIdx.x) * (60 * W);\n"
         "#pragma unroll\n"
         "      for (int c = 0; c < 60 * W; ++c) dst[c] = T.k[c];\n"
         "    }\n")


def build():
    import variant_lib
    variant_lib.main(["dumpt", "--patch", PATCH])


def run(N, gait, idx, rhos):
    import torch
    from quadrupedal_loco_amd import _lib, srbd
    _lib.LIB_PATH = os.path.join(HERE, "_var", "dumpt", "libqloco.so")
    import proto_lit as P
    import oracle_lib as O
    from srbd_ref import Instance
    W = 1 if N <= 10 else 2
    H = N if W == 1 else (N + 1) // 2
    x0, xr, ft, ct = srbd.generate(20261015, N, idx + 1, gait)
    x0, xr, ft, ct = (np.ascontiguousarray(a[idx:idx + 1]) for a in (x0, xr, ft, ct))
    dev = torch.device("cuda:0")
    # QSET: one of srbd.REFERENCE_WEIGHTS (default: the Go1 weights)
    qs = os.environ.get("QSET")
    q_w, r_w = srbd.REFERENCE_WEIGHTS[qs] if qs else (O.Q_W, O.R_W)
    wkw = dict(q_weights=q_w, r_weights=r_w) if qs else {}
    inst = Instance(O.srbd_spec(N=N, q_w=q_w, r_w=r_w), x0[0], xr[0], ft[0], ct[0])
    G, Vu = P.wrench_model(x0[0], ft[0], N, q_w=q_w)
    Pm, q, A, D, E, c = P.ruiz(inst.H, inst.g, inst.A)
    l, u = inst.lb * E, inst.ub * E
    Rdiag = np.diag(inst.H - Vu.T @ G @ Vu)
    # kernel row / column (wave w, lane l) -> global wrench index
    glob = {}
    for w in range(W):
        nw = H if w == 0 else N - H
        for ln in range(6 * nw):
            glob[(w, ln)] = 6 * (w * H + ln // 6) + ln % 6
    for rho in rhos:
        s = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=1, rho=rho, adaptive_rho=0, max_iter=0, **wkw)
        dump = torch.zeros((64 * W, 60 * W), dtype=torch.float32, device=dev)
        s.solve(*(torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)), warm=dump)
        torch.cuda.synchronize()
        Tk = dump.cpu().numpy().astype(np.float64)
        rv = np.where(u - l < 1e-4, 1e3 * rho, rho)
        ref = P.WrenchSolve(G, Vu, D, E, c, 1e-6, inst.A, rv, Rdiag, False).T
        Tg = np.zeros_like(ref)
        for (w, ln), gi in glob.items():
            for (w2, l2), gj in glob.items():
                Tg[gi, gj] = Tk[64 * w + ln, 60 * w2 + l2]
        err = np.abs(Tg - ref).max() / np.abs(ref).max()
        sym = np.abs(Tg - Tg.T).max() / np.abs(ref).max()
        # the solve it implies, on a random rhs (relative to the dense inverse)
        print("N=%d %s id %d rho %.0e: |T - T64| / |T64| %.3g  asym %.3g  |T64| %.3g" % (
            N, gait, idx, rho, err, sym, np.abs(ref).max()), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]), sys.argv[3], int(sys.argv[4]),
            [float(r) for r in sys.argv[5:]] or [0.1, 1e-2, 1e-3, 3e-4, 1e-4])
