"""Phase timing of the literal N <= 10 kernel (development aid).

    python tools/lit_phase.py build          # CPU: tools/_var/litphase/libqloco.so
    python tools/lit_phase.py run [B ...]    # GPU: per-phase s_memrealtime (10 ns ticks)

The variant stamps s_memrealtime at the phase boundaries of srbd_lit_one and
lane 0 writes the (float) tick counts over u[b, 0:8]: [0] inputs + model +
gradient, [1] Ruiz, [2] factorisation setup (W0, U, Cholesky, S rows; summed
over refactorisations), [3] S^-1, [4] Z and T, [5] start -> end of ADMM,
[6] residual checks, [7] number of factorisations."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

F = "qloco_srbd_lit.hip"
PATCHES = [
    ("  const int nvar = 12 * N, nw = 6 * N;\n",
     "  const int nvar = 12 * N, nw = 6 * N;\n  const long long tq0 = __builtin_amdgcn_s_memrealtime();\n"
     "  long long tqa = tq0, tqb = tq0, tf0 = 0, tf1 = 0, tf2 = 0;\n  float tph[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n"),
    ("  // ---------------- 5. modified Ruiz equilibration",
     "  tqa = __builtin_amdgcn_s_memrealtime(); tph[0] = (float)(tqa - tq0);\n"
     "  // ---------------- 5. modified Ruiz equilibration"),
    ("  const float cinv = 1.0f / cs;\n",
     "  const float cinv = 1.0f / cs;\n  tqb = __builtin_amdgcn_s_memrealtime(); tph[1] = (float)(tqb - tqa);\n"),
    ("      // opaque per factorisation: nothing derived",
     "      tf0 = __builtin_amdgcn_s_memrealtime(); tph[7] += 1.0f;\n"
     "      // opaque per factorisation: nothing derived"),
    ("      // S^-1 in place\n      lit_invert(S, lane, nw, T);\n",
     "      tf1 = __builtin_amdgcn_s_memrealtime(); tph[2] += (float)(tf1 - tf0);\n"
     "      lit_invert(S, lane, nw, T);\n"
     "      tf2 = __builtin_amdgcn_s_memrealtime(); tph[3] += (float)(tf2 - tf1);\n"),
    ("    bool refactor = false;\n",
     "    tph[4] += (float)(__builtin_amdgcn_s_memrealtime() - tf2);\n    bool refactor = false;\n"),
    ("      residuals(o, r, do_rho);\n",
     "      const long long tr0 = __builtin_amdgcn_s_memrealtime();\n      residuals(o, r, do_rho);\n"
     "      tph[6] += (float)(__builtin_amdgcn_s_memrealtime() - tr0);\n"),
    ("  // ---------------- 7. outputs",
     "  tph[5] = (float)(__builtin_amdgcn_s_memrealtime() - tqb);\n  // ---------------- 7. outputs"),
    ("  if (lane == 0) {\n    if (a.status) a.status[b] = status;",
     "  if (lane == 0 && a.u) {\n#pragma unroll\n    for (int k = 0; k < 8; ++k) a.u[b * 12 * N + k] = tph[k];\n  }\n"
     "  if (lane == 0) {\n    if (a.status) a.status[b] = status;"),
]


def build():
    import variant_lib
    argv = ["litphase"]
    for old, new in PATCHES:
        argv += ["--patch", "%s:%s=>%s" % (F, old, new)]
    variant_lib.main(argv)


def run(batches):
    import numpy as np
    import torch
    from quadrupedal_loco_amd import _lib, srbd
    _lib.LIB_PATH = os.path.join(HERE, "_var", "litphase", "libqloco.so")
    N = 10
    dev = torch.device("cuda:0")
    names = ["model+grad", "ruiz", "fac:W0..S", "fac:S^-1", "fac:Z,T", "admm total", "checks", "n_fac"]
    for B in batches:
        x0, xr, ft, ct = srbd.generate(20261015, N, B, "trot")
        args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
        s = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=1)
        for _ in range(2):
            out = s.solve(*args, full=True)
        torch.cuda.synchronize()
        t = out.u.cpu().numpy().reshape(B, -1)[:, :8]
        it = out.iters.cpu().numpy()
        print("B=%d iters mean %.1f" % (B, it.mean()))
        for k, nm in enumerate(names):
            v = t[:, k] * (0.01 if k < 7 else 1.0)
            print("  %-11s mean %8.2f  p50 %8.2f  max %8.2f %s" % (nm, v.mean(), np.median(v), v.max(),
                                                                "us" if k < 7 else ""))
        per_it = (t[:, 5] - t[:, 2] - t[:, 3] - t[:, 4] - t[:, 6]) * 0.01 / np.maximum(it, 1)
        print("  per ADMM iteration (total - factorisations - checks) / iters: mean %.3f us" % per_it.mean())


if __name__ == "__main__":
    if sys.argv[1] == "build":
        sys.path.insert(0, HERE)
        build()
    else:
        run([int(b) for b in sys.argv[2:]] or [256, 1024, 4096])
