"""Diagnostic: the literal mode's non-finite ends at eps 1e-6 -- rho carried in
the persistent record after a fixed number of iterations, for the instances
that end NaN and for normal ones.  python tools/literal_rho_diag.py (GPU)"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import torch  # noqa: E402

from quadrupedal_loco_amd import srbd  # noqa: E402

dev = torch.device("cuda:0")
N, B = 10, 24
x0, xr, ft, ct = srbd.generate(20261015, N, B, "trot")
args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
pick = [15, 16, 21, 0, 1]
for mi in (50, 75, 100, 125, 150, 175, 200, 225, 250, 300):
    s = srbd.PersistentConvexMpc(B, dev, horizon=N, literal_full_qp=1, eps_abs=1e-6, eps_rel=1e-6,
                                 max_iter=mi)
    out = s.solve(*args, full=True)
    torch.cuda.synchronize()
    rec = s.record.cpu().numpy()
    u = out.u.cpu().numpy()
    print("max_iter %4d" % mi, " ".join(
        "b%d:st%d ru%d rho %.3g |u|max %.3g" % (b, int(out.status[b]), int(out.rho_updates[b]),
                                               rec[b, 100 * N], np.abs(u[b]).max())
        for b in pick), flush=True)
