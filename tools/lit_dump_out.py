"""Write one literal batch's outputs (u, iters, status, rho_updates, obj) to
an .npz for a bit-identity comparison of two library builds (QLOCO_LIB).
    [QLOCO_LIB=...] python tools/lit_dump_out.py OUT.npz N B gait"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from quadrupedal_loco_amd import _lib, srbd

if os.environ.get("QLOCO_LIB"):
    _lib.LIB_PATH = os.environ["QLOCO_LIB"]
out, N, B, gait = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
x0, xr, ft, ct = srbd.generate(20261015, N, B, gait)
dev = torch.device("cuda:0")
r = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=1).solve(
    *(torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)), full=True)
torch.cuda.synchronize()
np.savez(out, **{k: getattr(r, k).cpu().numpy() for k in ("u", "iters", "status", "rho_updates", "obj")})
