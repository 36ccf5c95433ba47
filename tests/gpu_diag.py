"""Exploratory GPU run: solve a small batch and compare with the oracle."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
import torch

import oracle_lib as O
from quadrupedal_loco_amd import srbd
from srbd_ref import Instance

N = int(os.environ.get("N", 10))
B = int(os.environ.get("B", 64))
gait = os.environ.get("GAIT", "trot")
x0, xr, ft, ct = srbd.generate(20261015, N, B, gait)
dev = "cuda:0"
solver = srbd.BatchedConvexMpc(horizon=N)
t0 = time.time()
out = solver.solve(torch.from_numpy(x0).to(dev), torch.from_numpy(xr).to(dev),
                   torch.from_numpy(ft).to(dev), torch.from_numpy(ct).to(dev), full=True)
torch.cuda.synchronize()
print("gpu solve %.3f s" % (time.time() - t0))
u = out.u.cpu().numpy().astype(np.float64)
st = out.status.cpu().numpy()
it = out.iters.cpu().numpy()
ru = out.rho_updates.cpu().numpy()
sp = O.srbd_spec(N=N)
np.set_printoptions(precision=4, suppress=True, linewidth=200)
for b in range(min(B, 12)):
    inst = Instance(sp, x0[b], xr[b], ft[b], ct[b])
    xe, ste, ite = inst.exact()
    xa, info = inst.admm_reduced()
    fe = inst.obj(xe)
    print("b=%d status %d iters %d rho_upd %d | ref-reduced iters %d rho_upd %d | "
          "obj gpu %.6f ref %.6f exact %.6f | du0 vs ref %.4f vs exact %.4f viol %.2e"
          % (b, st[b], it[b], ru[b], info.iters, info.rho_updates, inst.obj(u[b]),
             inst.obj(xa), fe, np.abs(u[b][:12] - xa[:12]).max(),
             np.abs(u[b][:12] - xe[:12]).max(), inst.violation(u[b])))
