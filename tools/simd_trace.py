"""Per-instance placement and wall clock of the SRBD one-wave kernel
(development tool).  Needs a variant library built with -DQLOCO_TRACE_SIMD:
    python tools/variant_lib.py trace -DQLOCO_TRACE_SIMD [other -D flags]
    QLOCO_LIB=tools/_var/trace/libqloco.so python tools/simd_trace.py [B] [out.npz]
Each instance records HW_ID (CU / SIMD / SE), XCC_ID and s_memrealtime
(100 MHz) at its start and end.  Prints the spread of per-SIMD finish times
and what the SIMDs that finish last were running -- the load-balance
picture behind the kernel time at small batches.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedal_loco_amd import _lib, srbd  # noqa: E402

_lib.LIB_PATH = os.environ["QLOCO_LIB"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(os.environ.get("N", 10))
GAIT = os.environ.get("GAIT", "trot")
x0, xr, ft, ct = srbd.generate(20261015, N, B, GAIT)
dev = torch.device("cuda:0")
args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
s = srbd.BatchedConvexMpc(horizon=N)
out = s.alloc_outputs(B, dev)
legs = srbd.max_stance_legs(ct, N)
for _ in range(3):
    s.solve(*args, out=out, max_legs=legs)
torch.cuda.synchronize()
buf = np.zeros(4 * B, np.uint32)
dl = C.CDLL(_lib.LIB_PATH)
rc = dl.qloco_trace_read(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.size))
if rc != 0:
    raise SystemExit("qloco_trace_read failed %d" % rc)
tr = buf.reshape(B, 4).astype(np.int64)
hw, xcc = tr[:, 0], tr[:, 1] & 15
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
t0 = (tr[:, 2] - tr[:, 2].min()) * 10.0  # ns (100 MHz)
t1 = (tr[:, 3] - tr[:, 2].min()) * 10.0
key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
it = out.iters.cpu().numpy()
ru = out.rho_updates.cpu().numpy()
uk, inv = np.unique(key, return_inverse=True)
nk = len(uk)
cnt = np.bincount(inv, minlength=nk)
fin = np.zeros(nk)
np.maximum.at(fin, inv, t1)
work = np.bincount(inv, weights=it.astype(np.float64), minlength=nk)
inv_w = np.bincount(inv, weights=1.0 + ru, minlength=nk)
print("B=%d  SIMDs used %d  instances per SIMD min/median/max %d/%d/%d" % (
    B, nk, cnt.min(), int(np.median(cnt)), cnt.max()))
print("span %.1f us; per-SIMD finish time p10/p50/p90/max %.1f/%.1f/%.1f/%.1f us" % (
    t1.max() / 1e3, *(np.percentile(fin, [10, 50, 90, 100]) / 1e3)))
print("per-SIMD iteration sum mean %.0f p90 %.0f max %.0f; inverses mean %.2f max %.0f" % (
    work.mean(), np.percentile(work, 90), work.max(), inv_w.mean(), inv_w.max()))
dur = t1 - t0
print("instance wall time vs iterations (mean us): " + ", ".join(
    "%d:%.1f" % (k, dur[it == k].mean() / 1e3) for k in np.unique(it)))
last = np.argsort(fin)[-8:]
for k in last:
    m = inv == k
    print("  SIMD %5d finish %.1f us: %d instances, iterations %s, rho updates %s, starts %s us" % (
        uk[k], fin[k] / 1e3, m.sum(), it[m].tolist(), ru[m].tolist(),
        [round(v / 1e3, 1) for v in t0[m]]))
c = np.corrcoef(work, fin)[0, 1]
print("corr(per-SIMD iteration sum, finish time) %.3f" % c)
if len(sys.argv) > 2:
    np.savez(sys.argv[2], key=key, t0=t0, t1=t1, iters=it, rho_updates=ru)
