"""Where the headline's SIMD tail goes if the first pass is iteration-capped
(VERDICT r5 item 4).  For the literal N = 10 trot batch (B = 4096):
  - the full launch (time, iteration histogram);
  - the same launch capped at C iterations (max_iter = C: the pass-1 cost of
    a capped first pass, without its checkpoint writes);
  - the subset of instances still running at C, launched alone in full and
    capped at C: their difference estimates the resume pass (its setup and
    first C iterations excluded, its checkpoint reload not modelled).
    python tools/tail_probe.py [B] [REPS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from quadrupedal_loco_amd import _lib, srbd

if os.environ.get("QLOCO_LIB"):
    _lib.LIB_PATH = os.environ["QLOCO_LIB"]

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
N = int(os.environ.get("N", 10))
GAIT = os.environ.get("GAIT", "trot")
dev = torch.device("cuda:0")
host = srbd.generate(20261015, N, B, GAIT)


def timed(args, **kw):
    s = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=1, **kw)
    n = args[0].shape[0]
    out = s.alloc_outputs(n, dev)
    for _ in range(5):
        s.solve(*args, out=out)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(REPS + 1)]
    ev[0].record()
    for k in range(REPS):
        s.solve(*args, out=out)
        ev[k + 1].record()
    torch.cuda.synchronize()
    per = np.array([ev[k].elapsed_time(ev[k + 1]) for k in range(REPS)]) * 1e3
    return float(np.median(per)), out


full = [torch.from_numpy(a).to(dev) for a in host]
# warm the clocks
timed(full)
t_full, out = timed(full)
it = out.iters.cpu().numpy()
print("B=%d N=%d %s literal: full %.1f us  iters mean %.1f" % (B, N, GAIT, t_full, it.mean()))
vals, cnts = np.unique(it, return_counts=True)
print("  iteration histogram: " + ", ".join("%d:%d" % (v, c) for v, c in zip(vals, cnts)))
for cap in (50, 75, 100, 125, 150, 175, 200):
    t_cap, _ = timed(full, max_iter=cap)
    sel = np.nonzero(it > cap)[0]
    line = "  cap %3d: pass-1 %.1f us  unfinished %4d (%.1f%%)" % (cap, t_cap, len(sel), 100.0 * len(sel) / B)
    if len(sel):
        sub = [torch.from_numpy(np.ascontiguousarray(a[sel])).to(dev) for a in host]
        t_sf, _ = timed(sub)
        t_sc, _ = timed(sub, max_iter=cap)
        rem = it[sel] - cap
        line += "  subset full %.1f capped %.1f -> resume est %.1f us (remaining iters mean %.0f max %d)" % (
            t_sf, t_sc, t_sf - t_sc, rem.mean(), rem.max())
        line += "  => total est %.1f us" % (t_cap + t_sf - t_sc)
    print(line, flush=True)
