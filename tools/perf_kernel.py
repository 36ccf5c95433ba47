"""Run one SRBD kernel configuration repeatedly (for rocprofv3 counter passes
and batch-size scans).  Usage: python tools/perf_kernel.py VARIANT [B] [REPS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from quadrupedal_loco_amd import _lib, srbd

if os.environ.get("QLOCO_LIB"):  # experimental variant (tools/variant_lib.py)
    _lib.LIB_PATH = os.environ["QLOCO_LIB"]

VARIANTS = {
    "default": {},
    "iter1": dict(max_iter=1, check_termination=0, adaptive_rho=0),
    "iter1s20": dict(max_iter=1, check_termination=0, adaptive_rho=0, scaling=20),
    "iter1s0": dict(max_iter=1, check_termination=0, adaptive_rho=0, scaling=0),
    # 150 iterations with 30 residual checks that never pass (eps 1e-12): check cost
    "chk5": dict(max_iter=150, check_termination=5, adaptive_rho=0, eps_abs=1e-12, eps_rel=1e-12),
    "iter150": dict(max_iter=150, check_termination=0, adaptive_rho=0),
    "iter150s0": dict(max_iter=150, check_termination=0, adaptive_rho=0, scaling=0),
    "iter0": dict(max_iter=0, check_termination=0, adaptive_rho=0),
    "iter0s0": dict(max_iter=0, check_termination=0, adaptive_rho=0, scaling=0),
    "rho25": dict(max_iter=150, eps_abs=1e-12, eps_rel=1e-12, adaptive_rho=1,
                  adaptive_rho_interval=25, adaptive_rho_tolerance=1.0),
}
name = sys.argv[1] if len(sys.argv) > 1 else "default"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
N = int(os.environ.get("N", 10))
GAIT = os.environ.get("GAIT", "trot")
x0, xr, ft, ct = srbd.generate(20261015, N, B, GAIT)
dev = torch.device("cuda:0")
args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
legs = srbd.max_stance_legs(ct, N)
LIT = int(os.environ.get("LITERAL", 0))  # 1: the literal 12N-variable QP
if LIT:
    legs = 4 * N
s = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=LIT, **VARIANTS[name])
out = s.alloc_outputs(B, dev)
for _ in range(2):
    s.solve(*args, out=out, max_legs=legs)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    s.solve(*args, out=out, max_legs=legs)
e1.record()
torch.cuda.synchronize()
it = out.iters.float()
print("%-10s %-6s%s N=%-2d %-8s B=%6d  %9.1f us/launch  iters mean %.1f p99 %d max %d  rho_updates mean %.2f max %d" % (
    os.path.basename(os.path.dirname(os.environ.get("QLOCO_LIB", "/prod/x"))), GAIT,
    " lit" if LIT else "", N, name, B,
    e0.elapsed_time(e1) / reps * 1e3, it.mean().item(), int(it.quantile(0.99).item()), int(it.max().item()),
    out.rho_updates.float().mean().item(), int(out.rho_updates.max().item())), flush=True)
