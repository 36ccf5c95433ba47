"""Wall time per headline step with 0 / 1 / 2 / 3 timing events recorded per
step (bench.py records ev_s / ev_k / ev_e around every solve).  Usage:
    python tools/event_overhead.py [B] [STEPS]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from quadrupedal_loco_amd import srbd

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
N = 10
dev = torch.device("cuda:0")
x0, xr, ft, ct = [torch.from_numpy(a).to(dev) for a in srbd.generate(20261015, N, B, "trot")]
legs = srbd.max_stance_legs(ct.cpu().numpy(), N)
s = srbd.BatchedConvexMpc(horizon=N)
out = s.alloc_outputs(B, dev)
stream = torch.cuda.current_stream(dev)
for _ in range(20):
    s.solve(x0, xr, ft, ct, out=out, max_legs=legs, stream=stream.cuda_stream)
torch.cuda.synchronize(dev)
for rep in range(3):
    for nev in (0, 1, 2, 3):
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(nev)] for _ in range(K)]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(K):
            if nev >= 1:
                evs[i][0].record(stream)
            s.solve(x0, xr, ft, ct, out=out, max_legs=legs, stream=stream.cuda_stream)
            for e in evs[i][1:]:
                e.record(stream)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) / K * 1e3
        kern = (sum(evs[i][0].elapsed_time(evs[i][1]) for i in range(K)) / K) if nev >= 2 else float("nan")
        print("rep %d events/step %d  wall %.4f ms/step  kernel(ev) %.4f ms" % (rep, nev, wall, kern), flush=True)
