"""Measurement for SURVEY.md §8f row 4 (batched leg kinematics): one JSON line
per kernel with legs/s, the HBM roofline of the kernel and the CPU
restatement timed beside it.

    python tools/bench_kin.py [--legs N] [--steps K] [--warmup W]

Workload: N legs (default 4M = 1M robots x 4 legs, resident in HBM before the
timed region), world frame (servo.cpp:734-741 / :1038-1051 call the _g forms).
  fk: qloco_leg_fk  (Forward_kinematics_g + Jacobian_kin)
  ik: qloco_leg_ik  (Inverse_kinematics_g from q_target + U(-0.05, 0.05))
Algorithmic HBM bytes per leg (fp64 rows, int32 leg flag):
  fk: in q 24 + leg 4 + body_p 24 + body_r 24 = 76, out pos 24 + J 72 = 96 -> 172 B
  ik: in pos_des 24 + q_ini 24 + leg 4 + body 48 = 100,
      out q 24 + pos 24 + J 72 + updates 4 = 124 -> 224 B
Peak HBM 8.0 TB/s (MI355X_MICROARCH.md).  cpu_baseline: oracle/kinematics.c
batch drivers, 1 thread, on a bounded sample.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0
BYTES = {"fk": 172, "ik": 224}


def _traffic(kind, n):
    """measured HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, separate
    rocprofv3 passes) when profiled at this size (profiles/traffic_leg_*_4m.json)"""
    f = os.path.join(ROOT, "profiles", "traffic_leg_%s_4m.json" % kind)
    if n != 1 << 22 or not os.path.exists(f):
        return None
    with open(f) as fh:
        return json.load(fh).get("hbm_bytes_per_launch")


def inputs(n, seed=11):
    rng = np.random.default_rng(seed)
    q = np.stack([rng.uniform(-0.5, 0.5, n), rng.uniform(0.4, 1.4, n), rng.uniform(-2.2, -1.0, n)], 1)
    bp = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(0.27, 0.33, n)], 1)
    br = np.stack([rng.uniform(-0.2, 0.2, n), rng.uniform(-0.2, 0.2, n), rng.uniform(-3, 3, n)], 1)
    leg = (np.arange(n) % 4).astype(np.int32)
    dq = rng.uniform(-0.05, 0.05, (n, 3))
    return q, bp, br, leg, dq


def cpu_baseline(kind, q, bp, br, leg, pos_des, q_ini, budget_s=3.0):
    import oracle_lib as O
    L = O.lib()
    n = 1024
    while True:
        pos = np.zeros((n, 3))
        J = np.zeros((n, 9))
        t0 = time.perf_counter()
        if kind == "fk":
            L.qo_leg_fk_batch(n, q.ctypes.data, leg.ctypes.data, bp.ctypes.data, br.ctypes.data,
                              pos.ctypes.data, J.ctypes.data)
        else:
            qq = np.zeros((n, 3))
            upd = np.zeros(n, np.int32)
            L.qo_leg_ik_batch(n, pos_des.ctypes.data, q_ini.ctypes.data, leg.ctypes.data,
                              bp.ctypes.data, br.ctypes.data, qq.ctypes.data, pos.ctypes.data,
                              J.ctypes.data, upd.ctypes.data)
        dt = time.perf_counter() - t0
        if dt > budget_s / 4 or 2 * n > q.shape[0]:
            return n / dt, n
        n *= 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", type=int, default=4 << 20)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import torch
    from quadrupedal_loco_amd import kin
    n = args.legs
    q, bp, br, leg, dq = inputs(n)
    dev = torch.device("cuda:0")
    tq, tbp, tbr = (torch.from_numpy(a).to(dev) for a in (q, bp, br))
    tleg = torch.from_numpy(leg).to(dev)
    pos_des, _ = kin.leg_fk(tq, tleg, tbp, tbr)
    q_ini = tq + torch.from_numpy(dq).to(dev)
    torch.cuda.synchronize()
    for kind in ("fk", "ik"):
        def step():
            if kind == "fk":
                return kin.leg_fk(tq, tleg, tbp, tbr)
            return kin.leg_ik(pos_des, q_ini, tleg, tbp, tbr)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            out = step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        achieved = BYTES[kind] * n / (ms * 1e-3) / 1e9
        line = {"metric": "Go1 leg %s evaluations/sec (world frame, fp64)" %
                          ("FK_g + Jacobian" if kind == "fk" else "IK_g damped Newton"),
                "value": n / (ms * 1e-3), "unit": "legs/s", "n_gpus": 1, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
                "dtype": "f64", "data": "synthetic",
                "config": {"workload": "%s, %d legs (%d robots x 4)" % (kind, n, n // 4)},
                "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                             "algorithmic_bytes_per_leg": BYTES[kind],
                             "traffic": _traffic(kind, n)}}
        if kind == "ik":
            upd = out[3]
            line["newton_updates_mean"] = float(upd.float().mean().item())
        if not args.no_cpu_baseline:
            qh = q_ini.cpu().numpy()
            ph = pos_des.cpu().numpy()
            v, sample = cpu_baseline(kind, q, bp, br, leg, ph, qh)
            line["cpu_baseline"] = {"value": v, "unit": "legs/s", "cores": 1, "kind": "port",
                                    "sample": "%d legs, oracle/kinematics.c batch driver" % sample}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
