"""Measurement for SURVEY.md §8f row 1 / §8a rows a8-a11 (batched Go1 force
distribution QP, Dynamiccclass::force_distribution + force_opt, servo.cpp:
1224-1228): one JSON line with QP solves/s, the fp64 compute roofline and the
C restatement timed beside it.

    python tools/bench_qp.py [--robots B] [--steps K] [--warmup W]

Workload: B robots (default 65536), one qloco_force_qp_solve launch per step
(force_distribution heuristic + G/g0/CE/CI build + quirk-compatible
Goldfarb-Idnani, n = 12, p = 12 (6 live or 0), m = 24, fp64), inputs
resident in HBM (tests/cases.force_inputs: mixed modes 101/102/103 and
right_support 0/1/2), member state (grf_opt = F_prev, F_leg_ref) carried
between steps exactly as the servo's Dynamiccclass.
Algorithmic fp64 flops per solve (EiQuadProg.cpp structure, K = measured
active-set iterations): build A'A 2*6*12*12 = 1728, LLT n^3/3 = 576,
J = L^-T n^3/3 = 576, x0 2n^2 = 288, per iteration 2nm + 10n^2 = 2016.
Peak: 78.6 TFLOP/s fp64 vector (MI355X spec sheet; MICROARCH.md lists no
fp64 figure).  The kernel is latency-bound (one QP per 16-lane group, short
dependent chains), so the fraction is small by construction.
cpu_baseline: oracle/force_qp.c qo_force_batch, 1 thread, bounded sample.
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

PEAK_FP64_TFLOPS = 78.6
# algorithmic HBM bytes per robot: inputs com_des 3, leg_des 12, F_force_des 6,
# rfoot / lfoot 3 + 3, base_p 3, feet_p 12, FT_total_des 6, y_coef 1 doubles
# + mode, right_support int32 + the member state read (F_leg_ref, grf_opt: 24
# doubles) = 592 B; outputs grf_opt, F_leg_guess, F_leg_ref (36 doubles) +
# qp_solution, status, iters (int32) = 300 B
ALG_BYTES = 592 + 300
N, M = 12, 24


def flops(iters):
    return 1728 + N ** 3 / 3 + N ** 3 / 3 + 2 * N * N + iters * (2 * N * M + 10 * N * N)


def _traffic(B):
    f = os.path.join(ROOT, "profiles", "traffic_force_qp_b%d.json" % B)
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        return json.load(fh).get("hbm_bytes_per_launch_raw")


def cpu_baseline(inp, budget_s=6.0):
    import oracle_lib as O
    L = O.lib()
    L.qo_force_batch.argtypes = [C.c_int64, C.c_void_p, C.POINTER(O.ForceParams)] + [C.c_void_p] * 12
    prm = O.ForceParams()
    L.qo_force_params_default(C.byref(prm))
    n = 4096
    states = (O.DynState * n)()
    for s in states:
        L.qo_dyn_init(C.byref(s))
    arr = {k: np.ascontiguousarray(v[:n]) for k, v in inp.items()}
    out = np.zeros((n, 12))
    solves, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        L.qo_force_batch(n, C.cast(states, C.c_void_p), C.byref(prm),
                         *[arr[k].ctypes.data for k in ("com_des", "leg_des", "F_force_des",
                                                        "rfoot_des", "lfoot_des", "base_p",
                                                        "feet_p", "FT_total_des", "mode",
                                                        "right_support", "y_coef")],
                         out.ctypes.data)
        solves += n
    dt = time.perf_counter() - t0
    for s in states:
        L.qo_dyn_free(C.byref(s))
    return solves / dt, "%d robots x %d calls" % (n, solves // n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--order", choices=("given", "pattern", "iters"), default="given",
                    help="experiment: permute the robots on the host before timing -- grouped by "
                         "swing-leg pattern, or by pattern then by a first solve's iteration count")
    ap.add_argument("--ticks", type=int, default=1,
                    help="distinct input sets cycled over the steps (tests/cases.force_inputs, one rng "
                         "stream): with 1 every step re-solves the same inputs, so the grouping key (the "
                         "previous call's iteration count) predicts the next call exactly -- the best "
                         "case; with > 1 every call gets new inputs, as a servo tick does")
    ap.add_argument("--ungrouped", action="store_true",
                    help="the plain launch (qloco_force_qp_solve) instead of the grouped one")
    ap.add_argument("--servo", action="store_true",
                    help="time the whole servo force block (qloco_servo_force_block)")
    args = ap.parse_args()
    if args.servo:
        return servo_main(args)
    import torch
    if os.environ.get("QLOCO_LIB"):  # experimental variant (tools/variant_lib.py)
        from quadrupedal_loco_amd import _lib
        _lib.LIB_PATH = os.environ["QLOCO_LIB"]
    from cases import force_inputs
    from quadrupedal_loco_amd import qp
    B = args.robots
    dev = torch.device("cuda:0")
    inp = force_inputs(np.random.default_rng(3), B)
    if args.order != "given":
        m, rs = inp["mode"], inp["right_support"]
        pat = np.where(m == 102, np.where(rs == 0, 1, np.where(rs == 1, 2, 0)),
                       np.where(m == 101, np.where(rs == 0, 3, np.where(rs == 1, 4, 0)), 0))
        key = pat.astype(np.int64) * 1000
        if args.order == "iters":
            d0 = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in inp.items()}
            it0 = qp.ForceQP(batch=B, device=dev).step(**d0)["iters"].cpu().numpy()
            key = key + it0
        perm = np.argsort(key, kind="stable")
        inp = {k: v[perm] for k, v in inp.items()}
    sets = [{k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in inp.items()}]
    rng_t = np.random.default_rng(4)
    for _ in range(args.ticks - 1):
        sets.append({k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
                     for k, v in force_inputs(rng_t, B).items()})
    solver = qp.ForceQP(batch=B, device=dev, grouped=not args.ungrouped)
    for k in range(args.warmup):
        out = solver.step(**sets[k % len(sets)])
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ev[0].record(stream)
    for k in range(args.steps):
        out = solver.step(**sets[(args.warmup + k) % len(sets)])
        ev[k + 1].record(stream)
    torch.cuda.synchronize()
    per = np.array([ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)])
    ms = float(per.mean())
    iters = out["iters"].cpu().numpy()
    status = out["status"].cpu().numpy()
    f = float(flops(iters.astype(np.float64)).sum())
    achieved = f / (ms * 1e-3) / 1e12
    line = {"metric": "Go1 force-distribution QP solves/sec (Dynamiccclass force_distribution + "
                      "force_opt, EiQuadProg fp64)",
            "value": B / (ms * 1e-3), "unit": "solves/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms,
            "p99_batch_us": float(np.percentile(per, 99) * 1e3), "higher_is_better": True,
            "dtype": "f64", "data": "synthetic (tests/cases.force_inputs, seed 3)",
            "config": {"workload": "force QP, %d robots, modes 101/102/103, right_support 0/1/2%s%s%s" % (
                B, "" if args.order == "given" else ", host order: " + args.order,
                ", ungrouped launch" if args.ungrouped else ", grouped launch (pattern, previous iterations)",
                ", the same inputs every step" if args.ticks == 1 else
                ", %d distinct input sets cycled (new inputs every step)" % args.ticks)},
            "gi_iters_mean": float(iters.mean()), "status_ok_frac": float(np.mean(status == 0)),
            "roofline": {"bound": "valu-fp64", "achieved": achieved, "peak": PEAK_FP64_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / PEAK_FP64_TFLOPS,
                         "traffic": _traffic(B), "alg_bytes": ALG_BYTES * B,
                         "note": "fp64 VALU (no MFMA on this path); algorithmic flops per solve "
                                 "in the tool docstring; latency-bound active set"}}
    if not args.no_cpu_baseline:
        v, sample = cpu_baseline(inp)
        line["cpu_baseline"] = {"value": v, "unit": "solves/s", "cores": 1, "kind": "port",
                                "sample": sample + ", oracle/force_qp.c qo_force_batch"}
    print(json.dumps(line), flush=True)


def servo_main(args):
    """The go1 servo force block (servo.cpp:1052-1243): glue + force QP + the
    four legs' joint torques, one qloco_servo_force_block per step."""
    import torch
    import oracle_lib as O
    from quadrupedal_loco_amd.qp import ServoForceBlock, synth_servo_inputs
    B = args.robots
    dev = torch.device("cuda:0")
    sets = []
    for t in range(8):
        d = synth_servo_inputs(3, B, 100 + t)
        sets.append({k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()})
    blk = ServoForceBlock(B, dev)
    for k in range(args.warmup):
        blk.step(**sets[k % 8])
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ev[0].record(stream)
    for k in range(args.steps):
        blk.step(**sets[k % 8])
        ev[k + 1].record(stream)
    torch.cuda.synchronize()
    per = np.array([ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)])
    ms = float(per.mean())
    line = {"metric": "go1 servo force block ticks/sec (servo.cpp:1052-1243: glue + force QP + "
                      "joint torques, fp64)",
            "value": B / (ms * 1e-3), "unit": "robot-ticks/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms,
            "p99_batch_us": float(np.percentile(per, 99) * 1e3), "higher_is_better": True,
            "dtype": "f64", "data": "synthetic (quadrupedal_loco_amd.qp.synth_servo_inputs, 8 sets cycled)",
            "config": {"workload": "servo force block, %d robots" % B}}
    if not args.no_cpu_baseline:
        n = 4096
        orc = O.ServoOracle(n)
        L = O.lib()
        L.qo_servo_batch.argtypes = [C.c_int64, C.c_void_p, C.POINTER(O.ForceParams)] + [C.c_void_p] * 15
        d = {k: np.ascontiguousarray(v) for k, v in synth_servo_inputs(3, n, 100).items()}
        grf, tau = np.zeros((n, 12)), np.zeros((n, 12))
        keys = ("coma_des", "com_des", "rfoot_des", "lfoot_des", "body_p_des", "foot_des",
                "right_support", "gait_mode", "y_offset", "loop_count", "Jaco", "foot_rel_mea",
                "v_est_rel")
        calls, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 6.0:
            L.qo_servo_batch(n, C.cast(orc.states, C.c_void_p), C.byref(orc.prm),
                             *[d[k].ctypes.data for k in keys], grf.ctypes.data, tau.ctypes.data)
            calls += 1
        v = n * calls / (time.perf_counter() - t0)
        line["cpu_baseline"] = {"value": v, "unit": "robot-ticks/s", "cores": 1, "kind": "port",
                                "sample": "%d robots x %d ticks, oracle/servo_block.c qo_servo_batch"
                                          % (n, calls)}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
