"""Measurement for SURVEY.md §8f rows 2-3 (batched rt_mpc_qp node tick): one
JSON line with robot-ticks/s, the HBM roofline of a tick and the C
restatement timed beside it.

    python tools/bench_rt.py [--robots B] [--steps K] [--warmup W] [--sets M]

Workload: B robots (default 65536), one qloco_rt_tick per step = the rt
node's 100 Hz loop body for every robot (gait_fast.cpp:505-735: callbacks,
interpolation, Foot_trajectory_solve_mod2, XGetSolution_Foot_rotation,
body_theta_mpc, /rtMPC/traj + /rt2nrt/state).  M message sets
(synth_messages for ticks 0..M-1) are generated on the host and resident in
HBM before the timed region; step t uses set t mod M.  W warm-up ticks
(default 150) run first so every robot is past the 1 s height-offset phase
and into foot generation + body MPC (count_in_rt_mpc > 100).
Algorithmic HBM bytes per robot-tick (fp64), with foot generation running
(the steady state): messages in 125 x 8 = 1000 and out 125 x 8 = 1000; the
live node state the reference's loop reads (interpolation knots 48, swing
foot arrays 108, footholds 12, _tx scan 27, _ts/_td 8, lift 4, foot
rotation 8, body-MPC record 32, misc 2 = 249 doubles + 7 ints) and writes
(interpolation outputs 72 + knot shifts 24 (every other tick), foot arrays
108, footholds 6, foot rotation 8, generator outputs 60, /rt2nrt 25, body
record 32 = 335 doubles + 7 ints) = 4728 B -> 6728 B per robot-tick.
Peak 8.0 TB/s (MI355X_MICROARCH.md).  `traffic` = measured HBM bytes per
tick (profiles/traffic_rt_tick_b65536.json, FETCH_SIZE / WRITE_SIZE passes).
cpu_baseline: oracle/rt_tick.c (qo_rt_tick_n), 1 thread, bounded sample.

    python tools/bench_rt.py --support [--robots B]

measures the slow planner's contact-phase flag instead (qloco_support_phase,
SURVEY.md §8f row 2): default 4M robots, algorithmic bytes per robot
_ts + _tx rows 2 x 27 x 8 + t_int, t_end 8 + bjxx, bjx1, right_support 12 =
452 B; cpu_baseline oracle/support_phase.c, 1 thread.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0
BYTES_PER_ROBOT_TICK = 1000 + 1000 + (249 + 335) * 8 + 2 * 7 * 4
SEED = 20261016


def _traffic(B):
    """measured HBM bytes per tick (raw FETCH_SIZE + WRITE_SIZE) if profiled at this B"""
    f = os.path.join(ROOT, "profiles", "traffic_rt_tick_b%d.json" % B)
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        return json.load(fh).get("hbm_bytes_per_tick_raw")


def cpu_baseline(sets, budget_s=8.0):
    """robot-ticks/s of the C restatement over a bounded sample: 1024 robots
    warmed up 150 ticks untimed, then timed ticks until the budget."""
    import oracle_lib as O
    from quadrupedal_loco_amd.rt import synth_messages
    n = 1024
    orc = O.RtOracle(n)
    M = len(sets)
    msgs = [synth_messages(SEED, n, t) for t in range(M)]
    for t in range(150):
        orc.tick(*msgs[t % M])
    ticks, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        orc.tick(*msgs[(150 + ticks) % M])
        ticks += 1
    dt = time.perf_counter() - t0
    return n * ticks / dt, "%d robots x %d ticks (after 150 warm-up ticks)" % (n, ticks)


SUPPORT_BYTES = 2 * 27 * 8 + 8 + 12


def _support_traffic(B):
    """measured HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE) if profiled at this B"""
    f = os.path.join(ROOT, "profiles", "traffic_support_phase_b%d.json" % B)
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        return json.load(fh).get("hbm_bytes_per_launch")


def bench_support(args):
    import torch
    from quadrupedal_loco_amd.rt import support_phase, synth_schedules
    B = args.robots if args.robots != 65536 else 1 << 22
    dev = torch.device("cuda:0")
    host = synth_schedules(SEED, B)
    arrs = [torch.from_numpy(a).to(dev) for a in host]
    for _ in range(args.warmup if args.warmup != 150 else 5):
        support_phase(*arrs)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ev[0].record(stream)
    for k in range(args.steps):
        support_phase(*arrs)
        ev[k + 1].record(stream)
    torch.cuda.synchronize()
    per = np.array([ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)])
    ms = float(per.mean())
    achieved = SUPPORT_BYTES * B / (ms * 1e-3) / 1e9
    line = {"metric": "NLP contact-phase flags/sec (NLPClass schedule indices + right_support)",
            "value": B / (ms * 1e-3), "unit": "robots/s", "n_gpus": 1, "steps": args.steps,
            "ms_per_step": ms, "higher_is_better": True, "dtype": "f64",
            "data": "synthetic planner schedules (quadrupedal_loco_amd.rt.synth_schedules)",
            "config": {"workload": "support phase, %d robots" % B},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_robot": SUPPORT_BYTES,
                         "traffic": _support_traffic(B)}}
    if not args.no_cpu_baseline:
        import oracle_lib as O
        n = 1 << 20
        sub = [a[:n] for a in host]
        t0, reps = time.perf_counter(), 0
        while time.perf_counter() - t0 < 5.0:
            O.support_phase(*sub)
            reps += 1
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": n * reps / dt, "unit": "robots/s", "cores": 1,
                                "kind": "port", "sample": "%d x %d robots, oracle/support_phase.c"
                                % (reps, n)}
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=150)
    ap.add_argument("--sets", type=int, default=40)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--support", action="store_true")
    args = ap.parse_args()
    if args.support:
        return bench_support(args)
    import torch
    if os.environ.get("QLOCO_LIB"):  # experimental variant (tools/variant_lib.py)
        from quadrupedal_loco_amd import _lib
        _lib.LIB_PATH = os.environ["QLOCO_LIB"]
    from quadrupedal_loco_amd.rt import RtNodeBatch, synth_messages
    B, M = args.robots, args.sets
    dev = torch.device("cuda:0")
    sets = []
    for t in range(M):
        g, c = synth_messages(SEED, B, t)
        sets.append((torch.from_numpy(g).to(dev), torch.from_numpy(c).to(dev)))
    node = RtNodeBatch(B, dev)
    for t in range(args.warmup):
        node.tick(*sets[t % M], with_debug=False)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for k in range(args.steps):
        node.tick(*sets[(args.warmup + k) % M], with_debug=False)
        ev[k + 1].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    per = np.array([ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)])
    ms = float(per.mean())
    _, _, _, sched = node.tick(*sets[(args.warmup + args.steps) % M])  # one more tick, for its counts
    sched = sched.cpu().numpy()
    achieved = BYTES_PER_ROBOT_TICK * B / (ms * 1e-3) / 1e9
    line = {"metric": "rt_mpc_qp node ticks/sec (gait_fast loop body + PRMPCClass generators "
                      "+ body_theta_mpc, fp64)",
            "value": B / (ms * 1e-3), "unit": "robot-ticks/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "p99_tick_us": float(np.percentile(per, 99) * 1e3),
            "wall_ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True, "dtype": "f64",
            "data": "synthetic wire-format messages (quadrupedal_loco_amd.rt.synth_messages, "
                    "%d sets cycled)" % M,
            "config": {"workload": "rt node tick, %d robots" % B},
            "body_mpc_ran_frac": float(np.mean(sched[:, 5] >= 0)),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_robot_tick": BYTES_PER_ROBOT_TICK,
                         "traffic": _traffic(B),
                         "note": "whole tick (3 launches) against the state-streaming bytes"}}
    if not args.no_cpu_baseline:
        v, sample = cpu_baseline(sets)
        line["cpu_baseline"] = {"value": v, "unit": "robot-ticks/s", "cores": 1, "kind": "port",
                                "sample": sample + ", oracle/rt_tick.c"}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
