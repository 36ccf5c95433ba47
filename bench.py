#!/usr/bin/env python3
"""bench.py -- batched Go1 SRBD convex-MPC solves on MI355X.

Metric (BASELINE.json): "MPC QP solves/sec (Go1 SRBD N=10, 12 forces) at
1/2/4/8 GPUs; p99 solve µs".  Workload at N=1 GPU: configs[1] = Go1 trot
convex MPC N=10 fp32, batch 4096 per GPU.  One "step" = one pass of the hot
path over the batch: ONE fused kernel launch (condensed-QP build + OSQP
ADMM to termination + force extraction), inputs already resident in HBM;
for N>1 GPUs each rank solves its own 4096 instances (weak scaling, the
instance range is regenerated locally from (seed, global id)) and the solved
contact forces are all-gathered over RCCL/xGMI inside the timed step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                    [--horizon 10] [--gait trot] [--no-cpu-baseline] [--reduced]

The headline solves the reference's call as written: the literal
12N-variable QP, every force an ADMM variable and the swing legs held by
their fz in [0, 0] rows (spec.literal_full_qp = 1, A1RobotControl.cpp:557-578;
N <= 10 on one wavefront through the wrench space).  At N=1
the same line also carries `reduced_qp`: the same workload solved as the
stance-only reduction (swing forces eliminated exactly: same optimum,
different ADMM iterates), timed in the same run; `--reduced`
makes the reduction the headline (then the second line is `literal_full_qp`).

Rank 0 prints ONE JSON line.  Launch for N>1 GPUs:
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector == FP32 MFMA peak
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec
SEED = 20261015


def srbd_flops_alg(horizon, iters, rho_updates):
    """ALGORITHMIC flops of one solve, SURVEY.md §8(d) (the reference's 12N-variable
    formulation, whatever this kernel actually executes):
      F_B   = (N-1) 2*13^3 + N(N-1)/2 * 2*13*13*12     A powers + B_qp blocks
      F_H   = N(N+1)(N+2)/6 * 2*12*13*12               structure-aware B'QB
      F_g   = 2*13N*13 + 2*13N*12N                     gradient
      F_fac = (12N)^3 / 3 per (re)factorisation, R = 1 + rho_updates
      F_it  = 2(12N)^2 + 4*36N + 10*(12N + 20N)        per ADMM iteration, K = iters
    """
    N = float(horizon)
    it = np.asarray(iters, dtype=np.float64)
    ru = np.asarray(rho_updates, dtype=np.float64)
    nu = 12.0 * N
    F_B = (N - 1) * 2 * 13 ** 3 + N * (N - 1) / 2 * 2 * 13 * 13 * 12
    F_H = N * (N + 1) * (N + 2) / 6 * (2 * 12 * 13 * 12)
    F_g = 2 * 13 * N * 13 + 2 * 13 * N * nu
    F_fac = nu ** 3 / 3.0
    F_it = 2 * nu ** 2 + 4 * 36 * N + 10 * (nu + 20 * N)
    return F_B + F_H + F_g + it * F_it + (1.0 + ru) * F_fac


def srbd_flops_executed(n, iters, rho_updates, horizon, checks):
    """Useful FP32 flops the fused kernel executes for one solve:
    stance-only QP (n = 3 x stance (step, leg) pairs), closed-form P rows,
    Gauss-Jordan inverse (2n^3) per (re)factorisation, K^-1 matvec per iteration."""
    n = np.asarray(n, dtype=np.float64)
    it = np.asarray(iters, dtype=np.float64)
    ru = np.asarray(rho_updates, dtype=np.float64)
    ch = np.asarray(checks, dtype=np.float64)
    build = 12.0 * n * n + 20.0 * n * n + 40.0 * n + 60.0 * horizon
    fac = (1.0 + ru) * (2.0 * n ** 3 + 14.0 * n * n)
    iters = it * (2.0 * n * n + 30.0 * n)
    chk = ch * 70.0 * n
    return build + fac + iters + chk


def srbd_flops_executed_lit(horizon, iters, rho_updates, checks, scaling=10):
    """Useful flops of the wrench-space literal kernels, one wave (N <= 10,
    srbd_lit_kernel) or two (N = 11 .. 20, srbd_lit2_kernel,
    §3j), in the M = G^-1 / c + U form both run since round 5:
    n = 12N variables, w = 6N wrench rows (the kernels' 60 / 120-column rows
    beyond w are padding and not counted).
      build  Ruiz: 1 + scaling sweeps of the n x n P row norms (4 flops an
             entry), the gradient, the (beta, eps) tables; the G^-1 tables:
             six N x N float64 Gauss-Jordans per solve (2 N^3 each), counted
             twice (FP64 vector issues at half the FP32 rate)
      fac    per (re)factorisation, R = 1 + rho_updates: the W0^-1 leg rows
             (60 flops a variable, computed twice), the U rows (216 a wrench
             row), the M rows (4 an entry), the 2 w^3 Gauss-Jordan, the
             1 / scale pass (w^2)
      its    per ADMM iteration: the T matvec (2 w^2), 70 flops a variable
             (rhs, the two W0^-1 triple dots, update_x / z / y), 24 a wrench
             row (Vu a)
      chk    per residual check: P~x through the wrench rows (G w: 4N a
             wrench row, Te w, Vu' G w) and the residual maxima."""
    N = float(horizon)
    n, w = 12.0 * N, 6.0 * N
    it = np.asarray(iters, dtype=np.float64)
    ru = np.asarray(rho_updates, dtype=np.float64)
    ch = np.asarray(checks, dtype=np.float64)
    build = ((1.0 + scaling) * n * n * 4.0 + 12 * N * 8 + 16.0 * n + 144 * 6 * 14
             + 2.0 * 6 * (2.0 * N ** 3 + 10.0 * N * N))
    fac = (1.0 + ru) * (2.0 * w ** 3 + 5.0 * w * w + 216.0 * w + 120.0 * n)
    its = it * (2.0 * w * w + 70.0 * n + 24.0 * w)
    chk = ch * (4.0 * N * w + 40.0 * w + 55.0 * n)
    return build + fac + its + chk


def executed_flops(N, n_var, iters, rho_up, checks, literal):
    """Executed-flop model of the kernel the solve actually routes to: the
    wrench-space literal kernels for the literal QP at N <= 20 (the bench's
    Go1 weights satisfy their routing condition, qloco_srbd.hip), the
    stance-variable kernels otherwise."""
    if literal and N <= 20:
        return srbd_flops_executed_lit(N, iters, rho_up, checks)
    return srbd_flops_executed(n_var, iters, rho_up, N, checks)


def _config_tag(N, gait, B):
    """Which BASELINE.json config a bench line measures (per-GPU share for the
    8-GPU configs: 524288/8 = 65536, 1048576/8 = 131072)."""
    tags = {(10, "trot", 4096): " (BASELINE configs[1])",
            (16, "trot", 65536): " (BASELINE configs[2])",
            (20, "pace", 65536): " (BASELINE configs[3], 1/8 share)",
            (10, "mixed", 131072): " (BASELINE configs[4], 1/8 share)"}
    return tags.get((N, gait, B), "")


def usable_cores():
    """Host cores this process may actually run on: the affinity mask, capped by
    the cgroup CPU quota when one is set (the GPU box gives each GPU a CPU share
    smaller than the machine; os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N ranks through
    torch.distributed.run as a CHILD process (this process never touches the
    GPU, so nothing is exec'd from a GPU-initialised process), relay rank 0's
    JSON line and exit with the launcher's status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    for ln in lines:
        print(ln, flush=True)
    if p.returncode == 0 and len(lines) != 1:
        print("bench.py: expected one JSON line from rank 0, got %d" % len(lines), file=sys.stderr)
        return 1
    return p.returncode


def dist_selftest(args, rank, world):
    """CPU check of the multi-rank launch path (tests/test_bench_launch.py): gloo
    process group, the world size the launcher was asked for, and the step's one
    collective (ForceGather) -- no GPU, no solve."""
    import torch
    import torch.distributed as dist
    if "MASTER_ADDR" in os.environ:
        dist.init_process_group("gloo")
    else:  # --gpus 1 without a launcher
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % _free_port(),
                                rank=0, world_size=1)
    from quadrupedal_loco_amd.dist import ForceGather, shard_range
    B = 8
    first, _ = shard_range(B, rank)
    u0 = (torch.arange(B * 12, dtype=torch.float32).reshape(B, 12) + 12 * first)
    out = ForceGather(B)(u0)
    ok = bool(torch.equal(out, torch.arange(world * B * 12, dtype=torch.float32)
                          .reshape(world * B, 12)))
    t = torch.tensor([1.0 if ok else 0.0])
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(json.dumps({"selftest": "dist-launch", "n_gpus": world, "requested": args.gpus,
                          "allgather_ok": bool(t.item() == 1.0)}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU")
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--gait", default="trot")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--reduced", action="store_true",
                    help="headline = the stance-only reduction (literal_full_qp = 0) instead of "
                         "the reference's literal 12N-variable QP")
    ap.add_argument("--literal", action="store_true",
                    help="the literal QP as headline (the default; kept for old command lines)")
    ap.add_argument("--no-literal-line", "--no-second-line", dest="no_second_line",
                    action="store_true", help="skip the other formulation's side measurement at N = 1")
    ap.add_argument("--literal-steps", "--second-steps", dest="second_steps", type=int, default=50)
    ap.add_argument("--prewarm", type=int, default=64,
                    help="untimed headline solves before everything else (GPU clock ramp)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: every usable host core)")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--shard", choices=("auto", "contiguous", "interleaved"), default="auto",
                    help="instance ids per rank: contiguous ranges, or stride-interleaved "
                         "(SURVEY.md 8e; auto: interleaved for the mixed-schedule config 5)")
    ap.add_argument("--overlap", action="store_true",
                    help="N > 1: run each step's all-gather under the next solve (double-"
                         "buffered u0); off by default: on one GPU the RCCL kernel sharing "
                         "the CUs with the solve cost more than it hid (DESIGN.md §7)")
    ap.add_argument("--comm", choices=("torch", "capi"), default="torch",
                    help="N > 1: who shards and all-gathers -- torch.distributed (dist.py) or the "
                         "library's own C-ABI handles (qloco_mgpu_*: RCCL from C, include/qloco.h 10)")
    ap.add_argument("--force-dist", action="store_true",
                    help="testing: run the N > 1 code path (RCCL group, all-gather) at N = 1")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="testing (CPU): launch path + gloo all-gather only, no GPU")
    args = ap.parse_args()
    args.literal = not args.reduced
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # no launcher: spawn the ranks ourselves (before any GPU call)
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" % (os.environ["WORLD_SIZE"], args.gpus),
              file=sys.stderr)
        sys.exit(2)

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if args.dist_selftest:
        dist_selftest(args, rank, world)
        return

    import torch

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    json_out = sys.stdout
    if world > 1 or args.force_dist:
        # RCCL prints a version banner on stdout when its communicator comes
        # up: keep stdout for the one JSON line, library output goes to stderr
        sys.stdout.flush()
        json_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from quadrupedal_loco_amd import srbd

    B, N = args.batch, args.horizon
    from quadrupedal_loco_amd.dist import interleaved_shard, shard_range
    shard = args.shard if args.shard != "auto" else (
        "interleaved" if args.gait == "mixed" else "contiguous")
    if shard == "interleaved":
        first, stride, _ = interleaved_shard(B, world, rank)
    else:
        (first, _), stride = shard_range(B, rank), 1
    multi = world > 1 or args.force_dist
    capi = multi and args.comm == "capi" and not args.no_allgather
    if capi:
        # the C handles own the shard arithmetic: take this rank's ids from them
        from quadrupedal_loco_amd import mgpu
        mode = mgpu.INTERLEAVED if shard == "interleaved" else mgpu.CONTIGUOUS
        first, count, stride = mgpu.shard(B * world, world, rank, mode)
        assert count == B
    x0, xr, ft, ct = srbd.generate(SEED, N, B, args.gait, first=first, stride=stride)
    d_x0 = torch.from_numpy(x0).to(dev)
    d_xr = torch.from_numpy(xr).to(dev)
    d_ft = torch.from_numpy(ft).to(dev)
    d_ct = torch.from_numpy(ct).to(dev)
    solver = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=int(args.literal))
    legs = 4 * N if args.literal else srbd.max_stance_legs(ct, N)
    gather = None
    overlap = multi and not args.no_allgather and args.overlap and not capi
    handle = None
    if capi:
        cid = [mgpu.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(cid, src=0)
        handle = mgpu.MgpuSolver(solver.spec, B * world, world, rank, cid[0], mode)
    elif multi and not args.no_allgather:
        from quadrupedal_loco_amd.dist import ForceGather
        gather = [ForceGather(B, device=dev) for _ in range(2 if overlap else 1)]
    # two output sets when the all-gather of step i overlaps the solve of step
    # i + 1: step i solves into set i % 2, after the gather that last read it
    outs = [solver.alloc_outputs(B, dev) for _ in range(2 if overlap else 1)]
    out = outs[0]
    stream = torch.cuda.current_stream(dev)
    pending = [None, None]

    def step(i, ev=None):
        o = outs[i % len(outs)]
        if pending[i % 2] is not None:  # the gather that last read this u0 set
            pending[i % 2].wait()
            pending[i % 2] = None
        if ev is not None:
            ev[0].record(stream)
        if handle is not None:  # solve + all-gather + global order, all in the C library
            handle.solve(d_x0, d_xr, d_ft, d_ct, max_legs=legs,
                         stream=stream.cuda_stream)
            return
        solver.solve(d_x0, d_xr, d_ft, d_ct, out=o, max_legs=legs, stream=stream.cuda_stream)
        if ev is not None and ev[1] is not None:
            ev[1].record(stream)
        if gather is not None:
            if overlap:
                _, pending[i % 2] = gather[i % 2](o.u0, async_op=True)
            else:
                gather[0](o.u0)

    def drain():
        for k in range(2):
            if pending[k] is not None:
                pending[k].wait()
                pending[k] = None

    # Clock pre-warm: a cold GPU ramps its clocks over the first ~40 launches
    # (554 us per launch over the first 20, 515 us from launch 40 on,
    # profiles/r5a_step_timeline.txt), so W = 5 warm-up steps alone would time
    # part of the ramp.  A fixed number of untimed headline
    # solves (--prewarm, recorded in the line) runs first, whatever side
    # measurements the flags select, so the headline is timed at the clocks a
    # continuously running controller sees and does not move with the flag
    # set.  Then the side measurements, then W untimed warm-up steps and
    # exactly K timed steps.  Every rank runs the pre-warm and the two
    # rank-local side lines (its own shard, no collective), so an N-GPU run
    # times its headline at the same clocks as the 1-GPU run; the line
    # printed is rank 0's.
    for _ in range(args.prewarm):
        solver.solve(d_x0, d_xr, d_ft, d_ct, out=out, max_legs=legs, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    side = {}
    if not args.no_second_line:
        key = "reduced_qp" if args.literal else "literal_full_qp"
        side[key] = second_line(args, srbd, d_x0, d_xr, d_ft, d_ct, ct, stream, dev, not args.literal)
        try:  # side measurements: never lose the headline line over one
            side["shuffled_order"] = shuffled_line(args, srbd, d_x0, d_xr, d_ft, d_ct, ct, stream, dev,
                                                   args.literal)
        except Exception as e:  # noqa: BLE001
            side["shuffled_order"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_second_line:
        if args.horizon <= 20:
            try:
                side["persistent_literal"] = steady_line(args, srbd, stream, dev)
            except Exception as e:  # noqa: BLE001
                side["persistent_literal"] = {"error": repr(e)}
        if args.literal:
            try:
                side["reference_weights"] = weights_line(args, srbd, d_x0, d_xr, d_ft, d_ct, stream, dev)
            except Exception as e:  # noqa: BLE001
                side["reference_weights"] = {"error": repr(e)}
        try:
            side["pcie_inclusive"] = host_io_line(args, srbd, d_x0, d_xr, d_ft, d_ct, ct, stream, dev,
                                                  args.literal)
        except Exception as e:  # noqa: BLE001
            side["pcie_inclusive"] = {"error": repr(e)}

    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize(dev)

    K = args.steps
    # One timing event per step boundary (ev_b[i] starts step i, ev_b[K] ends
    # the last), plus one after the solve only when an all-gather follows it:
    # every event record costs the stream 2.5-5 us (tools/event_overhead.py,
    # profiles/r3_event_overhead.txt), so the timed loop records no more
    # than the numbers below need.  Without a gather, a step's span is its
    # solve launch.
    ev_b = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    ev_k = [torch.cuda.Event(enable_timing=True) if gather is not None else None
            for _ in range(K)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(K):
        step(i, (ev_b[i], ev_k[i]))
    drain()
    ev_b[K].record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    step_ms = np.array([ev_b[i].elapsed_time(ev_b[i + 1]) for i in range(K)])
    if gather is not None:
        kern_ms = np.array([ev_b[i].elapsed_time(ev_k[i]) for i in range(K)])
        gather_ms = np.array([ev_k[i].elapsed_time(ev_b[i + 1]) for i in range(K)])
    else:
        kern_ms = step_ms
        gather_ms = np.zeros(K)

    # per-instance stats of the solved batch (identical every step)
    if handle is not None:  # stats not gathered in the timed loop: one plain solve
        solver.solve(d_x0, d_xr, d_ft, d_ct, out=out, max_legs=legs, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
    status = out.status.cpu().numpy()
    iters = out.iters.cpu().numpy()
    rho_up = out.rho_updates.cpu().numpy()
    n_var = 12 * N * np.ones(B) if args.literal else 3 * ct.reshape(B, -1).sum(axis=1)
    checks = iters // 25 + iters // 100
    flops_alg = float(srbd_flops_alg(N, iters, rho_up).sum())
    flops_exec = float(executed_flops(N, n_var, iters, rho_up, checks, args.literal).sum())
    achieved_tflops = flops_alg / (kern_ms.mean() * 1e-3) / 1e12
    executed_tflops = flops_exec / (kern_ms.mean() * 1e-3) / 1e12

    value = B * world * K / elapsed
    res = {
        "metric": "MPC QP solves/sec (Go1 SRBD N=%d, 12 forces); p99 solve us" % N,
        "value": round(value, 1),
        "unit": "solves/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "prewarm_launches": args.prewarm,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (counter-based generator, seed %d, DESIGN.md §4)" % SEED,
        "config": {
            "workload": "Go1 %s convex MPC N=%d fp32, batch=%d per GPU%s"
                        % (args.gait, N, B, _config_tag(N, args.gait, B)),
            "horizon": N, "batch_per_gpu": B, "gait": args.gait,
            "solver": "OSQP-algorithm ADMM, default settings (eps 1e-3, adaptive rho), %s" % (
                "literal 12N-variable QP (literal_full_qp=1)" if args.literal else
                "stance-only reduction of the 12N-variable QP (same optimum)"),
            "parallelism": "dp%d (%s instance shards, RCCL all-gather of u0%s%s)" % (
                world, shard, ", overlapped with the next solve" if overlap else "",
                ", C-ABI handles qloco_mgpu_*" if capi else ""),
        },
        "p99_batch_us": round(float(np.percentile(step_ms, 99)) * 1e3, 2),
        "p50_batch_us": round(float(np.percentile(step_ms, 50)) * 1e3, 2),
        "kernel_us_avg": round(float(kern_ms.mean()) * 1e3, 2),
        "allgather_us_avg": (round(float(gather_ms.mean()) * 1e3, 2)
                             if gather is not None and not overlap else None),
        "admm_iters_p50_p99": [int(np.percentile(iters, 50)), int(np.percentile(iters, 99))],
        "status_ok_frac": float(np.mean(status == 0)),
        "roofline": {
            "bound": "valu-fp32",
            "achieved": round(achieved_tflops, 3),
            "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved_tflops / PEAK_FP32_TFLOPS, 4),
            "traffic": None,
            "algorithmic_flops_per_launch": flops_alg,
            "executed": round(executed_tflops, 3),
            "executed_frac": round(executed_tflops / PEAK_FP32_TFLOPS, 4),
            "note": ("FP32 VALU compute bound: no MFMA instruction runs on this path (the "
                     "closed-form Hessian removes the B'QB GEMM, DESIGN.md 3); peak = FP32 vector "
                     "157.3 TF.  achieved / frac count SURVEY.md 8(d)'s ALGORITHMIC flops of the "
                     "reference's 12N-variable QP (%.3g per launch) / mean kernel time (HIP events "
                     "on the launch stream, one per step boundary: without an all-gather a "
                     "step's span is its solve launch)%s; executed / executed_frac = the flops this kernel "
                     "actually performs (%.3g per launch, DESIGN.md 5) -- the number that rates "
                     "the kernel" % (flops_alg, "" if args.literal else
                                     ", which the stance-only kernel never builds", flops_exec)),
        },
    }
    tfile = os.path.join(ROOT, "profiles", "traffic_srbd_n%d_b%d%s.json" % (N, B, "_lit" if args.literal else ""))
    if os.path.exists(tfile):
        with open(tfile) as f:
            res["roofline"]["traffic"] = json.load(f).get("hbm_bytes_per_launch")

    res.update(side)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(N, args.gait, args.cpu_seconds, args.cpu_threads)
    if rank == 0:
        print(json.dumps(res), file=json_out, flush=True)
    if handle is not None:
        handle.close()
    if dist is not None:
        dist.destroy_process_group()


def second_line(args, srbd, d_x0, d_xr, d_ft, d_ct, ct, stream, dev, literal):
    """The same workload in the other formulation -- the reference's literal
    12N-variable QP (literal_full_qp = 1: swing forces kept as ADMM variables)
    or the stance-only reduction -- timed before the headline loop:
    barrier-free single-GPU timing, HIP events per launch."""
    import torch
    B, N, K = args.batch, args.horizon, args.second_steps
    solver = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=int(literal))
    legs = 4 * N if literal else srbd.max_stance_legs(ct, N)
    out = solver.alloc_outputs(B, dev)
    for _ in range(5):
        solver.solve(d_x0, d_xr, d_ft, d_ct, out=out, max_legs=legs, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for i in range(K):
        solver.solve(d_x0, d_xr, d_ft, d_ct, out=out, max_legs=legs, stream=stream.cuda_stream)
        ev[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    per = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(K)])
    iters = out.iters.cpu().numpy()
    rho_up = out.rho_updates.cpu().numpy()
    status = out.status.cpu().numpy()
    checks = iters // 25 + iters // 100
    fa = float(srbd_flops_alg(N, iters, rho_up).sum())
    n_var = 12 * N * np.ones(B) if literal else 3 * ct.reshape(B, -1).sum(axis=1)
    fe = float(executed_flops(N, n_var, iters, rho_up, checks, literal).sum())
    kt = float(per.mean()) * 1e-3
    return {"value": round(B * K / elapsed, 1), "unit": "solves/s", "steps": K,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "kernel_us_avg": round(float(per.mean()) * 1e3, 2),
            "p99_batch_us": round(float(np.percentile(per, 99)) * 1e3, 2),
            "admm_iters_p50_p99": [int(np.percentile(iters, 50)), int(np.percentile(iters, 99))],
            "status_ok_frac": float(np.mean(status == 0)),
            "frac": round(fa / kt / 1e12 / PEAK_FP32_TFLOPS, 4),
            "executed_frac": round(fe / kt / 1e12 / PEAK_FP32_TFLOPS, 4),
            "note": ("the reference's call as written (A1RobotControl.cpp:557-578): all 12N "
                     "forces ADMM variables, swing legs held by fz in [0, 0] equality rows; "
                     "%d variables per N = %d instance -> %s" % (
                         12 * N, N, "one wavefront, the OSQP solve through the per-step wrench "
                         "space (srbd_lit_kernel, DESIGN.md 3i)" if N <= 10
                         else "512-thread workgroups (srbd_admm_big_kernel)")) if literal else
                    "stance-only reduction of the same QPs (swing forces eliminated exactly: "
                    "same optimum, different ADMM iterates and Ruiz scaling; DESIGN.md 3): "
                    "closed-form P rows, K^-1 in registers, one wavefront for <= 20 stance legs"}


def shuffled_line(args, srbd, d_x0, d_xr, d_ft, d_ct, ct, stream, dev, literal):
    """The headline batch with its instances in a seeded random order: the
    generator's identity order puts instances of similar difficulty (the
    same trot phase) next to each other, so neighbouring workgroups finish
    together; a shuffled batch mixes long and short solves on every SIMD.
    Same solver, same K, HIP events per launch."""
    import torch
    B, N, K = args.batch, args.horizon, args.second_steps
    perm = torch.from_numpy(np.random.default_rng(SEED + 1).permutation(B)).to(dev)
    xs = [t.index_select(0, perm).contiguous() for t in (d_x0, d_xr, d_ft, d_ct)]
    solver = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=int(literal))
    legs = 4 * N if literal else srbd.max_stance_legs(ct, N)
    out = solver.alloc_outputs(B, dev)
    for _ in range(5):
        solver.solve(*xs, out=out, max_legs=legs, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for i in range(K):
        solver.solve(*xs, out=out, max_legs=legs, stream=stream.cuda_stream)
        ev[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    per = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(K)])
    iters = out.iters.cpu().numpy()
    return {"value": round(B * K / elapsed, 1), "unit": "solves/s", "steps": K,
            "kernel_us_avg": round(float(per.mean()) * 1e3, 2),
            "p99_batch_us": round(float(np.percentile(per, 99)) * 1e3, 2),
            "admm_iters_p50_p99": [int(np.percentile(iters, 50)), int(np.percentile(iters, 99))],
            "status_ok_frac": float(np.mean(out.status.cpu().numpy() == 0)),
            "note": "the headline workload, instances in a seeded random order (numpy default_rng(%d))"
                    % (SEED + 1)}


def steady_line(args, srbd, stream, dev, ticks=24, switch_every=6):
    """The reference's steady-state call: its member OSQP solver persists
    across control ticks (A1RobotControl.h:67) and every call after the first
    takes OSQP's update path with warm start (A1RobotControl.cpp:556-578) --
    PersistentConvexMpc(literal_full_qp=1), warm_start = 2.  B controllers
    over a `ticks`-call control loop (the synthetic instances drifting
    between 2.5 ms ticks, every controller flipping its trot phase each
    `switch_every` ticks, srbd.control_loop_sequence), inputs of every tick
    resident in HBM before timing.  Tick 0 (each controller's first, cold
    call) is untimed; the timed region is ticks 1 .. ticks-1, HIP events per
    launch on the launch stream."""
    import torch
    B, N = args.batch, args.horizon
    seq = srbd.control_loop_sequence(SEED, N, B, ticks, args.gait, switch_every=switch_every)
    d_seq = [[torch.from_numpy(a).to(dev) for a in tick] for tick in seq]
    ctl = srbd.PersistentConvexMpc(B, dev, horizon=N, literal_full_qp=1)
    outs = [ctl.alloc_outputs(B, dev) for _ in range(ticks)]
    ctl.solve(*d_seq[0], out=outs[0], stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(ticks)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for t in range(1, ticks):
        ctl.solve(*d_seq[t], out=outs[t], stream=stream.cuda_stream)
        ev[t].record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    per = np.array([ev[t - 1].elapsed_time(ev[t]) for t in range(1, ticks)])
    iters = np.concatenate([outs[t].iters.cpu().numpy() for t in range(1, ticks)])
    status = np.concatenate([outs[t].status.cpu().numpy() for t in range(1, ticks)])
    rho_up = np.concatenate([outs[t].rho_updates.cpu().numpy() for t in range(1, ticks)])
    it0 = outs[0].iters.cpu().numpy()
    return {"value": round(B * (ticks - 1) / elapsed, 1), "unit": "solves/s", "ticks_timed": ticks - 1,
            "batch": B, "kernel_us_avg": round(float(per.mean()) * 1e3, 2),
            "p99_batch_us": round(float(np.percentile(per, 99)) * 1e3, 2),
            "admm_iters_p50_p99": [int(np.percentile(iters, 50)), int(np.percentile(iters, 99))],
            "admm_iters_mean": round(float(iters.mean()), 2),
            "cold_first_tick_iters_mean": round(float(it0.mean()), 2),
            "rho_updates_mean": round(float(rho_up.mean()), 3),
            "status_ok_frac": float(np.mean(status == 0)),
            "note": ("the reference's steady-state call (A1RobotControl.cpp:556-578): member OSQP "
                     "solver kept across ticks, OSQP's update path + warm start on every call after "
                     "the first (PersistentConvexMpc, literal_full_qp=1, warm_start=2; "
                     "srbd_lit_kernel<true>); %d controllers x %d timed ticks of a drifting trot loop "
                     "with a phase flip every %d ticks" % (B, ticks - 1, switch_every))}


def weights_line(args, srbd, d_x0, d_xr, d_ft, d_ct, stream, dev):
    """The headline workload with the MPC weight sets the reference ships
    (config/{gazebo,hardware,isaac}_a1_mpc.yaml, srbd.REFERENCE_WEIGHTS):
    throughput, the kernel family qloco_srbd_route picks and the iteration
    counts, timed before the headline like the other side lines.  isaac's
    state weights (roll 8000) exceed the wrench-space kernels' float32 limit
    and run the generic literal kernels."""
    import torch
    B, N, K = args.batch, args.horizon, max(10, args.second_steps // 2)
    res = {}
    for name, (q, r) in srbd.REFERENCE_WEIGHTS.items():
        solver = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=1, q_weights=q, r_weights=r)
        out = solver.alloc_outputs(B, dev)
        for _ in range(3):
            solver.solve(d_x0, d_xr, d_ft, d_ct, out=out, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
        ev[0].record(stream)
        for i in range(K):
            solver.solve(d_x0, d_xr, d_ft, d_ct, out=out, stream=stream.cuda_stream)
            ev[i + 1].record(stream)
        torch.cuda.synchronize(dev)
        per = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(K)])
        it = out.iters.cpu().numpy()
        route = srbd.route(solver.spec)
        res[name] = {"value": round(B / (float(per.mean()) * 1e-3), 1), "unit": "solves/s", "steps": K,
                     "kernel_us_avg": round(float(per.mean()) * 1e3, 2),
                     "route": {1: "srbd_lit_kernel", 2: "srbd_lit2_kernel", 3: "generic literal kernels",
                               4: "reduced"}.get(route, str(route)),
                     "admm_iters_mean": round(float(it.mean()), 2),
                     "status_ok_frac": float(np.mean(out.status.cpu().numpy() == 0))}
    res["note"] = "the headline workload with the reference's shipped MPC weights (literal QP, same inputs)"
    return res


def host_io_line(args, srbd, d_x0, d_xr, d_ft, d_ct, ct, stream, dev, literal):
    """The headline workload with the boundary's host side included: every step
    copies the inputs (x0, x_ref, feet, contacts) from pinned host memory to
    HBM, solves, and copies u0 back -- what a host caller of the C ABI pays
    (the ROS node's ConvexMpc call, A1RobotControl.cpp:553-599).  The four
    inputs travel as ONE packed pinned buffer (one H2D copy per step; the
    solve reads typed views of the packed device buffer): each separate copy
    costs the stream a launch of its own.  One form, `serial` (copy, solve,
    copy back in order on one stream): the `pipelined` form of round 5 (the
    inputs of step i + 1 copied on a second HIP stream while step i solves,
    double-buffered) measured 0.924 ms per step against the serial form's
    0.569 at B = 4096 (round 6; the copy runs as a blit kernel on the compute
    queues and the cross-stream event hand-offs cost more than it hides).
    Reported beside the headline, never as `value` (inputs resident in HBM
    there)."""
    import torch
    B, N, K = args.batch, args.horizon, args.second_steps
    solver = srbd.BatchedConvexMpc(horizon=N, literal_full_qp=int(literal))
    legs = 4 * N if literal else srbd.max_stance_legs(ct, N)
    out = solver.alloc_outputs(B, dev)
    parts = [t.contiguous() for t in (d_x0, d_xr, d_ft, d_ct)]
    nbytes = [t.numel() * t.element_size() for t in parts]
    offs, o = [], 0
    for nb in nbytes:  # 16-byte aligned fields in the packed buffer
        offs.append(o)
        o += (nb + 15) // 16 * 16
    host = torch.empty(o, dtype=torch.uint8).pin_memory()
    for t, off, nb in zip(parts, offs, nbytes):
        host[off:off + nb].copy_(t.cpu().reshape(-1).view(torch.uint8))
    dbuf = torch.empty(o, dtype=torch.uint8, device=dev)
    dviews = [dbuf[off:off + nb].view(t.dtype).view(t.shape) for t, off, nb in zip(parts, offs, nbytes)]
    h_u0 = torch.empty(out.u0.shape, dtype=out.u0.dtype).pin_memory()

    def serial():
        dbuf.copy_(host, non_blocking=True)
        solver.solve(*dviews, out=out, max_legs=legs, stream=stream.cuda_stream)
        h_u0.copy_(out.u0, non_blocking=True)

    res = {"unit": "solves/s", "steps": K, "h2d_bytes_per_step": int(sum(nbytes)),
           "d2h_bytes_per_step": int(h_u0.numel() * h_u0.element_size()), "h2d_copies_per_step": 1}
    for _ in range(5):
        serial()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(K):
        serial()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    res["serial"] = {"value": round(B * K / elapsed, 1), "ms_per_step": round(elapsed / K * 1e3, 4)}
    res["note"] = ("PCIe-inclusive: the four inputs as one packed pinned buffer to HBM, the solve, u0 back, "
                   "every step on one stream; not the headline: `value` has the inputs resident in HBM.  "
                   "A pipelined form (next step's copy on a second stream under the solve) was slower at "
                   "every measurement (0.924 vs 0.569 ms, profiles/r6n_bench_default.json) and is dropped")
    return res


def cpu_baseline(N, gait, seconds, threads):
    """CPU-A baseline: the oracle's literal ConvexMpc build + OSQP-algorithm
    ADMM restatement (double, full 12N-variable QP) on host threads -- one per
    usable host core unless --cpu-threads says otherwise -- over a bounded
    sample of the same synthetic workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    import oracle_lib as O
    threads = threads if threads > 0 else usable_cores()
    sp = O.srbd_spec(N=N)
    st = O.admm_settings()
    g = {"trot": 0, "pace": 1, "mixed": 2, "stance": 3}.get(gait, 0)

    def run(count):
        x0, xr, ft, ct = O.gen_srbd(SEED, N, count, gait=g)
        secs = C.c_double(0)
        O.lib().qo_srbd_batch(C.byref(sp), C.byref(st), 0, count, O.P(x0, C.c_float),
                              O.P(xr, C.c_float), O.P(ft, C.c_float), 0, O.P(ct, C.c_uint8), 1,
                              None, None, None, None, threads, C.byref(secs))
        return secs.value

    probe = 4 * threads
    tp = run(probe)
    count = int(max(probe, min(2_000_000, probe * seconds / max(tp, 1e-6))))
    t = run(count)
    return {"value": round(count / t, 1), "unit": "solves/s", "cores": threads,
            "host_cores": os.cpu_count(), "cpu_model": cpu_model(),
            "kind": "port",
            "sample": "%d instances of the same workload (first %d of the seed), oracle CPU-A "
                      "(literal dense ConvexMpc build + OSQP-algorithm ADMM, fp64), %.1f s"
                      % (count, count, t)}


if __name__ == "__main__":
    main()
