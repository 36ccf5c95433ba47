"""Multi-GPU handles of the C ABI (include/qloco.h §10, qloco_mgpu.hip).

CPU: the C shard arithmetic (qloco_mgpu_shard) against quadrupedal_loco_amd/
dist.py, the gathered-row map (qloco_mgpu_gather_rows) as the exact inverse
of the shards, and a gloo world-2 run in which every rank takes ITS shard
from the C function, pads it to the common shard size, all-gathers and puts
the rows in global order with the C map -- the data movement
qloco_mgpu_solve does with RCCL.  GPU: the handle at world 1 (RCCL with one
rank on the box's one GPU) against qloco_srbd_solve_ex, bit for bit, for
both shard modes and with the gathered status / iterations.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as tdist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from quadrupedal_loco_amd import dist as qdist  # noqa: E402
from quadrupedal_loco_amd import mgpu  # noqa: E402

SEED, N = 20261015, 10


@pytest.mark.parametrize("total,world", [(4096, 1), (4096, 8), (4099, 8), (7, 8), (13, 3),
                                         (1_048_576, 8), (5, 2)])
def test_shard_arithmetic_matches_dist(total, world):
    seen_c = np.zeros(total, np.int32)
    seen_i = np.zeros(total, np.int32)
    for r in range(world):
        f, c, s = mgpu.shard(total, world, r, mgpu.CONTIGUOUS)
        assert (f, c) == qdist.strong_shard_range(total, world, r) and s == 1
        seen_c[f:f + c] += 1
        f, c, s = mgpu.shard(total, world, r, mgpu.INTERLEAVED)
        assert (f, s) == (r, world)
        ids = f + s * np.arange(c)
        assert c == len(range(r, total, world))
        seen_i[ids] += 1
    assert (seen_c == 1).all() and (seen_i == 1).all()


@pytest.mark.parametrize("mode", [mgpu.CONTIGUOUS, mgpu.INTERLEAVED])
@pytest.mark.parametrize("total,world", [(4099, 8), (8, 8), (13, 3), (1, 4)])
def test_gather_rows_inverts_the_shards(total, world, mode):
    P = -(-total // world)
    rows = mgpu.gather_rows(total, world, mode)
    assert len(np.unique(rows)) == total and rows.min() >= 0 and rows.max() < world * P
    for r in range(world):
        f, c, s = mgpu.shard(total, world, r, mode)
        ids = f + s * np.arange(c)
        assert (rows[ids] == r * P + np.arange(c)).all()


def test_shard_argument_checks():
    from quadrupedal_loco_amd import _lib
    import ctypes as C
    L = _lib.lib()
    z = C.c_int64()
    assert L.qloco_mgpu_shard(10, 0, 0, 0, C.byref(z), None, None) == 100
    assert L.qloco_mgpu_shard(10, 2, 2, 0, None, None, None) == 100
    assert L.qloco_mgpu_shard(10, 2, 0, 7, None, None, None) == 100
    assert L.qloco_mgpu_init(None, None, 1, 0, 10, 0) == 100
    assert L.qloco_mgpu_destroy(None) == 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_u0(ids):
    """A deterministic stand-in for the solved forces of global ids."""
    ids = np.asarray(ids, np.float32)
    return (ids[:, None] * 16 + np.arange(12, dtype=np.float32)[None, :]).astype(np.float32)


def _worker(rank, world, port, total, mode, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    from quadrupedal_loco_amd import mgpu as M
    f, c, s = M.shard(total, world, rank, mode)
    P = -(-total // world)
    send = np.zeros((P, 12), np.float32)
    send[:c] = _fake_u0(f + s * np.arange(c))
    parts = [torch.empty((P, 12)) for _ in range(world)]
    tdist.all_gather(parts, torch.from_numpy(send))
    stage = torch.cat(parts).numpy()
    out = stage[M.gather_rows(total, world, mode)]
    np.save(os.path.join(outdir, "u0_%d_%d.npy" % (mode, rank)), out)
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.parametrize("mode", [mgpu.CONTIGUOUS, mgpu.INTERLEAVED])
def test_gloo_world2_c_shards_gather_to_global_order(tmp_path, mode):
    total, world = 13, 2  # unequal shards: rank 0 owns 7, rank 1 owns 6
    mp.spawn(_worker, args=(world, _free_port(), total, mode, str(tmp_path)), nprocs=world, join=True)
    want = _fake_u0(np.arange(total))
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / ("u0_%d_%d.npy" % (mode, r))), want)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,gait,total", [(mgpu.CONTIGUOUS, "trot", 512),
                                             (mgpu.INTERLEAVED, "mixed", 301)])
def test_handle_world1_matches_single_gpu_solve(mode, gait, total):
    """RCCL with one rank: the handle's solve + all-gather + reorder gives the
    plain single-GPU solve's u0 / status / iterations bit for bit."""
    from quadrupedal_loco_amd import srbd
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    x0, xr, ft, ct = srbd.generate(SEED, N, total, gait)
    args = [torch.from_numpy(a).to(dev) for a in (x0, xr, ft, ct)]
    ref_solver = srbd.BatchedConvexMpc(horizon=N)
    ref = ref_solver.solve(*args)
    torch.cuda.synchronize()
    h = mgpu.MgpuSolver(srbd.default_spec(horizon=N), total, 1, 0, mgpu.unique_id(), mode)
    assert (h.first, h.count, h.stride) == (0, total, 1 if mode == mgpu.CONTIGUOUS else 1)
    for stats in (False, True):
        h.u0_all.fill_(float("nan"))
        u0 = h.solve(*args, stats=stats)
        torch.cuda.synchronize()
        assert torch.equal(u0, ref.u0)
        if stats:
            assert torch.equal(h.status_all, ref.status) and torch.equal(h.iters_all, ref.iters)
    h.close()


def test_solve_refuses_bad_tensors_before_the_c_call():
    """MgpuSolver.solve ran no input checks, so a CPU, float64 or
    non-contiguous tensor reached qloco_mgpu_solve as a bad device pointer.
    Both entry points now share srbd.check_inputs; every case below raises
    ValueError on the host (no GPU needed, no C call made), and
    each with its own check's message: layout checks run before the device
    check, so CPU tensors still reach the feet / x_ref / contacts checks."""
    from quadrupedal_loco_amd import srbd
    B, Nh = 4, 10
    spec = srbd.default_spec(horizon=Nh)
    x0 = torch.zeros((B, 13), dtype=torch.float32)
    xr = torch.zeros((B, 13 * Nh), dtype=torch.float32)
    ft = torch.zeros((B, 12), dtype=torch.float32)
    ct = torch.ones((B, 4), dtype=torch.uint8)
    h = mgpu.MgpuSolver.__new__(mgpu.MgpuSolver)  # no communicator: the checks come first
    h.spec, h.count, h.device, h._h = spec, B, torch.device("cuda", 0), None
    solver = srbd.BatchedConvexMpc(spec=spec)
    bad = [
        ((x0, xr, ft, ct), "x0 must be a device tensor"),                 # CPU tensors
        ((x0.double(), xr, ft, ct), "x0: need a contiguous"),             # float64
        ((x0, xr, torch.zeros((B, 24), dtype=torch.float32).t().contiguous().t()[:, :12], ct),
         "feet: need a contiguous"),                                      # non-contiguous feet
        ((x0, xr[:, :13 * Nh - 1].contiguous(), ft, ct), r"x_ref \(B,13N\)"),  # x_ref width
        ((x0, xr, ft, ct.to(torch.int32)), "contacts: need a contiguous"),  # contacts dtype
    ]
    for args, msg in bad:
        with pytest.raises(ValueError, match=msg):
            h.solve(*args)
        with pytest.raises(ValueError, match=msg):
            solver.solve(*args)
    with pytest.raises(ValueError):  # this rank's instance count
        h.solve(x0[:2], xr[:2], ft[:2], ct[:2])
    spec2 = srbd.default_spec(horizon=Nh, warm_start=2)
    assert srbd.warm_len(spec2) == srbd.persist_len(Nh) == 100 * Nh + 4
    assert srbd.warm_len(srbd.default_spec(horizon=Nh, warm_start=1)) == 32 * Nh


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [mgpu.CONTIGUOUS, mgpu.INTERLEAVED])
@pytest.mark.parametrize("total,world,width", [(13, 3, 12), (13, 3, 14), (4099, 8, 14), (16, 4, 12),
                                               (1048576, 8, 14), (1048573, 8, 14)])
def test_device_reorder_matches_gather_rows(total, world, width, mode):
    """the device reorder of qloco_mgpu_solve (mgpu_unpack_kernel,
    padded shards, interleaved owners, the width-14 stats rows) had only run
    at world 1, where it is skipped.  qloco_mgpu_reorder runs it on one GPU on
    a synthetic gathered buffer for world > 1: every global id's row must land
    where qloco_mgpu_gather_rows says, bit for bit, padding rows never read --
    up to BASELINE configs[4]'s whole batch (1,048,576 at world 8, and one
    short of it: padded shards)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda:0")
    P = -(-total // world)
    rng = np.random.default_rng(total * 31 + world)
    stage = rng.standard_normal((world, P, width)).astype(np.float32)
    rows = mgpu.gather_rows(total, world, mode)
    if width == 14:  # status / iterations as int32 bits, distinct per global id
        flat = stage.reshape(world * P, width)
        flat[rows, 12] = np.arange(total, dtype=np.int32).view(np.float32)
        flat[rows, 13] = (1000 + np.arange(total, dtype=np.int32)).view(np.float32)
    pad = np.setdiff1d(np.arange(world * P), rows)
    stage.reshape(world * P, width)[pad] = np.nan  # a padding row read would show up
    d_stage = torch.from_numpy(stage).to(dev)
    st = torch.full((total,), -1, dtype=torch.int32, device=dev) if width == 14 else None
    it = torch.full((total,), -1, dtype=torch.int32, device=dev) if width == 14 else None
    u0 = mgpu.reorder(d_stage, total, world, mode, status_all=st, iters_all=it)
    torch.cuda.synchronize()
    want = stage.reshape(world * P, width)[rows, :12]
    assert np.array_equal(u0.cpu().numpy().view(np.int32), want.view(np.int32))
    if width == 14:
        assert np.array_equal(st.cpu().numpy(), np.arange(total))
        assert np.array_equal(it.cpu().numpy(), 1000 + np.arange(total))
