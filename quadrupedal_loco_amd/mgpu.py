"""Multi-GPU handles of the C ABI (include/qloco.h §10), from Python.

The same sharding and the same one all-gather as quadrupedal_loco_amd/dist.py,
but done by libqloco.so itself (qloco_mgpu_*: RCCL loaded by the library,
shard ranges and the global-order reorder in C), so a C++ caller gets it
without torch.distributed.  The communicator id is made on rank 0 and shipped
to the other ranks by the caller (`bootstrap`: any callable that broadcasts
the 128 bytes, e.g. torch.distributed.broadcast_object_list).
"""
import ctypes as C

import numpy as np

from ._lib import check, lib, ptr

CONTIGUOUS, INTERLEAVED = 0, 1
ID_BYTES = 128


def shard(total, world, rank, mode=CONTIGUOUS):
    """(first, count, stride) of `rank`'s global ids (qloco_mgpu_shard)."""
    f, c, s = C.c_int64(), C.c_int64(), C.c_int64()
    check(lib().qloco_mgpu_shard(int(total), int(world), int(rank), int(mode), C.byref(f),
                                 C.byref(c), C.byref(s)), "qloco_mgpu_shard")
    return f.value, c.value, s.value


def gather_rows(total, world, mode=CONTIGUOUS):
    """Row of each global id in the gathered (world x P) buffer."""
    rows = np.zeros(int(total), np.int64)
    check(lib().qloco_mgpu_gather_rows(int(total), int(world), int(mode),
                                       rows.ctypes.data_as(C.c_void_p)), "qloco_mgpu_gather_rows")
    return rows


def reorder(stage, total, world, mode=CONTIGUOUS, status_all=None, iters_all=None, stream=None):
    """Gathered (world, P, width) shard rows -> u0 (total, 12) in global id
    order on the device (qloco_mgpu_reorder: the reorder step of
    qloco_mgpu_solve, for a caller that runs its own all-gather).  width 14
    rows carry status / iterations as int32 bits in columns 12 / 13."""
    import torch
    width = int(stage.shape[-1])
    P = -(-int(total) // int(world))
    if (stage.dtype != torch.float32 or not stage.is_cuda or not stage.is_contiguous()
            or stage.numel() != int(world) * P * width):
        raise ValueError("stage: contiguous float32 device tensor of %d x %d x %d" % (world, P, width))
    u0 = torch.empty((int(total), 12), dtype=torch.float32, device=stage.device)
    if stream is None:
        stream = torch.cuda.current_stream(stage.device).cuda_stream
    check(lib().qloco_mgpu_reorder(int(total), int(world), int(mode), width, ptr(stage), ptr(u0),
                                   ptr(status_all), ptr(iters_all), C.c_void_p(stream)),
          "qloco_mgpu_reorder")
    return u0


def unique_id():
    buf = (C.c_uint8 * ID_BYTES)()
    check(lib().qloco_mgpu_unique_id(buf), "qloco_mgpu_unique_id")
    return bytes(buf)


class MgpuSolver:
    """One rank of a multi-GPU SRBD solve through the C handles.

    `solve(x0, x_ref, feet, contacts)` takes this rank's shard (count
    instances, device tensors on the current device) and returns u0 of the
    whole batch (total, 12) in global id order, identical on every rank."""

    def __init__(self, spec, total, world, rank, comm_id, mode=CONTIGUOUS):
        import torch
        self.spec = spec
        self.total, self.world, self.rank, self.mode = int(total), int(world), int(rank), int(mode)
        self._h = C.c_void_p()
        idbuf = (C.c_uint8 * ID_BYTES).from_buffer_copy(comm_id)
        check(lib().qloco_mgpu_init(C.byref(self._h), idbuf, self.world, self.rank, self.total,
                                    self.mode), "qloco_mgpu_init")
        f, c, s, p = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        check(lib().qloco_mgpu_info(self._h, C.byref(f), C.byref(c), C.byref(s), C.byref(p)),
              "qloco_mgpu_info")
        self.first, self.count, self.stride, self.padded = f.value, c.value, s.value, p.value
        dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev  # the device the handle's communicator and buffers live on
        self.u0_all = torch.empty((self.total, 12), dtype=torch.float32, device=dev)
        self.status_all = torch.empty(self.total, dtype=torch.int32, device=dev)
        self.iters_all = torch.empty(self.total, dtype=torch.int32, device=dev)

    def solve(self, x0, x_ref, feet, contacts, stats=False, max_legs=0, warm=None, stream=None):
        import torch
        from .srbd import check_inputs
        N = self.spec.horizon
        if x0.shape[0] != self.count:
            raise ValueError("this rank owns %d instances, got %d" % (self.count, x0.shape[0]))
        # the checks BatchedConvexMpc.solve runs, on the handle's device: a CPU,
        # float64 or non-contiguous tensor is refused before the C call
        check_inputs(self.spec, x0, x_ref, feet, contacts, warm=warm, device=self.device)
        self.spec.feet_per_step = 1 if feet.shape[1] == 12 * N and N > 1 else 0
        self.spec.contacts_per_step = 1 if contacts.shape[1] == 4 * N and N > 1 else 0
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        check(lib().qloco_mgpu_solve(
            self._h, C.byref(self.spec), ptr(x0), ptr(x_ref), ptr(feet), ptr(contacts), ptr(warm),
            ptr(self.u0_all), ptr(self.status_all) if stats else None,
            ptr(self.iters_all) if stats else None, int(max_legs), C.c_void_p(stream)),
            "qloco_mgpu_solve")
        return self.u0_all

    def close(self):
        if self._h:
            check(lib().qloco_mgpu_destroy(self._h), "qloco_mgpu_destroy")
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
