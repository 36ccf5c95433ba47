"""Instance sharding and the one collective of the multi-GPU path.

The SRBD instances are independent, so the path shards with no exchange
during the solve: rank r owns the contiguous global range
[r*B, (r+1)*B) (weak scaling, B instances per GPU), or the stride-interleaved
ids r, r + world, ... (interleaved_shard), and regenerates its inputs locally
from (seed, global id).  The only collective is one all-gather
of the solved first-step forces u0 (12 fp32 per instance) so every rank ends
with the whole batch's forces — a single RCCL all-gather over xGMI (backend
"nccl" is RCCL on ROCm); the CPU tests drive the same code over gloo.
"""
import torch
import torch.distributed as tdist


def shard_range(per_rank, rank):
    """Global instance ids [first, first + count) owned by `rank` (weak scaling)."""
    if per_rank < 0 or rank < 0:
        raise ValueError("per_rank and rank must be non-negative")
    return rank * per_rank, per_rank


def interleaved_shard(per_rank, world, rank):
    """Stride-interleaved shard: rank r owns the
    global ids r, r + world, r + 2 world, ... -- (first, stride, count) for
    srbd.generate.  Mixed per-instance schedules diverge in iteration count;
    interleaving spreads any run of long instances in id order over all
    ranks instead of loading one rank with it."""
    if per_rank < 0 or rank < 0 or world < 1 or rank >= world:
        raise ValueError("need 0 <= rank < world and per_rank >= 0")
    return rank, world, per_rank


def strong_shard_range(total, world, rank):
    """Balanced contiguous split of `total` instances over `world` ranks."""
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


class ForceGather:
    """All-gather of per-rank u0 (B, 12) into a (world*B, 12) buffer, rank order.

    The output buffer is allocated once and reused every step, so the
    collective is the only work (no allocation inside the timed region).
    """

    def __init__(self, per_rank, width=12, device=None, group=None):
        self.group = group
        self.world = tdist.get_world_size(group)
        self.per_rank = per_rank
        self.out = torch.empty((self.world * per_rank, width), dtype=torch.float32, device=device)
        self._flat = tdist.get_backend(group) != "gloo"
        if not self._flat:
            self._views = list(self.out.split(per_rank))

    def global_order(self, out=None, interleaved=False):
        """The gathered rows in global id order: rank order for contiguous
        shards (the buffer itself), row k * world + r for interleaved shards
        (a reordering copy)."""
        out = self.out if out is None else out
        if not interleaved:
            return out
        w = out.shape[1]
        return out.view(self.world, self.per_rank, w).transpose(0, 1).reshape(-1, w)

    def __call__(self, u0, async_op=False):
        """Gather u0 of every rank into self.out.  async_op=True returns
        (out, work): the collective runs on the backend's stream (after the
        work already queued on the current one) and work.wait() makes the
        current stream wait for it -- so a caller can solve the next batch
        into another u0 buffer while this one is in flight."""
        if u0.shape[0] != self.per_rank:
            raise ValueError("u0 has %d rows, expected %d" % (u0.shape[0], self.per_rank))
        if self._flat:
            work = tdist.all_gather_into_tensor(self.out, u0.contiguous(), group=self.group,
                                                async_op=async_op)
        else:  # gloo has no flat all-gather
            work = tdist.all_gather(self._views, u0.contiguous(), group=self.group,
                                    async_op=async_op)
        return (self.out, work) if async_op else self.out
