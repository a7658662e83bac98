"""Instance sharding of a robot fleet over ranks.

The OCP instances are independent, so a multi-GPU job is one process per GPU, each owning a contiguous
range of robot indices of every model, with no collective on the solve path. The only collectives are
the harness's: a barrier around the timed region, a MAX all-reduce of the elapsed time, and (optional)
an all-gather of the per-tick commands to rank 0 for a fleet manager. Backend "nccl" (= RCCL over xGMI)
on the GPU box, "gloo" in the CPU tests.
"""
import time

import torch
import torch.distributed as dist


def shard_range(total, rank, world):
    """Balanced contiguous [lo, hi) of `total` instances for `rank` (the first total % world ranks get one
    more)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    q, r = divmod(int(total), world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def mixed_counts(total, models):
    """Split `total` robots over `models` as evenly as possible (remainder to the first models)."""
    q, r = divmod(int(total), len(models))
    return [(m, q + (1 if j < r else 0)) for j, m in enumerate(models)]


def world_info():
    """(rank, world, local_rank) from torchrun's environment (single process when unset)."""
    import os
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _sync(device):
    if device is not None and device.type == "cuda":
        torch.cuda.synchronize(device)


class TimedRegion:
    """Barrier + device sync on both sides, elapsed = MAX over ranks (bench.py contract)."""

    def __init__(self, device=None):
        self.device = device
        self.elapsed = None

    def __enter__(self):
        if dist.is_initialized():
            dist.barrier()
        _sync(self.device)
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        _sync(self.device)
        if dist.is_initialized():
            dist.barrier()
        el = time.perf_counter() - self._t0
        if dist.is_initialized():
            t = torch.tensor([el], dtype=torch.float64, device=self.device if self.device is not None else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        self.elapsed = el
        return False


class CommandGather:
    """All-gather of per-robot commands [rows][B_rank] to every rank (rank 0 keeps the fleet view).
    Ranks may hold different robot counts: buffers are padded to the largest shard.

    Two uses:
      * joined ticks: ``gather(parts)`` (or calling the object) copies the parts into the staging buffer and
        all-gathers it at once;
      * decoupled streams (FleetNode): each fleet copies its part into staging slot ``slot`` on its own stream
        when its tick is done (``stage``), and ``collect(slot)`` all-gathers that slot on the gather stream once
        every part has arrived. ``slots`` staging buffers rotate so that a fleet can run its next ticks while
        the gather of an earlier one is in flight."""

    def __init__(self, rows, counts, device, slots=2):
        self.rows, self.counts = rows, list(counts)
        self.pad = max(self.counts)
        self.slots = slots
        self.stage_bufs = [torch.zeros(rows, self.pad, device=device) for _ in range(slots)]
        self.recv = [[torch.zeros(rows, self.pad, device=device) for _ in self.counts] for _ in range(slots)]
        self.src = self.stage_bufs[0]
        self.bufs = self.recv[0]

    def stage(self, slot, off, part):
        """Copy one fleet's [r][b] part into staging slot `slot` at robot offset `off` (caller's stream)."""
        self.stage_bufs[slot][:part.shape[0], off:off + part.shape[1]].copy_(part)

    def collect(self, slot):
        """All-gather staging slot `slot` (on the current stream) -> [rows][total]."""
        src, bufs = self.stage_bufs[slot], self.recv[slot]
        if dist.is_initialized():  # (world size 1 too: bench.py --dist runs the RCCL call on one GPU)
            dist.all_gather(bufs, src)
        else:
            bufs[0].copy_(src)
        return torch.cat([b[:, :c] for b, c in zip(bufs, self.counts)], dim=1)

    def __call__(self, parts):
        """parts: list of [r_i][b_i] tensors (per model) concatenated along robots; returns [rows][total]."""
        off = 0
        self.src.zero_()
        for p in parts:
            self.stage(0, off, p)
            off += p.shape[1]
        return self.collect(0)
