"""Object sharding across ranks.

Carbonado objects are independent, so the multi-GPU layout is a contiguous
partition of the object index space over ranks with no exchange step: no
collective touches shard or stream bytes.  torch.distributed is used only for
the control plane (barrier, max-over-ranks time, optional input scatter).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class ObjectRange:
    rank: int
    world: int
    start: int  # first global object index owned by this rank
    count: int  # objects owned

    @property
    def stop(self) -> int:
        return self.start + self.count


def object_range(rank: int, world: int, total: int) -> ObjectRange:
    """Contiguous, balanced partition: the first total % world ranks get one extra."""
    if not (0 <= rank < world) or total < 0:
        raise ValueError("bad rank/world/total")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return ObjectRange(rank, world, start, base + (1 if rank < extra else 0))


def max_over_ranks(value: float) -> float:
    """MAX of a host scalar over the default process group (control plane)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: int) -> int:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def scatter_objects(local: torch.Tensor, full: torch.Tensor | None, src: int = 0) -> None:
    """Root `src` holds `full` [world * per_rank, n]; every rank receives its
    contiguous slice into `local` [per_rank, n].  With the nccl backend this is
    RCCL's scatter over xGMI (one peer link per receiver); used only to stage
    inputs, never inside the timed hot path."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    chunks = list(full.chunk(world, dim=0)) if rank == src else None
    if chunks is not None:
        chunks = [c.contiguous() for c in chunks]
    dist.scatter(local, chunks, src=src)
