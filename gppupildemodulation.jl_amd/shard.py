"""Multi-GPU layout of a series batch: series are independent, so each rank owns a
contiguous block of series (aligned to whole FC groups of 4) and fits it with no data-path
collective; the only exchange is one gather of the 64-byte parameter records to rank 0
(RCCL over xGMI under torch.distributed's "nccl" backend, gloo in CPU tests)."""
from __future__ import annotations

import numpy as np

GROUP = 4  # diodes sharing one fibre-coupler column (src/Modulation.jl:388-389)
RECORD_BYTES = 64  # gpd_param


def shard_range(n_total: int, world: int, rank: int, align: int = GROUP) -> tuple[int, int]:
    """[begin, end) of rank's contiguous block; boundaries on multiples of `align`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    groups = (n_total + align - 1) // align
    g0 = groups * rank // world
    g1 = groups * (rank + 1) // world
    return min(g0 * align, n_total), min(g1 * align, n_total)


def shard_counts(n_total: int, world: int, align: int = GROUP) -> list[int]:
    """Series per rank under shard_range."""
    return [e - b for b, e in (shard_range(n_total, world, r, align) for r in range(world))]


def weak_offset(per_rank: int, rank: int) -> int:
    """Global index of rank's first series when every rank owns `per_rank` series (weak scaling)."""
    if per_rank % GROUP:
        raise ValueError("per-rank series count must be a multiple of 4")
    return rank * per_rank


def gather_records(local, world: int, rank: int, dst: int = 0, group=None, counts=None,
                   force: bool = False):
    """Gather record tensors (uint8, n×64) to `dst`; returns the concatenation in rank order on
    dst, None elsewhere.  `counts` (records per rank, e.g. from shard_range) allows unequal
    shards: every rank sends max(counts) rows (one collective, the padding trimmed on dst).
    Works for CUDA tensors under nccl (RCCL) and CPU tensors under gloo.  At world size 1 the
    records are returned as they are, unless `force` (an initialised process group of one rank:
    the collective then runs, e.g. bench.py --dist-always)."""
    import torch
    import torch.distributed as dist

    if world == 1 and not force:
        return local
    n = local.shape[0]
    if counts is None:
        counts = [n] * world
    if counts[rank] != n:
        raise ValueError(f"rank {rank}: {n} records, counts says {counts[rank]}")
    m = max(counts)
    send = local
    if n < m:
        send = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        send[:n] = local
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send.contiguous(), gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


def records_to_numpy(t, dtype) -> np.ndarray:
    arr = t.detach().cpu().numpy()
    return arr.reshape(-1).view(dtype)
