"""Pair-level data parallelism: one process per GPU, pairs sharded in
contiguous blocks, optional gather of the int16 disparity maps to rank 0.

The reference processes one pair per call (``disparity_calculation.py:289``)
and has no distributed code.  Pairs are independent, so the
data path needs no collective; the only exchange is delivering results to
the root (BASELINE config "64 KITTI pairs sharded 8-per-GPU, gather over
xGMI"), done with ``torch.distributed.gather`` (RCCL on ROCm, gloo on CPU).
"""
from __future__ import annotations

from typing import Callable, Sequence


def shard_range(npairs: int, rank: int, world: int):
    """Contiguous block of pairs owned by ``rank``: returns (start, count).

    Blocks differ in size by at most one pair; lower ranks take the extra.
    """
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    if npairs < 0:
        raise ValueError("npairs < 0")
    base, extra = divmod(npairs, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def gather_to_root(local, npairs: int, group=None):
    """Gather each rank's [count, H, W] int16 block to rank 0 (pair order kept).

    ``local`` is a torch tensor on this rank's device (CUDA under RCCL, CPU
    under gloo).  Ranks with uneven counts are padded to the largest block.
    Returns the [npairs, H, W] tensor on rank 0 and None elsewhere.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [shard_range(npairs, r, world)[1] for r in range(world)]
    cmax = max(counts) if counts else 0
    H, W = local.shape[1:]
    buf = local
    if local.shape[0] < cmax:
        buf = torch.zeros((cmax, H, W), dtype=local.dtype, device=local.device)
        buf[:local.shape[0]] = local
    # RCCL/NCCL and gloo have no int16 type: move the maps as raw bytes.
    raw = buf.contiguous().view(torch.uint8)
    if rank == 0:
        parts = [torch.empty_like(raw) for _ in range(world)]
        dist.gather(raw, gather_list=parts, dst=0, group=group)
        return torch.cat([p.view(local.dtype)[:c] for p, c in zip(parts, counts)], 0)
    dist.gather(raw, dst=0, group=group)
    return None


def run_sharded(lefts: Sequence, rights: Sequence, compute_fn: Callable, gather: bool = True, group=None):
    """Compute this rank's shard with ``compute_fn(left, right) -> int16 tensor``
    and optionally gather all maps to rank 0."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    n = len(lefts)
    start, count = shard_range(n, rank, world)
    outs = [compute_fn(lefts[i], rights[i]) for i in range(start, start + count)]
    local = torch.stack(outs) if outs else None
    if not gather or world == 1:
        return local
    if local is None:
        H, W = lefts[0].shape
        local = torch.empty((0, H, W), dtype=torch.int16,
                            device=lefts[0].device if hasattr(lefts[0], "device") else "cpu")
    return gather_to_root(local, n, group)
