"""Pair-level data parallelism: one process per GPU, pairs sharded in
contiguous blocks, gather of the int16 disparity maps to rank 0.

The reference processes one pair per call (``disparity_calculation.py:289``)
and has no distributed code.  Pairs are independent, so the
data path needs no collective; the only exchange is delivering results to
the root (BASELINE config "64 KITTI pairs sharded 8-per-GPU, gather over
xGMI").

The gather is a set of point-to-point transfers (``torch.distributed``
``batch_isend_irecv``: RCCL on ROCm, gloo on CPU): rank r sends its block,
rank 0 receives it straight into rows ``[start_r, start_r + count_r)`` of a
preallocated ``[npairs, H, W]`` result, so there is no padding of uneven
blocks and no concatenation on the root, and rank 0 computes its own block
directly into its rows.  Each peer uses its own xGMI link to the root, so the
transfers form a one-hop star, not a ring.  ``OverlappedGather`` runs step k's
transfers on a side stream while step k+1 computes into the other of two
buffers ("gather pair i while computing pair i+1").
"""
from __future__ import annotations

from collections import namedtuple
from typing import Callable, Sequence

# one point-to-point transfer of a gather: kind "send" | "recv", the byte view, the peer rank
P2P = namedtuple("P2P", "kind tensor peer")


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


def _bytes(t):
    """Raw-byte view of a contiguous tensor (RCCL and gloo have no int16 type)."""
    import torch

    return t.contiguous().view(torch.uint8)


def _p2p_plan(local, out, npairs: int, rank: int, world: int):
    """The transfers of one gather (group ranks): non-root ranks send ``local`` to rank 0;
    rank 0 receives every other rank's block into its rows of ``out``."""
    ops = []
    if rank == 0:
        for r in range(1, world):
            s, c = shard_range(npairs, r, world)
            if c:
                ops.append(P2P("recv", _bytes(out[s:s + c]), r))
    elif local.shape[0]:
        ops.append(P2P("send", _bytes(local), 0))
    return ops


def dist_transport(plan, group=None):
    """The transfers of a plan as one ``batch_isend_irecv`` (RCCL / gloo); returns its works."""
    import torch.distributed as dist

    if not plan:
        return []
    ops = [dist.P2POp(dist.isend if o.kind == "send" else dist.irecv, o.tensor,
                      dist.get_global_rank(group, o.peer) if group is not None else o.peer, group) for o in plan]
    return dist.batch_isend_irecv(ops)


def _gather_ops(local, out, npairs: int, group=None):
    """torch P2P operations of one gather (see _p2p_plan)."""
    import torch.distributed as dist

    plan = _p2p_plan(local, out, npairs, dist.get_rank(group), dist.get_world_size(group))
    return [dist.P2POp(dist.isend if o.kind == "send" else dist.irecv, o.tensor,
                       dist.get_global_rank(group, o.peer) if group is not None else o.peer, group) for o in plan]


def gather_to_root(local, npairs: int, group=None, out=None):
    """Gather each rank's [count, H, W] block to rank 0 (pair order kept).

    ``local`` is a torch tensor on this rank's device (CUDA under RCCL, CPU
    under gloo).  On rank 0 the blocks land in ``out`` (a preallocated
    [npairs, H, W] tensor of local's dtype and device; allocated if None) by
    point-to-point receives into its row ranges: uneven blocks need no padding
    and the root concatenates nothing.  Rank 0's own block is copied into its
    rows unless ``local`` already is that view.  Returns ``out`` on rank 0 and
    None elsewhere.  Synchronous for the caller's stream.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    H, W = local.shape[1:]
    if rank == 0:
        if out is None:
            out = torch.empty((npairs, H, W), dtype=local.dtype, device=local.device)
        s, c = shard_range(npairs, 0, world)
        if c and local.data_ptr() != out[s:s + c].data_ptr():
            out[s:s + c].copy_(local)
    ops = _gather_ops(local, out, npairs, group)
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return out if rank == 0 else None


class OverlappedGather:
    """Double-buffered gather of each step's maps to rank 0, overlapped with the
    next step's compute.

    Step k computes into ``buffer(k)``: on rank 0 that is a view of the rows
    it owns in ``result(k)`` (the [npairs, H, W] maps of step k), elsewhere a
    [count, H, W] block.  ``launch(k)`` starts step k's transfers once the
    caller's current stream has produced the block; on CUDA they run on a side
    stream (RCCL's own stream waits for it), so the caller's stream goes on
    with step k+1 at once.  ``buffer(k + depth)`` makes the caller's stream
    wait for step k's transfers before the buffer is overwritten.  On CPU
    (gloo) the transfers are asynchronous works completed at the same points.

    ``exposed_ms()`` (CUDA): the time the caller's stream stood waiting for a
    gather (events around every wait, ``drain`` included), i.e. the part of
    the gather that compute did not hide.

    ``transport(plan) -> works`` moves one step's transfers (a list of ``P2P``);
    the default is ``dist_transport`` over the process group.  ``rank`` / ``world``
    default to the group's.  tests/test_gpu_gather.py runs the CUDA branch with a
    stream-ordered device-copy transport (two ranks' roles in one process on one
    GPU: RCCL refuses two ranks on one device and torch refuses a send to self).
    """

    def __init__(self, npairs: int, count: int, H: int, W: int, dtype, device, group=None, depth: int = 2,
                 rank: int | None = None, world: int | None = None, transport: Callable | None = None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.npairs, self.depth = npairs, depth
        self.world = dist.get_world_size(group) if world is None else world
        self.rank = dist.get_rank(group) if rank is None else rank
        self.transport = transport or (lambda plan: dist_transport(plan, group))
        self.start, c = shard_range(npairs, self.rank, self.world)
        if c != count:
            raise ValueError(f"rank {self.rank} owns {c} pairs, got count {count}")
        self.count = count
        self.cuda = getattr(device, "type", str(device)).startswith("cuda")
        if self.rank == 0:
            self.results = [torch.empty((npairs, H, W), dtype=dtype, device=device) for _ in range(depth)]
            self.blocks = [r[self.start:self.start + count] for r in self.results]
        else:
            self.results = [None] * depth
            self.blocks = [torch.empty((count, H, W), dtype=dtype, device=device) for _ in range(depth)]
        self.pending = [None] * depth  # CUDA: event on the side stream; CPU: list of works
        self.stream = torch.cuda.Stream(device) if self.cuda else None
        self.timing = False
        self.stalls = []  # CUDA: (start, end) events around each wait on the caller's stream
        self.spans = []   # CUDA: (start, end) events around each step's transfers on the side stream
        self.cpu_stall_s = 0.0  # CPU: host time spent completing works

    def buffer(self, k: int):
        """The block step k computes into (waits for step k - depth's transfers)."""
        slot = k % self.depth
        self._wait(slot)
        return self.blocks[slot]

    def result(self, k: int):
        """Rank 0: step k's [npairs, H, W] maps (complete after ``wait(k)``)."""
        return self.results[k % self.depth]

    def launch(self, k: int):
        """Start step k's transfers after the work already on the caller's stream."""
        slot = k % self.depth
        ops = _p2p_plan(self.blocks[slot], self.results[slot], self.npairs, self.rank, self.world)
        if not ops:  # world 1 (or an empty block): rank 0 computed into its rows already
            return
        if self.cuda:
            torch = self.torch
            cur = torch.cuda.current_stream()
            with torch.cuda.stream(self.stream):
                self.stream.wait_stream(cur)
                a = None
                if self.timing:
                    a = torch.cuda.Event(enable_timing=True)
                    a.record(self.stream)
                for w in self.transport(ops):
                    w.wait()  # the side stream waits for RCCL's stream (no host wait)
                ev = torch.cuda.Event(enable_timing=self.timing)
                ev.record(self.stream)
                if a is not None:
                    self.spans.append((a, ev))
            # the caller's allocator must not reuse the block before the transfer has read it
            self.blocks[slot].record_stream(self.stream)
            self.pending[slot] = ev
        else:
            self.pending[slot] = self.transport(ops)

    def wait(self, k: int):
        """The caller (its stream on CUDA) waits for step k's transfers."""
        self._wait(k % self.depth)

    def drain(self):
        for slot in range(self.depth):
            self._wait(slot)

    def _wait(self, slot: int):
        p = self.pending[slot]
        if p is None:
            return
        self.pending[slot] = None
        if self.cuda:
            torch = self.torch
            cur = torch.cuda.current_stream()
            if self.timing:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(cur)
                cur.wait_event(p)
                b.record(cur)
                self.stalls.append((a, b))
            else:
                cur.wait_event(p)
        else:
            import time

            t0 = time.perf_counter()
            for w in p:
                w.wait()
            if self.timing:
                self.cpu_stall_s += time.perf_counter() - t0

    def exposed_ms(self) -> float:
        """Summed stall of the caller on gathers since ``reset_stats`` (CUDA: of its
        stream, read after a device sync; CPU: host time completing the works)."""
        if self.cuda:
            return sum(a.elapsed_time(b) for a, b in self.stalls)
        return self.cpu_stall_s * 1e3

    def transfer_ms(self) -> float:
        """Summed duration of the transfers on the side stream (CUDA; rank 0: all
        receives of a step, other ranks: their send) since ``reset_stats``."""
        return sum(a.elapsed_time(b) for a, b in self.spans)

    def reset_stats(self, timing: bool = True):
        self.timing = timing
        self.stalls, self.spans, self.cpu_stall_s = [], [], 0.0


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
