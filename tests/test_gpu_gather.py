"""BASELINE config 4's overlapped gather (stereo_match_amd.batch.OverlappedGather) through
its CUDA branch with bytes in flight, on the one GPU a test box has.

RCCL refuses two ranks on one device and torch refuses a send to the own rank, so the
transfers go through an injected transport: a device copy enqueued on the side stream the
gather runs them on (exactly where RCCL's kernels would be ordered), preceded by a delay
kernel.  The two roles of a 2-rank gather are driven in one process: the sender (rank 1),
whose block must not be overwritten before its send has read it, and the root (rank 0),
which receives the peer's block into its rows of the double-buffered result.  Slow producer
kernels before each send, and slow transfers after each step, make a missing
``wait_stream`` / ``wait_event`` show as wrong bytes."""
import pytest
import torch

from stereo_match_amd.batch import OverlappedGather

pytestmark = pytest.mark.gpu

H, W, COUNT = 375, 1242, 2  # two KITTI-size int16 maps per rank: 1.9 MB per transfer
SLOW = 4_000_000  # torch.cuda._sleep cycles (~ms): longer than a step's other work


def pattern(k, rank, npairs=2 * COUNT):
    """Step k's maps of `rank`'s block, distinct per step, pair and pixel."""
    i = torch.arange(COUNT * H * W, device="cuda", dtype=torch.int32).reshape(COUNT, H, W)
    return ((i * 7 + k * 131 + rank * 977) % 30011).to(torch.int16)


class DeviceCopyTransport:
    """transport(plan): each transfer is a copy on the current stream (the gather's side
    stream), after a delay kernel of `delay` cycles.  A send lands in sink[n] (n = call
    number); a receive copies source[n] into the plan's destination rows."""

    def __init__(self, delay=0, sink=None, source=None):
        self.delay, self.sink, self.source, self.calls = delay, sink, source, 0

    def __call__(self, plan):
        n = self.calls
        self.calls += 1
        for o in plan:
            if self.delay:
                torch.cuda._sleep(self.delay)
            if o.kind == "send":
                self.sink[n].view(torch.uint8).view(-1).copy_(o.tensor.view(-1))
            else:
                o.tensor.view(-1).copy_(self.source[n].view(torch.uint8).view(-1))
        return []  # stream-ordered: nothing for the side stream to wait on


def _sender_run(steps, producer_sleep, transfer_delay):
    sink = [torch.full((COUNT, H, W), -1, dtype=torch.int16, device="cuda") for _ in range(steps)]
    tr = DeviceCopyTransport(transfer_delay, sink=sink)
    og = OverlappedGather(2 * COUNT, COUNT, H, W, torch.int16, torch.device("cuda", 0), rank=1, world=2,
                          transport=tr)
    og.reset_stats(timing=True)
    for k in range(steps):
        buf = og.buffer(k)  # waits for step k - 2's send before the block is rewritten
        if producer_sleep:
            torch.cuda._sleep(producer_sleep)  # the block's producer is slow
        buf.copy_(pattern(k, 1))
        og.launch(k)
    og.drain()
    torch.cuda.synchronize()
    return og, sink


def test_sender_waits_for_the_producer():
    """A slow producer before every send: the side stream must wait for the caller's stream
    (wait_stream) or the copies read the previous step's bytes."""
    og, sink = _sender_run(6, SLOW, 0)
    for k in range(6):
        assert torch.equal(sink[k], pattern(k, 1)), f"step {k}: the send read the block before it was written"
    assert og.transfer_ms() > 0


def test_sender_buffer_not_overwritten_before_its_send():
    """Slow transfers: buffer(k) must make the caller's stream wait for step k - 2's send
    (wait_event), else step k's data overwrites a block still being sent.  The caller's
    stream then stood waiting, so exposed_ms is > 0."""
    og, sink = _sender_run(6, 0, SLOW)
    for k in range(6):
        assert torch.equal(sink[k], pattern(k, 1)), f"step {k}: its block was overwritten before the send"
    assert og.transfer_ms() > 0 and og.exposed_ms() > 0


def test_root_receives_in_pair_order_while_computing_the_next_step():
    """Rank 0: its own rows are computed in place, rank 1's rows arrive by the (slow)
    receive of step k while step k + 1 computes into the other result buffer."""
    steps = 5
    source = [torch.empty((COUNT, H, W), dtype=torch.int16, device="cuda") for _ in range(steps)]
    tr = DeviceCopyTransport(SLOW, source=source)
    og = OverlappedGather(2 * COUNT, COUNT, H, W, torch.int16, torch.device("cuda", 0), rank=0, world=2,
                          transport=tr)
    og.reset_stats(timing=True)
    for k in range(steps):
        buf = og.buffer(k)
        source[k].copy_(pattern(k, 1))  # what rank 1 sends at step k
        torch.cuda._sleep(SLOW // 4)
        buf.copy_(pattern(k, 0))
        og.launch(k)
        if k >= 1:  # step k - 1's result is complete once its receive finished
            og.wait(k - 1)
            res = og.result(k - 1)
            assert torch.equal(res[:COUNT], pattern(k - 1, 0)), f"step {k - 1}: rank 0's rows"
            assert torch.equal(res[COUNT:], pattern(k - 1, 1)), f"step {k - 1}: rank 1's rows"
    og.drain()
    res = og.result(steps - 1)
    assert torch.equal(res[COUNT:], pattern(steps - 1, 1)) and torch.equal(res[:COUNT], pattern(steps - 1, 0))
    torch.cuda.synchronize()
    assert og.transfer_ms() > 0 and og.exposed_ms() > 0
