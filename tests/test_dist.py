"""world_size-2 gloo coverage of the pair sharding + gather (CPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stereo_match_amd.batch import gather_to_root, run_sharded, shard_range


@pytest.mark.parametrize("n,world", [(64, 8), (10, 3), (2, 4), (0, 2), (7, 1)])
def test_shard_range_partitions(n, world):
    spans = [shard_range(n, r, world) for r in range(world)]
    covered = [i for s, c in spans for i in range(s, s + c)]
    assert covered == list(range(n))
    counts = [c for _, c in spans]
    assert max(counts) - min(counts) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lefts = [torch.full((3, 5), i, dtype=torch.uint8) for i in range(n)]
        rights = [torch.full((3, 5), 2 * i, dtype=torch.uint8) for i in range(n)]
        seen = []

        def fake(l, r):  # stands in for the GPU matcher: encodes which pair it saw
            seen.append(int(l[0, 0]))
            return (l.to(torch.int16) * 16 + r.to(torch.int16))

        out = run_sharded(lefts, rights, fake, gather=True)
        if rank == 0:
            q.put(("out", out.tolist()))
        q.put(("seen", rank, seen))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [5, 4])
def test_gloo_two_ranks_gather(n):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=120) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = [m for m in msgs if m[0] == "out"][0][1]
    expect = [[[i * 16 + 2 * i] * 5] * 3 for i in range(n)]
    assert out == expect
    seen = {m[1]: m[2] for m in msgs if m[0] == "seen"}
    s0, c0 = shard_range(n, 0, world)
    assert seen[0] == list(range(s0, s0 + c0))
    assert sorted(seen[0] + seen[1]) == list(range(n))


def _oracle_worker(rank, world, port, n, q):
    """Real pairs through the C restatement on every rank (stands in for the
    per-GPU matcher), gathered to rank 0 as bench.py does over RCCL."""
    import numpy as np

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import ref_c
        from stereo_match_amd import synthetic

        pairs = [synthetic.random_dot_pair(20, 70, 16, seed=200 + i)[:2] for i in range(n)]
        p = synthetic.headline_params(16)
        out = run_sharded([torch.from_numpy(a) for a, _ in pairs], [torch.from_numpy(b) for _, b in pairs],
                          lambda l, r: torch.from_numpy(ref_c.compute(l.numpy(), r.numpy(), p)), gather=True)
        if rank == 0:
            q.put(out.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 5), (4, 6), (4, 3)])
def test_gloo_sharded_matches_single_process(world, n):
    """every shard's output equals the single-process output."""
    import numpy as np

    from oracle import ref_c
    from stereo_match_amd import synthetic

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_oracle_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    p = synthetic.headline_params(16)
    for i in range(n):
        a, b, _ = synthetic.random_dot_pair(20, 70, 16, seed=200 + i)
        assert np.array_equal(got[i], ref_c.compute(a, b, p)), i


def _overlap_worker(rank, world, port, n, steps, q):
    """OverlappedGather over gloo: step k writes pair i's block as (k, i)-coded maps; every
    step's result on rank 0 must hold all pairs in order, although step k+1 computes while
    step k's transfers are in flight."""
    from stereo_match_amd.batch import OverlappedGather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, count = shard_range(n, rank, world)
        og = OverlappedGather(n, count, 3, 4, torch.int16, torch.device("cpu"))
        og.reset_stats(timing=True)
        ok = []
        for k in range(steps):
            buf = og.buffer(k)
            assert buf.shape == (count, 3, 4)
            for j in range(count):
                buf[j].fill_(100 * k + start + j)
            og.launch(k)
            if rank == 0 and k >= 1:  # the previous step's maps, completed after wait(k - 1)
                og.wait(k - 1)
                got = og.result(k - 1)
                ok.append(all(bool((got[i] == 100 * (k - 1) + i).all()) for i in range(n)))
        og.drain()
        if rank == 0:
            got = og.result(steps - 1)
            ok.append(all(bool((got[i] == 100 * (steps - 1) + i).all()) for i in range(n)))
            # rank 0's own block is a view of its rows (nothing copied)
            assert og.buffer(steps).data_ptr() == og.result(steps)[start:].data_ptr()
            q.put((ok, og.exposed_ms()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 4), (4, 8), (4, 6), (3, 2)])
def test_gloo_overlapped_gather_pair_order(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, n, 5, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, exposed = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok and all(ok), ok
    assert exposed >= 0


def _root_out_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 5
        s, c = shard_range(n, rank, world)
        local = torch.stack([torch.full((2, 3), i, dtype=torch.int16) for i in range(s, s + c)])
        out = torch.full((n, 2, 3), -1, dtype=torch.int16) if rank == 0 else None
        res = gather_to_root(local, n, out=out)
        if rank == 0:
            q.put((res.data_ptr() == out.data_ptr(), res.tolist()))
    finally:
        dist.destroy_process_group()


def test_gather_to_root_fills_preallocated_out():
    # uneven blocks (3 + 2 pairs) land in the caller's tensor, no padding, no concatenation
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_root_out_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    same, got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same
    assert got == [[[i] * 3] * 2 for i in range(5)]
