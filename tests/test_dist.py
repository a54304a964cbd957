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
