"""Multi-GPU partition sharding on the CPU: world_size 2 over gloo.

Each rank owns a contiguous partition range (redpanda_amd/shard.py,
SURVEY.md §8e), validates only its own batches and reduces them to
per-partition summaries; the one exchange is the all-gather of those
summaries.  Here the batch results come from the oracle (the GPU is not
needed for the sharding logic under test); rank 0 checks the gathered table
against a single-process computation over every batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

PARTS = 13  # not a multiple of the world size: unequal ranges


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def arena():
    from redpanda_amd import engine

    spec = engine.make_spec(seed=0x5EED0E00, partitions=PARTS, records_per_batch=3, key_len=4, value_len=60,
                            corrupt_ppm=150_000, corrupt_mask=0x1FF)
    return engine.build_arena(spec, 700, nthreads=2)


def worker(rank: int, world: int, port: int, q):
    import oracle.oracle as orc
    from redpanda_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data, descs = arena()
        lo, hi = shard.partition_range(rank, world, PARTS)
        mine = descs[(descs["partition"] >= lo) & (descs["partition"] < hi)]
        res, _, _ = orc.validate_arena(data, mine)
        local = shard.partition_summaries(torch.from_numpy(res.view(np.uint8).copy()),
                                          torch.from_numpy(mine["partition"].astype(np.int64)), lo, hi)
        table = shard.gather_summaries(local, world, PARTS)
        q.put((rank, table.numpy()))
    finally:
        dist.destroy_process_group()


def test_partition_ranges_cover():
    from redpanda_amd import shard

    for world in (1, 2, 3, 8):
        for P in (1, 13, 4096, 65536):
            rs = [shard.partition_range(g, world, P) for g in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == P
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_summaries_match_numpy(built):
    import oracle.oracle as orc
    from redpanda_amd import shard

    data, descs = arena()
    res, _, _ = orc.validate_arena(data, descs)
    got = shard.partition_summaries(torch.from_numpy(res.view(np.uint8).copy()),
                                    torch.from_numpy(descs["partition"].astype(np.int64)), 0, PARTS).numpy()
    assert np.array_equal(got, shard.summaries_numpy(res, descs["partition"], 0, PARTS))
    assert len(np.unique(res["verdict"])) >= 4


def test_two_rank_gloo_gather(built):
    import oracle.oracle as orc
    from redpanda_amd import shard

    world, port = 2, free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data, descs = arena()
    res, _, _ = orc.validate_arena(data, descs)
    want = shard.summaries_numpy(res, descs["partition"], 0, PARTS)
    for r in range(world):
        assert np.array_equal(out[r], want), r
