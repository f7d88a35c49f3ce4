"""world_size-2 gloo rehearsal of the multi-GPU path (host logic on CPU):
shards tile the buffer in rank order on segment boundaries, and the timing
reduction takes the maximum over ranks."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from zt_shard import SEGMENT, max_over_ranks, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lo, hi = shard_range(n, world, rank)
    t = torch.tensor([lo, hi], dtype=torch.int64)
    got = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(got, t)
    m = max_over_ranks(1.0 + rank, dist)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, [tuple(x.tolist()) for x in got], m))


@pytest.mark.parametrize("n", [0, 1, SEGMENT - 1, 3 * SEGMENT + 17, 8 << 30])
def test_gloo_world2_shards_and_timing(n):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ranges, m in res:
        assert m == float(world)  # max over ranks
        assert ranges[0][0] == 0 and ranges[-1][1] == n
        for (a, b), (c, d) in zip(ranges, ranges[1:]):
            assert b == c and a <= b
        for a, b in ranges:
            assert a % SEGMENT == 0 or a == n


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_tiles(world):
    for n in [0, 5, SEGMENT, 10 * SEGMENT + 3]:
        rs = [shard_range(n, world, r) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
