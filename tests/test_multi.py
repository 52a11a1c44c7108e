"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 bench path: streams shard
one per rank with no data-path collective; only the timing uses a MAX reduction."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        elapsed = 1.0 + rank  # rank 1 is the slow one
        m = bench.max_over_ranks(elapsed, dist)
        q.put((rank, m, bench.aggregate_fps(world, 60, m), bench.stream_seed(0x5EED0001, rank)))
    finally:
        dist.destroy_process_group()


def test_two_rank_timing_and_sharding():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank sees the max elapsed; value = all ranks' frames / that time
    assert [r[1] for r in res] == [2.0, 2.0]
    assert res[0][2] == pytest.approx(2 * 60 / 2.0)
    # independent streams per rank
    assert res[0][3] != res[1][3]


def test_single_rank_passthrough():
    assert bench.max_over_ranks(1.5, None) == 1.5
    assert bench.aggregate_fps(1, 60, 2.0) == 30.0
