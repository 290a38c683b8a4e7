"""Multi-rank diff propagation (gallocy_amd/exchange.py) on CPU: world_size 2 and 3 over gloo,
with the C oracle producing and applying the streams. Checks that every home shard's REPLICA
ends equal to the CURRENT content written by the other ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gallocy_amd import exchange
from oracle import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, mode, ppm, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seed = 31
        twin, cur = oracle.gen_pages(n, seed=seed, mode=mode, ppm=ppm, first_page=rank, stride=world)
        ro, data = oracle.diff_pages(twin, cur)
        b = exchange.dest_bounds(rank, world, n)
        off, rdata, sent_remote, received = exchange.exchange_stream(
            torch.from_numpy(ro.astype(np.int64)), torch.from_numpy(data), b, world)
        _, _, rep = oracle.gen_pages(n, seed=seed, mode=mode, ppm=ppm, first_page=rank * n, replica=True)
        rc = oracle.apply(rep, off.numpy().astype(np.uint64), rdata.numpy(), ids=exchange.recv_ids(world, n))
        _, want = oracle.gen_pages(n, seed=seed, mode=mode, ppm=ppm, first_page=rank * n)
        q.put((rank, rc, bool(np.array_equal(rep, want)), sent_remote, received, int(ro[-1])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,ppm", [(2, 0, 10000), (3, 1, 100000), (4, 0, 200000)])
def test_exchange_gloo(world, mode, ppm):
    n = 48 * world
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, mode, ppm, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, rc, ok, sent_remote, received, total in res:
        assert rc == 0 and ok, (rank, rc)
        assert 0 < sent_remote < total


def test_dest_bounds_partition():
    for world in (1, 2, 3, 8):
        n = 24 * world
        seen = np.zeros(world * n, int)
        for r in range(world):
            b = exchange.dest_bounds(r, world, n)
            assert b[0] == 0 and b[-1] == n
            for d in range(world):
                pages = np.arange(b[d], b[d + 1]) * world + r
                assert np.all(pages // n == d)
                seen[pages] += 1
        assert np.all(seen == 1)
        ids = exchange.recv_ids(world, n)
        assert sorted(ids.tolist()) == list(range(n))
