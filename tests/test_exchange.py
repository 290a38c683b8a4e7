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
        b = exchange.dest_bounds(rank, world, n)
        sids = exchange.send_ids(rank, world, n)
        send = []
        for d in range(world):  # one stream per destination, as the GPU shard diffs them
            ro, data = oracle.diff_pages(twin, cur, ids=np.arange(b[d], b[d + 1], dtype=np.uint32))
            send.append((ro, sids[d], data))
        got = exchange.GlooTransport().exchange(send)
        _, _, rep = oracle.gen_pages(n, seed=seed, mode=mode, ppm=ppm, first_page=rank * n, replica=True)
        rc = 0
        for ro, ids, data in got:  # the home applies every source's stream
            rc |= oracle.apply(rep, ro, data, ids=ids)
        _, want = oracle.gen_pages(n, seed=seed, mode=mode, ppm=ppm, first_page=rank * n)
        sent_remote = sum(int(s[0][-1]) for d, s in enumerate(send) if d != rank)
        total = sum(int(s[0][-1]) for s in send)
        received = sum(int(g[0][-1]) for s, g in enumerate(got) if s != rank)
        q.put((rank, rc, bool(np.array_equal(rep, want)), sent_remote, received, total))
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
        assert 0 < sent_remote < total and received > 0


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
        # every home index is received exactly once, from its writer
        got = np.concatenate([exchange.send_ids(r, world, n)[d] + d * n
                              for r in range(world) for d in range(world)])
        assert sorted(got.tolist()) == list(range(world * n))
        assert all(len(x) == 0 or x.max() < n for r in range(world)
                   for x in exchange.send_ids(r, world, n))


def test_budget_covers_and_is_aligned():
    for b in (0, 1, 4, 1000, 123456, 1 << 30):
        x = exchange.budget(b)
        assert x >= b + 4096 and x % 256 == 0


def _hang_worker(rank, world, port, deadline):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wd = exchange.Watchdog(rank).arm(deadline, "first exchange")
    if rank == 1:
        import time
        time.sleep(600)  # the peer that hangs
    n = 16
    twin, cur = oracle.gen_pages(n, seed=1, mode=0, ppm=10000, first_page=rank, stride=world)
    sids = exchange.send_ids(rank, world, n)
    b = exchange.dest_bounds(rank, world, n)
    send = []
    for d in range(world):
        ro, data = oracle.diff_pages(twin, cur, ids=np.arange(b[d], b[d + 1], dtype=np.uint32))
        send.append((ro, sids[d], data))
    exchange.GlooTransport().exchange(send)  # blocks: rank 1 never joins
    wd.disarm()


def test_watchdog_ends_ranks_blocked_on_a_hung_peer():
    """World size 2 over gloo on the CPU: rank 1 hangs before the first exchange, rank 0 blocks
    in it. Both ranks' watchdogs (exchange.Watchdog, the one bench.py --deadline arms) end their
    processes with status 3 within about the deadline, instead of the job hanging."""
    import time
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_hang_worker, args=(r, 2, port, 5.0)) for r in range(2)]
    t0 = time.monotonic()
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=90)
    assert all(p.exitcode == 3 for p in procs), [p.exitcode for p in procs]
    assert time.monotonic() - t0 < 80
