"""Coherence across GPUs (docs/SPEC.md §5b) restated over gloo on CPU, world_size 2-4: each rank
is a DSM node of the test_mmult trace AND the home of a block of pages. Per round, every node
splits its stamped fault events by home, an all-to-all delivers them, each home merges them by
(page, seq), folds them into its page-table shard with the C oracle and returns the notices
(access changes) to the nodes with a second all-to-all. The shards and the notices must equal the
oracle's sequential fold of the whole trace (oracle.route_round). The GPU code of the same
protocol (gdsm_route_events / gdsm_coherence_notify) is tests/test_gpu_route.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gallocy_amd.trace import MmultTrace, mmult_layout
from oracle import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _a2a(parts):
    """all_to_all of variable-length uint64 arrays (gloo, int64 on the wire)."""
    world = dist.get_world_size()
    sizes = torch.tensor([len(p) for p in parts], dtype=torch.int64)
    got = torch.empty_like(sizes)
    dist.all_to_all_single(got, sizes)
    inp = torch.from_numpy(np.concatenate(parts).view(np.int64) if sum(map(len, parts))
                           else np.zeros(0, np.int64))
    out = torch.empty(int(got.sum()), dtype=torch.int64)
    dist.all_to_all_single(out, inp, output_split_sizes=got.tolist(),
                           input_split_sizes=[len(p) for p in parts])
    return [x.numpy().view(np.uint64) for x in torch.split(out, got.tolist())] if world else []


def _worker(rank, world, port, ndim, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = mmult_layout(ndim)
        T = MmultTrace(L, world, seed=11)
        Z = L.n_pages
        per = -(-Z // world)
        base = min(Z, rank * per)
        nh = max(0, min(Z, base + per) - base)
        st = np.full(nh, (1 << rank) | (rank << 8) | (2 << 16), np.uint32)  # SPEC §5 initial
        fl = np.zeros(nh, np.uint32)
        gst, gfl = oracle.coh_init(Z, world)   # the sequential reference, whole table
        ok = True
        acc = np.zeros(10, np.int64)
        for r in range(T.rounds):
            stamped = T.round_stamped(r)
            mine = stamped[rank]
            # node side: split by home (the list is sorted, homes are contiguous page blocks)
            keys = (np.arange(world + 1, dtype=np.uint64) * np.uint64(per)) << np.uint64(36)
            b = np.searchsorted(mine, keys, side="left")
            b[-1] = len(mine)
            runs = _a2a([mine[b[d]:b[d + 1]] for d in range(world)])
            # home side: merge by (page, seq), fold, notices
            ev = np.sort(np.concatenate(runs), kind="stable")
            plain = ((((ev >> np.uint64(36)) - np.uint64(base)) << np.uint64(4))
                     | (ev & np.uint64(15))).astype(np.uint64)
            pages = np.unique((plain >> np.uint64(4)).astype(np.int64))
            pre = st[pages].copy()
            rc, tot = oracle.coherence(st, fl, plain, n_nodes=world)
            ok &= rc == 0
            acc += [tot["invalidations"], tot["transfers"], *tot["node_faults"]]
            per_node = oracle.notices(pre, st[pages], pages.astype(np.uint64) + np.uint64(base),
                                      world)
            got = np.concatenate(_a2a(per_node))   # from every home, in home (= page) order
            # the sequential reference of the same round
            rc2, _, want = oracle.route_round(gst, gfl, stamped, world, Z)
            ok &= rc2 == 0 and bool(np.array_equal(got, want[rank]))
        ok &= bool(np.array_equal(st, gst[base:base + nh]) and np.array_equal(fl, gfl[base:base + nh]))
        t = torch.tensor(acc)
        dist.all_reduce(t)
        q.put((rank, ok, t.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,ndim", [(2, 64), (3, 96), (4, 128)])
def test_route_and_notify_gloo(world, ndim):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ndim, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T = MmultTrace(mmult_layout(ndim), world, seed=11)
    st, fl = oracle.coh_init(mmult_layout(ndim).n_pages, world)
    rc, tot = oracle.coherence(st, fl, T.all_events(), n_nodes=world)
    want = [tot["invalidations"], tot["transfers"], *tot["node_faults"]]
    for rank, ok, t in res:
        assert ok, rank
        assert t == want


def test_notice_rule():
    """SPEC §5b on hand-made words: a write by node 2 to a page SHARED by {0, 1} owned by 0
    invalidates 0 and 1, makes 2 the writer, and tells the old owner; a read by 3 of a page
    EXCLUSIVE at 1 downgrades 1 to read and grants 3 read."""
    sh = (0b11) | (0 << 8) | (1 << 16)
    ex2 = (1 << 2) | (2 << 8) | (2 << 16) | (1 << 18)
    ex1 = (1 << 1) | (1 << 8) | (2 << 16)
    sh13 = (1 << 1) | (1 << 3) | (1 << 8) | (1 << 16)
    out = oracle.notices([sh, ex1], [ex2, sh13], [5, 9], 4)
    dec = [[(int(x) & 0xFFFFFFFF, (int(x) >> 32) & 3, (int(x) >> 34) & 3, (int(x) >> 40) & 0xFF,
             (int(x) >> 48) & 0xFF) for x in o] for o in out]
    assert dec[0] == [(5, 1, 0, 0, 2)]
    assert dec[1] == [(5, 1, 0, 0, 2), (9, 2, 1, 1, 1)]
    assert dec[2] == [(5, 0, 2, 0, 2)]
    assert dec[3] == [(9, 0, 1, 1, 1)]
