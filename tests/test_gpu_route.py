"""Coherence across GPUs on ONE GPU (docs/SPEC.md §5b): G ranks as threads, each a DSM node with its
own page-table shard context on cuda:0, wired by the loopback communicator. Every batch goes
through gdsm_route_events (nodes -> homes, merged by (page, seq)) and gdsm_coherence_notify (fold
+ notices back); the shards, the per-batch totals and every node's notices must equal the
oracle's sequential fold of all nodes' events (oracle.route_round). Also: empty nodes, empty
batches, and the collective refusals (-EINVAL for an unsorted list, -ENOSPC for a small buffer)
returned on every rank with nothing moved."""
import errno
import threading

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd import exchange
from oracle import oracle

pytestmark = pytest.mark.gpu


def run_ranks(G, fn):
    errs = [None] * G

    def body(r):
        try:
            fn(r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e
    th = [threading.Thread(target=body, args=(r,)) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=110)
    assert not any(t.is_alive() for t in th), "a rank is stuck"
    for e in errs:
        if e is not None:
            raise e


def stamped_batch(rng, G, Z, n_per_node, hot=0):
    """Random stamped events per node: pages uniform (plus `hot` events on page 0 from every
    node), seq = a global clock shuffled over the batch, 20 % writes."""
    tot = n_per_node * G + hot * G
    clock = rng.permutation(tot).astype(np.uint64)
    out, k = [], 0
    for t in range(G):
        m = n_per_node + hot
        pages = np.concatenate([rng.integers(0, Z, n_per_node), np.zeros(hot, np.int64)])
        rw = (rng.random(m) < 0.2).astype(np.uint64)
        seq = clock[k:k + m]
        k += m
        e = (pages.astype(np.uint64) << np.uint64(36)) | (seq << np.uint64(4)) \
            | np.uint64(t << 1) | rw
        out.append(np.sort(e))
    return out


class Shard:
    def __init__(self, rank, G, Z):
        self.per = -(-Z // G)
        self.base = min(Z, rank * self.per)
        self.nh = max(0, min(Z, self.base + self.per) - self.base)
        self.ctx = ga.Context(max(1, self.nh), arenas=())
        self.ctx.coh_init(G)
        if self.nh:
            self.ctx.coh_upload(np.full(self.nh, (1 << rank) | (rank << 8) | (2 << 16), np.uint32),
                                np.zeros(self.nh, np.uint32))


@pytest.mark.parametrize("G,Z,n,hot", [(2, 5000, 3000, 0), (3, 4099, 20000, 500), (4, 777, 4000, 0),
                                       (8, 9001, 3000, 300), (8, 64, 2000, 0)])
def test_route_notify_equal_sequential_fold(G, Z, n, hot):
    rng = np.random.default_rng(G * 1000 + Z)
    shards = [Shard(r, G, Z) for r in range(G)]
    comms = exchange.Comm.loopback([s.ctx for s in shards])
    gst, gfl = oracle.coh_init(Z, G)
    try:
        for batch in range(3):
            # node 1 sends nothing in batch 1; batch 2 is empty on every node
            stamped = stamped_batch(rng, G, Z, n if batch < 2 else 0, hot if batch < 2 else 0)
            if batch == 1:
                stamped[1] = stamped[1][:0]
            rc_ref, tot_ref, want = oracle.route_round(gst, gfl, stamped, G, Z)
            assert rc_ref == 0
            got, tots, nb = [None] * G, [None] * G, [None] * G

            def rank(r):
                s, c = shards[r], comms[r]
                ev = s.ctx.buffer(max(8, 8 * len(stamped[r]))).upload(stamped[r])
                cap = sum(len(x) for x in stamped) + 1
                bt = s.ctx.buffer(8 * cap)
                nt = s.ctx.buffer(8 * (Z + 1))
                tot = s.ctx.buffer(80)
                nb[r] = exchange.route_events(s.ctx, c, ev.ptr, len(stamped[r]), Z, bt.ptr, cap)
                k = exchange.coherence_notify(s.ctx, c, bt.ptr, nb[r], s.base, tot.ptr, nt.ptr,
                                              Z + 1)
                s.ctx.sync()
                got[r] = nt.download(np.uint64, k) if k else np.zeros(0, np.uint64)
                tots[r] = tot.download(np.uint64, 10).astype(np.int64)
                for b in (ev, bt, nt, tot):
                    b.free()
            run_ranks(G, rank)
            assert sum(nb) == sum(len(x) for x in stamped)
            for r in range(G):
                assert np.array_equal(got[r], want[r]), (batch, r, len(got[r]), len(want[r]))
            assert np.sum(tots, axis=0).tolist() == [tot_ref["invalidations"],
                                                     tot_ref["transfers"], *tot_ref["node_faults"]]
        for r, s in enumerate(shards):
            if s.nh:
                st, fl = s.ctx.coh_download()
                assert np.array_equal(st, gst[s.base:s.base + s.nh])
                assert np.array_equal(fl, gfl[s.base:s.base + s.nh])
    finally:
        for c in comms:
            c.close()
        for s in shards:
            s.ctx.close()


def test_route_refusals_are_collective():
    """One node's unsorted list: every rank gets -EINVAL from gdsm_route_events. One home's batch
    buffer too small: every rank gets -ENOSPC. A notice buffer too small on one node: every rank
    gets -ENOSPC from gdsm_coherence_notify. Afterwards the group still works."""
    G, Z = 3, 3000
    rng = np.random.default_rng(5)
    shards = [Shard(r, G, Z) for r in range(G)]
    comms = exchange.Comm.loopback([s.ctx for s in shards])
    lib = ga.gdsm.lib()
    try:
        stamped = stamped_batch(rng, G, Z, 2000)
        bad = stamped[2].copy()
        bad[[10, 11]] = bad[[11, 10]]
        rcs = {}

        def call(r, evs, cap, ncap):
            import ctypes as C
            s, c = shards[r], comms[r]
            ev = s.ctx.buffer(8 * len(evs[r])).upload(evs[r])
            bt = s.ctx.buffer(8 * max(cap, 1))
            nt = s.ctx.buffer(8 * max(ncap, 1))
            tot = s.ctx.buffer(80)
            nb, nn = C.c_uint64(0), C.c_uint64(0)
            rc1 = lib.gdsm_route_events(s.ctx.handle, c.handle, ev.ptr, len(evs[r]), Z, bt.ptr,
                                        cap, C.byref(nb))
            rc2 = None
            if rc1 == 0:
                rc2 = lib.gdsm_coherence_notify(s.ctx.handle, c.handle, bt.ptr, nb.value, s.base,
                                                tot.ptr, nt.ptr, ncap, C.byref(nn))
            s.ctx.sync()
            return rc1, rc2

        def case(name, evs, caps, ncaps):
            def rank(r):
                rcs[(name, r)] = call(r, evs, caps[r], ncaps[r])
            run_ranks(G, rank)
            return [rcs[(name, r)] for r in range(G)]

        big = 3 * 2000 + 1
        assert case("unsorted", [stamped[0], stamped[1], bad], [big] * 3, [Z] * 3) == \
            [(-errno.EINVAL, None)] * 3
        assert case("small batch", stamped, [big, 10, big], [Z] * 3) == [(-errno.ENOSPC, None)] * 3
        assert case("small notices", stamped, [big] * 3, [Z, Z, 1]) == [(0, -errno.ENOSPC)] * 3
        assert case("ok", stamped, [big] * 3, [Z] * 3) == [(0, 0)] * 3
        # the refusals changed nothing: the shards equal one sequential fold of the batch
        gst, gfl = oracle.coh_init(Z, G)
        assert oracle.route_round(gst, gfl, stamped, G, Z)[0] == 0
        for s in shards:
            st, fl = s.ctx.coh_download()
            assert np.array_equal(st, gst[s.base:s.base + s.nh])
            assert np.array_equal(fl, gfl[s.base:s.base + s.nh])
    finally:
        for c in comms:
            c.close()
        for s in shards:
            s.ctx.close()


def test_route_notify_8_nodes_full_copyset():
    """The production group size, GDSM_MAX_NODES = 8 ranks: in batch 0 every node reads pages
    0-99 (their copysets become all 8 nodes), in batch 1 every node writes some of them (a write
    to a page all 8 share invalidates 7 copies), then a random batch. Shards, totals and every
    node's notices equal the oracle's sequential fold."""
    G, Z = 8, 4096
    rng = np.random.default_rng(88)
    shards = [Shard(r, G, Z) for r in range(G)]
    comms = exchange.Comm.loopback([s.ctx for s in shards])
    gst, gfl = oracle.coh_init(Z, G)
    try:
        def batch_of(pages_per_node, rw_of):
            tot = sum(len(p) for p in pages_per_node)
            clock = rng.permutation(tot).astype(np.uint64)
            out, k = [], 0
            for t, pages in enumerate(pages_per_node):
                m = len(pages)
                rw = rw_of(t, m)
                e = (np.asarray(pages, np.uint64) << np.uint64(36)) \
                    | (clock[k:k + m] << np.uint64(4)) | np.uint64(t << 1) | rw
                k += m
                out.append(np.sort(e))
            return out
        reads = batch_of([np.arange(100)] * G, lambda t, m: np.zeros(m, np.uint64))
        writes = batch_of([rng.choice(100, 10, replace=False) for _ in range(G)],
                          lambda t, m: np.ones(m, np.uint64))
        mixed = batch_of([rng.integers(0, Z, 3000) for _ in range(G)],
                         lambda t, m: (rng.random(m) < 0.2).astype(np.uint64))
        for bi, stamped in enumerate((reads, writes, mixed)):
            rc_ref, tot_ref, want = oracle.route_round(gst, gfl, stamped, G, Z)
            assert rc_ref == 0
            if bi == 0:
                assert np.all(gst[:100] & 0xFF == 0xFF)  # every page shared by all 8 nodes
            if bi == 1:
                assert tot_ref["invalidations"] >= 7
            got, tots = [None] * G, [None] * G

            def rank(r):
                s, c = shards[r], comms[r]
                ev = s.ctx.buffer(max(8, 8 * len(stamped[r]))).upload(stamped[r])
                cap = sum(len(x) for x in stamped) + 1
                bt, nt, tot = s.ctx.buffer(8 * cap), s.ctx.buffer(8 * (Z + 1)), s.ctx.buffer(80)
                nb = exchange.route_events(s.ctx, c, ev.ptr, len(stamped[r]), Z, bt.ptr, cap)
                k = exchange.coherence_notify(s.ctx, c, bt.ptr, nb, s.base, tot.ptr, nt.ptr, Z + 1)
                s.ctx.sync()
                got[r] = nt.download(np.uint64, k) if k else np.zeros(0, np.uint64)
                tots[r] = tot.download(np.uint64, 10).astype(np.int64)
                for b in (ev, bt, nt, tot):
                    b.free()
            run_ranks(G, rank)
            for r in range(G):
                assert np.array_equal(got[r], want[r]), (bi, r)
            assert np.sum(tots, axis=0).tolist() == [tot_ref["invalidations"],
                                                     tot_ref["transfers"], *tot_ref["node_faults"]]
        for s in shards:
            st, fl = s.ctx.coh_download()
            assert np.array_equal(st, gst[s.base:s.base + s.nh])
            assert np.array_equal(fl, gfl[s.base:s.base + s.nh])
    finally:
        for c in comms:
            c.close()
        for s in shards:
            s.ctx.close()


def test_route_notify_local_failure_is_collective():
    """One rank's own failure (a workspace it cannot allocate, forced by gdsm_debug_fail_alloc)
    inside gdsm_route_events or gdsm_coherence_notify: that rank returns -ENOMEM and every other
    rank -ECANCELED, together (no peer is left waiting in a transfer), nothing changes, and the
    group works afterwards. notify grows five workspaces (pre-fold words, per-block counts and
    offsets, the fold's workspace, the notice staging); a failure is forced at each in turn."""
    import ctypes as C
    G, Z = 3, 3000
    rng = np.random.default_rng(6)
    shards = [Shard(r, G, Z) for r in range(G)]
    comms = exchange.Comm.loopback([s.ctx for s in shards])
    lib = ga.gdsm.lib()
    try:
        stamped = stamped_batch(rng, G, Z, 2000)
        cap = sum(len(x) for x in stamped) + 1
        bufs = []
        for r, s in enumerate(shards):
            bufs.append((s.ctx.buffer(8 * len(stamped[r])).upload(stamped[r]),
                         s.ctx.buffer(8 * cap), s.ctx.buffer(8 * Z), s.ctx.buffer(80)))
        nbs = [C.c_uint64(0) for _ in range(G)]

        def route_all():
            rcs = [None] * G

            def rank(r):
                s, c = shards[r], comms[r]
                ev, bt, _, _ = bufs[r]
                rcs[r] = lib.gdsm_route_events(s.ctx.handle, c.handle, ev.ptr, len(stamped[r]), Z,
                                               bt.ptr, cap, C.byref(nbs[r]))
            run_ranks(G, rank)
            return rcs

        def notify_all():
            rcs = [None] * G

            def rank(r):
                s, c = shards[r], comms[r]
                _, bt, nt, tot = bufs[r]
                nn = C.c_uint64(0)
                rcs[r] = lib.gdsm_coherence_notify(s.ctx.handle, c.handle, bt.ptr, nbs[r].value,
                                                   s.base, tot.ptr, nt.ptr, Z, C.byref(nn))
                s.ctx.sync()
            run_ranks(G, rank)
            return rcs

        assert lib.gdsm_debug_fail_alloc(shards[1].ctx.handle, 1) == 0
        assert route_all() == [-errno.ECANCELED, -errno.ENOMEM, -errno.ECANCELED]
        assert route_all() == [0, 0, 0]
        init = [s.ctx.coh_download() for s in shards]
        fails = 0
        for _ in range(8):
            # the first call fails the first growth; each later one lets the growth that failed
            # last time happen and fails the next one
            assert lib.gdsm_debug_fail_alloc(shards[2].ctx.handle, 2 if fails else 1) == 0
            rcs = notify_all()
            if rcs == [0, 0, 0]:
                break
            assert rcs == [-errno.ECANCELED, -errno.ECANCELED, -errno.ENOMEM], rcs
            fails += 1
            for s, (st0, fl0) in zip(shards, init):  # no page table changed
                st, fl = s.ctx.coh_download()
                assert np.array_equal(st, st0) and np.array_equal(fl, fl0)
        assert fails == 5 and rcs == [0, 0, 0]
        assert lib.gdsm_debug_fail_alloc(shards[2].ctx.handle, 0) == 0
        gst, gfl = oracle.coh_init(Z, G)
        assert oracle.route_round(gst, gfl, stamped, G, Z)[0] == 0
        for s in shards:
            st, fl = s.ctx.coh_download()
            assert np.array_equal(st, gst[s.base:s.base + s.nh])
            assert np.array_equal(fl, gfl[s.base:s.base + s.nh])
    finally:
        for c in comms:
            c.close()
        for s in shards:
            s.ctx.close()


def test_notify_ignores_a_stale_event_error_bit():
    """An error bit an earlier, never-synchronised gdsm_coherence_batch_async left behind (an
    unsorted batch) does not make the next gdsm_coherence_notify refuse: only its own fold's
    rejection counts. The stale bit is still reported by the next gdsm_sync."""
    G, Z = 2, 2000
    rng = np.random.default_rng(7)
    shards = [Shard(r, G, Z) for r in range(G)]
    comms = exchange.Comm.loopback([s.ctx for s in shards])
    lib = ga.gdsm.lib()
    try:
        # rank 0: an unsorted local batch folded asynchronously, never synchronised
        bad = np.array([(5 << 4) | 1, (3 << 4)], np.uint64)
        s0 = shards[0]
        evb, tb = s0.ctx.buffer(16).upload(bad), s0.ctx.buffer(80)
        assert lib.gdsm_coherence_batch_async(s0.ctx.handle, evb.ptr, 2, tb.ptr) == 0
        stamped = stamped_batch(rng, G, Z, 1000)
        got = [None] * G

        def rank(r):
            s, c = shards[r], comms[r]
            ev = s.ctx.buffer(8 * len(stamped[r])).upload(stamped[r])
            cap = sum(len(x) for x in stamped) + 1
            bt, nt, tot = s.ctx.buffer(8 * cap), s.ctx.buffer(8 * (Z + 1)), s.ctx.buffer(80)
            nb = exchange.route_events(s.ctx, c, ev.ptr, len(stamped[r]), Z, bt.ptr, cap)
            got[r] = exchange.coherence_notify(s.ctx, c, bt.ptr, nb, s.base, tot.ptr, nt.ptr,
                                               Z + 1)
        run_ranks(G, rank)
        assert all(k is not None for k in got)
        assert lib.gdsm_sync(s0.ctx.handle) == -errno.EINVAL  # the earlier batch's error
        assert lib.gdsm_sync(shards[1].ctx.handle) == 0
    finally:
        for c in comms:
            c.close()
        for s in shards:
            s.ctx.close()


@pytest.mark.parametrize("refusal", ["enospc", "enomem"])
def test_refused_notify_keeps_a_stale_event_error_bit(refusal):
    """The stale bit survives a notify that is REFUSED: every rank gets -ENOSPC (a notice buffer
    too small) or the failing rank -ENOMEM and the others -ECANCELED (a workspace growth forced to
    fail on rank 0), and the next gdsm_sync on rank 0 still reports the earlier batch's
    rejection (-EINVAL) while rank 1's is clean."""
    import ctypes as C
    G, Z = 2, 2000
    rng = np.random.default_rng(17)
    shards = [Shard(r, G, Z) for r in range(G)]
    comms = exchange.Comm.loopback([s.ctx for s in shards])
    lib = ga.gdsm.lib()
    try:
        s0 = shards[0]
        bad = np.array([(5 << 4) | 1, (3 << 4)], np.uint64)
        evb, tb = s0.ctx.buffer(16).upload(bad), s0.ctx.buffer(80)
        stamped = stamped_batch(rng, G, Z, 1000)
        cap = sum(len(x) for x in stamped) + 1
        bufs = [(s.ctx.buffer(8 * len(stamped[r])).upload(stamped[r]), s.ctx.buffer(8 * cap),
                 s.ctx.buffer(8 * (Z + 1)), s.ctx.buffer(80)) for r, s in enumerate(shards)]
        nbs = [0] * G

        def route(r):
            ev, bt, _, _ = bufs[r]
            nbs[r] = exchange.route_events(shards[r].ctx, comms[r], ev.ptr, len(stamped[r]), Z,
                                           bt.ptr, cap)
        run_ranks(G, route)
        assert lib.gdsm_coherence_batch_async(s0.ctx.handle, evb.ptr, 2, tb.ptr) == 0
        if refusal == "enomem":
            assert lib.gdsm_debug_fail_alloc(s0.ctx.handle, 1) == 0
        ncap = 1 if refusal == "enospc" else Z + 1
        rcs = [None] * G

        def notify(r):
            s, c = shards[r], comms[r]
            _, bt, nt, tot = bufs[r]
            nn = C.c_uint64(0)
            rcs[r] = lib.gdsm_coherence_notify(s.ctx.handle, c.handle, bt.ptr, nbs[r], s.base,
                                               tot.ptr, nt.ptr, ncap, C.byref(nn))
        run_ranks(G, notify)
        want = ([-errno.ENOSPC] * G if refusal == "enospc"
                else [-errno.ENOMEM, -errno.ECANCELED])
        assert rcs == want
        assert lib.gdsm_debug_fail_alloc(s0.ctx.handle, 0) == 0
        assert lib.gdsm_sync(s0.ctx.handle) == -errno.EINVAL  # the earlier batch's error
        assert lib.gdsm_sync(shards[1].ctx.handle) == 0
        assert lib.gdsm_sync(s0.ctx.handle) == 0  # reported once
    finally:
        for c in comms:
            c.close()
        for s in shards:
            s.ctx.close()
