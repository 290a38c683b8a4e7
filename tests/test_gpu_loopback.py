"""gdsm_exchange's multi-rank C++ path on ONE GPU: G ranks as threads of this process, each with its
own context on cuda:0, wired by libgdsm's loopback communicator (gdsm_comm_init_loopback). The
peer loop, the whole-stream checks, the remote applies, gdsm_comm_agree and the over-budget
recovery all run exactly as over RCCL; only the move is a device-to-device copy. Replaces the
reference's per-peer HTTP fan-out of page updates (gallocy/http/client.cpp:39-91).

Layout as exchange.py: writer(p) = p mod G (writer r's TWIN/CURRENT arena index i = global page
i*G + r), home(p) = p // n (REPLICA of rank d = global pages [d*n, (d+1)*n))."""
import ctypes as C
import errno
import threading

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd import exchange
from gallocy_amd._lib import GdsmRuns

pytestmark = pytest.mark.gpu

SEED = 31


def run_ranks(G, fn):
    """fn(rank) on G threads; re-raises the first failure."""
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


def make_group(G, n, mode=ga.GEN_UNIFORM, ppm=10000):
    ctxs = [ga.Context(n) for _ in range(G)]
    for r, ctx in enumerate(ctxs):
        ctx.gen_pages(seed=SEED, mode=mode, ppm=ppm, first_global=r, stride=G,
                      arenas=("twin", "current"))
        ctx.gen_pages(seed=SEED, mode=mode, ppm=ppm, first_global=r * n, stride=1,
                      arenas=("replica",))
    comms = exchange.Comm.loopback(ctxs)
    return ctxs, comms


def close_group(ctxs, comms):
    for c in comms:
        c.close()
    for x in ctxs:
        x.close()


def homes_equal_writers(ctxs, n):
    """Every home block equals the writers' CURRENT contents of those pages (host check)."""
    G = len(ctxs)
    glob = np.empty((G * n, 4096), np.uint8)
    for r, ctx in enumerate(ctxs):
        glob[r::G] = ctx.download("current")
    return all(np.array_equal(ctx.download("replica"), glob[d * n:(d + 1) * n])
               for d, ctx in enumerate(ctxs))


@pytest.mark.parametrize("G", [2, 3, 4, 8])
def test_loopback_shard_exact_then_fixed(G):
    """Release 0 with exact sizes (all-to-all of sizes, agreement, grouped moves), calibrate(),
    then pipelined fixed-budget releases with no host synchronisation: every home REPLICA equals
    its pages' CURRENT, and nothing asked for a recovery."""
    n = 4096 * G
    ctxs, comms = make_group(G, n)
    shards = [exchange.Shard(ctxs[r], r, G, n, 1024, transport="loopback", comm=comms[r])
              for r in range(G)]
    try:
        def rank(r):
            s = shards[r]
            s.run(1, pipelined=False)
            s.drain()
            s.calibrate()
            assert s.flags == exchange.XCHG_FIXED
            s.run(3, pipelined=True)
            s.drain()
            assert s.recoveries == 0
        run_ranks(G, rank)
        assert homes_equal_writers(ctxs, n)
        # exchanged bytes: every rank received the streams of every other rank
        assert all(s.received > 0 and s.sent_remote > 0 for s in shards)
    finally:
        for s in shards:
            s.close()
        close_group(ctxs, comms)


@pytest.mark.parametrize("G", [3, 8])
def test_loopback_over_budget_is_rejected_then_recovered(G):
    """After calibrate(), rank 0 writes 4x as many words: its fixed-budget streams (n/G > 256
    records each) no longer fit their budgets. The homes reject them whole (nothing of rank 0's
    release applied, -EOVERFLOW on the homes and on rank 0), drain() has every rank agree and redo
    the release with exact sizes, and every home ends equal to the writers' CURRENT."""
    n = G * 4096
    ctxs, comms = make_group(G, n)
    shards = [exchange.Shard(ctxs[r], r, G, n, 1024, transport="loopback", comm=comms[r])
              for r in range(G)]
    try:
        def rank(r):
            s = shards[r]
            s.run(1, pipelined=False)
            s.drain()
            s.calibrate()
        run_ranks(G, rank)
        # rank 0's words at 4 % instead of 1 % (a superset of the old writes, SPEC §6)
        ctxs[0].gen_pages(seed=SEED, mode=ga.GEN_UNIFORM, ppm=40000, first_global=0, stride=G,
                          arenas=("current",))
        ctxs[0].sync()
        before = [c.download("replica") for c in ctxs]
        rcs = [None] * G

        def fixed_release(r):
            shards[r].run(1, pipelined=False)
            rcs[r] = ga.gdsm.lib().gdsm_sync(ctxs[r].handle)
        run_ranks(G, fixed_release)
        # homes 1 and 2 rejected rank 0's streams, rank 0 learned it too (and rejected its own
        # stream to itself, checked like the others)
        assert rcs == [-errno.EOVERFLOW] * G, rcs
        g = np.empty((G * n, 4096), np.uint8)
        for r, ctx in enumerate(ctxs):
            g[r::G] = ctx.download("current")
        for d in range(G):
            now = ctxs[d].download("replica")
            mine = np.arange(d * n, (d + 1) * n)
            from0 = (mine % G) == 0
            # nothing of rank 0's rejected stream was applied at any home
            assert np.array_equal(now[from0], before[d][from0])
            # the other writers' streams were applied
            assert np.array_equal(now[~from0], g[mine[~from0]])
        # the budgets are still too small: the next fixed release fails the same way, and
        # drain() recovers it (agreement -> exact release -> new budgets)

        def recovering(r):
            shards[r].run(1, pipelined=False)
            shards[r].drain()
            assert shards[r].recoveries == 1
            shards[r].run(2, pipelined=True)   # the new budgets hold
            shards[r].drain()
            assert shards[r].recoveries == 1
        run_ranks(G, recovering)
        assert homes_equal_writers(ctxs, n)
    finally:
        for s in shards:
            s.close()
        close_group(ctxs, comms)


def _exchange(ctx, comm, send, sids, recv, rids, flags=0):
    G = comm.world
    s_arr = (GdsmRuns * G)(*[r.s for r in send])
    r_arr = (GdsmRuns * G)(*[r.s for r in recv])
    sid = (C.c_void_p * G)(*sids)
    rid = (C.c_void_p * G)(*rids)
    rc = ga.gdsm.lib().gdsm_exchange(ctx.handle, comm.handle, s_arr, sid, r_arr, rid, ga.REPLICA,
                                     flags)
    for s in range(G):
        recv[s].s.n = r_arr[s].n
    return rc


def test_loopback_bad_receive_ids_and_offsets_write_nothing():
    """A received stream naming a page index past the home's arena, and one with decreasing
    offsets: each is rejected whole (-EINVAL at the home's next gdsm_sync, nothing of it
    written), while a good stream in the same exchange is applied."""
    G, n = 3, 2048
    ctxs, comms = make_group(G, n)
    try:
        per = 64
        # rank r diffs its arena pages 0..per-1 for every home d, to land at the home's REPLICA
        # indices [r*per, (r+1)*per), whose base content is set to the writer's TWIN of them
        for r, ctx in enumerate(ctxs):
            tw = ctx.download("twin", 0, per)
            for d in range(G):
                ctxs[d].upload("replica", tw, first=r * per)
        streams, ids_bufs = [], []
        for r, ctx in enumerate(ctxs):
            src = ctx.ids(np.arange(per, dtype=np.uint32))
            st = []
            ib = []
            for d in range(G):
                st.append(ctx.diff(src, n=per, cap=per * 1024))
                dest = np.arange(r * per, (r + 1) * per, dtype=np.uint32)
                if r == 1 and d == 0:
                    dest[17] = n + 5          # out of range at home 0
                ib.append(ctx.ids(dest))
            streams.append(st)
            ids_bufs.append(ib)
            ctx.sync()
        # rank 2's stream to home 0: decreasing offsets
        ro = streams[2][0].to_host().rec_off.copy()
        ro[10], ro[11] = ro[11], ro[10]
        if ro[10] == ro[11]:
            ro[11] += 4
        lib = ga.gdsm.lib()
        assert lib.gdsm_memcpy_h2d(ctxs[2].handle, streams[2][0].s.rec_off, ro.ctypes.data,
                                   ro.nbytes) == 0
        before = [c.download("replica") for c in ctxs]
        recv = [[ga.Runs(ctxs[d], per, cap=per * 1024) if s != d else ga.Runs(ctxs[d], 1, cap=16)
                 for s in range(G)] for d in range(G)]
        rids = [[ctxs[d].buffer(4 * per) for s in range(G)] for d in range(G)]
        rcs = [None] * G

        def rank(r):
            rc = _exchange(ctxs[r], comms[r], streams[r], [b.ptr for b in ids_bufs[r]], recv[r],
                           [b.ptr for b in rids[r]])
            assert rc == 0
            rcs[r] = lib.gdsm_sync(ctxs[r].handle)
        run_ranks(G, rank)
        assert rcs == [-errno.EINVAL, 0, 0], rcs
        for d in range(G):
            now = ctxs[d].download("replica")
            for r in range(G):
                blk = slice(r * per, (r + 1) * per)
                cur_r = ctxs[r].download("current", 0, per)
                if d == 0 and r in (1, 2):
                    assert np.array_equal(now[blk], before[d][blk]), (d, r)
                else:
                    assert np.array_equal(now[blk], cur_r), (d, r)
        for row in recv:
            for x in row:
                x.free()
    finally:
        close_group(ctxs, comms)


def test_loopback_checked_ids_regrow_with_several_sources():
    """The exchange's checked-index scratch starts small (one page per source) and must grow
    for the next exchange (every page from every source) while earlier work is queued; both
    rounds land every stream at its home."""
    G, n = 4, 4 * 2048
    ctxs, comms = make_group(G, n, mode=ga.GEN_CLUSTERED, ppm=100000)
    try:
        sids_all = exchange.send_ids
        bounds = [exchange.dest_bounds(r, G, n) for r in range(G)]
        rmax = n // G + 1

        def rank(r):
            ctx = ctxs[r]
            iota = ctx.ids(np.arange(n, dtype=np.uint32))
            sid = [ctx.ids(x) for x in sids_all(r, G, n)]
            recv = [ga.Runs(ctx, rmax, cap=rmax * 1024) if s != r else ga.Runs(ctx, 1, cap=16)
                    for s in range(G)]
            rid = [ctx.buffer(4 * rmax) for _ in range(G)]
            for take_all in (False, True):
                send = []
                for d in range(G):
                    cnt = bounds[r][d + 1] - bounds[r][d]
                    if not take_all:
                        cnt = min(cnt, 1)
                    send.append(ctx.diff(iota.ptr + 4 * bounds[r][d], n=cnt,
                                         cap=max(4096, cnt * 1024)))
                assert _exchange(ctx, comms[r], send, [b.ptr for b in sid], recv,
                                 [b.ptr for b in rid]) == 0
                ctx.sync()
                for x in send:
                    x.free()
            for x in recv:
                x.free()
        run_ranks(G, rank)
        assert homes_equal_writers(ctxs, n)
    finally:
        close_group(ctxs, comms)


def test_loopback_agree():
    """gdsm_comm_agree returns the maximum of the ranks' values on every rank."""
    G, n = 2, 1024
    ctxs, comms = make_group(G, n)
    try:
        got = [None] * G

        def rank(r):
            got[r] = comms[r].agree(ctxs[r], 10 + 5 * r)
        run_ranks(G, rank)
        assert got == [15, 15]
    finally:
        close_group(ctxs, comms)


@pytest.mark.parametrize("G", [4, 8])
def test_loopback_bench_step_pipelined_timed(G):
    """bench.py's N > 1 step at the production group size, reduced total: every rank diffs its
    pages into one stream per home (one gdsm_diff_split launch), release 0 exact, calibrate(),
    then pipelined fixed-budget releases with profiling on, then the same releases with
    GDSM_XCHG_TIMED (the device barrier before each transfer that bench.py uses to time the link
    alone): both runs record the exchange and exchange_wait stages, nothing recovers, and every
    home REPLICA equals its pages' CURRENT (checked on the device by Shard.verify and on the host)."""
    n = 8192 * G // 4 * 4
    ctxs, comms = make_group(G, n)
    shards = [exchange.Shard(ctxs[r], r, G, n, 128, transport="loopback", comm=comms[r])
              for r in range(G)]
    profs = [None] * G
    try:
        def rank(r):
            s = shards[r]
            s.run(1, pipelined=False)
            s.drain()
            s.calibrate()
            s.run(2, pipelined=True)
            s.drain()
            out = []
            for timed in (False, True):
                if timed:
                    s.flags |= exchange.XCHG_TIMED
                ctxs[r].prof_enable(True)
                s.run(3, pipelined=True)
                s.drain()
                out.append(ctxs[r].prof_read())
                s.flags &= ~exchange.XCHG_TIMED
            assert s.recoveries == 0
            profs[r] = out
        run_ranks(G, rank)
        for r in range(G):
            for p in profs[r]:
                assert p["diff"][1] == 3 and p["exchange"][1] == 3 and p["exchange_wait"][1] == 3
                # the wait-inclusive span contains the transfer
                assert p["exchange_wait"][0] >= p["exchange"][0] * 0.999
        assert all(shards[r].verify(SEED, ga.GEN_UNIFORM, 10000) for r in range(G))
        assert homes_equal_writers(ctxs, n)
    finally:
        for s in shards:
            s.close()
        close_group(ctxs, comms)


def test_exchange_rejects_unknown_flags():
    G, n = 2, 1024
    ctxs, comms = make_group(G, n)
    try:
        runs = [ga.Runs(ctxs[0], 1, cap=16) for _ in range(G)]
        rids = [None] * G
        assert _exchange(ctxs[0], comms[0], runs, [0] * G, runs, rids, flags=4) == -errno.EINVAL
    finally:
        close_group(ctxs, comms)


def test_loopback_init_failure_frees_the_group():
    """gdsm_comm_init_loopback with a NULL context among valid ones: -EINVAL, nothing leaked or
    double-freed (the group is deleted by whoever holds the last reference)."""
    lib = ga.gdsm.lib()
    ctx = ga.Context(64)
    try:
        hs = (C.c_void_p * 3)()
        cs = (C.c_void_p * 3)(ctx.handle, None, ctx.handle)
        assert lib.gdsm_comm_init_loopback(hs, cs, 3) == -errno.EINVAL
        assert all(h is None for h in hs)
        for _ in range(3):  # repeated builds and teardowns of a valid group
            comms = exchange.Comm.loopback([ctx])
            for c in comms:
                c.close()
    finally:
        ctx.close()
