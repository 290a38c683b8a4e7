"""Config 5 end to end on the GPU: the test_mmult trace replayed through coherence batches and
twin/diff/apply propagation (gallocy_amd/replay.py). The home copies must equal the zone after
the whole multiplication, and the page table must equal the oracle's fold of the same events."""
import numpy as np
import pytest

from gallocy_amd.replay import MmultReplay
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ndim,nodes,graph,fused", [
    (64, 1, False, True), (64, 2, False, True), (96, 4, False, True), (64, 8, False, True),
    (257, 3, False, True), (1000, 1, False, True), (1000, 2, False, True), (1000, 4, False, True),
    (1000, 8, False, True), (96, 4, True, True), (1000, 4, True, True), (257, 3, False, False),
    (1000, 4, False, False), (1000, 4, True, False)])
def test_mmult_replay_end_to_end(ndim, nodes, graph, fused):
    """NDIM = 1000 is BASELINE config 5's size (test/test_mmult.cpp:103-180 uses
    NDIM up to 1021 before the reference heap aborts). graph: every round recorded into one HIP
    graph (gdsm_capture_*) and replayed by one launch, or issued eagerly (the default: the C++
    round loop, gallocy_amd/native/replay.cpp). fused: the diff kernel applies the runs to the
    home copies (gdsm_diff_apply_ids), or a separate apply of the stream does (Python rounds)."""
    _check_replay(MmultReplay(ndim=ndim, nodes=nodes, seed=7, fused=fused), nodes, graph)


@pytest.mark.parametrize("ndim,nodes,retwin,driver", [
    (1000, 4, True, "python"), (257, 3, False, "python"), (64, 8, True, "python"),
    (1000, 4, True, "native2"), (257, 3, False, "native2"),
    (64, 1, True, "device"), (257, 3, True, "device"), (1000, 1, True, "device"),
    (1000, 2, True, "device"), (1000, 4, True, "device"), (1000, 8, True, "device"),
    (1000, 1, True, "device-grid"), (1000, 4, True, "device-grid"),
    (1000, 1, True, "device-gridfold"), (1000, 8, True, "device-gridfold")])
def test_mmult_replay_other_drivers(ndim, nodes, retwin, driver, monkeypatch):
    """The same replay with every round issued from Python (MmultReplay.round, driver="python"),
    by two C++ threads, one per context (driver="native2"), or on the device (driver="device":
    gdsm_rounds, one persistent launch per context with device-wide barriers between a round's
    steps), with and without the re-twinning release: the same home copies, totals and page
    table. "device-grid": gdsm_rounds on the whole grid (GDSM_ROUNDS_XCD=0) instead of the
    one-XCD team it takes for rounds this small; "device-gridfold": the page-table rounds on the
    persistent grid (GDSM_ROUNDS_LDS=0) instead of one workgroup with the table in LDS."""
    if driver == "device-grid":
        monkeypatch.setenv("GDSM_ROUNDS_XCD", "0")
        driver = "device"
    if driver == "device-gridfold":
        monkeypatch.setenv("GDSM_ROUNDS_LDS", "0")
        driver = "device"
    _check_replay(MmultReplay(ndim=ndim, nodes=nodes, seed=7, retwin=retwin, driver=driver),
                  nodes, False)


@pytest.mark.parametrize("xcd", ["0", "1"])
@pytest.mark.parametrize("ndim,nodes", [(1000, 1), (257, 3), (1000, 8)])
def test_device_rounds_stream_equals_the_issued_rounds(ndim, nodes, xcd, monkeypatch):
    """gdsm_rounds (every round in one persistent launch per context) leaves the same last-round
    stream, the same TWIN and CURRENT views and the same home copy as the C++-issued rounds (one
    chained release launch per round): the stream checks the record bytes and offsets that no
    home-copy comparison sees. Both forms of the launch: the whole grid with write-through
    hand-offs (GDSM_ROUNDS_XCD=0) and the one-XCD team whose hand-offs meet in its L2 (=1, the
    default at these round sizes)."""
    monkeypatch.setenv("GDSM_ROUNDS_XCD", xcd)
    Rs = [MmultReplay(ndim=ndim, nodes=nodes, seed=11, driver=d) for d in ("native", "device")]
    try:
        out = []
        for R in Rs:
            R.run()
            h = R._runs.to_host()
            n = int(R.id_off[-1] - R.id_off[-2])
            out.append((h.rec_off[:n + 1].copy(), h.data[:int(h.rec_off[n])].copy(),
                        R.data.download("twin"), R.data.download("current"), R.home_copy(),
                        R.totals.copy()))
        for a, b in zip(*out):
            assert np.array_equal(a, b)
        assert out[0][0][-1] > 0  # the last round ships records
    finally:
        for R in Rs:
            R.close()


def _check_replay(R, nodes, graph):
    try:
        R.run(graph=graph)
        assert np.array_equal(R.home_copy(), R.final_image())
        st, fl = oracle.coh_init(R.Z, nodes)
        acc = np.zeros(10, np.int64)
        for r in range(R.T.rounds):
            rc, t = oracle.coherence(st, fl, R.T.round_events(r), n_nodes=nodes)
            assert rc == 0
            acc += [t["invalidations"], t["transfers"], *t["node_faults"]]
        assert R.totals.tolist() == acc.tolist()
        gst, gfl = R.pt.coh_download()
        assert np.array_equal(gst, st) and np.array_equal(gfl, fl)
    finally:
        R.close()


def _check_rank_replays(Rs, world):
    """Every home block equals the product zone; the page-table shards, the totals summed over
    ranks and every node's notices of every round equal the oracle's sequential fold of the whole
    trace (SPEC §5b, oracle.route_round)."""
    T = Rs[0].T
    st, fl = oracle.coh_init(Rs[0].Z, world)
    acc = np.zeros(10, np.int64)
    for r in range(T.rounds):
        rc, t, want = oracle.route_round(st, fl, T.round_stamped(r), world, Rs[0].Z)
        assert rc == 0
        acc += [t["invalidations"], t["transfers"], *t["node_faults"]]
        for R in Rs:
            assert np.array_equal(R.notices_of(r), want[R.rank]), (r, R.rank)
    assert np.sum([R.totals for R in Rs], axis=0).tolist() == acc.tolist()
    for R in Rs:
        assert np.array_equal(R.home_block(), R.final_block())
        if R.nh:
            gst, gfl = R.pt.coh_download()
            assert np.array_equal(gst[:R.nh], st[R.base:R.base + R.nh])
            assert np.array_equal(gfl[:R.nh], fl[R.base:R.base + R.nh])


def test_rank_replay_single_rank_rccl():
    """Config 5 with one process per DSM node (gallocy_amd.replay.MmultRankReplay), here the
    1-rank case on RCCL (two communicators: page data, coherence): NDIM = 1000."""
    from gallocy_amd.replay import MmultRankReplay
    R = MmultRankReplay(0, 1, ndim=1000, seed=7)
    try:
        R.run()
        _check_rank_replays([R], 1)
    finally:
        R.close()


@pytest.mark.parametrize("ranks,ndim", [(2, 300), (3, 257), (4, 1000), (8, 1000)])
def test_rank_replay_multi_rank_loopback(ranks, ndim):
    """MmultRankReplay with `ranks` DSM nodes as threads on cuda:0 over the loopback communicator:
    every round routes each node's own fault events to the homes (gdsm_route_events), folds them
    there and returns the notices (gdsm_coherence_notify), then ships the row writes' diffs to
    the homes (gdsm_exchange) -- the multi-GPU code path, with device-to-device copies for the
    moves."""
    import threading

    from gallocy_amd.replay import MmultRankReplay
    Rs = [MmultRankReplay(r, ranks, ndim=ndim, seed=7, transport="loopback")
          for r in range(ranks)]
    try:
        MmultRankReplay.wire_loopback(Rs)
        errs = [None] * ranks

        def body(r):
            try:
                Rs[r].run()
            except BaseException as e:  # noqa: BLE001
                errs[r] = e
        th = [threading.Thread(target=body, args=(r,)) for r in range(ranks)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=110)
        assert not any(t.is_alive() for t in th)
        for e in errs:
            if e is not None:
                raise e
        _check_rank_replays(Rs, ranks)
    finally:
        for R in Rs:
            R.close()


@pytest.mark.parametrize("case", ["outside", "misaligned", "ok"])
def test_rounds_refuse_writes_outside_released_pages(case):
    """gdsm_rounds lays a round's writes onto the pages the round releases (no copy step), so a
    write into a page the round does not release, or one that is not 8-B aligned, is reported by
    gdsm_sync (-EINVAL) instead of being lost silently; a write inside the released page lands in
    CURRENT, REPLICA (home apply) and TWIN (re-twin)."""
    import ctypes as C
    import errno
    import gallocy_amd as ga
    from gallocy_amd import gdsm
    L = gdsm.lib()
    with ga.Context(8) as d, ga.Context(8, arenas=()) as pt:
        z = np.zeros((8, 4096), np.uint8)
        for a in ("twin", "current", "replica"):
            d.upload(a, z)
        pt.coh_init(2)
        src = d.buffer(4096).upload(np.arange(4096, dtype=np.uint64).view(np.uint8)[:4096])
        base = d.arena_ptr("current")
        dst_page = 2 if case == "outside" else 1
        off = 8 if case != "misaligned" else 12
        desc = np.array([base + dst_page * 4096 + off, src.ptr, 256], np.uint64)
        dd = d.buffer(24).upload(desc)
        ids = d.ids([1])
        home = d.ids([1])
        ev = pt.buffer(8).upload(np.array([(1 << 4) | 1], np.uint64))
        tot = pt.buffer(80)
        runs = gdsm.Runs(d, 1, cap=10244)
        z2 = np.array([0, 1], np.int64)
        rc = L.gdsm_rounds(d.handle, pt.handle, 1, ev.ptr, z2.ctypes.data, tot.ptr, ids.ptr,
                           home.ptr, z2.ctypes.data, dd.ptr, z2.ctypes.data, C.byref(runs.s))
        assert rc == 0
        rc_d = L.gdsm_sync(d.handle)
        assert L.gdsm_sync(pt.handle) == 0
        if case == "ok":
            assert rc_d == 0
            want = np.frombuffer(src.download(np.uint8, 256).tobytes(), np.uint8)
            for a in ("current", "replica", "twin"):
                got = d.download(a, 1, 1).reshape(-1)
                assert np.array_equal(got[8:264], want), a
                assert not got[:8].any() and not got[264:].any(), a
        else:
            assert rc_d == -errno.EINVAL
        runs.free()
