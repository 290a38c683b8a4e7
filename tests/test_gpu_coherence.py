"""GPU parity of the batched page-coherence state machine (docs/SPEC.md §5) against the C oracle
fold, through the C-ABI. Bit-exact: page-table words, per-page faults and the batch totals."""
import ctypes as C

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd.gdsm import GdsmError
from oracle import oracle
from tests.helpers import zipf_counts

pytestmark = pytest.mark.gpu


def _run_both(n_pages, batches, n_nodes=8):
    with ga.Context(n_pages, arenas=()) as c:
        c.coh_init(n_nodes)
        st, fl = oracle.coh_init(n_pages, n_nodes)
        for ev in batches:
            tot = c.coherence_batch(ev)
            rc, otot = oracle.coherence(st, fl, ev, n_nodes=n_nodes)
            assert rc == 0
            assert tot == otot
        gst, gfl = c.coh_download()
        assert np.array_equal(gst, st), np.flatnonzero(gst != st)[:10]
        assert np.array_equal(gfl, fl), np.flatnonzero(gfl != fl)[:10]


def test_golden_batch(golden):
    g = golden["coherence"]
    with ga.Context(64, arenas=()) as c:
        c.coh_init(8)
        tot = c.coherence_batch(g["events"])
        assert [tot["invalidations"], tot["transfers"], *tot["node_faults"]] == g["totals"].tolist()
        st, fl = c.coh_download()
        assert np.array_equal(st, g["state"]) and np.array_equal(fl, g["faults"])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_uniform_counts(seed):
    rng = np.random.default_rng(seed)
    n = 20000
    counts = rng.integers(0, 30, n).astype(np.uint64)
    ev = oracle.gen_events(counts, seed=seed, write_pct=20)
    _run_both(n, [ev])


def test_zipf_with_pages_spanning_many_blocks():
    n = 50000
    counts = zipf_counts(n, 400000, s=0.8, seed=4)
    counts[17] = 50000  # a hot page spanning ~12 blocks of 4096 events
    ev = oracle.gen_events(counts, seed=9, write_pct=20)
    _run_both(n, [ev])


def test_block_boundary_alignment_and_write_mix():
    for counts in ([4096, 4096, 1, 4095, 4097], [1] * 5000, [8191, 0, 0, 1]):
        n = max(64, len(counts))
        cts = np.zeros(n, np.uint64)
        cts[:len(counts)] = counts
        for wp in (0, 50, 100):
            ev = oracle.gen_events(cts, seed=len(counts) + wp, write_pct=wp)
            _run_both(n, [ev])


@pytest.mark.parametrize("write_pct", [0, 3, 20, 100])
def test_hot_page_heads_at_every_sampling_offset(write_pct):
    """A page whose segment starts at many offsets inside a 2048-event block and runs past its
    end: pass A finds such a block's last head by sampling every 32nd event, then the 32 before
    the hit (tail without a head but with a write), or folds the block (no write in the tail)."""
    offsets = [0, 1, 2, 31, 32, 33, 63, 64, 65, 1000, 1951, 1952, 1983, 1984, 1985, 2047]
    counts = []
    for o in offsets:
        counts += [o, 2048 * 2 + 17, 1, 0, 2048 - (o % 7) - 1, 3]
    n = len(counts) + 8
    cts = np.zeros(n, np.uint64)
    cts[:len(counts)] = counts
    ev = oracle.gen_events(cts, seed=71 + write_pct, write_pct=write_pct)
    _run_both(n, [ev, ev])


def test_multi_batch_persistence_and_fewer_nodes():
    n = 3000
    rng = np.random.default_rng(8)
    batches = []
    for b in range(4):
        counts = rng.integers(0, 12, n).astype(np.uint64)
        batches.append(oracle.gen_events(counts, seed=100 + b, n_nodes=3, write_pct=30))
    _run_both(n, batches, n_nodes=3)


def test_single_and_empty_batches():
    _run_both(10, [np.array([(4 << 4) | (3 << 1) | 1], np.uint64), np.zeros(0, np.uint64)])


def test_unsorted_batch_is_rejected():
    with ga.Context(16, arenas=()) as c:
        c.coh_init(8)
        with pytest.raises(GdsmError) as ei:
            c.coherence_batch(np.array([5 << 4, 2 << 4], np.uint64))
        assert ei.value.errno == 22
        with pytest.raises(GdsmError):
            c.coherence_batch(np.array([99 << 4], np.uint64))  # page out of range


def test_node_outside_the_table_is_rejected():
    """gdsm_coherence_batch rejects an event naming a node >= the n_nodes of gdsm_coh_init, like
    the oracle."""
    with ga.Context(16, arenas=()) as c:
        c.coh_init(3)
        with pytest.raises(GdsmError) as ei:
            c.coherence_batch(np.array([(1 << 4) | (3 << 1), (2 << 4) | (7 << 1) | 1], np.uint64))
        assert ei.value.errno == 22
        c.coh_init(3)
        c.coherence_batch(np.array([(1 << 4) | (2 << 1)], np.uint64))


def test_node_outside_the_table_is_rejected_in_whole_blocks():
    """The same rejection when the bad event sits in a whole 2048-event block (the vector-load
    instance, whose node check reads the block's LDS copy after the walk) — its first, middle and
    last events, a later block, and the partial block at the end — and a clean batch still folds
    like the oracle."""
    n = 4096
    counts = zipf_counts(n, 3 * 2048 + 5, seed=7)
    good = oracle.gen_events(counts, seed=11, n_nodes=5, write_pct=25)
    with ga.Context(n, arenas=()) as c:
        for pos in (0, 1000, 2047, 2048, 4095, 6143, 6146):
            ev = good.copy()
            ev[pos] = (ev[pos] & ~np.uint64(14)) | np.uint64(6 << 1)  # node 6 of 5
            c.coh_init(5)
            with pytest.raises(GdsmError) as ei:
                c.coherence_batch(ev)
            assert ei.value.errno == 22, pos
        c.coh_init(5)
        tot = c.coherence_batch(good)
        st, fl = oracle.coh_init(n, 5)
        rc, otot = oracle.coherence(st, fl, good, n_nodes=5)
        assert rc == 0 and tot == otot
        gst, gfl = c.coh_download()
        assert np.array_equal(gst, st) and np.array_equal(gfl, fl)


def _batch_from(c, host, unaligned):
    """Device copy of a host event batch: 16-B aligned, or one u64 in (8-B aligned only), which
    takes the scalar-load instance of pass C."""
    buf = c.buffer(8 * (len(host) + 1))
    if unaligned:
        buf.upload(np.concatenate([np.zeros(1, np.uint64), host]))
        return buf, buf.ptr + 8
    buf.upload(host)
    return buf, buf.ptr


@pytest.mark.parametrize("unaligned", [False, True])
def test_unaligned_events_match_oracle(unaligned):
    """Event arrays that are not 16-B aligned (pass C with scalar loads) are bit-exact too."""
    L = ga.gdsm.lib()
    n = 5000
    counts = zipf_counts(n, 90000, seed=4)
    host = oracle.gen_events(counts, seed=9, n_nodes=8, write_pct=25)
    with ga.Context(n, arenas=()) as c:
        c.coh_init(8)
        _, ptr = _batch_from(c, host, unaligned)
        tot = (C.c_uint64 * 10)()
        assert L.gdsm_coherence_batch(c.handle, ptr, len(host), tot) == 0
        st, fl = oracle.coh_init(n, 8)
        rc, otot = oracle.coherence(st, fl, host)
        assert rc == 0
        assert list(tot) == [otot["invalidations"], otot["transfers"], *otot["node_faults"]]
        gst, gfl = c.coh_download()
        assert np.array_equal(gst, st) and np.array_equal(gfl, fl)


@pytest.mark.parametrize("unaligned", [False, True])
def test_arbitrary_page_table_states(unaligned):
    """Uploaded page-table words in any SPEC §5 state (INVALID, SHARED, EXCLUSIVE, the unused
    state 3, owners >= 8, dirty or not, fault counts up to 2^32 - 1): pass C folds them exactly
    like the oracle, over Zipf batches with hot pages and single-event pages. (The round-1
    block-scan kernel, retired in round 2, lost bit 31 of large fault counts here.)"""
    L = ga.gdsm.lib()
    n = 6000
    rng = np.random.default_rng(77 + unaligned)
    with ga.Context(n, arenas=()) as c:
        c.coh_init(8)
        st = rng.integers(0, 1 << 19, n).astype(np.uint32)
        fl = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        c.coh_upload(st, fl)
        for b in range(3):
            counts = zipf_counts(n, 70000, s=0.9, seed=200 + b)
            counts[rng.integers(0, n, 5)] = rng.integers(2000, 9000, 5)
            ev = oracle.gen_events(counts, seed=300 + b, n_nodes=8, write_pct=(5, 30, 70)[b])
            _, ptr = _batch_from(c, ev, unaligned)
            tot = (C.c_uint64 * 10)()
            assert L.gdsm_coherence_batch(c.handle, ptr, len(ev), tot) == 0
            rc, otot = oracle.coherence(st, fl, ev)
            assert rc == 0
            assert list(tot) == [otot["invalidations"], otot["transfers"], *otot["node_faults"]]
            gst, gfl = c.coh_download()
            assert np.array_equal(gst, st), np.flatnonzero(gst != st)[:10]
            assert np.array_equal(gfl, fl), np.flatnonzero(gfl != fl)[:10]


def test_out_of_range_page_writes_nothing():
    """A rejected batch whose segment lies on a page >= n_pages must not store its final state
    anywhere: the state word it computed is not a page id (a read by node 0 ends in state 1, which
    once landed on page 1's entry)."""
    with ga.Context(16, arenas=()) as c:
        c.coh_init(8)
        st0, fl0 = c.coh_download()
        for e in ((99 << 4), (99 << 4) | (3 << 1), (40 << 4) | 1):
            with pytest.raises(GdsmError) as ei:
                c.coherence_batch(np.array([e], np.uint64))
            assert ei.value.errno == 22
            st, fl = c.coh_download()
            assert np.array_equal(st, st0) and np.array_equal(fl, fl0), hex(e)


def test_device_event_generation_matches_oracle():
    n = 4000
    counts = zipf_counts(n, 60000, seed=2)
    with ga.Context(n, arenas=()) as c:
        ev = c.gen_events(counts, seed=21, n_nodes=8, write_pct=20)
        got = ev.download(np.uint64, ev.count)
    assert np.array_equal(got, oracle.gen_events(counts, seed=21, n_nodes=8, write_pct=20))


def test_config4_scaled_parity():
    """Config 4 shape (Zipf 0.8 over the pages, 8 nodes, 20 % writes) at 1M pages x 16M events,
    generated on the device, checked against the oracle fold of the same events."""
    n = 1 << 20
    counts = zipf_counts(n, 16 << 20, s=0.8, seed=44)
    with ga.Context(n, arenas=()) as c:
        ev = c.gen_events(counts, seed=44)
        c.coh_init(8)
        tot = c.coherence_batch(ev)
        host_ev = ev.download(np.uint64, ev.count)
        gst, gfl = c.coh_download()
    st, fl = oracle.coh_init(n, 8)
    rc, otot = oracle.coherence(st, fl, host_ev)
    assert rc == 0 and tot == otot
    assert np.array_equal(gst, st) and np.array_equal(gfl, fl)


@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_config4_full_size_parity(dist):
    """BASELINE config 4 at its full size (16M pages, 8 nodes, 1B events, 20 % writes), the
    events generated on the device as bench.py does, and the whole batch folded by the C oracle
    on the host: page-table words, per-page faults and totals bit-exact. Also the checksum
    property Σ per-page faults == Σ per-node faults (both start at 0)."""
    from gallocy_amd.workloads import event_counts
    n, total = 16 << 20, 1 << 30
    counts = event_counts(n, total, dist=dist, seed=2026)
    with ga.Context(n, arenas=()) as c:
        ev = c.gen_events(counts, seed=2026)
        c.coh_init(8)
        tot = c.coherence_batch(ev)
        host_ev = ev.download(np.uint64, ev.count)
        ev.free()
        gst, gfl = c.coh_download()
    assert len(host_ev) == total
    assert int(gfl.astype(np.uint64).sum()) == sum(tot["node_faults"])
    st, fl = oracle.coh_init(n, 8)
    rc, otot = oracle.coherence(st, fl, host_ev)
    del host_ev
    assert rc == 0 and tot == otot
    assert np.array_equal(gst, st), np.flatnonzero(gst != st)[:10]
    assert np.array_equal(gfl, fl), np.flatnonzero(gfl != fl)[:10]


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_every_selectable_coherence_variant(variant):
    """Every coherence path the product library can select (gdsm_tune "coh_variant": 0 =
    automatic, the streaming fold with 256-event spans for this small batch; 1 = the streaming
    fold with 4096-event spans; 2 = the single-pass fold at every size) is bit-exact on Zipf batches with hot
    pages, uploaded arbitrary states, fewer nodes and a partial last block."""
    L = ga.gdsm.lib()
    assert L.gdsm_tune(b"coh_variant", variant) == 0
    try:
        n = 9000
        rng = np.random.default_rng(500 + variant)
        counts = zipf_counts(n, 130000, s=0.9, seed=31)
        counts[rng.integers(0, n, 3)] = rng.integers(5000, 12000, 3)
        ev = oracle.gen_events(counts, seed=32, n_nodes=5, write_pct=25)
        with ga.Context(n, arenas=()) as c:
            c.coh_init(5)
            st = rng.integers(0, 1 << 19, n).astype(np.uint32)
            fl = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
            c.coh_upload(st, fl)
            tot = c.coherence_batch(ev)
            rc, otot = oracle.coherence(st, fl, ev, n_nodes=5)
            assert rc == 0 and tot == otot
            gst, gfl = c.coh_download()
            assert np.array_equal(gst, st) and np.array_equal(gfl, fl)
    finally:
        L.gdsm_tune(b"coh_variant", 0)


def test_coherence_at_the_maximum_table_size():
    """GDSM_MAX_COH_PAGES = 2^28 pages, where the top page's events use every bit of the event's
    low dword (page << 4): one batch on the lowest and the highest 4096 pages, the top page hot
    (its events cross many 2048-event blocks), bit-exact against the oracle over the whole
    2 GiB page table; a table one page larger is refused."""
    n = 1 << 28
    rng = np.random.default_rng(28)
    lo = rng.integers(0, 40, 4096).astype(np.uint64)
    hi = rng.integers(0, 40, 4096).astype(np.uint64)
    hi[-1] = 20000
    ev = np.concatenate([oracle.gen_events(lo, seed=5, write_pct=20),
                         oracle.gen_events(hi, seed=6, write_pct=20, first_page=n - 4096)])
    assert int(ev[-1] >> 4) == n - 1
    with ga.Context(n, arenas=()) as c:
        c.coh_init(8)
        tot = c.coherence_batch(ev)
        gst, gfl = c.coh_download()
    st, fl = oracle.coh_init(n, 8)
    rc, otot = oracle.coherence(st, fl, ev)
    assert rc == 0 and tot == otot
    assert np.array_equal(gst, st), np.flatnonzero(gst != st)[:10]
    assert np.array_equal(gfl, fl), np.flatnonzero(gfl != fl)[:10]
    del gst, gfl, st, fl
    with ga.Context(n + 1, arenas=()) as c:
        with pytest.raises(GdsmError):
            c.coh_init(8)


@pytest.mark.parametrize("span", [4, 1])
def test_chained_small_batches_across_launches_and_graphs(span):
    """Batches of up to 2^20 events take the chained one-launch fold (CohChain: epoch-tagged
    status granules; ticket counters, totals row and completion counter zeroed by the previous
    launch; the last span to finish copies the totals out). Twenty-odd batches in a row of varying
    size, mixed with whole-GPU batches (> 2^20 events, the zeroing path), a graph of a small batch
    replayed between them (captured launches take the zeroing form), the chain switched off and
    on, and a rejected batch: every batch's totals and the final page table equal the oracle's.
    span: the chained fold's 64-event chunks per span (gdsm_tune "coh_span"; 4 is the default)."""
    n, nodes = 6000, 8
    rng = np.random.default_rng(31)
    L = ga.gdsm.lib()

    def batch(k, seed):
        counts = np.bincount(rng.integers(0, n, k), minlength=n).astype(np.uint64)
        return oracle.gen_events(counts, seed=seed, n_nodes=nodes, write_pct=25)

    assert L.gdsm_tune(b"coh_span", span) == 0
    with ga.Context(n, arenas=()) as c:
        c.coh_init(nodes)
        st, fl = oracle.coh_init(n, nodes)
        gev = batch(3000, 7)
        d_gev = c.buffer(gev.nbytes).upload(gev)
        d_gtot = c.buffer(80)
        ga.gdsm.check(L.gdsm_reserve(c.handle, 0, 1 << 21), "gdsm_reserve")
        c.sync()
        c.capture_begin()
        ga.gdsm.check(L.gdsm_coherence_batch_async(c.handle, d_gev.ptr, len(gev), d_gtot.ptr),
                      "coherence")
        graph = c.capture_end()
        sizes = [1, 300, 8000, 257, 256, 70000, 1 << 20, 4096, (1 << 20) + 5, 50000, 12, 9000]
        try:
            for it, k in enumerate(sizes * 2):
                if it == 6:
                    assert L.gdsm_tune(b"coh_chain", 0) == 0
                if it == 9:
                    assert L.gdsm_tune(b"coh_chain", 1) == 0
                ev = batch(k, 100 + it)
                tot = c.coherence_batch(ev)
                rc, otot = oracle.coherence(st, fl, ev, n_nodes=nodes)
                assert rc == 0 and tot == otot, (it, k)
                if it % 5 == 2:
                    graph.launch(c)
                    c.sync()
                    rc, otot = oracle.coherence(st, fl, gev, n_nodes=nodes)
                    got = d_gtot.download(np.uint64, 10)
                    assert rc == 0
                    assert got.tolist() == [otot["invalidations"], otot["transfers"],
                                            *otot["node_faults"]], it
            gst, gfl = c.coh_download()
            assert np.array_equal(gst, st) and np.array_equal(gfl, fl)
            with pytest.raises(GdsmError) as ei:  # rejected inside the chain, which goes on
                c.coherence_batch(np.array([5 << 4, 2 << 4], np.uint64))
            assert ei.value.errno == 22
            c.coh_init(nodes)
            st, fl = oracle.coh_init(n, nodes)
            for it in range(5):
                ev = batch(1000 * (it + 1), 500 + it)
                tot = c.coherence_batch(ev)
                rc, otot = oracle.coherence(st, fl, ev, n_nodes=nodes)
                assert rc == 0 and tot == otot, it
            gst, gfl = c.coh_download()
            assert np.array_equal(gst, st) and np.array_equal(gfl, fl)
        finally:
            L.gdsm_tune(b"coh_chain", 1)
            L.gdsm_tune(b"coh_span", 4)
            graph.destroy()
