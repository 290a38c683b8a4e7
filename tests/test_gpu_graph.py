"""HIP graph capture through the C ABI (gdsm_capture_*, include/gdsm.h): recorded libgdsm calls
replay bit-exactly like the same calls issued eagerly, across two joined contexts, and the
capture refuses what it cannot record (workspace growth, host synchronisation)."""
import errno

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd.gdsm import GdsmError, Runs
from oracle import oracle

pytestmark = pytest.mark.gpu


def _pages(n, seed):
    twin, cur = oracle.gen_pages(n, seed=seed, mode=0, ppm=20000)
    return twin, cur


def test_graph_replays_twin_diff_apply_and_coherence():
    n = 3000
    twin, cur = _pages(n, 5)
    ids = np.arange(0, n, 3, dtype=np.uint32)
    counts = np.random.default_rng(3).integers(0, 9, 500).astype(np.uint64)
    ev = oracle.gen_events(counts, seed=4, n_nodes=8, write_pct=30)
    with ga.Context(n) as c, ga.Context(500, arenas=()) as pt:
        c.upload("twin", twin)
        c.upload("current", cur)
        c.upload("replica", twin)
        pt.coh_init(8)
        d_ids = c.ids(ids)
        d_ev = pt.buffer(ev.nbytes).upload(ev)
        d_tot = pt.buffer(80)
        runs = Runs(c, len(ids), cap=len(ids) * 4200)
        ga.gdsm.check(ga.gdsm.lib().gdsm_reserve(c.handle, len(ids), 0), "reserve")
        ga.gdsm.check(ga.gdsm.lib().gdsm_reserve(pt.handle, 0, len(ev)), "reserve")
        c.sync()
        c.capture_begin(pt)
        ga.gdsm.check(ga.gdsm.lib().gdsm_coherence_batch_async(pt.handle, d_ev.ptr, len(ev),
                                                                d_tot.ptr), "coherence")
        c.diff(d_ids.ptr, n=len(ids), out=runs)
        c.apply(runs, "replica", d_ids.ptr)
        g = c.capture_end()
        # nothing ran yet
        assert np.array_equal(c.download("replica"), twin)
        g.launch(c)
        c.sync()
        exp = twin.copy()
        exp[ids] = cur[ids]
        assert np.array_equal(c.download("replica"), exp)
        st, fl = oracle.coh_init(500, 8)
        rc, otot = oracle.coherence(st, fl, ev)
        tot = d_tot.download(np.uint64, 10)
        assert rc == 0
        assert tot.tolist() == [otot["invalidations"], otot["transfers"], *otot["node_faults"]]
        gst, gfl = pt.coh_download()
        assert np.array_equal(gst, st) and np.array_equal(gfl, fl)
        g.destroy()
        runs.free()


def test_capture_refuses_workspace_growth_and_host_sync():
    n = 512
    twin, cur = _pages(n, 6)
    with ga.Context(n) as c:
        c.upload("twin", twin)
        c.upload("current", cur)
        runs = Runs(c, n, cap=n * 4200)
        ga.gdsm.check(ga.gdsm.lib().gdsm_reserve(c.handle, 16, 0), "reserve")
        c.sync()
        c.capture_begin()
        with pytest.raises(GdsmError) as ei:
            c.diff(n=n, out=runs)  # needs a larger workspace than reserved
        assert ei.value.errno == errno.EBUSY
        with pytest.raises(GdsmError) as ei:
            c.sync()  # a recording stream cannot be waited for
        assert ei.value.errno == errno.EBUSY
        c.capture_end().destroy()
        # after the capture the context works eagerly again
        c.diff(n=n, out=runs)
        c.sync()
        h = runs.to_host()
        ro, data = oracle.diff_pages(twin, cur)
        assert np.array_equal(h.rec_off, ro) and np.array_equal(h.data[:int(ro[-1])], data)
        runs.free()
        with pytest.raises(GdsmError) as ei:
            c.capture_end()
        assert ei.value.errno == errno.EINVAL


def test_capture_end_on_joined_context_is_refused():
    """Only the context that began a capture may end it: gdsm_capture_end on a context that was
    joined into another's capture returns -EINVAL and leaves the recording open, which the
    originating context then ends (round-2 advice, gdsm_capi.cpp capture_origin)."""
    import ctypes as C
    L = ga.gdsm.lib()
    with ga.Context(64) as a, ga.Context(64) as b:
        a.sync()
        b.sync()
        a.capture_begin(b)
        g = C.c_void_p()
        assert L.gdsm_capture_end(b.handle, C.byref(g)) == -errno.EINVAL
        assert not g.value
        a.capture_end().destroy()
        # both contexts work eagerly again
        a.sync()
        b.sync()


def _hip():
    import ctypes as C
    h = C.CDLL("libamdhip64.so")
    vp = C.c_void_p
    h.hipStreamBeginCapture.argtypes = [vp, C.c_int]
    h.hipStreamEndCapture.argtypes = [vp, C.POINTER(vp)]
    h.hipGraphInstantiate.argtypes = [C.POINTER(vp), vp, vp, vp, C.c_size_t]
    h.hipGraphLaunch.argtypes = [vp, vp]
    h.hipGraphExecDestroy.argtypes = [vp]
    h.hipGraphDestroy.argtypes = [vp]
    return h


def test_direct_capture_of_the_context_stream_replays_twice():
    """A caller that captures gdsm_stream() itself (hipStreamBeginCapture, not gdsm_capture_*):
    the recorded short release and small coherence batch must replay correctly more than once
    (round-5 advice: the chained one-launch forms carry a per-launch epoch that a replay would
    repeat, so every call checks hipStreamIsCapturing and records the zeroing forms). CURRENT
    and the event buffer change between the two replays; each replay's stream, REPLICA and page
    table equal the oracle's."""
    import ctypes as C
    hip = _hip()
    n = 48
    twin, cur1 = _pages(n, 11)
    _, cur2 = oracle.gen_pages(n, seed=12, mode=0, ppm=60000)
    counts = np.random.default_rng(13).integers(0, 9, 300).astype(np.uint64)
    ev1 = oracle.gen_events(counts, seed=14, n_nodes=8, write_pct=30)
    ev2 = oracle.gen_events(counts, seed=15, n_nodes=8, write_pct=30)
    m = len(ev1)
    assert len(ev2) == m and not np.array_equal(ev1, ev2)
    with ga.Context(n) as c, ga.Context(300, arenas=()) as pt:
        c.upload("twin", twin)
        c.upload("current", cur1)
        c.upload("replica", twin)
        pt.coh_init(8)
        d_ev = pt.buffer(8 * m)
        d_tot = pt.buffer(80)
        d_ids = c.ids(np.arange(n, dtype=np.uint32))
        runs = Runs(c, n, cap=n * 4200)
        ga.gdsm.check(ga.gdsm.lib().gdsm_reserve(c.handle, n, 0), "reserve")
        ga.gdsm.check(ga.gdsm.lib().gdsm_reserve(pt.handle, 0, m), "reserve")
        c.sync()
        pt.sync()
        graphs = []
        for ctx, record in ((c, lambda: c.diff(d_ids.ptr, n=n, out=runs, apply_to="replica")),
                            (pt, None)):
            s = C.c_void_p(ctx.stream)
            assert hip.hipStreamBeginCapture(s, 2) == 0  # relaxed mode
            if record:
                record()
            else:
                ga.gdsm.check(ga.gdsm.lib().gdsm_coherence_batch_async(
                    pt.handle, d_ev.ptr, m, d_tot.ptr), "coherence")
            g, ge = C.c_void_p(), C.c_void_p()
            assert hip.hipStreamEndCapture(s, C.byref(g)) == 0
            assert hip.hipGraphInstantiate(C.byref(ge), g, None, None, 0) == 0
            graphs.append((s, g, ge))
        st, fl = oracle.coh_init(300, 8)
        for cur, ev in ((cur1, ev1), (cur2, ev2)):
            c.upload("current", cur)
            c.upload("replica", twin)
            d_ev.upload(ev)
            for s, _, ge in graphs:
                assert hip.hipGraphLaunch(ge, s) == 0
            c.sync()
            pt.sync()
            h = runs.to_host()
            ro, data = oracle.diff_pages(twin, cur)
            assert np.array_equal(h.rec_off, ro)
            assert np.array_equal(h.data[:int(ro[-1])], data)
            assert np.array_equal(c.download("replica"), cur)
            rc, otot = oracle.coherence(st, fl, ev)
            assert rc == 0
            tot = d_tot.download(np.uint64, 10)
            assert tot.tolist() == [otot["invalidations"], otot["transfers"], *otot["node_faults"]]
            gst, gfl = pt.coh_download()
            assert np.array_equal(gst, st) and np.array_equal(gfl, fl)
        for _, g, ge in graphs:
            hip.hipGraphExecDestroy(ge)
            hip.hipGraphDestroy(g)
        runs.free()
