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
