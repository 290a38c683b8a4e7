"""GPU parity of the page hot path (twin / run diff / apply) against the C oracle, through the
C-ABI (libgdsm.so). Bit-exact: this is byte work, docs/SPEC.md §2-4."""
import ctypes as C

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd import _lib
from gallocy_amd._lib import GdsmRuns
from gallocy_amd.gdsm import GdsmError, HostRuns, Runs
from oracle import oracle
from tests.helpers import (RAW_RANGES, REF_WINDOW_SETS, c1_windows, np_diff, raw_range_pages,
                           runs_positions, window_pages)

pytestmark = pytest.mark.gpu


def _eq_runs(host: HostRuns, ro, data):
    assert np.array_equal(host.rec_off, ro), "rec_off differs"
    assert np.array_equal(host.data, data), "data differs"


@pytest.fixture(scope="module")
def ctx64():
    with ga.Context(64) as c:
        yield c


def test_gen_matches_oracle(ctx64):
    ctx64.gen_pages(seed=1, mode=ga.GEN_UNIFORM, ppm=10000, first_global=7)
    ctx64.sync()
    t, c, r = oracle.gen_pages(64, seed=1, mode=0, ppm=10000, first_page=7, replica=True)
    assert np.array_equal(ctx64.download("twin"), t)
    assert np.array_equal(ctx64.download("current"), c)
    assert np.array_equal(ctx64.download("replica"), r)
    ctx64.gen_pages(seed=4, mode=ga.GEN_CLUSTERED, ppm=100000, first_global=1 << 30)
    t, c = oracle.gen_pages(64, seed=4, mode=1, ppm=100000, first_page=1 << 30)
    assert np.array_equal(ctx64.download("current"), c)


def test_config1_diff_apply_bit_exact(ctx64, golden):
    """BASELINE config 1 (64 x 4 KiB, 1 % word writes, seed 1) on the GPU."""
    ctx64.gen_pages(seed=1, mode=ga.GEN_UNIFORM, ppm=10000)
    runs = ctx64.diff()
    h = runs.to_host()
    _eq_runs(h, golden["pages"]["c1_rec_off"], golden["pages"]["c1_data"])
    ctx64.apply(runs)
    ctx64.sync()
    assert np.array_equal(ctx64.download("replica"), ctx64.download("current"))
    runs.free()


def test_edge_pages_golden(golden):
    g = golden["pages"]
    n = g["edge_twin"].shape[0]
    with ga.Context(n) as c:
        c.upload("twin", g["edge_twin"])
        c.upload("current", g["edge_cur"])
        c.upload("replica", g["edge_twin"])
        runs = c.diff()
        _eq_runs(runs.to_host(), g["edge_rec_off"], g["edge_data"])
        c.apply(runs)
        c.sync()
        assert np.array_equal(c.download("replica"), g["edge_cur"])


@pytest.mark.parametrize("n", [700, 300])
@pytest.mark.parametrize("density", [0.001, 0.05, 0.3, 0.5, 0.9, 1.0])
def test_random_byte_density(density, n):
    """n = 700: not a multiple of the 64-page block (four pages per workgroup, chained); n = 300:
    the page-per-workgroup release kernel."""
    rng = np.random.default_rng(int(density * 1000) + n)
    twin = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
    cur = twin.copy()
    mask = rng.random((n, 4096)) < density
    cur[mask] ^= rng.integers(1, 256, int(mask.sum()), dtype=np.uint8)
    with ga.Context(n) as c:
        c.upload("twin", twin)
        c.upload("current", cur)
        c.upload("replica", twin)
        runs = c.diff()
        ro, data = oracle.diff_pages(twin, cur)
        _eq_runs(runs.to_host(), ro, data)
        c.apply(runs)
        c.sync()
        assert np.array_equal(c.download("replica"), cur)


def test_page_id_lists_and_duplicates():
    n = 300
    t, cur = oracle.gen_pages(n, seed=8, mode=1, ppm=100000)
    rng = np.random.default_rng(5)
    ids = rng.integers(0, n, 513).astype(np.uint32)  # duplicates allowed for diff (read only)
    with ga.Context(n) as c:
        c.upload("twin", t)
        c.upload("current", cur)
        d_ids = c.ids(ids)
        runs = c.diff(d_ids)
        ro, data = oracle.diff_pages(t, cur, ids=ids)
        _eq_runs(runs.to_host(), ro, data)
        # apply needs unique ids: apply a permutation into CURRENT-shaped replica
        perm = rng.permutation(n).astype(np.uint32)
        d_perm = c.ids(perm)
        runs2 = c.diff(d_perm)
        c.upload("replica", t)
        c.apply(runs2, "replica", d_perm)
        c.sync()
        assert np.array_equal(c.download("replica"), cur)
        # twin(ids): snapshot only the listed pages
        few = np.array([3, 10, 299], np.uint32)
        c.twin(c.ids(few))
        c.sync()
        tw = c.download("twin")
        assert np.array_equal(tw[few], cur[few])
        rest = np.setdiff1d(np.arange(n), few)
        assert np.array_equal(tw[rest], t[rest])


def test_out_of_range_page_ids_touch_no_listed_page_and_fail():
    """Context-level id lists are checked on the device: an id >= n_pages goes to the arenas'
    guard page (never outside them), the valid ids are processed as usual and the next
    gdsm_sync reports -EINVAL."""
    n = 16
    t, cur = oracle.gen_pages(n, seed=9, mode=0, ppm=50000)
    ids = np.array([2, 16, 5, 0xFFFFFFFF, 7], np.uint32)
    ok = np.array([0, 2, 4])
    rest = np.setdiff1d(np.arange(n), ids[ok])
    with ga.Context(n) as c:
        c.upload("twin", t)
        c.upload("current", cur)
        c.upload("replica", t)
        d_ids = c.ids(ids)
        runs = c.diff(d_ids)
        with pytest.raises(GdsmError) as ei:
            c.sync()
        assert ei.value.errno == 22
        host = runs.to_host()
        for i in ok:
            assert host.record(i) == oracle.diff_pages(t[ids[i]][None], cur[ids[i]][None])[1].tobytes()
        for apply in (c.apply, c.apply_async):
            c.upload("replica", t)
            apply(runs, "replica", d_ids)
            with pytest.raises(GdsmError):
                c.sync()
            rep = c.download("replica")
            assert np.array_equal(rep[ids[ok]], cur[ids[ok]])
            assert np.array_equal(rep[rest], t[rest])
        c.twin(d_ids)
        with pytest.raises(GdsmError):
            c.sync()
        tw = c.download("twin")
        assert np.array_equal(tw[ids[ok]], cur[ids[ok]]) and np.array_equal(tw[rest], t[rest])
        assert np.array_equal(c.download("current"), cur)
        c.sync()  # the error word was cleared


def test_raw_diff_workspace_contract():
    """gdsm_diff_raw with the workspace gdsm_diff_workspace_bytes(n) names works; a smaller one is
    rejected with -EINVAL before anything runs."""
    n = 1000
    t, cur = oracle.gen_pages(n, seed=12, mode=0, ppm=40000)
    L = _lib.load()
    with ga.Context(n) as c:
        c.upload("twin", t)
        c.upload("current", cur)
        ws_bytes = L.gdsm_diff_workspace_bytes(n)
        ws = c.buffer(ws_bytes)
        ro_buf = c.buffer((n + 1) * 8)
        cap = n * 2048
        data_buf = c.buffer(cap)
        assert L.gdsm_diff_raw(c.arena_ptr("twin"), c.arena_ptr("current"), None, n, ro_buf.ptr,
                               data_buf.ptr, cap, ws.ptr, 64, c.stream) == -22
        rc = L.gdsm_diff_raw(c.arena_ptr("twin"), c.arena_ptr("current"), None, n, ro_buf.ptr,
                             data_buf.ptr, cap, ws.ptr, ws_bytes, c.stream)
        assert rc == 0
        c.sync()
        ro_h = ro_buf.download(np.uint64, n + 1)
        ro, data = oracle.diff_pages(t, cur)
        assert np.array_equal(ro_h, ro)
        assert np.array_equal(data_buf.download(np.uint8, int(ro[-1])), data)


def test_capacity_overflow_reports_enospc():
    n = 64
    t, cur = oracle.gen_pages(n, seed=3, mode=1, ppm=300000)
    with ga.Context(n) as c:
        c.upload("twin", t)
        c.upload("current", cur)
        ro, data = oracle.diff_pages(t, cur)
        cap = int(ro[n // 2]) + 16
        runs = c.diff(cap=cap)
        with pytest.raises(GdsmError) as ei:
            runs.total()
        assert ei.value.errno == 28
        got = np.empty(n + 1, np.uint64)
        L = _lib.load()
        assert L.gdsm_memcpy_d2h(c.handle, got.ctypes.data, runs.s.rec_off, got.nbytes) == 0
        assert np.array_equal(got, ro)  # rec_off is complete even when data overflowed
        # every record that ends inside the capacity was written (fast and re-read pages alike)
        fit = int(ro[ro <= cap].max())
        part = np.empty(fit, np.uint8)
        assert L.gdsm_memcpy_d2h(c.handle, part.ctypes.data, runs.s.data, fit) == 0
        assert np.array_equal(part, data[:fit])


def test_apply_rejects_malformed_stream():
    n = 8
    t, cur = oracle.gen_pages(n, seed=2, mode=0, ppm=50000)
    ro, data = oracle.diff_pages(t, cur)
    bad = data.copy()
    i = int(np.flatnonzero(np.diff(ro))[0])
    bad[int(ro[i]):int(ro[i]) + 4] = np.frombuffer(np.uint32(4000).tobytes(), np.uint8)  # nruns
    with ga.Context(n) as c:
        c.upload("replica", t)
        r = Runs.from_host(c, HostRuns(ro, bad))
        c.apply(r)
        with pytest.raises(GdsmError) as ei:
            c.sync()
        assert ei.value.errno == 22
        # the good records were still applied; the bad page was left alone
        rep = c.download("replica")
        good = [k for k in range(n) if k != i and ro[k + 1] > ro[k]]
        assert np.array_equal(rep[good], cur[good])
        assert np.array_equal(rep[i], t[i])


def test_empty_batch():
    with ga.Context(4) as c:
        runs = c.diff(n=0)
        assert runs.total() == 0
        c.apply(runs)
        c.sync()


def _sample_parity(c, n, seed, mode, ppm, k=64):
    """Diff of a random sample of pages (by id) equals the oracle on the same global pages."""
    rng = np.random.default_rng(seed)
    ids = np.sort(rng.choice(n, k, replace=False)).astype(np.uint32)
    runs = c.diff(c.ids(ids), cap=k * 10244)
    h = runs.to_host()
    for j, p in enumerate(ids):
        t, cur = oracle.gen_pages(1, seed=seed, mode=mode, ppm=ppm, first_page=int(p))
        ro, data = oracle.diff_pages(t, cur)
        assert h.record(j) == data.tobytes()
    runs.free()


def test_config2_full_size_properties():
    """BASELINE config 2 at full size: 1M pages, 1 % word writes. Size-independent checks:
    sampled records equal the oracle, apply makes REPLICA == CURRENT (diff(REPLICA, CURRENT) is
    empty), a second apply is idempotent, and twin() empties the diff."""
    n = 1 << 20
    L = _lib.load()
    with ga.Context(n) as c:
        c.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
        runs = c.diff(cap=256 << 20)
        total = runs.total()
        # E|D| ~ 61 B/page at this density
        assert 50 * n < total < 72 * n
        ro = np.empty(n + 1, np.uint64)
        assert L.gdsm_memcpy_d2h(c.handle, ro.ctypes.data, runs.s.rec_off, ro.nbytes) == 0
        assert ro[0] == 0 and np.all(np.diff(ro.astype(np.int64)) >= 0) and ro[-1] == total
        assert np.all(np.diff(ro) % 4 == 0)
        dirty = int((np.diff(ro) > 0).sum())
        assert abs(dirty / n - (1 - 0.99 ** 512)) < 0.002  # 99.4 % of pages dirty
        c.apply(runs)
        c.apply(runs)
        c.sync()
        chk = ga.Runs(c, n, cap=1 << 20)
        ws = c.buffer(L.gdsm_diff_workspace_bytes(n))
        rc = L.gdsm_diff_raw(c.arena_ptr("replica"), c.arena_ptr("current"), None, n,
                             chk.s.rec_off, chk.s.data, chk.cap, ws.ptr, ws.nbytes, c.stream)
        assert rc == 0 and chk.total() == 0
        _sample_parity(c, n, 2026, 0, 10000)
        c.twin()
        assert c.diff(cap=1 << 20).total() == 0


def test_config2_full_stream_bit_exact():
    """BASELINE config 2 at full size (1M pages, 1 % word writes, the bench's seed): the whole
    diff stream (rec_off and record bytes) equals the C oracle's over the same pages, and the
    device-generated arenas equal the oracle's generator page for page."""
    n = 1 << 20
    twin, cur = oracle.gen_pages(n, seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
    oro, odata = oracle.diff_pages(twin, cur, cap=256 << 20)
    del twin
    with ga.Context(n) as c:
        c.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
        h = c.diff(cap=256 << 20).to_host()
        assert np.array_equal(c.download("current"), cur)
    assert np.array_equal(h.rec_off, oro), np.flatnonzero(h.rec_off != oro)[:10]
    assert len(h.data) == len(odata) and np.array_equal(h.data, odata)


def test_north_star_16M_pages_1pct():
    """The north-star size on one GPU: 16M x 4 KiB pages (3 arenas = 192 GiB of HBM), 1 % random
    word writes. The WHOLE stream equals the oracle's record by record (oracle.check_stream
    regenerates every page on the host); apply makes REPLICA == CURRENT (the diff of the two is
    empty), a second apply changes nothing, and twin() empties the diff."""
    n = 16 << 20
    L = _lib.load()
    with ga.Context(n) as c:
        c.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
        runs = c.diff(cap=2 << 30)
        total = runs.total()
        assert 50 * n < total < 72 * n
        ro = np.empty(n + 1, np.uint64)
        assert L.gdsm_memcpy_d2h(c.handle, ro.ctypes.data, runs.s.rec_off, ro.nbytes) == 0
        sizes = np.diff(ro.astype(np.int64))
        assert ro[0] == 0 and ro[-1] == total and (sizes >= 0).all() and (sizes % 4 == 0).all()
        assert abs((sizes > 0).mean() - (1 - 0.99 ** 512)) < 0.001
        del sizes
        data = np.empty(total, np.uint8)
        assert L.gdsm_memcpy_d2h(c.handle, data.ctypes.data, runs.s.data, total) == 0
        assert oracle.check_stream(ro, data, 0, n, 2026, 0, 10000) == -1
        del data, ro
        c.apply(runs)
        c.apply(runs)
        c.sync()
        runs.free()
        chk = ga.Runs(c, n, cap=1 << 20)
        ws = c.buffer(L.gdsm_diff_workspace_bytes(n))
        assert L.gdsm_diff_raw(c.arena_ptr("replica"), c.arena_ptr("current"), None, n,
                               chk.s.rec_off, chk.s.data, chk.cap, ws.ptr, ws.nbytes,
                               c.stream) == 0
        assert chk.total() == 0
        ws.free()
        c.twin()
        assert c.diff(out=chk).total() == 0


def test_config3_16M_clustered_whole_stream():
    """BASELINE config 3's 16M clustered pages (10 % of 64-B clusters) on ONE GPU, in the dense
    diff geometry the context picks after a first release: the whole 7.4 GB stream equals the
    oracle's record by record, and apply makes REPLICA == CURRENT."""
    n = 16 << 20
    L = _lib.load()
    with ga.Context(n) as c:
        c.gen_pages(seed=2026, mode=ga.GEN_CLUSTERED, ppm=100000)
        runs = c.diff(cap=8 << 30)
        total = runs.total()  # the context now knows the density: the second diff is 16 pages
        runs = c.diff(out=runs)
        assert runs.total() == total and 400 * n < total < 480 * n
        ro = np.empty(n + 1, np.uint64)
        assert L.gdsm_memcpy_d2h(c.handle, ro.ctypes.data, runs.s.rec_off, ro.nbytes) == 0
        data = np.empty(total, np.uint8)
        assert L.gdsm_memcpy_d2h(c.handle, data.ctypes.data, runs.s.data, total) == 0
        assert oracle.check_stream(ro, data, 0, n, 2026, 1, 100000) == -1
        del data, ro
        c.apply(runs)
        c.sync()
        runs.free()
        chk = ga.Runs(c, n, cap=1 << 20)
        ws = c.buffer(L.gdsm_diff_workspace_bytes(n))
        assert L.gdsm_diff_raw(c.arena_ptr("replica"), c.arena_ptr("current"), None, n,
                               chk.s.rec_off, chk.s.data, chk.cap, ws.ptr, ws.nbytes,
                               c.stream) == 0
        assert chk.total() == 0


def test_config3_shard_properties():
    """BASELINE config 3 shard shape (2M pages = 16M / 8 GPUs, clustered 10 %), one GPU."""
    n = 2 << 20
    with ga.Context(n) as c:
        c.gen_pages(seed=77, mode=ga.GEN_CLUSTERED, ppm=100000, first_global=3 * n)
        runs = c.diff(cap=2 << 30)
        total = runs.total()
        assert 300 * n < total < 600 * n
        c.apply(runs)
        c.sync()
        L = _lib.load()
        chk = ga.Runs(c, n, cap=1 << 20)
        ws = c.buffer(L.gdsm_diff_workspace_bytes(n))
        assert L.gdsm_diff_raw(c.arena_ptr("replica"), c.arena_ptr("current"), None, n,
                               chk.s.rec_off, chk.s.data, chk.cap, ws.ptr, ws.nbytes,
                               c.stream) == 0
        assert chk.total() == 0
        rng = np.random.default_rng(1)
        ids = np.sort(rng.choice(n, 32, replace=False)).astype(np.uint32)
        h = c.diff(c.ids(ids), cap=32 * 10244).to_host()
        for j, p in enumerate(ids):
            t, cur = oracle.gen_pages(1, seed=77, mode=1, ppm=100000, first_page=3 * n + int(p))
            assert h.record(j) == oracle.diff_pages(t, cur)[1].tobytes()


def test_config3_shard_full_stream_bit_exact():
    """BASELINE config 3 shard (2M pages of the 16M-page space, clustered 10 %): the whole diff
    stream equals the C oracle's for the same global pages."""
    n = 2 << 20
    twin, cur = oracle.gen_pages(n, seed=77, mode=ga.GEN_CLUSTERED, ppm=100000, first_page=5 * n)
    oro, odata = oracle.diff_pages(twin, cur, cap=2 << 30)
    del twin, cur
    with ga.Context(n) as c:
        c.gen_pages(seed=77, mode=ga.GEN_CLUSTERED, ppm=100000, first_global=5 * n)
        h = c.diff(cap=2 << 30).to_host()
    assert np.array_equal(h.rec_off, oro), np.flatnonzero(h.rec_off != oro)[:10]
    assert len(h.data) == len(odata) and np.array_equal(h.data, odata)


def _one_record(runs, pay_fill=0xAB):
    hdr = [o | (ln << 16) for o, ln in runs]
    pay = bytes([pay_fill]) * sum(max(0, ln) for _, ln in runs)
    pay += b"\0" * ((-len(pay)) % 4)
    rec = np.array([len(runs)] + hdr, "<u4").tobytes() + pay
    return np.array([0, len(rec)], np.uint64), np.frombuffer(rec, np.uint8).copy()


@pytest.mark.parametrize("runs", [
    [(100, 8), (50, 8)],          # unsorted
    [(100, 8), (104, 8)],         # overlapping
    [(10, 0)],                    # empty run
    [(4090, 8)],                  # past the page end
])
def test_apply_rejects_bad_runs_like_oracle(runs):
    ro, data = _one_record(runs)
    page = np.zeros((1, 4096), np.uint8)
    assert oracle.apply(page.copy(), ro, data) == -22
    with ga.Context(1) as c:
        c.upload("replica", page)
        c.apply(Runs.from_host(c, HostRuns(ro, data)))
        with pytest.raises(GdsmError):
            c.sync()
        assert not c.download("replica").any()


def test_apply_many_runs_and_long_runs():
    """Records mixing long runs (many chunks, pair-spread path) and dense short runs."""
    rng = np.random.default_rng(17)
    n = 257
    twin = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
    cur = twin.copy()
    for i in range(n):
        kind = i % 4
        if kind == 0:    # a few long runs at odd offsets
            for _ in range(3):
                o = int(rng.integers(0, 3000))
                cur[i, o:o + int(rng.integers(17, 1000))] ^= 0xFF
        elif kind == 1:  # 70..300 short runs (more than one 64-run group)
            pos = np.sort(rng.choice(2048, int(rng.integers(70, 300)), replace=False)) * 2
            cur[i, pos] ^= 0x5A
        elif kind == 2:  # one run over the whole page
            cur[i] ^= 0x01
        # kind 3: clean
    ro, data = oracle.diff_pages(twin, cur)
    with ga.Context(n) as c:
        c.upload("replica", twin)
        c.apply(Runs.from_host(c, HostRuns(ro, data)))
        c.sync()
        assert np.array_equal(c.download("replica"), cur)


def test_apply_async_double_buffered_releases():
    """gdsm_apply_async: diff k+1 overlaps apply k, two run buffers alternate. Step k releases
    a distinct page subset; if diff k+2 overwrote buffer k%2 before apply k had read it, apply k
    would write another subset's records onto these pages and the replica would differ."""
    n, steps = 4096, 8
    t, cur = oracle.gen_pages(n, seed=21, mode=1, ppm=200000)
    rng = np.random.default_rng(3)
    perm = rng.permutation(n).astype(np.uint32)
    subsets = np.array_split(perm, steps)
    with ga.Context(n) as c:
        c.upload("twin", t)
        c.upload("current", cur)
        c.upload("replica", t)
        d_ids = [c.ids(s) for s in subsets]
        runs = [Runs(c, n, cap=n * 2048) for _ in range(2)]
        for k in range(steps):
            r = runs[k % 2]
            c.diff(d_ids[k], n=len(subsets[k]), out=r)
            c.apply_async(r, "replica", d_ids[k])
        c.sync()
        assert np.array_equal(c.download("replica"), cur)
        # a later synchronous call is ordered after the async applies (joins the second stream)
        c.upload("replica", t)
        for k in range(steps):
            c.diff(d_ids[k], n=len(subsets[k]), out=runs[k % 2])
            c.apply_async(runs[k % 2], "replica", d_ids[k])
        c.twin()  # TWIN <- CURRENT, must run after every apply
        c.sync()
        assert np.array_equal(c.download("replica"), cur)
        assert np.array_equal(c.download("twin"), cur)


def test_apply_async_reports_malformed_stream():
    n = 8
    t, cur = oracle.gen_pages(n, seed=2, mode=0, ppm=50000)
    ro, data = oracle.diff_pages(t, cur)
    bad = data.copy()
    i = int(np.flatnonzero(np.diff(ro))[0])
    bad[int(ro[i]) + 4:int(ro[i]) + 8] = np.frombuffer(np.uint32(4090 | (100 << 16)).tobytes(),
                                                      np.uint8)  # run past the page end
    with ga.Context(n) as c:
        c.upload("replica", t)
        c.apply_async(Runs.from_host(c, HostRuns(ro, bad)))
        with pytest.raises(GdsmError) as ei:
            c.sync()
        assert ei.value.errno == 22


def _mixed_density_pages(rng, n):
    """Pages whose dirty-chunk counts straddle the compacted kernel's 64-chunk fast path: clean,
    sparse, exactly 64 / 65 dirty 16-B chunks, dense, fully changed, in random order."""
    tw = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
    cu = tw.copy()
    for i in range(n):
        kind = rng.integers(0, 6)
        if kind == 1:
            m = rng.random(4096) < 0.003
        elif kind in (2, 3):
            m = np.zeros(4096, bool)
            chunks = rng.choice(256, 64 if kind == 2 else 65, replace=False)
            for ch in chunks:
                m[ch * 16 + rng.integers(0, 16, rng.integers(1, 17))] = True
        elif kind == 4:
            m = rng.random(4096) < 0.4
        elif kind == 5:
            m = np.ones(4096, bool)
        else:
            continue
        cu[i, m] ^= rng.integers(1, 256, int(m.sum()), dtype=np.uint8)
    return tw, cu


def _lds_overflow_pages(rng, n):
    """Pages with <= 64 dirty 16-B chunks but large records (alternating bytes in 60 chunks:
    2404-B records), so a wave's 8 KiB LDS buffer fills after three of them and the rest of the
    unit is emitted from the arenas after the look-back."""
    tw = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
    cu = tw.copy()
    for i in range(n):
        if i % 5 == 4:
            continue
        for ch in rng.choice(256, 60, replace=False):
            cu[i, ch * 16:ch * 16 + 16:2] ^= 0x3C
    return tw, cu


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8])
def test_diff_variants_bit_exact(variant, golden):
    """Every diff geometry (gdsm_tune "diff_variant": automatic, 16, 32, 2 or 64 pages per wave,
    64 pages per wave with the global spill slot) is bit-exact on edge pages, random byte
    densities (pages past the 64-dirty-chunk fast path), records that overflow the wave's LDS
    buffer (and, for 5, its spill slot), and clustered and uniform synthetic writes."""
    L = _lib.load()
    assert L.gdsm_tune(b"diff_variant", variant) == 0
    try:
        g = golden["pages"]
        cases = [(g["edge_twin"], g["edge_cur"])]
        rng = np.random.default_rng(100 + variant)
        for density in (0.002, 0.02, 0.2, 0.7):
            tw = rng.integers(0, 256, (130, 4096), dtype=np.uint8)
            cu = tw.copy()
            mask = rng.random(tw.shape) < density
            cu[mask] ^= rng.integers(1, 256, int(mask.sum()), dtype=np.uint8)
            cases.append((tw, cu))
        cases.append(oracle.gen_pages(200, seed=9, mode=1, ppm=100000))
        cases.append(oracle.gen_pages(200, seed=9, mode=0, ppm=10000))
        cases.append(_mixed_density_pages(rng, 300))
        cases.append(_lds_overflow_pages(rng, 200))
        for tw, cu in cases:
            with ga.Context(len(tw)) as c:
                c.upload("twin", tw)
                c.upload("current", cu)
                ro, data = oracle.diff_pages(tw, cu)
                _eq_runs(c.diff(cap=max(64, int(ro[-1]))).to_host(), ro, data)
    finally:
        L.gdsm_tune(b"diff_variant", 0)


def test_c1_windows_pinned_by_reference_diff(golden):
    """BASELINE config 1 pinned to the REFERENCE diff() (gallocy/utils/diff.cpp:73-167): the
    remapped config-1 pages, cut into 1024-B windows, were aligned by oracle/_ref (fixture
    tests/golden/c1_windows.npz, every alignment gap-free). On the GPU, per window:
    {i : out1[i] != out2[i]} equals the union of gdsm_diff's runs, and gdsm_apply of the stream
    to the twin gives out2 (whose crc32 the fixture holds)."""
    import zlib
    g = golden["c1_windows"]
    t, cur = c1_windows()
    assert g["gapfree"].all()
    ref = np.unpackbits(g["mask"], axis=1).astype(bool)
    with ga.Context(64) as c:
        c.upload("twin", t)
        c.upload("current", cur)
        c.upload("replica", t)
        runs = c.diff()
        h = runs.to_host()
        pos = runs_positions(h.rec_off, h.data, 64).reshape(-1, 1024)
        bad = np.flatnonzero((pos != ref).any(axis=1))
        assert len(bad) == 0, f"windows whose runs differ from the reference alignment: {bad[:8]}"
        c.apply(runs)
        c.sync()
        rep = c.download("replica").reshape(-1, 1024)
    for w in range(len(rep)):
        assert zlib.crc32(rep[w].tobytes()) == int(g["crc"][w][1]), w


@pytest.mark.parametrize("variant", [0, 7, 8])
@pytest.mark.parametrize("name", REF_WINDOW_SETS)
def test_ref_windows_pinned_by_reference_diff(name, variant, golden):
    """Config 3's clustered pages, a dense set and the SPEC edge pages pinned to the REFERENCE
    diff() (gallocy/utils/diff.cpp:73-167; fixture tests/golden/ref_windows.npz from oracle/_ref):
    for every window whose reference alignment is gap-free, {i : out1[i] != out2[i]} equals the
    union of gdsm_diff's runs (in the default geometry, the 16-page spill geometry and the
    one-page-per-wave geometry), and gdsm_apply of the stream to the twin gives out2 (crc32)."""
    import zlib
    pre = name + "_"
    crc, gapfree, mask = (golden["ref_windows"][pre + k] for k in ("crc", "gapfree", "mask"))
    ref = np.unpackbits(mask, axis=1).astype(bool)
    t, cur = window_pages(name, golden)
    n = t.shape[0]
    L = ga.gdsm.lib()
    L.gdsm_tune(b"diff_variant", variant)
    try:
        with ga.Context(n) as c:
            c.upload("twin", t)
            c.upload("current", cur)
            c.upload("replica", t)
            runs = c.diff(cap=n * 10244)
            h = runs.to_host()
            pos = runs_positions(h.rec_off, h.data, n).reshape(-1, 1024)
            bad = [i for i in np.flatnonzero(gapfree) if not np.array_equal(pos[i], ref[i])]
            assert not bad, f"windows whose runs differ from the reference alignment: {bad[:8]}"
            c.apply(runs)
            c.sync()
            rep = c.download("replica").reshape(-1, 1024)
    finally:
        L.gdsm_tune(b"diff_variant", 0)
    for w in np.flatnonzero(gapfree):
        assert zlib.crc32(rep[w].tobytes()) == int(crc[w][1]), w
    assert np.array_equal(rep.reshape(n, 4096), cur)


@pytest.mark.parametrize("r", [0, 1])
def test_raw_windows_pinned_by_reference_diff(r, golden):
    """BASELINE's own bytes, no remap (tests/golden/raw_windows.npz, the reference diff() through
    oracle/_ref): the north-star pages of range r generated ON THE GPU (gdsm_gen_pages, seed
    2026, uniform 1 %, the bench's generator) and diffed whole by gdsm_diff in the bench's
    geometry. For every reference window (no NUL / '-' byte, all gap-free): the twin and current
    bytes are the reference's out1 / out2 (crc32), the runs cover exactly {i : out1[i] !=
    out2[i]}, and gdsm_apply of the stream to REPLICA gives out2."""
    import zlib
    g = golden["raw_windows"]
    pre = f"r{r}_"
    first, n = (int(x) for x in g[pre + "range"])
    assert (first, n) == RAW_RANGES[r]
    win, crc, mask = (g[pre + k] for k in ("win", "crc", "mask"))
    ref = np.unpackbits(mask, axis=1).astype(bool)
    with ga.Context(n) as c:
        c.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000, first_global=first)
        runs = c.diff(cap=n * 128)
        c.apply(runs)
        c.sync()
        h = runs.to_host()
        pages = np.unique(win // 4)
        tw = np.concatenate([c.download("twin", int(p), 1) for p in pages]).reshape(-1, 1024)
        cw = np.concatenate([c.download("current", int(p), 1) for p in pages]).reshape(-1, 1024)
        rw = np.concatenate([c.download("replica", int(p), 1) for p in pages]).reshape(-1, 1024)
    where = {int(p): i for i, p in enumerate(pages)}
    for j, w in enumerate(win):
        k = 4 * where[int(w) // 4] + int(w) % 4
        assert [zlib.crc32(tw[k].tobytes()), zlib.crc32(cw[k].tobytes())] == crc[j].tolist(), w
        assert zlib.crc32(rw[k].tobytes()) == int(crc[j][1]), w
        p = int(w) // 4
        a, b = int(h.rec_off[p]), int(h.rec_off[p + 1])
        pos = runs_positions(np.array([0, b - a], np.uint64), h.data[a:b], 1).reshape(4, 1024)
        assert np.array_equal(pos[int(w) % 4], ref[j]), w
    # and the host generator agrees with the device one on these pages
    t, cu = raw_range_pages(first, n)
    assert np.array_equal(t[pages].reshape(-1, 1024), tw)
    assert np.array_equal(cu[pages].reshape(-1, 1024), cw)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8])
def test_diff_apply_fused_equals_diff_then_apply(variant, golden):
    """gdsm_diff_apply (the diff kernel also applying the runs to a home copy on this GPU) writes
    the same stream as gdsm_diff, and leaves the target exactly as gdsm_apply of that stream
    would, also when the target is NOT the twin (bytes outside the runs keep their old values),
    with id lists, in every diff geometry."""
    L = _lib.load()
    assert L.gdsm_tune(b"diff_variant", variant) == 0
    try:
        rng = np.random.default_rng(300 + variant)
        g = golden["pages"]
        cases = [(g["edge_twin"], g["edge_cur"])]
        for density in (0.002, 0.05, 0.7):
            tw = rng.integers(0, 256, (130, 4096), dtype=np.uint8)
            cu = tw.copy()
            mask = rng.random(tw.shape) < density
            cu[mask] ^= rng.integers(1, 256, int(mask.sum()), dtype=np.uint8)
            cases.append((tw, cu))
        cases.append(oracle.gen_pages(300, seed=5, mode=0, ppm=10000))
        cases.append(oracle.gen_pages(300, seed=5, mode=1, ppm=100000))
        cases.append(_lds_overflow_pages(rng, 120))
        for tw, cu in cases:
            n = len(tw)
            rep = rng.integers(0, 256, tw.shape, dtype=np.uint8)  # a home copy unlike the twin
            ids = rng.permutation(n).astype(np.uint32)
            ro, data = oracle.diff_pages(tw, cu, ids=ids)
            want = rep.copy()
            assert oracle.apply(want, ro, data, ids=ids) == 0
            with ga.Context(n) as c:
                c.upload("twin", tw)
                c.upload("current", cu)
                c.upload("replica", rep)
                d_ids = c.ids(ids)
                runs = c.diff(d_ids, cap=max(64, int(ro[-1])), apply_to="replica")
                _eq_runs(runs.to_host(), ro, data)
                assert np.array_equal(c.download("replica"), want)
    finally:
        L.gdsm_tune(b"diff_variant", 0)


def test_diff_apply_applies_every_page_past_capacity():
    """With a stream too small for the records, gdsm_diff_apply still applies every page (the
    stream reports -ENOSPC; records past the capacity are not stored)."""
    n = 500
    tw, cu = oracle.gen_pages(n, seed=12, mode=1, ppm=100000)
    with ga.Context(n) as c:
        c.upload("twin", tw)
        c.upload("current", cu)
        c.upload("replica", tw)
        runs = c.diff(cap=4096, apply_to="replica")
        with pytest.raises(GdsmError) as ei:
            runs.total()
        assert ei.value.errno == 28
        assert np.array_equal(c.download("replica"), cu)


def test_diff_apply_config2_full_size():
    """BASELINE config 2 at full size through the fused path the bench times: the whole stream
    equals gdsm_diff's, REPLICA == CURRENT afterwards (the diff of the two is empty)."""
    n = 1 << 20
    L = _lib.load()
    with ga.Context(n) as c:
        c.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
        a = c.diff(cap=256 << 20).to_host()
        b = c.diff(cap=256 << 20, apply_to="replica").to_host()
        assert np.array_equal(a.rec_off, b.rec_off) and np.array_equal(a.data, b.data)
        chk = ga.Runs(c, n, cap=1 << 20)
        ws = c.buffer(L.gdsm_diff_workspace_bytes(n))
        rc = L.gdsm_diff_raw(c.arena_ptr("replica"), c.arena_ptr("current"), None, n,
                             chk.s.rec_off, chk.s.data, chk.cap, ws.ptr, ws.nbytes, c.stream)
        assert rc == 0 and chk.total() == 0


def _long_list_apply_case(rng, n):
    """A stream of n > 16384 records (the long-list apply path) mixing every record shape: clean
    pages, 1 % words, clustered 64-B runs, dense random bytes, alternating bytes (many runs), a
    few long runs, whole-page runs, records larger than a 4 or 8 KiB staging window; and some
    malformed records (bad run count, unsorted / overlapping / empty / past-the-page runs, a size
    that does not add up), which must write nothing while the rest is applied."""
    tw = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
    cu = tw.copy()
    kinds = rng.integers(0, 9, n)
    for i in np.flatnonzero(kinds == 1):  # 1 % of 8-B words
        w = np.flatnonzero(rng.random(512) < 0.01)
        cu[i].reshape(512, 8)[w] ^= 0x11
    for i in np.flatnonzero(kinds == 2):  # clustered: 10 % of 64-B clusters
        c = np.flatnonzero(rng.random(64) < 0.1)
        cu[i].reshape(64, 64)[c] ^= 0x77
    for i in np.flatnonzero(kinds == 3):  # dense random bytes
        m = rng.random(4096) < 0.3
        cu[i, m] ^= 0x0F
    for i in np.flatnonzero(kinds == 4):  # alternating bytes over part of the page
        o = int(rng.integers(0, 2048))
        cu[i, o:o + 1500:2] ^= 0xA5
    for i in np.flatnonzero(kinds == 5):  # a few long runs
        for _ in range(3):
            o = int(rng.integers(0, 3000))
            cu[i, o:o + int(rng.integers(100, 1000))] ^= 0xFF
    for i in np.flatnonzero(kinds == 6):  # the whole page
        cu[i] ^= 0x01
    for i in np.flatnonzero(kinds == 7):  # > 8 KiB records: alternating bytes everywhere
        cu[i, ::2] ^= 0x3C
    ro, data = oracle.diff_pages(tw, cu)
    data = data.copy()
    w = data.view("<u4")
    dirty = np.flatnonzero(np.diff(ro))
    bad = rng.choice(dirty, 40, replace=False)
    for t, i in enumerate(bad):
        b = int(ro[i]) // 4
        nr = int(w[b])
        kind = t % 6
        if kind == 0:
            w[b] = 5000                              # run count past 2048
        elif kind == 1 and nr >= 2:                  # unsorted runs
            w[b + 1], w[b + 2] = w[b + 2], w[b + 1]
        elif kind == 2:                              # empty run
            w[b + 1] = w[b + 1] & 0xFFFF
        elif kind == 3:                              # past the page end
            w[b + 1] = 4095 | (int(w[b + 1] >> 16) + 2 << 16)
        elif kind == 4 and nr >= 2:                  # overlapping runs
            o0, l0 = int(w[b + 1] & 0xFFFF), int(w[b + 1] >> 16)
            o1, l1 = int(w[b + 2] & 0xFFFF), int(w[b + 2] >> 16)
            w[b + 2] = (o0 + l0 - 1) | (l1 << 16) if o0 + l0 - 1 < o1 else w[b + 2]
            if not o0 + l0 - 1 < o1:
                w[b] = 5000
        else:                                        # sizes do not add up
            w[b + 1] = (w[b + 1] & 0xFFFF) | ((int(w[b + 1] >> 16) + 4) << 16)
    rc = oracle.apply(tw.copy(), ro, data)  # the oracle stops at the first malformed record
    want = tw.copy()
    for i in np.flatnonzero(np.diff(ro)):   # the GPU applies every well-formed one (SPEC §4)
        one = data[int(ro[i]):int(ro[i + 1])]
        oracle.apply(want, np.array([0, len(one)], np.uint64), one, ids=np.array([i], np.uint32))
    return tw, ro, data, want, rc


@pytest.mark.parametrize("variant", list(range(8)))
def test_apply_variants_long_lists(variant):
    """Every apply geometry on a long list (gdsm_tune "apply_variant": flat with a 4 KiB window
    filled 16 B per lane (default) or dword by dword, with more or fewer nontemporal stores;
    records by rows with an 8 or 4 KiB window; flat with an 8 or 2 KiB window) leaves REPLICA exactly as the oracle's apply of the same stream, malformed records included (nothing
    of them written, -EINVAL at sync)."""
    L = _lib.load()
    rng = np.random.default_rng(900 + variant)
    n = 20000
    tw, ro, data, want, rc = _long_list_apply_case(rng, n)
    assert rc == -22
    assert L.gdsm_tune(b"apply_variant", variant) == 0
    try:
        with ga.Context(n) as c:
            c.upload("replica", tw)
            r = Runs.from_host(c, HostRuns(ro, data))
            c.apply(r)
            with pytest.raises(GdsmError) as ei:
                c.sync()
            assert ei.value.errno == 22
            got = c.download("replica")
            diffp = np.flatnonzero((got != want).any(axis=1))
            assert len(diffp) == 0, diffp[:10]
            # a permuted id list through the same path
            perm = rng.permutation(n).astype(np.uint32)
            ro2, data2 = oracle.diff_pages(tw[perm], want[perm])
            c.upload("replica", tw)
            c.apply(Runs.from_host(c, HostRuns(ro2, data2)), "replica", c.ids(perm))
            c.sync()
            assert np.array_equal(c.download("replica"), want)
    finally:
        L.gdsm_tune(b"apply_variant", 0)


@pytest.mark.parametrize("variant", [0, 1, 3, 4, 5, 6, 7, 8])
def test_diff_split_equals_per_range_diffs(variant):
    """gdsm_diff_split (one launch, G <= 8 streams, each with its own look-back chain) writes
    exactly the stream gdsm_diff writes for each range, in every diff geometry: ranges that are
    not unit multiples, empty ranges, a single page, uniform and clustered pages, and the
    largest-record pages; bad arguments are refused."""
    L = _lib.load()
    assert L.gdsm_tune(b"diff_variant", variant) == 0
    rng = np.random.default_rng(1200 + variant)
    try:
        n = 40000
        tw, cu = oracle.gen_pages(n, seed=12, mode=1, ppm=100000)
        tw[:300] = rng.integers(0, 256, (300, 4096), dtype=np.uint8)
        cu[:300] = tw[:300]
        cu[:300, ::2] ^= 0x5A  # 2048 runs per page: the largest records
        cu[300:20000] = tw[300:20000]
        w = rng.random((19700, 512)) < 0.01
        cu[300:20000].reshape(19700, 512, 8)[w] ^= 0x11
        with ga.Context(n) as c:
            c.upload("twin", tw)
            c.upload("current", cu)
            for G, bounds in [(1, [0, n]), (2, [0, 17, n]), (8, None), (5, [0, 0, 1, 1, 30000, n]),
                              (3, [100, 100, 100, 100])]:
                if bounds is None:
                    bounds = [0] + sorted(rng.integers(0, n, G - 1).tolist()) + [n]
                outs = [Runs(c, max(1, bounds[d + 1] - bounds[d]),
                             cap=max(64, 11000 * (bounds[d + 1] - bounds[d]))) for d in range(G)]
                c.diff_split(bounds, outs)
                for d in range(G):
                    a, b = bounds[d], bounds[d + 1]
                    got = outs[d].to_host()
                    assert outs[d].n == b - a
                    ro, data = oracle.diff_pages(tw[a:b], cu[a:b])
                    _eq_runs(got, ro, data)
                for o in outs:
                    o.free()
            one = [Runs(c, 10, cap=4096) for _ in range(2)]
            b = (C.c_uint64 * 3)(0, 10, 5)  # decreasing
            arr = (GdsmRuns * 2)(*[o.s for o in one])
            assert L.gdsm_diff_split(c.handle, b, 2, arr) == -22
            b = (C.c_uint64 * 3)(0, 5, n + 1)  # past the arenas
            assert L.gdsm_diff_split(c.handle, b, 2, arr) == -22
            arr = (GdsmRuns * 2)(one[0].s, one[0].s)  # one stream twice
            b = (C.c_uint64 * 3)(0, 5, 10)
            assert L.gdsm_diff_split(c.handle, b, 2, arr) == -22
            b = (C.c_uint64 * 10)(*range(10))
            assert L.gdsm_diff_split(c.handle, b, 9, (GdsmRuns * 9)()) == -22
    finally:
        L.gdsm_tune(b"diff_variant", 0)


@pytest.mark.parametrize("m", [700, 12, 1])
def test_diff_apply_ids_applies_at_other_indices(m):
    """gdsm_diff_apply_ids: list entry i (page ids[i] of TWIN / CURRENT) is applied to page
    target_ids[i] of REPLICA by the diff kernel itself, the stream being the same as gdsm_diff's;
    an out-of-range target id writes nothing and is reported by the next sync. m = 700 takes the
    grid with its separate id check; m <= 16 the one-workgroup release that guards both lists
    inside the kernel."""
    n = 3000
    rng = np.random.default_rng(77)
    twin, cur = oracle.gen_pages(n, seed=77, mode=1, ppm=100000)
    ids = rng.choice(n, m, replace=False).astype(np.uint32)
    tids = rng.permutation(n)[:m].astype(np.uint32)
    with ga.Context(n) as c:
        base = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
        c.upload("twin", twin)
        c.upload("current", cur)
        # the home copy starts as the twin's pages, moved to their target indices
        rep = base.copy()
        rep[tids] = twin[ids]
        c.upload("replica", rep)
        r = c.diff(c.ids(ids), apply_to="replica", target_ids=c.ids(tids))
        c.sync()
        h = r.to_host()
        ro, data = oracle.diff_pages(twin, cur, ids)
        assert np.array_equal(h.rec_off, ro) and np.array_equal(h.data[:int(ro[-1])], data)
        want = rep.copy()
        want[tids] = cur[ids]
        assert np.array_equal(c.download("replica"), want)
        bad = tids.copy()
        k = min(5, m - 1)
        bad[k] = n + 3
        c.upload("replica", rep)
        r2 = c.diff(c.ids(ids), apply_to="replica", target_ids=c.ids(bad))
        with pytest.raises(GdsmError) as ei:
            c.sync()
        assert ei.value.errno == 22
        h2 = r2.to_host()  # the stream is still gdsm_diff's
        assert np.array_equal(h2.rec_off, ro) and np.array_equal(h2.data[:int(ro[-1])], data)
        got = c.download("replica")
        keep = np.ones(m, bool)
        keep[k] = False
        want2 = rep.copy()
        want2[tids[keep]] = cur[ids[keep]]
        assert np.array_equal(got, want2)


def test_memcpy_batch():
    """gdsm_memcpy_batch: several copies in one launch, in 16-, 8-, 4- and 1-B words by the
    alignment of dst and src, with and without a remainder after the words, next to bytes that
    must stay untouched."""
    rng = np.random.default_rng(5)
    with ga.Context(8, arenas=()) as c:
        src = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
        d_src = c.buffer(src.nbytes).upload(src)
        d_dst = c.buffer(1 << 16).upload(np.zeros(1 << 16, np.uint8))
        copies = [(0, 0, 8000), (16384, 32, 4096), (30001, 7, 999), (40000, 50000, 3),
                  (8200, 56008, 8000), (20488, 24000, 4103), (45004, 52012, 1030),
                  (36000, 1, 3000), (28000, 4000, 1)]
        desc = np.array([[d_dst.ptr + d, d_src.ptr + s, b] for d, s, b in copies],
                        np.uint64).reshape(-1)
        d_desc = c.buffer(desc.nbytes).upload(desc)
        assert ga.gdsm.lib().gdsm_memcpy_batch(c.handle, d_desc.ptr, len(copies)) == 0
        c.sync()
        got = d_dst.download(np.uint8, 1 << 16)
        want = np.zeros(1 << 16, np.uint8)
        for d, s, b in copies:
            want[d:d + b] = src[s:s + b]
        assert np.array_equal(got, want)
        assert ga.gdsm.lib().gdsm_memcpy_batch(c.handle, None, 1) == -22
        assert ga.gdsm.lib().gdsm_memcpy_batch(c.handle, None, 0) == 0


@pytest.mark.parametrize("m", [1, 4, 5, 12, 16, 17, 31, 32, 33, 700, 3000])
@pytest.mark.parametrize("home", [False, True])
def test_release_retwin(m, home):
    """gdsm_release with GDSM_RELEASE_RETWIN: the stream is gdsm_diff's, the runs land at the
    home copy (target ids) when asked, and afterwards TWIN == CURRENT for exactly the listed
    pages (unlisted twins untouched), so a second release of the same pages is empty. m <= 4:
    the one-workgroup kernel, a page per wave, re-twins in place; up to 2048 pages the chained
    grid of one-page waves does too; 3000 pages (two-page units, whose late pages are read
    again): a guarded re-twin launch after the grid. The first three listed pages are dense
    (every byte changed: late records)."""
    n = 3000
    rng = np.random.default_rng(100 + m)
    twin, cur = oracle.gen_pages(n, seed=5, mode=1, ppm=100000)
    ids = rng.choice(n, m, replace=False).astype(np.uint32)
    cur[ids[:3]] ^= 0x5A
    tids = rng.permutation(n)[:m].astype(np.uint32)
    with ga.Context(n) as c:
        c.upload("twin", twin)
        c.upload("current", cur)
        base = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
        rep = base.copy()
        rep[tids] = twin[ids]
        c.upload("replica", rep)
        if home:
            r = c.release(c.ids(ids), apply_to="replica", target_ids=c.ids(tids))
        else:
            r = c.release(c.ids(ids))
        c.sync()
        h = r.to_host()
        ro, data = oracle.diff_pages(twin, cur, ids)
        assert np.array_equal(h.rec_off, ro) and np.array_equal(h.data[:int(ro[-1])], data)
        want_t = twin.copy()
        want_t[ids] = cur[ids]
        assert np.array_equal(c.download("twin"), want_t)
        want_r = rep.copy()
        if home:
            want_r[tids] = cur[ids]
        assert np.array_equal(c.download("replica"), want_r)
        r2 = c.release(c.ids(ids))
        c.sync()
        assert r2.total() == 0


def test_release_retwin_keeps_pages_that_did_not_fit():
    """A release whose stream overflows its capacity: the pages whose records were not stored
    keep their old TWIN (they stay dirty), the stored ones are re-twinned; a second release with a
    large enough stream ships exactly the rest (one-workgroup, chained and, inside a graph
    capture, zeroing-launch paths)."""
    for m, captured in ((4, False), (10, False), (24, False), (400, False), (10, True),
                        (24, True), (400, True)):
        n = 1000
        twin, cur = oracle.gen_pages(n, seed=9, mode=1, ppm=100000)
        ids = np.arange(0, 2 * m, 2, dtype=np.uint32)
        ro, data = oracle.diff_pages(twin, cur, ids)
        cap = int(ro[m // 2])  # the first half of the records fit
        with ga.Context(n) as c:
            c.upload("twin", twin)
            c.upload("current", cur)
            r = ga.Runs(c, m, cap=cap)
            d_ids = c.ids(ids)
            if captured:
                ga.gdsm.check(ga.gdsm.lib().gdsm_reserve(c.handle, m, 0), "gdsm_reserve")
                c.sync()
                c.capture_begin()
                c.release(d_ids, out=r)
                g = c.capture_end()
                g.launch(c)
                c.sync()
                g.destroy()
            else:
                c.release(d_ids, out=r)
            with pytest.raises(GdsmError):
                r.total()
            got = c.download("twin")
            stored = ro[1:] <= cap
            assert stored.sum() == m // 2
            want = twin.copy()
            want[ids[stored]] = cur[ids[stored]]
            assert np.array_equal(got, want), (m, captured)
            r2 = c.release(c.ids(ids), cap=m * 10244)
            c.sync()
            ro2, data2 = oracle.diff_pages(want, cur, ids)
            h2 = r2.to_host()
            assert np.array_equal(h2.rec_off, ro2) and np.array_equal(h2.data[:int(ro2[-1])], data2)
            assert np.array_equal(c.download("twin")[ids], cur[ids])


def test_chained_short_lists_across_launches_and_graphs():
    """Lists of 17-2048 pages take the chained one-launch diff (DiffChain: epoch-tagged look-back
    granules, ticket counters the previous launch zeroed, no zeroing launch). Forty launches in a
    row of varying length and kind (diff, diff_apply_ids, release), mixed with one-workgroup
    (<= 16 pages) and zeroing-launch (3000 pages) diffs, a graph of a short diff replayed between
    them (captured launches take the zeroing form), every chained form in turn (gdsm_tune
    "diff_chain": zeroing grid, one or four pages per workgroup, a page per four-wave workgroup,
    automatic), and a
    list with an out-of-range id (-EINVAL at the sync, the valid records still right): every
    stream equals the oracle's and every home-copy page is right."""
    n = 4096
    rng = np.random.default_rng(77)
    twin, cur = oracle.gen_pages(n, seed=21, mode=1, ppm=60000)
    cur[rng.choice(n, 40, replace=False)] ^= 0x33  # some dense pages (late records)
    L = ga.gdsm.lib()
    with ga.Context(n) as c:
        c.upload("twin", twin)
        c.upload("current", cur)
        c.upload("replica", twin)
        gids = rng.choice(n, 100, replace=False).astype(np.uint32)
        d_g = c.ids(gids)
        g_runs = Runs(c, 100, cap=100 * 10244)
        ga.gdsm.check(L.gdsm_reserve(c.handle, n, 0), "gdsm_reserve")  # no growth while capturing
        c.sync()
        c.capture_begin()
        c.diff(d_g.ptr, n=100, out=g_runs)
        graph = c.capture_end()
        g_ro, g_data = oracle.diff_pages(twin, cur, gids)
        sizes = [17, 2048, 1, 300, 3000, 64, 16, 1999, 33, 500] * 4
        try:
            for it, m in enumerate(sizes):
                # every chained form: the zeroing grid, one / four pages per workgroup, a page
                # per four-wave workgroup at every length, then automatic
                toggles = {20: 0, 24: 1, 28: 4, 32: 3, 37: 2}
                if it in toggles:
                    assert L.gdsm_tune(b"diff_chain", toggles[it]) == 0
                ids = rng.choice(n, m, replace=False).astype(np.uint32)
                kind = it % 3
                if kind == 0:
                    r = c.diff(c.ids(ids))
                elif kind == 1:
                    tids = rng.permutation(n)[:m].astype(np.uint32)
                    rep = twin.copy()
                    rep[tids] = twin[ids]  # the home copy holds the pages' last release
                    c.upload("replica", rep)
                    r = c.diff(c.ids(ids), apply_to="replica", target_ids=c.ids(tids))
                else:
                    r = c.release(c.ids(ids), retwin=False)
                c.sync()
                h = r.to_host()
                ro, data = oracle.diff_pages(twin, cur, ids)
                assert np.array_equal(h.rec_off, ro), (it, m)
                assert np.array_equal(h.data[:int(ro[-1])], data), (it, m)
                if kind == 1:
                    assert np.array_equal(c.download("replica")[tids], cur[ids]), (it, m)
                r.free()
                if it % 7 == 3:
                    graph.launch(c)
                    c.sync()
                    hg = g_runs.to_host()
                    assert np.array_equal(hg.rec_off, g_ro)
                    assert np.array_equal(hg.data[:int(g_ro[-1])], g_data)
            bad = rng.choice(n, 40, replace=False).astype(np.uint32)
            bad[[5, 30]] = [n, 0xFFFFFFFF]
            r = c.diff(c.ids(bad))
            with pytest.raises(GdsmError) as ei:
                c.sync()
            assert ei.value.errno == 22
            h = r.to_host()
            for i in range(40):
                if i not in (5, 30):
                    want = oracle.diff_pages(twin[bad[i]][None], cur[bad[i]][None])[1].tobytes()
                    assert h.record(i) == want, i
            ids = rng.choice(n, 700, replace=False).astype(np.uint32)
            r = c.diff(c.ids(ids))
            c.sync()
            ro, data = oracle.diff_pages(twin, cur, ids)
            h = r.to_host()
            assert np.array_equal(h.rec_off, ro) and np.array_equal(h.data[:int(ro[-1])], data)
        finally:
            L.gdsm_tune(b"diff_chain", 2)
            graph.destroy()


def test_chained_releases_from_concurrent_host_threads():
    """Three contexts, each driven by its own host thread (a context is driven by one thread at a
    time; gallocy's runtime is threaded), each issuing thirty chained releases of 5-2048 pages
    with home applies and re-twins back to back, CURRENT moving on between some of them: every
    context's streams, home copies and twins equal the oracle's."""
    import threading

    n = 2600
    twin0, cur0 = oracle.gen_pages(n, seed=41, mode=1, ppm=80000)
    errors = []

    def worker(k):
        try:
            rng = np.random.default_rng(900 + k)
            twin, cur, rep = twin0.copy(), cur0.copy(), twin0.copy()
            with ga.Context(n) as c:
                c.upload("twin", twin)
                c.upload("current", cur)
                c.upload("replica", rep)
                for it in range(30):
                    m = int(rng.choice([5, 40, 300, 513, 2048]))
                    ids = rng.choice(n, m, replace=False).astype(np.uint32)
                    r = c.release(c.ids(ids), apply_to="replica")
                    c.sync()
                    ro, data = oracle.diff_pages(twin, cur, ids)
                    h = r.to_host()
                    assert np.array_equal(h.rec_off, ro), (k, it)
                    assert np.array_equal(h.data[:int(ro[-1])], data), (k, it)
                    twin[ids] = cur[ids]
                    rep[ids] = cur[ids]
                    r.free()
                    if it % 10 == 9:
                        assert np.array_equal(c.download("twin"), twin), (k, it)
                        assert np.array_equal(c.download("replica"), rep), (k, it)
                    if it % 7 == 6:  # new writes: CURRENT moves on for some pages
                        cur[rng.choice(n, 64, replace=False)] ^= 0x11
                        c.upload("current", cur)
        except Exception as e:  # surfaced below
            errors.append((k, repr(e)))

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(3)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in threads)
    assert not errors, errors
