"""Pins the C oracle (oracle/gdsm_oracle.c) before it is trusted as the GPU parity checker.

NW diff: against the reference's own golden strings (test/test_diff.cpp:13-16, 29-31), the
SURVEY §8c KATs, and vectors produced by the reference itself (tests/golden/nw_ref.npz, made by
oracle/_ref from gallocy/utils/diff.cpp), plus live reference runs when oracle/_ref exists.
Page diff / apply / coherence: parity unpinned by the reference (no implementation there);
checked against independent numpy / pure-Python restatements and the SPEC bridge to NW.
"""
import numpy as np
import pytest

from oracle import oracle
from tests.helpers import (RAW_RANGES, REF_WINDOW_SETS, c1_windows, raw_range_pages, raw_windows, hash3, np_diff, np_runs, py_coherence,
                           runs_positions, window_pages, zipf_counts)


# ---------------------------------------------------------------- NW (reference diff())
def test_nw_reference_test_diff_goldens():
    # test/test_diff.cpp:13-16 and :24-31
    assert oracle.nw_diff(b"GGAATGG", b"ATG") == (b"GGAATGG", b"---AT-G")
    assert oracle.nw_diff(b"FOO BOP BOOP", b"FOOO BOOP BOP") == (b"F-OO B-OP BOOP", b"FOOO BOOP B-OP")


@pytest.mark.parametrize("a,b,o1,o2", [
    (b"", b"", b"", b""), (b"", b"ABC", b"---", b"ABC"), (b"ABC", b"", b"ABC", b"---"),
    (b"AB", b"BA", b"AB", b"BA"), (b"ABCD", b"BCDA", b"ABCD-", b"-BCDA"),
    (b"AAAA", b"AA", b"AAAA", b"--AA"), (b"AA", b"AAAA", b"--AA", b"AAAA"),
    (b"ACGT", b"TGCA", b"ACGT", b"TGCA"), (b"HELLO", b"YELLOW", b"HELLO-", b"YELLOW"),
    (b"0123456789", b"0123X56789", b"0123456789", b"0123X56789")])
def test_nw_survey_kats(a, b, o1, o2):
    assert oracle.nw_diff(a, b) == (o1, o2)


def _nw_golden_cases(golden):
    g = golden["nw_ref"]
    blob = g["blob"].tobytes()
    i = 0
    for n, m, L in g["lens"]:
        a, b = blob[i:i + n], blob[i + n:i + n + m]
        i += n + m
        o1, o2 = blob[i:i + L], blob[i + L:i + 2 * L]
        i += 2 * L
        yield a, b, o1, o2


def test_nw_reference_vectors(golden):
    cases = list(_nw_golden_cases(golden))
    assert len(cases) >= 30
    for a, b, o1, o2 in cases:
        assert oracle.nw_diff(a, b) == (o1, o2), (len(a), len(b))


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (no reference tree)")
def test_nw_live_reference_random():
    rng = np.random.default_rng(99)
    cases = []
    for _ in range(40):
        n, m = int(rng.integers(0, 200)), int(rng.integers(0, 200))
        a = bytes(rng.integers(1, 4, n, dtype=np.uint8) + 64)  # small alphabet: many ties
        b = bytes(rng.integers(1, 4, m, dtype=np.uint8) + 64)
        cases.append((a, b))
    for (a, b), ref in zip(cases, oracle.ref_nw_batch(cases)):
        assert oracle.nw_diff(a, b) == ref


def test_nw_bridge_to_page_runs(golden):
    """for equal-length substitution-only inputs whose NW alignment is gap-free,
    {i : out1[i] != out2[i]} is exactly the union of the page-diff runs."""
    checked = 0
    for a, b, o1, o2 in _nw_golden_cases(golden):
        if len(a) != len(b) or len(o1) != len(a) or b"-" in o1 + o2:
            continue
        ta, tb = np.frombuffer(a, np.uint8), np.frombuffer(b, np.uint8)
        nw_pos = {i for i in range(len(o1)) if o1[i] != o2[i]}
        run_pos = {o + k for o, ln in np_runs(ta, tb) for k in range(ln)}
        assert nw_pos == run_pos
        checked += 1
    assert checked >= 5


# ---------------------------------------------------------------- synthetic inputs
def test_gen_matches_spec_hash():
    t, c = oracle.gen_pages(3, seed=42, mode=0, ppm=10000, first_page=100)
    for i in range(3):
        for w in (0, 1, 255, 511):
            v = hash3(42 ^ 0xDA7A, 100 + i, w)
            assert int(t[i, w * 8:w * 8 + 8].view("<u8")[0]) == v
            changed = hash3(42 ^ 0x5E1EC7ED, 100 + i, w) % 1000000 < 10000
            x = hash3(42 ^ 0x0F11E5, 100 + i, w) if changed else 0
            x = 1 if (changed and x == 0) else x
            assert int(c[i, w * 8:w * 8 + 8].view("<u8")[0]) == v ^ x


def test_gen_density():
    t, c = oracle.gen_pages(256, seed=5, mode=0, ppm=10000)
    words = (t.view("<u8") != c.view("<u8")).mean()
    assert 0.008 < words < 0.012
    t, c = oracle.gen_pages(256, seed=5, mode=1, ppm=100000)
    cl = (t.view("<u8").reshape(256, 64, 8) != c.view("<u8").reshape(256, 64, 8))
    assert (cl.all(axis=2) == cl.any(axis=2)).all()  # whole 64-B clusters
    assert 0.08 < cl.any(axis=2).mean() < 0.12


# ---------------------------------------------------------------- page diff / apply
def test_diff_edge_pages_vs_numpy(golden):
    g = golden["pages"]
    ro, data = oracle.diff_pages(g["edge_twin"], g["edge_cur"])
    ro2, data2 = np_diff(g["edge_twin"], g["edge_cur"])
    assert np.array_equal(ro, ro2) and np.array_equal(data, data2)
    assert np.array_equal(ro, g["edge_rec_off"]) and np.array_equal(data, g["edge_data"])
    sizes = np.diff(ro)
    assert sizes[0] == 0                       # clean page: empty record
    assert sizes[1] == 4 + 4 + 4096            # one full-page run
    assert sizes[2] == 4 + 4 * 2048 + 2048     # alternating bytes: the largest record


def test_diff_config1_golden(golden):
    """BASELINE config 1: 64 x 4 KiB pages, 1 % random word writes, seed 1 (CPU)."""
    g = golden["pages"]
    t, c = oracle.gen_pages(64, seed=1, mode=0, ppm=10000)
    ro, data = oracle.diff_pages(t, c)
    assert np.array_equal(ro, g["c1_rec_off"]) and np.array_equal(data, g["c1_data"])
    ro2, data2 = np_diff(t, c)
    assert np.array_equal(ro, ro2) and np.array_equal(data, data2)
    rep = t.copy()
    assert oracle.apply(rep, ro, data) == 0
    assert np.array_equal(rep, c)


def test_diff_ids_and_capacity():
    t, c = oracle.gen_pages(32, seed=9, mode=1, ppm=100000)
    ids = np.array([5, 3, 31, 0, 3], np.uint32)
    ro, data = oracle.diff_pages(t, c, ids=ids)
    ro2, data2 = np_diff(t, c, ids.tolist())
    assert np.array_equal(ro, ro2) and np.array_equal(data, data2)
    ro3, data3 = oracle.diff_pages(t, c, ids=ids, cap=int(ro[2]))
    assert np.array_equal(ro3, ro)            # rec_off is complete even past capacity
    assert np.array_equal(data3, data[:int(ro[2])])


def test_apply_idempotent_and_rejects_malformed():
    t, c = oracle.gen_pages(8, seed=2, mode=0, ppm=50000)
    ro, data = oracle.diff_pages(t, c)
    rep = t.copy()
    assert oracle.apply(rep, ro, data) == 0
    assert oracle.apply(rep, ro, data) == 0
    assert np.array_equal(rep, c)
    bad = data.copy()
    i = int(np.flatnonzero(np.diff(ro))[0])
    bad[int(ro[i]):int(ro[i]) + 4] = np.frombuffer(np.uint32(4000).tobytes(), np.uint8)
    assert oracle.apply(t.copy(), ro, bad) == -22


# ---------------------------------------------------------------- coherence
def test_coherence_vs_python_fold(golden):
    g = golden["coherence"]
    st, fl = oracle.coh_init(64, 8)
    rc, tot = oracle.coherence(st, fl, g["events"])
    assert rc == 0
    assert np.array_equal(st, g["state"]) and np.array_equal(fl, g["faults"])
    assert [tot["invalidations"], tot["transfers"], *tot["node_faults"]] == g["totals"].tolist()
    st2, fl2 = oracle.coh_init(64, 8)
    tot2 = py_coherence(st2, fl2, g["events"], 64)
    assert np.array_equal(st, st2) and np.array_equal(fl, fl2)
    assert tot2 == g["totals"].tolist()


def test_coherence_initial_state_and_rules():
    st, fl = oracle.coh_init(16, 8)
    assert ((st >> 8) & 0xFF).tolist() == [p // 2 for p in range(16)]   # home = p / ceil(16/8)
    ev = np.array([(3 << 4) | (5 << 1) | 0,   # read by 5: fault, SHARED
                   (3 << 4) | (5 << 1) | 0,   # read again: nothing
                   (3 << 4) | (5 << 1) | 1,   # write by 5: fault, invalidates home 1, transfer
                   (3 << 4) | (5 << 1) | 1],  # write by owner in EXCLUSIVE: no fault
                  np.uint64)
    rc, tot = oracle.coherence(st, fl, ev)
    assert rc == 0
    assert tot["invalidations"] == 1 and tot["transfers"] == 1 and tot["node_faults"][5] == 2
    assert st[3] == (1 << 5) | (5 << 8) | (2 << 16) | (1 << 18) and fl[3] == 2


def test_coherence_rejects_unsorted():
    st, fl = oracle.coh_init(8, 8)
    rc, _ = oracle.coherence(st, fl, np.array([5 << 4, 2 << 4], np.uint64))
    assert rc == -22


def test_gen_events_and_zipf_counts():
    counts = zipf_counts(1000, 20000, s=0.8, seed=1)
    assert counts.sum() == 20000 and counts.max() > 10 * counts.mean()
    ev = oracle.gen_events(counts, seed=3)
    pages = ev >> 4
    assert np.all(np.diff(pages.astype(np.int64)) >= 0)
    assert abs((ev & 1).mean() - 0.2) < 0.02


# ---------------------------------------------------------------- config 1 pinned by the reference
def test_c1_windows_pinned_by_reference_diff(golden):
    """BASELINE config 1 cut into 256 windows of 1024 B (test/test_diff.cpp:38-57 shape) and run
    through the REFERENCE diff() (gallocy/utils/diff.cpp:73-167, oracle/_ref; fixture made by
    tests/golden/make_golden.py). Where its alignment is gap-free (all 256 windows), out1 / out2
    are the window's twin / current bytes and {i : out1[i] != out2[i]} must equal the positions
    the oracle's page-diff runs cover; applying the oracle stream to the twin gives out2."""
    import zlib
    g = golden["c1_windows"]
    t, c = c1_windows()
    assert g["gapfree"].all() and (g["L"] == 1024).all()
    tw, cw = t.reshape(-1, 1024), c.reshape(-1, 1024)
    for i in range(len(tw)):
        assert [zlib.crc32(tw[i].tobytes()), zlib.crc32(cw[i].tobytes())] == g["crc"][i].tolist()
    ro, data = oracle.diff_pages(t, c)
    pos = runs_positions(ro, data, 64).reshape(-1, 1024)
    ref = np.unpackbits(g["mask"], axis=1).astype(bool)
    assert ref.any(axis=1).sum() > 150  # 1 - 0.99^128 = 72 % of windows hold a write
    assert np.array_equal(pos, ref)
    rep = t.copy()
    assert oracle.apply(rep, ro, data) == 0
    assert np.array_equal(rep, c)
    # the oracle's own NW restatement agrees with the reference on a sample of the windows
    for i in range(0, 256, 32):
        o1, o2 = oracle.nw_diff(tw[i].tobytes(), cw[i].tobytes())
        assert [zlib.crc32(o1), zlib.crc32(o2)] == g["crc"][i].tolist()


@pytest.mark.parametrize("name", REF_WINDOW_SETS)
def test_ref_windows_pinned_by_reference_diff(name, golden):
    """More page sets pinned to the REFERENCE diff() (gallocy/utils/diff.cpp:73-167 through
    oracle/_ref; fixture tests/golden/ref_windows.npz): config 3's clustered pages, a dense set
    (>= 30 % of the bytes changed) and the SPEC edge pages, remapped and cut into 1024-B windows
    (test/test_diff.cpp:38-57 shape). Every gap-free window's {i : out1[i] != out2[i]} equals the
    positions the oracle's runs cover, and its out1 / out2 are the window's twin / current bytes
    (crc32); the oracle's apply gives out2. Windows whose reference alignment has gaps (it slid
    a changed run along a shifted match) are pinned through the oracle's NW restatement: same
    length and crc32 as the reference's."""
    import zlib
    pre = name + "_"
    L, crc, gapfree, mask = (golden["ref_windows"][pre + k] for k in ("L", "crc", "gapfree", "mask"))
    t, c = window_pages(name, golden)
    n = t.shape[0]
    tw, cw = t.reshape(-1, 1024), c.reshape(-1, 1024)
    assert len(L) == len(tw) and gapfree.sum() >= len(tw) - 8
    if name == "dense":
        assert (t != c).mean() >= 0.30
    ro, data = oracle.diff_pages(t, c)
    pos = runs_positions(ro, data, n).reshape(-1, 1024)
    ref = np.unpackbits(mask, axis=1).astype(bool)
    for i in np.flatnonzero(gapfree):
        assert [zlib.crc32(tw[i].tobytes()), zlib.crc32(cw[i].tobytes())] == crc[i].tolist(), i
        assert np.array_equal(pos[i], ref[i]), i
    assert ref[gapfree].any(axis=1).sum() > (4 if name == "edge" else len(tw) // 2)
    rep = t.copy()
    assert oracle.apply(rep, ro, data) == 0
    assert np.array_equal(rep, c)
    for i in np.flatnonzero(~gapfree):
        o1, o2 = oracle.nw_diff(tw[i].tobytes(), cw[i].tobytes())
        assert len(o1) == L[i] and [zlib.crc32(o1), zlib.crc32(o2)] == crc[i].tolist(), i


@pytest.mark.parametrize("r", [0, 1])
def test_raw_windows_pinned_by_reference_diff(r, golden):
    """BASELINE's own bytes, no remap (tests/helpers.py:RAW_RANGES; fixture
    tests/golden/raw_windows.npz from the reference diff(), gallocy/utils/diff.cpp:73-167, run
    through oracle/_ref, test/test_diff.cpp:38-57 window shape): the north-star generator's pages
    at seed 2026 in the first and the last 65 536 of the 16M. The windows are the ones holding
    no NUL and no '-' byte, which the selection rule reproduces; every one is gap-free, so
    {i : out1[i] != out2[i]} must equal the positions the oracle's runs cover, out1 / out2 the
    window's twin / current bytes (crc32), and the oracle's apply must give out2."""
    import zlib
    g = golden["raw_windows"]
    pre = f"r{r}_"
    first, n = (int(x) for x in g[pre + "range"])
    assert (first, n) == RAW_RANGES[r]
    win, crc, gapfree, mask = (g[pre + k] for k in ("win", "crc", "gapfree", "mask"))
    t, c = raw_range_pages(first, n)
    assert np.array_equal(raw_windows(t, c), win)
    assert gapfree.all() and len(win) >= 60
    ref = np.unpackbits(mask, axis=1).astype(bool)
    assert ref.any(axis=1).sum() >= 50  # most windows hold changed words
    pages = np.unique(win // 4)
    tp, cp = t[pages], c[pages]
    ro, data = oracle.diff_pages(tp, cp)
    pos = runs_positions(ro, data, len(pages)).reshape(len(pages), 4, 1024)
    tw, cw = t.reshape(-1, 1024), c.reshape(-1, 1024)
    where = {int(p): i for i, p in enumerate(pages)}
    for j, w in enumerate(win):
        assert [zlib.crc32(tw[w].tobytes()), zlib.crc32(cw[w].tobytes())] == crc[j].tolist(), w
        assert np.array_equal(pos[where[int(w) // 4], int(w) % 4], ref[j]), w
    rep = tp.copy()
    assert oracle.apply(rep, ro, data) == 0
    assert np.array_equal(rep, cp)


def test_coherence_rejects_node_outside_the_table():
    """A page table initialised for n nodes rejects an event naming node >= n (include/gdsm.h
    gdsm_coherence_batch: -EINVAL)."""
    st, fl = oracle.coh_init(8, 3)
    rc, _ = oracle.coherence(st, fl, np.array([(1 << 4) | (3 << 1)], np.uint64), n_nodes=3)
    assert rc == -22
    st, fl = oracle.coh_init(8, 3)
    rc, _ = oracle.coherence(st, fl, np.array([(1 << 4) | (2 << 1)], np.uint64), n_nodes=3)
    assert rc == 0


def test_check_stream_finds_the_first_bad_record():
    """oracle.check_stream (the whole-stream checker of the full-size GPU tests) accepts the
    oracle's own stream of a workload slice and names the page of the first corrupted record."""
    n = 5000
    for mode, ppm in ((0, 10000), (1, 100000)):
        tw, cu = oracle.gen_pages(n, seed=3, mode=mode, ppm=ppm, first_page=777)
        ro, data = oracle.diff_pages(tw, cu)
        assert oracle.check_stream(ro, data, 777, n, 3, mode, ppm, threads=4) == -1
        assert oracle.check_stream(ro, data, 778, n, 3, mode, ppm, threads=4) != -1
        bad = data.copy()
        p = 3210 + int(np.flatnonzero(np.diff(ro[3210:].astype(np.int64)) > 8)[0])
        bad[int(ro[p]) + 5] ^= 0x40
        assert oracle.check_stream(ro, bad, 777, n, 3, mode, ppm, threads=4) == p
