"""gdsm_rounds' page-table side on its own (docs/SPEC.md §5, rounds folded in order): random
multi-round batches against the C oracle's sequential fold, round by round (page-table words,
per-page faults, every round's totals row). Both forms of the launch: workgroups that keep
slices of the page table in LDS (GDSM_ROUNDS_LDS=1, the default wherever it fits: up to 16 slices
of <= 8192 pages, rounds of <= 16384 events, <= 2048 rounds) and the persistent grid
(GDSM_ROUNDS_LDS=0, the form larger tables and rounds take). The data
side gets empty rounds (no pages), so only the fold runs."""
import ctypes as C

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd.gdsm import GdsmError, check, lib
from oracle import oracle
from tests.helpers import zipf_counts

pytestmark = pytest.mark.gpu

LDS_PAGES, LDS_EVENTS = 8192, 16384


def _round_events(n_pages, n_ev, n_nodes, seed, write_pct):
    counts = zipf_counts(n_pages, n_ev, s=0.9, seed=seed) if n_ev else np.zeros(n_pages, np.int64)
    return oracle.gen_events(counts, seed=seed + 1, n_nodes=n_nodes, write_pct=write_pct)


def _run_rounds(n_pages, n_nodes, rounds, st0=None, fl0=None):
    """gdsm_rounds over `rounds` (host event arrays, one per round) with empty page-data rounds;
    returns (state, faults, totals[R, 10])."""
    R = len(rounds)
    with ga.Context(4) as data, ga.Context(n_pages, arenas=()) as pt:
        pt.coh_init(n_nodes)
        if st0 is not None:
            pt.coh_upload(st0, fl0)
        ev = np.concatenate(rounds).astype(np.uint64) if R else np.zeros(0, np.uint64)
        ev_off = np.zeros(R + 1, np.int64)
        ev_off[1:] = np.cumsum([len(r) for r in rounds])
        d_ev = pt.buffer(8 * max(1, len(ev)))
        if len(ev):
            d_ev.upload(ev)
        d_tot = pt.buffer(80 * max(1, R))
        d_ids = data.buffer(16)
        d_desc = data.buffer(64)
        zeros = np.zeros(R + 1, np.int64)
        runs = ga.Runs(data, 1, cap=1 << 16)
        check(lib().gdsm_rounds(data.handle, pt.handle, R, d_ev.ptr, ev_off.ctypes.data,
                                d_tot.ptr, d_ids.ptr, d_ids.ptr, zeros.ctypes.data, d_desc.ptr,
                                zeros.ctypes.data, C.byref(runs.s)), "gdsm_rounds")
        data.sync()
        pt.sync()
        tot = d_tot.download(np.uint64, 10 * R).reshape(R, 10) if R else np.zeros((0, 10))
        st, fl = pt.coh_download()
        return st, fl, tot


def _oracle_rounds(n_pages, n_nodes, rounds, st0=None, fl0=None):
    st, fl = oracle.coh_init(n_pages, n_nodes)
    if st0 is not None:
        st[:], fl[:] = st0, fl0
    tots = []
    for ev in rounds:
        rc, t = oracle.coherence(st, fl, ev, n_nodes=n_nodes)
        assert rc == 0
        tots.append([t["invalidations"], t["transfers"], *t["node_faults"]])
    return st, fl, np.array(tots, np.uint64).reshape(len(rounds), 10)


@pytest.mark.parametrize("lds", ["1", "0", "1-wg3"])
@pytest.mark.parametrize("n_pages,n_nodes,sizes", [
    (6011, 8, [2012, 2012, 0, 16096, 1, 5000]),   # config 5's table; an empty and a 1-event round
    (LDS_PAGES, 5, [LDS_EVENTS, 3, LDS_EVENTS]),   # both LDS limits at once
    (100, 2, [900, 1200, 64, 7]),                 # long page runs across thread chunks
])
def test_rounds_fold_matches_oracle(n_pages, n_nodes, sizes, lds, monkeypatch):
    """lds "1-wg3": the LDS form on three workgroups (GDSM_ROUNDS_LDS_WG=3), each folding the
    events of its third of the table."""
    monkeypatch.setenv("GDSM_ROUNDS_LDS", lds[0])
    if lds.endswith("wg3"):
        monkeypatch.setenv("GDSM_ROUNDS_LDS_WG", "3")
    rounds = [_round_events(n_pages, n, n_nodes, seed=40 + i, write_pct=(10, 35, 70)[i % 3])
              for i, n in enumerate(sizes)]
    got = _run_rounds(n_pages, n_nodes, rounds)
    want = _oracle_rounds(n_pages, n_nodes, rounds)
    for g, w in zip(got, want):
        assert np.array_equal(g, w), np.argwhere(g != w)[:10]


@pytest.mark.parametrize("lds", ["1", "0"])
def test_rounds_fold_arbitrary_table_states(lds, monkeypatch):
    """Uploaded words in any state (INVALID, the unused state 3, owners >= 8, dirty, fault counts
    near 2^32, which wrap)."""
    monkeypatch.setenv("GDSM_ROUNDS_LDS", lds)
    n = 3000
    rng = np.random.default_rng(5)
    st0 = rng.integers(0, 1 << 19, n).astype(np.uint32)
    fl0 = rng.integers((1 << 32) - 40, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    rounds = [_round_events(n, 4000, 8, seed=70 + i, write_pct=30) for i in range(4)]
    got = _run_rounds(n, 8, rounds, st0, fl0)
    want = _oracle_rounds(n, 8, rounds, st0, fl0)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)


def test_rounds_fold_past_the_lds_limits_takes_the_grid():
    """A round of more than 16384 events (or a table of more than 8192 pages) folds on the
    persistent grid by default, and GDSM_ROUNDS_LDS=1 refuses it."""
    n = LDS_PAGES + 1
    rounds = [_round_events(n, LDS_EVENTS + 1, 8, seed=90, write_pct=25)]
    got = _run_rounds(n, 8, rounds)
    want = _oracle_rounds(n, 8, rounds)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)


def test_rounds_fold_lds_forced_past_its_limits_is_refused(monkeypatch):
    monkeypatch.setenv("GDSM_ROUNDS_LDS", "1")
    with pytest.raises(GdsmError) as ei:
        _run_rounds(16, 8, [_round_events(16, LDS_EVENTS + 1, 8, seed=3, write_pct=25)])
    assert ei.value.errno == 22


@pytest.mark.parametrize("lds", ["1", "0"])
@pytest.mark.parametrize("bad", ["unsorted", "page", "node", "high"])
def test_rounds_fold_rejects_bad_events(bad, lds, monkeypatch):
    """An unsorted round, a page outside the table, a node >= n_nodes or a set high dword fails
    the call (EINVAL at the sync), as gdsm_coherence_batch does."""
    monkeypatch.setenv("GDSM_ROUNDS_LDS", lds)
    good = _round_events(500, 3000, 4, seed=11, write_pct=25)
    ev = good.copy()
    if bad == "unsorted":
        ev[0], ev[-1] = ev[-1], ev[0]  # (the largest page first)
    elif bad == "page":
        ev[-1] = np.uint64(600 << 4)
    elif bad == "node":
        ev[1000] = (ev[1000] & ~np.uint64(14)) | np.uint64(6 << 1)
    else:
        ev[2000] |= np.uint64(1 << 40)
    with pytest.raises(GdsmError) as ei:
        _run_rounds(500, 4, [good, ev, good])
    assert ei.value.errno == 22


@pytest.mark.parametrize("lds", ["auto", "1"])
def test_rounds_fold_more_rounds_than_lds_offsets(lds, monkeypatch):
    """2049 rounds: more event offsets than the LDS form stages (2048), so the default takes the
    persistent grid and GDSM_ROUNDS_LDS=1 refuses the call; 2048 rounds still fold in LDS."""
    if lds == "1":
        monkeypatch.setenv("GDSM_ROUNDS_LDS", "1")
    rounds = [_round_events(64, 3, 4, seed=500 + i, write_pct=40) for i in range(2049)]
    if lds == "1":
        with pytest.raises(GdsmError) as ei:
            _run_rounds(64, 4, rounds)
        assert ei.value.errno == 22
        rounds = rounds[:2048]
    got = _run_rounds(64, 4, rounds)
    want = _oracle_rounds(64, 4, rounds)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("wg", ["", "3"])
def test_rounds_fold_lds_slices_a_larger_table(wg, monkeypatch):
    """A table of 20000 pages (more than one workgroup's 8192) in the LDS form: three or four
    slices, Zipf rounds whose runs cross the slices' edges, and 8192-page multiples."""
    monkeypatch.setenv("GDSM_ROUNDS_LDS", "1")
    if wg:
        monkeypatch.setenv("GDSM_ROUNDS_LDS_WG", wg)
    n = 20000
    rounds = [_round_events(n, m, 8, seed=600 + i, write_pct=30)
              for i, m in enumerate([16000, 9000, 1, 12000])]
    got = _run_rounds(n, 8, rounds)
    want = _oracle_rounds(n, 8, rounds)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("bad", ["unsorted", "across"])
def test_rounds_fold_lds_slices_reject_unsorted_rounds(bad, monkeypatch):
    """Unsorted rounds on three slices: a swap inside one slice, and one that moves an event into
    another slice's index range."""
    monkeypatch.setenv("GDSM_ROUNDS_LDS", "1")
    monkeypatch.setenv("GDSM_ROUNDS_LDS_WG", "3")
    good = _round_events(600, 6000, 4, seed=21, write_pct=25)
    ev = good.copy()
    if bad == "unsorted":
        pg = ev >> np.uint64(4)
        i = int(np.flatnonzero(pg[1:] != pg[:-1])[len(pg) // 4 // 100])  # a page change inside
        ev[i], ev[i + 1] = ev[i + 1], ev[i]                              # the first slices
    else:
        ev[0], ev[-1] = ev[-1], ev[0]
    with pytest.raises(GdsmError) as ei:
        _run_rounds(600, 4, [good, ev])
    assert ei.value.errno == 22
