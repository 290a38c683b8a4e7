"""The config-5 trace generator: heap-layout model against the reference application heap itself
(tests/golden/ref_layout.npz) and SURVEY §8f's figures, and properties of the mmult access
trace."""
import numpy as np
import pytest

from gallocy_amd.trace import (AppHeap, HeapExhausted, MmultTrace, c_row_values, mmult_layout,
                               zone_image)
from oracle import oracle


@pytest.mark.parametrize("ndim", [4, 64, 1000, 1021])
def test_layout_matches_the_reference_heap(ndim, golden):
    """Every object of test_mmult (a, b, c: row pointers and rows; threads; args) sits at the zone
    offset the REFERENCE custom_malloc hands out (tests/golden/ref_layout.npz, made by
    oracle/_ref/ref_layout_driver, linked with libgallocy.cpp and internal.cpp in place)."""
    g = golden["ref_layout"]
    L = mmult_layout(ndim)
    assert [L.a_rp, L.b_rp, L.c_rp] == g[f"n{ndim}_rp"].tolist()
    rows = g[f"n{ndim}_rows"]
    assert np.array_equal(L.a_rows, rows[0]) and np.array_equal(L.b_rows, rows[1])
    assert np.array_equal(L.c_rows, rows[2])
    threads, args, end = g[f"n{ndim}_tail"].tolist()
    assert [L.threads, L.args] == [threads, args]
    assert L.args + 4 * 40 == end and L.zone_bytes >= end


def test_layout_survey_figures():
    """SURVEY §8f's quoted figures agree too (NDIM=4 relative offsets; NDIM=1000 row stride,
    matrix bases, ~6010 pages, last object at ~24.6 MB)."""
    L = mmult_layout(4)
    first = L.a_rp
    got = [L.a_rp, *L.a_rows.tolist(), L.b_rp, L.c_rp, L.threads, L.args]
    assert [g - first for g in got] == [0, 48, 96, 144, 192, 240, 480, 720, 768]
    assert L.n_pages == 5 and (L.args + 160) // 4096 == 0
    L = mmult_layout(1000)
    f = L.a_rp
    assert L.a_rows[1] - f == 16392 and L.b_rp - f == 8204016 and L.c_rp - f == 16408392
    assert 6000 <= L.n_pages <= 6020
    assert abs(L.zone_bytes - 24.6e6) < 0.1e6


def test_layout_limit_1021(golden):
    """NDIM 1021 is the largest that fits the 32 MiB zone; at 1022 the reference prints
    ---ENOMEM--- and aborts (source.h:23-24) after the same number of objects as the model
    allocates before HeapExhausted (fixture: the reference's exit status and object count)."""
    mmult_layout(1021)
    with pytest.raises(HeapExhausted):
        mmult_layout(1022)
    status, objects = golden["ref_layout"]["abort_1022"].tolist()
    assert status == -6  # SIGABRT
    h = AppHeap()
    done = 0
    with pytest.raises(HeapExhausted):
        for _ in range(3):
            h.malloc(8 * 1022)
            done += 1
            for _ in range(1022):
                h.malloc(8 * 1022)
                done += 1
    assert done == objects


def test_c_rows_and_image():
    L = mmult_layout(16)
    a = np.add.outer(np.arange(16.0), np.arange(16.0))
    c = a @ a
    for i in range(16):
        assert np.array_equal(c_row_values(L, i), c[i])
    z = zone_image(L).view("<f8")
    assert z[L.a_rows[3] // 8 + 5] == 8.0 and z[L.b_rows[2] // 8] == 2.0
    assert z[L.c_rows[1] // 8: L.c_rows[1] // 8 + 16].sum() == 0


@pytest.mark.parametrize("nodes", [1, 2, 4, 8])
def test_trace_shape_and_oracle_fold(nodes):
    L = mmult_layout(64)
    T = MmultTrace(L, nodes, seed=3)
    ev = T.all_events()
    pages = (ev >> 4).astype(np.int64)
    assert np.all(np.diff(pages) >= 0) and pages.max() < L.n_pages
    writes = ev[(ev & 1) == 1]
    # every row writes its c row pages exactly once, by its node
    n_w = sum(len(T.row_sets(i)[1]) for i in range(64))
    assert len(writes) == n_w
    st, fl = oracle.coh_init(L.n_pages, nodes)
    rc, tot = oracle.coherence(st, fl, ev, n_nodes=nodes)
    assert rc == 0
    if nodes == 1:
        assert tot["invalidations"] == 0 and tot["transfers"] == 0
    else:
        assert tot["transfers"] > 0


def test_round_batches_equal_whole_trace():
    """Folding the rounds one batch at a time == folding the whole trace as one batch."""
    L = mmult_layout(48)
    T = MmultTrace(L, 4, seed=1)
    st1, fl1 = oracle.coh_init(L.n_pages, 4)
    acc = np.zeros(10, np.int64)
    for r in range(T.rounds):
        rc, t = oracle.coherence(st1, fl1, T.round_events(r), n_nodes=4)
        assert rc == 0
        acc += [t["invalidations"], t["transfers"], *t["node_faults"]]
    st2, fl2 = oracle.coh_init(L.n_pages, 4)
    rc, t = oracle.coherence(st2, fl2, T.all_events(), n_nodes=4)
    assert np.array_equal(st1, st2) and np.array_equal(fl1, fl2)
    assert acc.tolist() == [t["invalidations"], t["transfers"], *t["node_faults"]]
