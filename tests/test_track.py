"""Host write-fault capture (gdsm_track_*, gallocy_amd/csrc/gdsm_track.cpp): the protect ->
SIGSEGV -> twin -> writable step the reference describes but does not implement
(resources/NUTSHELL.md:52-69, resources/IMPLEMENTATION.md:246-249). CPU only: no GPU needed.
The oracle (tests only) checks that the captured twin and the current pages form a diff that
turns the twin into the current contents."""
import ctypes as C
import mmap
import subprocess
import sys
import threading
from pathlib import Path

import numpy as np
import pytest

import gallocy_amd as ga
from oracle import oracle

ROOT = Path(__file__).resolve().parents[1]


def _region(n_pages, seed):
    mm = mmap.mmap(-1, n_pages * 4096)
    v = np.frombuffer(mm, np.uint8)
    v[:] = np.random.default_rng(seed).integers(0, 256, v.size, dtype=np.uint8)
    return mm


def test_first_write_captures_twin_and_lists_page():
    mm = _region(64, 1)
    before = np.frombuffer(mm, np.uint8).reshape(64, 4096).copy()
    with ga.Tracker(mm) as t:
        pg = t.pages()
        assert t.dirty().size == 0 and t.faults() == 0
        pg[17, 100:108] = 7
        pg[3, 0] ^= 0xFF
        pg[40, 4095] ^= 1
        pg[17, 200] = 9           # same page again: no new fault
        assert t.dirty().tolist() == [3, 17, 40]
        assert t.faults() == 3
        tw = t.twin()
        for p in (3, 17, 40):
            assert np.array_equal(tw[p], before[p])
        cur = pg.copy()
        assert np.array_equal(cur[[0, 1, 2, 4, 63]], before[[0, 1, 2, 4, 63]])
        # the captured interval is a diff that turns the twins into the current pages
        ids = t.dirty()
        ro, data = oracle.diff_pages(tw[ids].copy(), cur[ids])
        rep = tw[ids].copy()
        assert oracle.apply(rep, ro, data) == 0
        assert np.array_equal(rep, cur[ids])


def test_rearm_starts_a_new_interval():
    mm = _region(16, 2)
    with ga.Tracker(mm) as t:
        pg = t.pages()
        pg[5, :] = 1
        pg[6, :] = 2
        assert t.dirty().tolist() == [5, 6]
        t.rearm()
        assert t.dirty().size == 0
        snap = pg[6].copy()
        pg[6, 10] = 99
        assert t.dirty().tolist() == [6]
        assert np.array_equal(t.twin()[6], snap)   # twin = contents at the release point
        assert t.faults() == 3


def test_concurrent_first_writes_from_threads():
    n = 256
    mm = _region(n, 3)
    with ga.Tracker(mm) as t:
        base = t.base
        rng = np.random.default_rng(4)
        pages = [rng.choice(n, 40, replace=False) for _ in range(8)]

        def writer(ps, val):
            for p in ps:  # ctypes calls run without the GIL: real concurrent faults
                C.memset(base + int(p) * 4096 + int(val) * 8, val, 8)

        th = [threading.Thread(target=writer, args=(pages[i], i + 1)) for i in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        want = sorted(set(np.concatenate(pages).tolist()))
        assert t.dirty().tolist() == want
        assert t.faults() == len(want)
        v = t.pages()
        for i, ps in enumerate(pages):
            for p in ps:
                assert np.all(v[p, (i + 1) * 8:(i + 2) * 8] == i + 1)


def test_end_restores_write_access():
    mm = _region(4, 5)
    t = ga.Tracker(mm)
    t.close()
    v = np.frombuffer(mm, np.uint8)
    v[:] = 3  # would fault forever if still protected and untracked
    assert v.sum() == 3 * v.size


def test_unrelated_segfault_still_terminates():
    """A fault outside every tracked region goes to the previous handler (default: the process
    dies of SIGSEGV), it is not swallowed."""
    code = ("import mmap, ctypes, gallocy_amd as ga\n"
            "mm = mmap.mmap(-1, 8 * 4096)\n"
            "t = ga.Tracker(mm)\n"
            "t.pages()[1, 0] = 1\n"
            "print('tracked ok', flush=True)\n"
            "ctypes.string_at(0)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert "tracked ok" in r.stdout
    assert r.returncode == -11, (r.returncode, r.stderr[-500:])


def test_rejects_unaligned_region():
    L = ga.gdsm.lib()
    buf = (C.c_uint8 * (3 * 4096))()
    addr = C.addressof(buf)
    h = C.c_void_p()
    if addr % 4096 == 0:
        addr += 1
    assert L.gdsm_track_begin(C.byref(h), addr, 1) == -22


def test_non_write_fault_in_tracked_page_is_not_swallowed():
    """Only write faults belong to a tracker: an instruction fetch from a tracked (PROT_READ,
    not executable) page goes to the previous handler, so the process dies of SIGSEGV instead of
    retrying the fetch forever."""
    code = ("import mmap, ctypes, gallocy_amd as ga\n"
            "mm = mmap.mmap(-1, 4 * 4096)\n"
            "t = ga.Tracker(mm)\n"
            "t.pages()[2, 0] = 1\n"
            "print('tracked ok', flush=True)\n"
            "fn = ctypes.CFUNCTYPE(None)(t.base + 4096)\n"
            "fn()\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert "tracked ok" in r.stdout
    assert r.returncode == -11, (r.returncode, r.stderr[-500:])
