"""Shared test helpers: independent pure-numpy restatements used to cross-check the C oracle."""
from __future__ import annotations

import numpy as np


def np_runs(twin_page: np.ndarray, cur_page: np.ndarray):
    """Maximal runs of differing bytes, by numpy (independent of oracle/gdsm_oracle.c)."""
    d = (twin_page != cur_page).astype(np.int8)
    edges = np.diff(np.concatenate([[0], d, [0]]))
    starts = np.flatnonzero(edges == 1)
    ends = np.flatnonzero(edges == -1)
    return [(int(s), int(e - s)) for s, e in zip(starts, ends)]


def np_record(twin_page, cur_page) -> bytes:
    runs = np_runs(twin_page, cur_page)
    if not runs:
        return b""
    hdr = np.array([o | (ln << 16) for o, ln in runs], "<u4").tobytes()
    pay = b"".join(cur_page[o:o + ln].tobytes() for o, ln in runs)
    pay += b"\0" * ((-len(pay)) % 4)
    return np.array([len(runs)], "<u4").tobytes() + hdr + pay


def np_diff(twin, cur, ids=None):
    ids = range(twin.shape[0]) if ids is None else ids
    recs = [np_record(twin[p], cur[p]) for p in ids]
    off = np.zeros(len(recs) + 1, np.uint64)
    off[1:] = np.cumsum([len(r) for r in recs])
    return off, np.frombuffer(b"".join(recs), np.uint8)


C1_NUL, C1_DASH = 0xFE, 0xFD  # replacement bytes for 0x00 and '-' (0x2D)


def c1_remap(pages: np.ndarray) -> np.ndarray:
    """The byte remap of the config-1 windows (tests/golden/c1_windows.npz): 0x00 -> 0xFE,
    '-' -> 0xFD, others unchanged, so the reference diff(), which returns NUL-terminated
    alignments with '-' gaps (gallocy/utils/diff.h:9-11), can take the bytes. Applied to TWIN and
    CURRENT alike; the remapped pages are the inputs of every side of the comparison."""
    out = pages.copy()
    out[pages == 0] = C1_NUL
    out[pages == 0x2D] = C1_DASH
    return out


def c1_windows():
    """Remapped BASELINE config-1 pages (64 x 4 KiB, SPEC §6 seed 1, 1 % word writes):
    (twin', cur'), each (64, 4096) uint8; window w = bytes [1024 w, 1024 w + 1024) of the flat
    arrays."""
    from oracle import oracle
    t, c = oracle.gen_pages(64, seed=1, mode=0, ppm=10000)
    return c1_remap(t), c1_remap(c)


# Further page sets aligned window by window by the REFERENCE diff() (tests/golden/
# ref_windows.npz, tests/golden/make_golden.py): name -> how the pages are made.
#   cl     BASELINE config 3's workload (SPEC §6 CLUSTERED, 100 000 ppm, bench seed 2026): 64
#          pages from global page 5 000 000 of the 16M
#   dense  SPEC §6 UNIFORM at 400 000 ppm (40 % of the words rewritten, >= 30 % of the bytes)
#   edge   the SPEC edge pages of tests/golden/pages.npz (clean, all bytes, alternating bytes,
#          first / last byte, chunk and lane edges, tail run, sparse bytes, partial words)
REF_WINDOW_SETS = ("cl", "dense", "edge")
CL_FIRST = 5_000_000


def window_pages(name: str, golden=None):
    """(twin', cur') of a reference-window set, remapped as c1_remap; window w = bytes
    [1024 w, 1024 w + 1024) of the flat arrays."""
    from oracle import oracle
    if name == "cl":
        t, c = oracle.gen_pages(64, seed=2026, mode=1, ppm=100000, first_page=CL_FIRST)
    elif name == "dense":
        t, c = oracle.gen_pages(16, seed=2026, mode=0, ppm=400000)
    elif name == "edge":
        t, c = golden["pages"]["edge_twin"], golden["pages"]["edge_cur"]
    else:
        raise KeyError(name)
    return c1_remap(t), c1_remap(c)


# Windows of BASELINE's own bytes, no remap (tests/golden/raw_windows.npz): the north-star /
# config-2 generator (SPEC §6 UNIFORM, 10 000 ppm, bench seed 2026; config 2's 1M pages are the
# north star's first 1M), two ranges of 65 536 pages (the first and the last of the 16M). Every
# 1024-B window whose twin and current bytes hold neither 0x00 nor '-' (0x2D) is taken as it is:
# the reference diff() returns NUL-terminated alignments with '-' gaps (diff.h:9-11), so those
# two bytes are the only ones it cannot carry.
RAW_RANGES = ((0, 65536), ((16 << 20) - 65536, 65536))


def raw_range_pages(first: int, n: int):
    """(twin, current) of north-star pages [first, first + n): BASELINE's bytes, unremapped."""
    from oracle import oracle
    return oracle.gen_pages(n, seed=2026, mode=0, ppm=10000, first_page=first)


def raw_windows(t: np.ndarray, c: np.ndarray) -> np.ndarray:
    """Indices of the 1024-B windows of (t, c) that hold no 0x00 and no 0x2D byte on either side."""
    tw, cw = t.reshape(-1, 1024), c.reshape(-1, 1024)
    return np.flatnonzero(~((tw == 0) | (tw == 0x2D) | (cw == 0) | (cw == 0x2D)).any(axis=1))


def runs_positions(rec_off, data, n_pages: int) -> np.ndarray:
    """bool[n_pages * 4096]: True at every byte covered by a run of the stream (SPEC §3),
    record i describing page i."""
    out = np.zeros(n_pages * 4096, bool)
    w = np.frombuffer(np.ascontiguousarray(data).tobytes() + b"\0" * 4, "<u4")
    for i in range(n_pages):
        a, b = int(rec_off[i]), int(rec_off[i + 1])
        if a == b:
            continue
        nr = int(w[a // 4])
        for h in w[a // 4 + 1:a // 4 + 1 + nr]:
            o, ln = int(h & 0xFFFF), int(h >> 16)
            out[i * 4096 + o:i * 4096 + o + ln] = True
    return out


def mix64(z):
    M = (1 << 64) - 1
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M
    z ^= z >> 31
    return z


def hash3(s, a, b):
    M = (1 << 64) - 1
    return mix64((mix64(s ^ ((a * 0x9E3779B97F4A7C15) & M)) + b * 0xC2B2AE3D27D4EB4F + 0x165667B19E3779F9) & M)


def py_coherence(state, faults, events, n_pages):
    """Pure-Python sequential fold of docs/SPEC.md §5 (small cases only)."""
    tot = [0] * 10
    for e in events.tolist():
        p, node, wr = e >> 4, (e >> 1) & 7, e & 1
        s = int(state[p])
        cs, owner, st, dirty = s & 0xFF, (s >> 8) & 0xFF, (s >> 16) & 3, (s >> 18) & 1
        bit = 1 << node
        if not wr:
            if not cs & bit:
                faults[p] += 1
                tot[2 + node] += 1
                cs |= bit
                if st == 2:
                    st = 1
        else:
            dirty = 1
            if not (st == 2 and owner == node):
                faults[p] += 1
                tot[2 + node] += 1
                tot[0] += bin(cs & ~bit).count("1")
                tot[1] += owner != node
            owner, cs, st = node, bit, 2
        state[p] = cs | (owner << 8) | (st << 16) | (dirty << 18)
    return tot


from gallocy_amd.workloads import zipf_counts  # noqa: E402,F401
