"""BASELINE config 5: the `test_mmult` distributed matrix-multiply access pattern, replayed
through the engine (coherence + diff propagation).

1. `AppHeap` reproduces the address assignment of the reference application heap
   `ApplicationHeapType` (gallocy/include/gallocy/heaplayers/application.h:20-29) on a fresh
   zone: StdlibHeap rounds to max(8·⌈sz/8⌉, 16) (stdlibheap.h:13-18), FirstFitHeap passes fresh
   requests through (nothing is freed before the end), SizeHeap adds a 16-B header
   (sizeheap.h:32-37), ZoneHeap bump-allocates 16368-B arenas behind a 24-B arena header, a new
   arena when the request does not fit (zoneheap.h:52-83), and SourceMmapHeap bumps arenas back
   to back inside one 32 MiB zone (source.h:15-38). Checked in tests/test_trace.py against the
   reference heap itself (libgallocy.cpp's custom_malloc compiled in place by oracle/Makefile's
   `layout` target: every object's zone offset at NDIM 4, 64, 1000, 1021 and the abort at 1022,
   tests/golden/ref_layout.npz) and SURVEY §8f's figures.
2. `mmult_layout` allocates in test_mmult's order: init_matrix(a), (b), (c) — a row-pointer
   array then NDIM rows each (test/test_mmult.cpp:31-37, 137-139) — then `threads` and `args`
   (:152-154).
3. `MmultTrace` is the access trace of `mm()` (test_mmult.cpp:51-64) at the reference's -O0: for
   row i, every (j, k) reads a's row pointer i, a[i][k], b's row pointer k and b[k][j]; every j
   reads c's row pointer i and writes c[i][j]. A DSM faults once per page until invalidated, so
   a node's accesses for one row collapse to one R and/or one W event per page (R before W).
   Node t computes rows i ≡ t (mod P); rows run in rounds (round r: row t + r·P of every node),
   the nodes of a round in a seeded permutation (the jitter of SURVEY §8d).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

PAGE_SZ = 4096
ZONE_SZ = 32 << 20                  # utils/constants.h:11
ZONE_CHUNK = 16384 - 16             # DEFAULT_ZONE_SZ, heaplayers/application.h
ARENA_HDR = 24                      # ZoneHeap::Arena {next, space, double}, zoneheap.h:85-90
SIZE_HDR = 16                       # SizeHeap freeObject {dummy, sz}, sizeheap.h:19-22
U64 = (1 << 64) - 1


class HeapExhausted(MemoryError):
    """SourceMmapHeap prints ---ENOMEM--- and aborts (source.h:21-24, 35-36)."""


class AppHeap:
    """Zone offsets handed out by the reference application heap (see module docstring)."""

    def __init__(self):
        self.zone_used = 0           # SourceMmapHeap bump
        self.arena_base = None       # current arena's zone offset
        self.space = 0               # ZoneHeap arenaSpace (zone offset)
        self.remaining = U64         # sizeRemaining, uint64 (starts at -1)
        self.headers = []            # (zone offset, requested size) of each SizeHeap header
        self.arenas = []             # zone offsets of arena headers
        self.arena_space = []        # each arena's final arenaSpace (zone offset)

    def malloc(self, sz: int) -> int:
        sz = max(sz, 16)
        sz = (sz + 7) & ~7                      # StdlibHeap
        req = (sz + SIZE_HDR + 7) & ~7          # SizeHeap header, ZoneHeap align
        if self.arena_base is None or self.remaining < req:
            alloc = max(ZONE_CHUNK, req) + ARENA_HDR
            if not (ZONE_SZ - self.zone_used > alloc):   # source.h:29 `bytes_left > sz`
                raise HeapExhausted(f"zone exhausted at {self.zone_used} + {alloc}")
            if self.arena_base is not None:
                self.arena_space[-1] = self.space
            self.arena_base = self.zone_used
            self.zone_used += alloc
            self.arenas.append(self.arena_base)
            self.arena_space.append(0)
            self.space = self.arena_base + ARENA_HDR
            self.remaining = ZONE_CHUNK                  # zoneheap.h:75 (even for big chunks)
        ptr = self.space
        self.space += req
        self.arena_space[-1] = self.space
        self.remaining = (self.remaining - req) & U64
        self.headers.append((ptr, sz))
        return ptr + SIZE_HDR


@dataclass
class MmultLayout:
    ndim: int
    nthreads: int
    a_rp: int
    b_rp: int
    c_rp: int
    a_rows: np.ndarray
    b_rows: np.ndarray
    c_rows: np.ndarray
    threads: int
    args: int
    heap: AppHeap

    @property
    def zone_bytes(self) -> int:
        return self.heap.zone_used

    @property
    def n_pages(self) -> int:
        return -(-self.heap.zone_used // PAGE_SZ)


PARM_SZ = 40  # struct parm {int id, noproc, dim; double **a, **b, **c;} test_mmult.cpp:23-28


def mmult_layout(ndim: int, nthreads: int = 4) -> MmultLayout:
    h = AppHeap()
    mats = []
    for _ in range(3):                                   # init_matrix(&a), (&b), (&c)
        rp = h.malloc(8 * ndim)
        rows = np.array([h.malloc(8 * ndim) for _ in range(ndim)], np.int64)
        mats.append((rp, rows))
    threads = h.malloc(nthreads * 8)                     # pthread_t[n]
    args = h.malloc(nthreads * PARM_SZ)                  # parm[n]
    (a_rp, a_rows), (b_rp, b_rows), (c_rp, c_rows) = mats
    return MmultLayout(ndim, nthreads, a_rp, b_rp, c_rp, a_rows, b_rows, c_rows, threads, args, h)


def _span_pages(start: int, nbytes: int) -> np.ndarray:
    return np.arange(start // PAGE_SZ, (start + nbytes - 1) // PAGE_SZ + 1, dtype=np.int64)


class MmultTrace:
    """Access events of mm() for P nodes, grouped in rounds (see module docstring)."""

    def __init__(self, layout: MmultLayout, nodes: int, seed: int = 0):
        if not 1 <= nodes <= 8:
            raise ValueError("1..8 nodes")
        self.L, self.P, self.seed = layout, nodes, seed
        n = layout.ndim
        # pages every row reads regardless of i: b's row-pointer array and all of b's rows
        b_pages = [_span_pages(layout.b_rp, 8 * n)] + [_span_pages(int(r), 8 * n)
                                                        for r in layout.b_rows]
        self.b_read = np.unique(np.concatenate(b_pages))
        self.rounds = -(-n // nodes)
        rng = np.random.default_rng(seed)
        self.order = [rng.permutation(nodes) for _ in range(self.rounds)]

    def row_sets(self, i: int):
        """(R pages, W pages) of one row's computation (test_mmult.cpp:54-61)."""
        L, n = self.L, self.L.ndim
        r = np.concatenate([[(L.a_rp + 8 * i) // PAGE_SZ], _span_pages(int(L.a_rows[i]), 8 * n),
                            self.b_read, [(L.c_rp + 8 * i) // PAGE_SZ]])
        return np.unique(r), _span_pages(int(L.c_rows[i]), 8 * n)

    def round_rows(self, r: int):
        """[(node, row)] of round r in execution order."""
        return [(int(t), int(t) + r * self.P) for t in self.order[r] if int(t) + r * self.P < self.L.ndim]

    def round_events(self, r: int) -> np.ndarray:
        """Events of round r (docs/SPEC.md §5 packing), sorted by page, sequence order kept."""
        evs = []
        for t, i in self.round_rows(r):
            rp, wp = self.row_sets(i)
            pages = np.union1d(rp, wp)
            isr = np.isin(pages, rp)
            isw = np.isin(pages, wp)
            # R then W of the same page; rows of the round in execution order
            e_r = (pages[isr] << 4) | (t << 1)
            e_w = (pages[isw] << 4) | (t << 1) | 1
            evs.append(np.concatenate([e_r, e_w]))
        if not evs:
            return np.zeros(0, np.uint64)
        ev = np.concatenate(evs).astype(np.uint64)
        # stable by page: rows stay in execution order, and inside a row R precedes W
        return ev[np.argsort(ev >> 4, kind="stable")]

    def round_stamped(self, r: int) -> list:
        """Per node t: its own events of round r as SPEC §5b stamped events (page << 36 | seq << 4
        | node << 1 | rw), sorted. seq = 2 * (the row's position in the round's execution order)
        + rw, a logical clock every node knows locally; merging all nodes' lists by (page, seq)
        gives exactly round_events(r)."""
        out = [np.zeros(0, np.uint64) for _ in range(self.P)]
        for pos, (t, i) in enumerate(self.round_rows(r)):
            rp, wp = self.row_sets(i)
            e = np.concatenate([(rp.astype(np.uint64) << np.uint64(36))
                                | np.uint64((2 * pos) << 4 | (t << 1)),
                                (wp.astype(np.uint64) << np.uint64(36))
                                | np.uint64((2 * pos + 1) << 4 | (t << 1) | 1)])
            out[t] = np.sort(np.concatenate([out[t], e]))
        return out

    def all_events(self) -> np.ndarray:
        """The whole trace as ONE page-sorted batch (per-page order = execution order)."""
        ev = np.concatenate([self.round_events(r) for r in range(self.rounds)])
        return ev[np.argsort(ev >> 4, kind="stable")]


# ---------------------------------------------------------------- page contents
ZONE_BASE = 0x7F5A00000000  # the zone's virtual address in the model (global_base(), any page)


def zone_image(L: MmultLayout) -> np.ndarray:
    """Bytes of the application zone right after test_mmult's setup (test_mmult.cpp:137-160):
    arena and size headers, row-pointer arrays, a[i][j] = b[i][j] = i + j, c = 0."""
    z = np.zeros(L.n_pages * PAGE_SZ, np.uint8)
    u64 = z.view("<u8")
    arenas = L.heap.arenas
    for k, a in enumerate(arenas):  # Arena{next, space, dummy}: a retired arena points at the
        last = k + 1 == len(arenas)  # previous one (zoneheap.h:59-62); the current one at NULL
        u64[a // 8] = 0 if (k == 0 or last) else ZONE_BASE + arenas[k - 1]
        u64[a // 8 + 1] = ZONE_BASE + L.heap.arena_space[k]
    for off, sz in L.heap.headers:                      # SizeHeap {dummy, sz}
        u64[off // 8 + 1] = sz
    n = L.ndim
    idx = np.arange(n, dtype=np.float64)
    for rp, rows in ((L.a_rp, L.a_rows), (L.b_rp, L.b_rows), (L.c_rp, L.c_rows)):
        u64[rp // 8: rp // 8 + n] = (ZONE_BASE + rows).astype(np.uint64)
    f64 = z.view("<f8")
    for rows in (L.a_rows, L.b_rows):
        for i, r in enumerate(rows):
            f64[r // 8: r // 8 + n] = idx + i
    return z


def c_row_values(L: MmultLayout, i: int) -> np.ndarray:
    """c[i][j] = sum_k (i + k)(k + j), exactly representable in float64 for NDIM <= 1021."""
    n = L.ndim
    k = np.arange(n, dtype=np.float64)
    return ((i + k)[None, :] * (k[:, None] + np.arange(n, dtype=np.float64)[None, :]).T).sum(axis=1)
