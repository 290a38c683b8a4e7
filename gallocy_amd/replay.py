"""End-to-end replay of the test_mmult trace (BASELINE config 5) through the engine.

P simulated DSM nodes share one GPU (the multi-GPU layout of exchange.py puts one node per
rank; here the per-node views live side by side in one arena):

  data context:  arena pages [t·Z, (t+1)·Z) = node t's view of the Z-page application zone
                 (CURRENT and its TWIN); REPLICA pages [0, Z) = the home copies.
  page table:    a second, arena-less context over the Z zone pages (home = page-shard).

Per round (one row per node, gallocy_amd/trace.py):
  1. coherence batch of the round's R/W fault events (SPEC §5);
  2. twin of every c[i] page the round writes (SPEC §2), taken in each writer's view;
  3. each writer stores its row c[i][*] into its own view (the application's writes);
  4. one diff of all those pages (SPEC §3) — release;
  5. apply of the stream to the home copies (SPEC §4). Rows sharing a page are written by
     different nodes at disjoint bytes: their records hit the same home page with disjoint
     runs, which the store-only apply handles without a read-modify-write race.
The trace, the rows' values and the page lists are prepared on the host before the timed
replay; a round is then only asynchronous launches on two streams (page table, page data).
At the end the home copies must equal the zone after the whole multiplication, and the page
table / totals must equal the oracle's sequential fold of the same events.
"""
from __future__ import annotations

import time

import numpy as np

from . import gdsm
from .trace import PAGE_SZ, MmultTrace, c_row_values, mmult_layout, zone_image


class MmultReplay:
    def __init__(self, ndim: int = 1000, nodes: int = 4, seed: int = 0, device: int = 0):
        self.L = mmult_layout(ndim)
        self.T = MmultTrace(self.L, nodes, seed)
        self.P = nodes
        self.Z = self.L.n_pages
        self.image = zone_image(self.L)
        L = self.L
        # ---- host preparation (not part of the replay time)
        ev_parts, id_parts, home_parts = [], [], []
        self.ev_off, self.rows, n_ids = [0], [], []
        for r in range(self.T.rounds):
            rows = self.T.round_rows(r)
            ev = self.T.round_events(r)
            ev_parts.append(ev)
            self.ev_off.append(self.ev_off[-1] + len(ev))
            k = 0
            for t, i in rows:
                wp = np.arange(int(L.c_rows[i]) // PAGE_SZ,
                               (int(L.c_rows[i]) + 8 * L.ndim - 1) // PAGE_SZ + 1)
                id_parts.append(t * self.Z + wp)
                home_parts.append(wp)
                k += len(wp)
            n_ids.append(k)
            self.rows.append(rows)
        events = np.concatenate(ev_parts).astype(np.uint64)
        ids = np.concatenate(id_parts).astype(np.uint32)
        home = np.concatenate(home_parts).astype(np.uint32)
        self.id_off = np.concatenate([[0], np.cumsum(n_ids)]).astype(np.int64)
        rowvals = np.stack([c_row_values(L, i) for i in range(L.ndim)]).view(np.uint8)
        # ---- device state
        self.data = gdsm.Context(self.Z * nodes, device=device)
        self.pt = gdsm.Context(self.Z, device=device, arenas=())
        pages = self.image.reshape(self.Z, PAGE_SZ)
        for t in range(nodes):
            self.data.upload("current", pages, first=t * self.Z)
            self.data.upload("twin", pages, first=t * self.Z)
        self.data.upload("replica", pages, first=0)
        self.pt.coh_init(nodes)
        self.d_events = self.pt.buffer(max(8, events.nbytes)).upload(events)
        self.d_tot = self.pt.buffer(8 * 10 * self.T.rounds)
        self.d_ids = self.data.buffer(max(4, ids.nbytes)).upload(ids)
        self.d_home = self.data.buffer(max(4, home.nbytes)).upload(home)
        self.d_rows = self.data.buffer(rowvals.nbytes).upload(rowvals)
        self.row_bytes = 8 * L.ndim
        max_ids = int(np.max(np.diff(self.id_off))) if len(self.id_off) > 1 else 1
        self._runs = gdsm.Runs(self.data, max_ids, cap=max_ids * 10244)
        max_ev = int(np.max(np.diff(self.ev_off))) if len(self.ev_off) > 1 else 1
        gdsm.check(gdsm.lib().gdsm_reserve(self.data.handle, max_ids, 0), "reserve")
        gdsm.check(gdsm.lib().gdsm_reserve(self.pt.handle, 0, max_ev), "reserve")
        self.events_total = len(events)
        self.pages_diffed = len(ids)
        self.totals = None

    def round(self, r: int):
        lib = gdsm.lib()
        e0, e1 = self.ev_off[r], self.ev_off[r + 1]
        gdsm.check(lib.gdsm_coherence_batch_async(self.pt.handle, self.d_events.ptr + 8 * e0, e1 - e0,
                                                  self.d_tot.ptr + 80 * r), "coherence")   # 1
        a, b = int(self.id_off[r]), int(self.id_off[r + 1])
        ids, home, n = self.d_ids.ptr + 4 * a, self.d_home.ptr + 4 * a, b - a
        self.data.twin(ids, n=n)                                                           # 2
        base = self.data.arena_ptr("current")
        for t, i in self.rows[r]:                                                          # 3
            dst = base + t * self.Z * PAGE_SZ + int(self.L.c_rows[i])
            gdsm.check(lib.gdsm_memcpy_d2d(self.data.handle, dst, self.d_rows.ptr + i * self.row_bytes,
                                           self.row_bytes), "row write")
        self.data.diff(ids, n=n, out=self._runs)                                           # 4
        self.data.apply(self._runs, "replica", home)                                       # 5

    def run(self) -> float:
        self.data.sync()
        self.pt.sync()
        t0 = time.perf_counter()
        for r in range(self.T.rounds):
            self.round(r)
        self.data.sync()
        self.pt.sync()
        dt = time.perf_counter() - t0
        self.totals = self.d_tot.download(np.uint64, 10 * self.T.rounds).reshape(-1, 10).sum(0).astype(np.int64)
        return dt

    def final_image(self) -> np.ndarray:
        z = self.image.copy()
        f64 = z.view("<f8")
        n = self.L.ndim
        for i in range(n):
            o = int(self.L.c_rows[i]) // 8
            f64[o:o + n] = c_row_values(self.L, i)
        return z

    def home_copy(self) -> np.ndarray:
        return self.data.download("replica", 0, self.Z).reshape(-1)

    def close(self):
        self._runs.free()
        self.data.close()
        self.pt.close()
