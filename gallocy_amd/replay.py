"""End-to-end replay of the test_mmult trace (BASELINE config 5) through the engine.

P simulated DSM nodes share one GPU (the multi-GPU layout of exchange.py puts one node per
rank; here the per-node views live side by side in one arena):

  data context:  arena pages [t·Z, (t+1)·Z) = node t's view of the Z-page application zone
                 (CURRENT and its TWIN); REPLICA pages [0, Z) = the home copies.
  page table:    a second, arena-less context over the Z zone pages (home = page-shard).

Per round (one row per node, gallocy_amd/trace.py):
  1. coherence batch of the round's R/W fault events (SPEC §5);
  2. each writer stores its row c[i][*] into its own view (the application's writes; all of the
     round's rows as one batched copy, gdsm_memcpy_batch);
  3. one release of all those pages (gdsm_release, SPEC §3) whose kernel also applies the runs to
     the home copies (view page t·Z + p -> home page p) and then sets the pages' TWIN to their
     CURRENT (GDSM_RELEASE_RETWIN), so the next round starts from clean twins without a twin
     step (the views are uploaded with TWIN == CURRENT). retwin=False: a twin step (SPEC §2)
     before the writes and gdsm_diff_apply_ids (fused=False: a separate apply, SPEC §4). Rows
     sharing a page are written by different nodes at disjoint bytes: their records hit the same
     home page with disjoint runs, which the store-only apply handles without a
     read-modify-write race.
The trace, the rows' values and the page lists are prepared on the host before the timed
replay; a round is then only asynchronous launches on two streams (page table, page data),
issued by the C++ round loop (driver="native", gallocy_amd/native/replay.cpp: the host side of a
C++ DSM runtime over the C ABI) or by Python (driver="python", round()), or, with
run(graph=True), one HIP graph of all rounds recorded beforehand.
At the end the home copies must equal the zone after the whole multiplication, and the page
table / totals must equal the oracle's sequential fold of the same events.
"""
from __future__ import annotations

import ctypes as C
import time
from pathlib import Path

import numpy as np

from . import _lib, gdsm
from .trace import PAGE_SZ, MmultTrace, c_row_values, mmult_layout, zone_image


_NATIVE = None


def native_driver():
    """gallocy_amd/lib/libgdsm_replay.so (gallocy_amd/native/replay.cpp), which links the in-tree
    libgdsm.so: only with that library loaded (not a GDSM_LIB build: two copies of the library in
    one process would not share contexts)."""
    global _NATIVE
    if _NATIVE is None:
        libdir = Path(_lib.__file__).resolve().parent / "lib"
        if _lib.LIB_PATH.resolve() != (libdir / "libgdsm.so").resolve():
            raise RuntimeError(f"driver='native' needs the in-tree libgdsm.so, not {_lib.LIB_PATH}")
        _lib.load()
        path = libdir / "libgdsm_replay.so"
        if not path.exists():
            raise RuntimeError(f"{path} is missing: build it (python -m gallocy_amd.build)")
        d = C.CDLL(str(path))
        vp, i64p = C.c_void_p, C.c_void_p
        for fn in (d.gdsm_replay_mmult, d.gdsm_replay_mmult_threads):
            fn.restype = C.c_int
            fn.argtypes = [vp, vp, C.c_uint32, C.c_uint32, vp, i64p, vp, vp, vp, i64p, vp, i64p,
                           vp, C.c_int]
        _NATIVE = d
    return _NATIVE


class MmultReplay:
    def __init__(self, ndim: int = 1000, nodes: int = 4, seed: int = 0, device: int = 0,
                 fused: bool = True, retwin: bool = True, driver: str = "native"):
        if driver not in ("native", "native2", "python", "device"):
            raise ValueError(driver)
        if driver == "device" and not (fused and retwin):
            raise ValueError("driver='device' runs the re-twinning release (gdsm_rounds)")
        self.driver = driver
        self.fused = fused
        # retwin: every release refreshes its pages' twins (gdsm_release, GDSM_RELEASE_RETWIN), so
        # a round needs no twin step: TWIN == CURRENT from the upload on, as after a release
        self.retwin = retwin and fused
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
        # the rounds' row writes as (dst, src, bytes) copy descriptors, back to back
        base = self.data.arena_ptr("current")
        desc, self.desc_off = [], [0]
        for rows in self.rows:
            for t, i in rows:
                desc += [base + t * self.Z * PAGE_SZ + int(L.c_rows[i]),
                         self.d_rows.ptr + i * self.row_bytes, self.row_bytes]
            self.desc_off.append(len(desc) // 3)
        desc = np.array(desc or [0, 0, 0], np.uint64)
        self.d_desc = self.data.buffer(desc.nbytes).upload(desc)
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
        if not self.retwin:
            self.data.twin(ids, n=n)                                                       # 2
        d0, d1 = self.desc_off[r], self.desc_off[r + 1]                                    # 3
        gdsm.check(lib.gdsm_memcpy_batch(self.data.handle, self.d_desc.ptr + 24 * d0, d1 - d0),
                   "row writes")
        if self.retwin:                                                                    # 4
            self.data.release(ids, n=n, out=self._runs, apply_to="replica", target_ids=home)
        elif self.fused:
            self.data.diff(ids, n=n, out=self._runs, apply_to="replica", target_ids=home)
        else:
            self.data.diff(ids, n=n, out=self._runs)
            self.data.apply(self._runs, "replica", home)

    def run(self, graph: bool = False) -> float:
        """Replays every round once; returns the seconds from the first launch to the end.
        graph=False (default): the calls are issued eagerly on the two streams. graph=True: the
        rounds' calls on both contexts are recorded once into one HIP graph (gdsm_capture_*,
        untimed) and the replay is one graph launch. On MI355X the graph replay is the slower of
        the two (0.40 vs 0.35 ms per round at NDIM = 1000): a round is ~20 dependent tiny
        operations, bound by their device-side cost, not by the host issuing them."""
        self.data.sync()
        self.pt.sync()
        self.graph_build_s = 0.0
        if graph:
            tb = time.perf_counter()
            self.data.capture_begin(self.pt)
            try:
                for r in range(self.T.rounds):
                    self.round(r)
            finally:
                g = self.data.capture_end()
            self.graph_build_s = time.perf_counter() - tb
            t0 = time.perf_counter()
            g.launch(self.data)
            self.data.sync()
            dt = time.perf_counter() - t0
            g.destroy()
        elif self.driver == "device":
            # every round in one persistent launch per context (gdsm_rounds)
            ev_off = np.ascontiguousarray(self.ev_off, np.int64)
            id_off = np.ascontiguousarray(self.id_off, np.int64)
            desc_off = np.ascontiguousarray(self.desc_off, np.int64)
            t0 = time.perf_counter()
            gdsm.check(gdsm.lib().gdsm_rounds(
                self.data.handle, self.pt.handle, self.T.rounds, self.d_events.ptr,
                ev_off.ctypes.data, self.d_tot.ptr, self.d_ids.ptr, self.d_home.ptr,
                id_off.ctypes.data, self.d_desc.ptr, desc_off.ctypes.data,
                C.byref(self._runs.s)), "gdsm_rounds")
            self.data.sync()
            self.pt.sync()
            dt = time.perf_counter() - t0
        elif self.driver in ("native", "native2") and self.fused:
            d = native_driver()
            drv_fn = d.gdsm_replay_mmult_threads if self.driver == "native2" else d.gdsm_replay_mmult
            ev_off = np.ascontiguousarray(self.ev_off, np.int64)
            id_off = np.ascontiguousarray(self.id_off, np.int64)
            desc_off = np.ascontiguousarray(self.desc_off, np.int64)
            t0 = time.perf_counter()
            rc = drv_fn(self.data.handle, self.pt.handle, 0, self.T.rounds, self.d_events.ptr,
                        ev_off.ctypes.data, self.d_tot.ptr, self.d_ids.ptr, self.d_home.ptr,
                        id_off.ctypes.data, self.d_desc.ptr, desc_off.ctypes.data,
                        C.byref(self._runs.s), int(self.retwin))
            gdsm.check(rc, "gdsm_replay_mmult")
            self.data.sync()
            self.pt.sync()
            dt = time.perf_counter() - t0
        else:
            t0 = time.perf_counter()
            for r in range(self.T.rounds):
                self.round(r)
            self.data.sync()
            self.pt.sync()
            dt = time.perf_counter() - t0
        self.pt.sync()
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


class MmultRankReplay:
    """Config 5 with one process (one GPU) per DSM node: rank t of P = node t of the trace.

    Pages are homed in contiguous blocks, home(p) = p // ceil(Z / P), which is also the home the
    page table is initialised with (SPEC §5). Per round, on every rank (SPEC §5b):
      1. coherence: the node's OWN fault events of the round (stamped with the round's logical
         clock, MmultTrace.round_stamped) go to their pages' homes with gdsm_route_events; each
         home folds the merged batch into its page-table shard and returns the access-change
         notices to the nodes with gdsm_coherence_notify (kept per round in `notices_of(r)`);
      2. twin, then the node's own row writes c[i][*] in its view of the zone (CURRENT);
      3. release: the written pages are diffed into one stream per home rank and shipped with
         gdsm_exchange, each home applying what it receives to its REPLICA (indexed by global
         page: the home block is REPLICA[base, base + per)).
    At the end every home block equals the zone after the multiplication, the page-table shards
    together equal the sequential fold of the whole trace, and every node's notices equal the
    ones the sequential fold implies (tests/test_gpu_replay.py).
    Two communicators: one for page data (on the data context), one for coherence (on the
    page-table context), so the two kinds of collective never share an RCCL communicator across
    streams. transport "rccl" creates them; transport "loopback" (several ranks as threads of one
    process on one GPU) takes them from `wire_loopback`."""

    def __init__(self, rank: int, world: int, ndim: int = 1000, seed: int = 0, device: int = 0,
                 transport: str = "rccl", group=None):
        from . import exchange
        self.rank, self.P = rank, world
        self.L = mmult_layout(ndim)
        self.T = MmultTrace(self.L, world, seed)
        self.Z = self.L.n_pages
        self.per = -(-self.Z // world)
        self.base = min(self.Z, rank * self.per)
        self.nh = max(0, min(self.Z, self.base + self.per) - self.base)
        L, Z = self.L, self.Z
        self.image = zone_image(L)
        home = lambda p: p // self.per  # noqa: E731
        # ---- host preparation (not part of the replay time)
        self.rounds = []
        rowvals = np.stack([c_row_values(L, i) for i in range(L.ndim)]).view(np.uint8)
        max_per_dest, bcap, ncap = 1, 1, 1

        def written(rows):
            return np.unique(np.concatenate(
                [np.arange(int(L.c_rows[i]) // PAGE_SZ,
                           (int(L.c_rows[i]) + 8 * L.ndim - 1) // PAGE_SZ + 1) for _, i in rows])
                             ) if rows else np.zeros(0, np.int64)
        evs = []
        for r in range(self.T.rounds):
            all_rows = self.T.round_rows(r)
            for t in range(world):  # receive streams are sized for the largest sender
                wp = written([x for x in all_rows if x[0] == t])
                if len(wp):
                    max_per_dest = max(max_per_dest, int(np.bincount(home(wp)).max()))
            rows = [(t, i) for t, i in all_rows if t == rank]
            pages = written(rows)
            by_dest = [pages[home(pages) == d].astype(np.uint32) for d in range(world)]
            stamped = self.T.round_stamped(r)
            evs.append(stamped[rank])
            total = sum(len(x) for x in stamped)
            bcap = max(bcap, total)  # a home may receive the whole round
            ncap = max(ncap, len(np.unique(np.concatenate(stamped) >> np.uint64(36)))
                       if total else 1)  # one notice per node and page at most
            self.rounds.append((rows, pages.astype(np.uint32), by_dest))
            max_per_dest = max([max_per_dest] + [len(x) for x in by_dest])
        # ---- device state
        self.data = gdsm.Context(Z, device=device)
        self.pt = gdsm.Context(max(1, self.nh), device=device, arenas=())
        pages_img = self.image.reshape(Z, PAGE_SZ)
        for a in ("current", "twin", "replica"):
            self.data.upload(a, pages_img)
        self.pt.coh_init(world)
        if self.nh:  # every page of this shard is homed here (SPEC §5 initial state)
            st = np.full(self.nh, (1 << rank) | (rank << 8) | (2 << 16), np.uint32)
            self.pt.coh_upload(st, np.zeros(self.nh, np.uint32))
        self.d_rows = self.data.buffer(rowvals.nbytes).upload(rowvals)
        self.row_bytes = 8 * L.ndim
        # per round: written pages (twin list) and per-destination lists, in one device buffer
        flat, self.offs = [], []
        pos = 0
        for rows, pages, by_dest in self.rounds:
            o = [pos]
            flat.append(pages)
            pos += len(pages)
            for x in by_dest:
                o.append(pos)
                flat.append(x)
                pos += len(x)
            self.offs.append(o)
        allids = np.concatenate(flat).astype(np.uint32) if pos else np.zeros(1, np.uint32)
        self.d_ids = self.data.ids(allids)
        # this node's stamped events of every round, back to back; the home batch; the notices
        self.ev_off = np.concatenate([[0], np.cumsum([len(e) for e in evs])]).astype(np.int64)
        allev = np.concatenate(evs).astype(np.uint64) if self.ev_off[-1] else np.zeros(1, np.uint64)
        self.d_ev = self.pt.buffer(max(8, allev.nbytes)).upload(allev)
        self.bcap, self.ncap = bcap, ncap
        self.d_batch = self.pt.buffer(8 * bcap)
        self.d_notices = self.pt.buffer(8 * ncap * max(1, self.T.rounds))
        self.n_notices = np.zeros(self.T.rounds, np.int64)
        self.n_batch = np.zeros(self.T.rounds, np.int64)
        self.d_tot = self.pt.buffer(8 * 10 * max(1, self.T.rounds))
        cap = max_per_dest * 10244
        self.send = [gdsm.Runs(self.data, max_per_dest, cap=cap) for _ in range(world)]
        self.recv = [gdsm.Runs(self.data, max_per_dest, cap=cap) if s != rank
                     else gdsm.Runs(self.data, 1, cap=16) for s in range(world)]
        self.rids = [self.data.buffer(4 * max_per_dest) for _ in range(world)]
        gdsm.check(gdsm.lib().gdsm_reserve(self.data.handle, max_per_dest, 0), "reserve")
        gdsm.check(gdsm.lib().gdsm_reserve(self.pt.handle, 0, bcap), "reserve")
        self.transport = transport
        self.comm = self.coh_comm = None
        if transport == "rccl":
            self.comm = exchange.Comm(self.data, rank, world, group)
            self.coh_comm = exchange.Comm(self.pt, rank, world, group)
        elif transport != "loopback":
            raise ValueError("transport: rccl or loopback")
        self.events_total = int(self.ev_off[-1])
        self.pages_diffed = sum(len(p) for _, p, _ in self.rounds)
        self.totals = None

    @staticmethod
    def wire_loopback(replays: list):
        """Loopback communicators for replays built with transport="loopback" (one per rank,
        all in this process, each then driven by its own thread)."""
        from . import exchange
        data = exchange.Comm.loopback([R.data for R in replays])
        coh = exchange.Comm.loopback([R.pt for R in replays])
        for R, a, b in zip(replays, data, coh):
            R.comm, R.coh_comm = a, b

    def round(self, r: int):
        from . import exchange
        lib = gdsm.lib()
        rows, pages, by_dest = self.rounds[r]
        e0, e1 = int(self.ev_off[r]), int(self.ev_off[r + 1])
        nb = exchange.route_events(self.pt, self.coh_comm, self.d_ev.ptr + 8 * e0, e1 - e0,  # 1
                                   self.Z, self.d_batch.ptr, self.bcap)
        self.n_batch[r] = nb
        self.n_notices[r] = exchange.coherence_notify(
            self.pt, self.coh_comm, self.d_batch.ptr, nb, self.base, self.d_tot.ptr + 80 * r,
            self.d_notices.ptr + 8 * self.ncap * r, self.ncap)
        o = self.offs[r]
        if len(pages):
            # (no twin step: every release below refreshes its pages' twins, and the views were
            # uploaded with TWIN == CURRENT)
            base = self.data.arena_ptr("current")
            for _, i in rows:
                gdsm.check(lib.gdsm_memcpy_d2d(self.data.handle, base + int(self.L.c_rows[i]),
                                               self.d_rows.ptr + i * self.row_bytes,
                                               self.row_bytes), "row write")
        counts = [len(x) for x in by_dest]
        sids = [self.d_ids.ptr + 4 * o[1 + d] for d in range(self.P)]
        for d in range(self.P):                                                          # 3
            # the release for home d, re-twinning its pages (n = 0: rec_off[0] = 0)
            self.data.release(sids[d], n=counts[d], out=self.send[d])
        exchange.exchange_runs(self.data, self.comm, self.send, sids, self.recv,
                               [b.ptr for b in self.rids])

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

    def notices_of(self, r: int) -> np.ndarray:
        """The notices this node received in round r (SPEC §5b), sorted by page."""
        n = int(self.n_notices[r])
        out = np.empty(n, np.uint64)
        if n:
            gdsm.check(gdsm.lib().gdsm_memcpy_d2h(self.pt.handle, out.ctypes.data,
                                                  self.d_notices.ptr + 8 * self.ncap * r, 8 * n),
                       "d2h")
        return out

    def home_block(self) -> np.ndarray:
        """REPLICA pages [base, base + per) (this rank's home block)."""
        if not self.nh:
            return np.zeros(0, np.uint8)
        return self.data.download("replica", self.base, self.nh).reshape(-1)

    def final_block(self) -> np.ndarray:
        z = self.image.copy()
        f64 = z.view("<f8")
        n = self.L.ndim
        for i in range(n):
            o = int(self.L.c_rows[i]) // 8
            f64[o:o + n] = c_row_values(self.L, i)
        return z[self.base * PAGE_SZ:(self.base + self.nh) * PAGE_SZ]

    def close(self):
        for c in (self.comm, self.coh_comm):
            if c is not None:
                c.close()
        self.comm = self.coh_comm = None
        for r in self.send + self.recv:
            r.free()
        self.data.close()
        self.pt.close()
