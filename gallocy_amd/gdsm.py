"""Host-side mirror of the gdsm C-ABI (include/gdsm.h) for Python callers and tests.

Names follow the reference's domain: pages, twins, diffs (run records), replicas, the page
table. `diff()` keeps the reference utility's name and meaning
(gallocy/utils/diff.cpp:73-167); the page-level engine is `Context`.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import GdsmError, GdsmRuns, check

PAGE_SZ = 4096
MAX_RUNS = 2048
MAX_RECORD = 10244
TWIN, CURRENT, REPLICA = 0, 1, 2
GEN_UNIFORM, GEN_CLUSTERED = 0, 1
RELEASE_RETWIN = 1  # gdsm.h GDSM_RELEASE_RETWIN
_ARENA = {"twin": TWIN, "current": CURRENT, "replica": REPLICA,
          TWIN: TWIN, CURRENT: CURRENT, REPLICA: REPLICA}


def lib():
    return _lib.load()


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().gdsm_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def version() -> str:
    return lib().gdsm_version().decode()


class DeviceBuffer:
    """A device allocation owned by a Context (freed with it, or by .free())."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(lib().gdsm_dev_alloc(ctx.handle, self.nbytes, C.byref(p)), "gdsm_dev_alloc")
        self.ptr = p.value

    def upload(self, arr: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(arr)
        if a.nbytes > self.nbytes:
            raise ValueError("array larger than the device buffer")
        check(lib().gdsm_memcpy_h2d(self.ctx.handle, self.ptr, a.ctypes.data, a.nbytes), "h2d")
        return self

    def download(self, dtype, count: int) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if out.nbytes > self.nbytes:
            raise ValueError("read past the device buffer")
        check(lib().gdsm_memcpy_d2h(self.ctx.handle, out.ctypes.data, self.ptr, out.nbytes), "d2h")
        return out

    def free(self):
        if self.ptr and self.ctx.handle:
            check(lib().gdsm_dev_free(self.ctx.handle, self.ptr), "gdsm_dev_free")
        self.ptr = None


@dataclass
class HostRuns:
    """A diff stream on the host: rec_off[n+1] (uint64) and data (uint8), SPEC §3."""
    rec_off: np.ndarray
    data: np.ndarray

    @property
    def n(self) -> int:
        return len(self.rec_off) - 1

    def record(self, i: int) -> bytes:
        return self.data[self.rec_off[i]:self.rec_off[i + 1]].tobytes()

    def runs(self, i: int):
        """[(off, len, payload bytes)] of record i."""
        r = self.record(i)
        if not r:
            return []
        nr = int(np.frombuffer(r[:4], "<u4")[0])
        hdr = np.frombuffer(r[4:4 + 4 * nr], "<u4")
        out, p = [], 4 + 4 * nr
        for h in hdr:
            o, ln = int(h & 0xFFFF), int(h >> 16)
            out.append((o, ln, r[p:p + ln]))
            p += ln
        return out


class Runs:
    """A device diff stream (gdsm_runs)."""

    def __init__(self, ctx: "Context", n: int, cap: int = 0):
        self.ctx = ctx
        self.s = GdsmRuns()
        check(lib().gdsm_runs_alloc(ctx.handle, n, cap, C.byref(self.s)), "gdsm_runs_alloc")
        self.cap_alloc = self.s.cap  # bytes allocated; s.cap may be lowered to a byte budget

    @property
    def n(self) -> int:
        return self.s.n

    @property
    def cap(self) -> int:
        return self.s.cap

    def total(self) -> int:
        t = C.c_uint64(0)
        rc = lib().gdsm_runs_total(self.ctx.handle, C.byref(self.s), C.byref(t))
        if rc == -28:
            raise GdsmError(28, f"diff stream needs {t.value} bytes, capacity {self.cap}")
        check(rc, "gdsm_runs_total")
        return t.value

    def to_host(self) -> HostRuns:
        total = self.total()
        ro = np.empty(self.n + 1, np.uint64)
        check(lib().gdsm_memcpy_d2h(self.ctx.handle, ro.ctypes.data, self.s.rec_off, ro.nbytes), "d2h")
        data = np.empty(total, np.uint8)
        if total:
            check(lib().gdsm_memcpy_d2h(self.ctx.handle, data.ctypes.data, self.s.data, total), "d2h")
        return HostRuns(ro, data)

    @classmethod
    def from_host(cls, ctx: "Context", host: HostRuns, cap: Optional[int] = None) -> "Runs":
        r = cls(ctx, host.n, cap if cap is not None else max(16, len(host.data)))
        ro = np.ascontiguousarray(host.rec_off, dtype=np.uint64)
        check(lib().gdsm_memcpy_h2d(ctx.handle, r.s.rec_off, ro.ctypes.data, ro.nbytes), "h2d")
        if len(host.data):
            d = np.ascontiguousarray(host.data, dtype=np.uint8)
            check(lib().gdsm_memcpy_h2d(ctx.handle, r.s.data, d.ctypes.data, d.nbytes), "h2d")
        return r

    def free(self):
        if self.s.owned:
            check(lib().gdsm_runs_free(self.ctx.handle, C.byref(self.s)), "gdsm_runs_free")


class Graph:
    """An instantiated HIP graph of recorded libgdsm calls (Context.capture_end)."""

    def __init__(self, handle: int):
        self.handle = handle

    def launch(self, ctx: "Context"):
        check(lib().gdsm_graph_launch(ctx.handle, self.handle), "gdsm_graph_launch")

    def destroy(self):
        if self.handle:
            lib().gdsm_graph_destroy(self.handle)
            self.handle = None


class Context:
    """One shard of pages on one GPU: TWIN / CURRENT / REPLICA arenas + the page table."""

    def __init__(self, n_pages: int, device: int = 0, arenas: Sequence = ("twin", "current", "replica")):
        flags = 0
        for a in arenas:
            flags |= 1 << _ARENA[a]
        if not flags:
            flags = 1 << 31  # GDSM_NO_ARENAS: page-table-only context
        h = C.c_void_p()
        check(lib().gdsm_init(C.byref(h), device, n_pages, flags), "gdsm_init")
        self.handle = h.value
        self.n_pages = n_pages
        self.device = device

    # -- lifetime
    def close(self):
        if self.handle:
            lib().gdsm_fini(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- plumbing
    def arena_ptr(self, which) -> int:
        p = C.c_void_p()
        check(lib().gdsm_arena(self.handle, _ARENA[which], C.byref(p)), "gdsm_arena")
        return p.value

    @property
    def stream(self) -> int:
        return lib().gdsm_stream(self.handle)

    def sync(self):
        check(lib().gdsm_sync(self.handle), "gdsm_sync")

    # -- HIP graphs (gdsm_capture_*): record a launch-bound sequence once, replay it at once
    def capture_begin(self, *others: "Context"):
        """Starts recording this context's asynchronous calls (and those of `others`, joined in
        order) into one graph; end with capture_end()."""
        check(lib().gdsm_capture_begin(self.handle), "gdsm_capture_begin")
        for o in others:
            check(lib().gdsm_capture_join(self.handle, o.handle), "gdsm_capture_join")

    def capture_end(self) -> "Graph":
        g = C.c_void_p()
        check(lib().gdsm_capture_end(self.handle, C.byref(g)), "gdsm_capture_end")
        return Graph(g.value)

    PROF_STAGES = ("diff", "apply", "twin", "coh_fold", "coh_reduce", "nw_fill", "nw_trace",
                   "exchange", "route", "exchange_wait")

    def prof_enable(self, on: bool = True):
        check(lib().gdsm_prof_enable(self.handle, int(on)), "gdsm_prof_enable")

    def prof_read(self) -> dict:
        """{stage: (total_ms, launches)} from HIP events on the context stream."""
        ms = (C.c_double * len(self.PROF_STAGES))()
        ln = (C.c_uint64 * len(self.PROF_STAGES))()
        check(lib().gdsm_prof_read(self.handle, ms, ln), "gdsm_prof_read")
        return {k: (ms[i], ln[i]) for i, k in enumerate(self.PROF_STAGES)}

    def upload(self, which, pages: np.ndarray, first: int = 0):
        a = np.ascontiguousarray(pages, dtype=np.uint8).reshape(-1, PAGE_SZ)
        check(lib().gdsm_upload(self.handle, _ARENA[which], first, a.shape[0], a.ctypes.data), "upload")

    def download(self, which, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.n_pages - first if n is None else n
        out = np.empty((n, PAGE_SZ), np.uint8)
        check(lib().gdsm_download(self.handle, _ARENA[which], first, n, out.ctypes.data), "download")
        return out

    def buffer(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def ids(self, page_ids) -> DeviceBuffer:
        a = np.ascontiguousarray(page_ids, dtype=np.uint32)
        return DeviceBuffer(self, max(4, a.nbytes)).upload(a)

    @staticmethod
    def _ptr(ids) -> Optional[int]:
        if ids is None:
            return None
        if isinstance(ids, DeviceBuffer):
            return ids.ptr
        return int(ids)

    # -- hot path
    def gen_pages(self, seed: int, mode: int = GEN_UNIFORM, ppm: int = 10000, first_global: int = 0,
                  stride: int = 1, arenas: Sequence = ()):
        """SPEC §6 synthetic pages; arena page i is global page first_global + i * stride."""
        mask = 0
        for a in arenas:
            mask |= 1 << _ARENA[a]
        check(lib().gdsm_gen_pages(self.handle, mask, first_global, stride, seed, mode, ppm),
              "gdsm_gen_pages")

    def twin(self, ids=None, n: Optional[int] = None):
        n = self._count(ids, n)
        check(lib().gdsm_twin(self.handle, self._ptr(ids), n), "gdsm_twin")

    def diff_split(self, bounds, outs) -> None:
        """One diff launch for several destinations (gdsm_diff_split): arena pages
        [bounds[d], bounds[d+1]) into outs[d], each stream exactly what diff() of that range
        writes."""
        G = len(outs)
        b = (C.c_uint64 * (G + 1))(*[int(x) for x in bounds])
        arr = (GdsmRuns * G)(*[o.s for o in outs])
        check(lib().gdsm_diff_split(self.handle, b, G, arr), "gdsm_diff_split")
        for d, o in enumerate(outs):
            o.s.n = arr[d].n

    def diff(self, ids=None, n: Optional[int] = None, out: Optional[Runs] = None, cap: int = 0,
             apply_to: Optional[str] = None, target_ids=None) -> Runs:
        """TWIN vs CURRENT -> Runs; with apply_to (normally "replica"), the same kernel also
        applies the runs to that arena (gdsm_diff_apply: a home copy on this GPU), at the pages
        target_ids (device list, gdsm_diff_apply_ids) when they are not the same ids."""
        n = self._count(ids, n)
        out = out or Runs(self, n, cap)
        if apply_to is None:
            check(lib().gdsm_diff(self.handle, self._ptr(ids), n, C.byref(out.s)), "gdsm_diff")
        elif target_ids is not None:
            check(lib().gdsm_diff_apply_ids(self.handle, self._ptr(ids), n, C.byref(out.s),
                                            _ARENA[apply_to], self._ptr(target_ids)),
                  "gdsm_diff_apply_ids")
        else:
            check(lib().gdsm_diff_apply(self.handle, self._ptr(ids), n, C.byref(out.s),
                                        _ARENA[apply_to]), "gdsm_diff_apply")
        return out

    def release(self, ids=None, n: Optional[int] = None, out: Optional[Runs] = None,
                cap: int = 0, apply_to: Optional[str] = None, target_ids=None,
                retwin: bool = True) -> Runs:
        """gdsm_release: the diff of the listed pages (applied to `apply_to` at target_ids as
        diff() does) and, with retwin, TWIN := CURRENT for every page whose record fit. Up to
        2048 pages this is one kernel launch (outside graph capture: no zeroing launch)."""
        n = self._count(ids, n)
        out = out or Runs(self, n, cap)
        check(lib().gdsm_release(self.handle, self._ptr(ids), n, C.byref(out.s),
                                 -1 if apply_to is None else _ARENA[apply_to],
                                 self._ptr(target_ids), RELEASE_RETWIN if retwin else 0),
              "gdsm_release")
        return out

    def apply(self, runs: Runs, target="replica", ids=None):
        check(lib().gdsm_apply(self.handle, _ARENA[target], self._ptr(ids), C.byref(runs.s)), "gdsm_apply")

    def apply_async(self, runs: Runs, target="replica", ids=None):
        """gdsm_apply_async: the apply overlaps the diffs enqueued after it (double buffering)."""
        check(lib().gdsm_apply_async(self.handle, _ARENA[target], self._ptr(ids), C.byref(runs.s)),
              "gdsm_apply_async")

    def _count(self, ids, n):
        if n is not None:
            return int(n)
        if ids is None:
            return self.n_pages
        if isinstance(ids, DeviceBuffer):
            return ids.nbytes // 4
        raise ValueError("pass n= with a raw device pointer")

    # -- page table (coherence)
    def coh_init(self, n_nodes: int = 8):
        check(lib().gdsm_coh_init(self.handle, n_nodes), "gdsm_coh_init")

    def coherence_batch(self, events) -> dict:
        """events: a DeviceBuffer of uint64 (page-sorted) or a numpy array (uploaded here)."""
        tmp = None
        if isinstance(events, np.ndarray):
            ev = np.ascontiguousarray(events, dtype=np.uint64)
            tmp = DeviceBuffer(self, max(8, ev.nbytes)).upload(ev)
            ptr, n = tmp.ptr, len(ev)
        else:
            ptr, n = events.ptr, events.nbytes // 8
        tot = (C.c_uint64 * 10)()
        try:
            check(lib().gdsm_coherence_batch(self.handle, ptr, n, tot), "gdsm_coherence_batch")
        finally:
            if tmp is not None:
                tmp.free()
        t = list(tot)
        return {"invalidations": t[0], "transfers": t[1], "node_faults": t[2:10]}

    def coh_download(self):
        st = np.empty(self.n_pages, np.uint32)
        fl = np.empty(self.n_pages, np.uint32)
        check(lib().gdsm_coh_download(self.handle, st.ctypes.data, fl.ctypes.data), "gdsm_coh_download")
        return st, fl

    def coh_upload(self, state: np.ndarray, faults: np.ndarray):
        s = np.ascontiguousarray(state, np.uint32)
        f = np.ascontiguousarray(faults, np.uint32)
        check(lib().gdsm_coh_upload(self.handle, s.ctypes.data, f.ctypes.data), "gdsm_coh_upload")

    def gen_events(self, counts: np.ndarray, seed: int, n_nodes: int = 8, write_pct: int = 20,
                   first_page: int = 0) -> DeviceBuffer:
        counts = np.ascontiguousarray(counts, dtype=np.uint64)
        offs = np.zeros(len(counts) + 1, np.uint64)
        np.cumsum(counts, out=offs[1:])
        total = int(offs[-1])
        d_off = DeviceBuffer(self, offs.nbytes).upload(offs)
        ev = DeviceBuffer(self, max(8, total * 8))
        check(lib().gdsm_gen_events(self.handle, ev.ptr, d_off.ptr, first_page, len(counts), seed,
                                    n_nodes, write_pct), "gdsm_gen_events")
        self.sync()
        d_off.free()
        ev.count = total
        return ev

    def nw_diff_batch(self, pairs: Sequence, max_len: Optional[int] = None) -> list:
        """GPU diff() over a batch: [(mem1, mem2), ...] -> [(out1, out2), ...] (bytes), the
        alignment of gallocy/utils/diff.cpp:73-167 for every pair (gdsm_nw_diff_batch)."""
        n = len(pairs)
        if n == 0:
            return []
        la = np.array([len(p[0]) for p in pairs], np.uint64)
        lb = np.array([len(p[1]) for p in pairs], np.uint64)
        a_off = np.zeros(n + 1, np.uint64)
        b_off = np.zeros(n + 1, np.uint64)
        np.cumsum(la, out=a_off[1:])
        np.cumsum(lb, out=b_off[1:])
        ml = int(max(la.max(), lb.max())) if max_len is None else int(max_len)
        a = np.frombuffer(b"".join(bytes(p[0]) for p in pairs) or b"\0", np.uint8)
        b = np.frombuffer(b"".join(bytes(p[1]) for p in pairs) or b"\0", np.uint8)
        out_bytes = int(a_off[-1] + b_off[-1]) + n
        bufs = [self.buffer(max(x.nbytes, 1)).upload(x) for x in (a, a_off, b, b_off)]
        o1, o2, ol = self.buffer(out_bytes), self.buffer(out_bytes), self.buffer(8 * n)
        try:
            check(lib().gdsm_nw_diff_batch(self.handle, bufs[0].ptr, bufs[1].ptr, bufs[2].ptr,
                                           bufs[3].ptr, n, ml, o1.ptr, o2.ptr, ol.ptr),
                  "gdsm_nw_diff_batch")
            h1 = o1.download(np.uint8, out_bytes)
            h2 = o2.download(np.uint8, out_bytes)
            lens = ol.download(np.uint64, n)
        finally:
            for x in (*bufs, o1, o2, ol):
                x.free()
        res = []
        for i in range(n):
            o = int(a_off[i] + b_off[i]) + i
            L = int(lens[i])
            res.append((h1[o:o + L].tobytes(), h2[o:o + L].tobytes()))
        return res

    # -- diff wire format (docs/SPEC.md §7): Raft log command text
    def wire_encode(self, runs: Runs, ids=None) -> bytes:
        """The command text "GDSM1:" + base64(frame) of `runs` (pages `ids`, a DeviceBuffer or
        None = 0..n-1), encoded on the GPU (gdsm_wire_encode)."""
        need = C.c_uint64(0)
        rc = lib().gdsm_wire_encode(self.handle, self._ptr(ids), C.byref(runs.s), None, 0,
                                    C.byref(need))
        if rc != -28:
            check(rc, "gdsm_wire_encode")
        buf = C.create_string_buffer(need.value + 1)
        check(lib().gdsm_wire_encode(self.handle, self._ptr(ids), C.byref(runs.s), buf,
                                     need.value + 1, C.byref(need)), "gdsm_wire_encode")
        return buf.raw[:need.value]

    def wire_decode(self, text: bytes, n_cap: int, cap: int):
        """-> (ids DeviceBuffer, Runs) decoded and verified on the GPU (gdsm_wire_decode)."""
        ids = self.buffer(4 * max(n_cap, 1))
        out = Runs(self, n_cap, cap)
        n = C.c_uint64(0)
        try:
            check(lib().gdsm_wire_decode(self.handle, text, len(text), ids.ptr, C.byref(out.s),
                                         C.byref(n)), "gdsm_wire_decode")
        except Exception:
            ids.free()
            out.free()
            raise
        return ids, out

    def wire_apply(self, text: bytes, target="replica") -> int:
        """Follower try_apply: verify the command text and apply it to `target`; -> records."""
        n = C.c_uint64(0)
        check(lib().gdsm_wire_apply(self.handle, _ARENA[target], text, len(text), C.byref(n)),
              "gdsm_wire_apply")
        return n.value


def wire_size(n: int, data_bytes: int) -> int:
    return lib().gdsm_wire_size(n, data_bytes)


def set_diff_device(ctx: Optional["Context"], min_cells: int = 0):
    """Routes diff() / gdsm_nw_diff through the GPU of ctx for inputs with n*m >= min_cells
    (None: back to the CPU path)."""
    check(lib().gdsm_set_diff_device(ctx.handle if ctx is not None else None, int(min_cells)),
          "gdsm_set_diff_device")


class Tracker:
    """Write-fault capture over a host region (include/gdsm.h gdsm_track_*): the region is
    protected read-only, the first write to a page in an interval copies it to the twin and
    lists it as dirty. `region` is an anonymous mmap (page-aligned) or any page-aligned buffer
    exporting the buffer protocol; n_pages = len(region) // 4096."""

    def __init__(self, region):
        self._region = region
        self._view = np.frombuffer(region, dtype=np.uint8)
        self.n_pages = len(self._view) // PAGE_SZ
        base = self._view.ctypes.data
        h = C.c_void_p()
        check(lib().gdsm_track_begin(C.byref(h), base, self.n_pages), "gdsm_track_begin")
        self.handle = h
        self.base = base

    def pages(self) -> np.ndarray:
        """A (n_pages, 4096) uint8 view of the tracked region (writes are tracked)."""
        return self._view[: self.n_pages * PAGE_SZ].reshape(self.n_pages, PAGE_SZ)

    def dirty(self) -> np.ndarray:
        n = C.c_uint64(0)
        check(lib().gdsm_track_dirty(self.handle, None, 0, C.byref(n)), "gdsm_track_dirty")
        ids = np.empty(max(1, n.value), np.uint32)
        check(lib().gdsm_track_dirty(self.handle, ids.ctypes.data, len(ids), C.byref(n)),
              "gdsm_track_dirty")
        return ids[: n.value]

    def twin(self) -> np.ndarray:
        """The twin buffer as a (n_pages, 4096) array (rows of dirty pages are valid)."""
        ptr = C.c_void_p()
        check(lib().gdsm_track_twin(self.handle, C.byref(ptr)), "gdsm_track_twin")
        buf = (C.c_uint8 * (self.n_pages * PAGE_SZ)).from_address(ptr.value)
        return np.frombuffer(buf, dtype=np.uint8).reshape(self.n_pages, PAGE_SZ)

    def faults(self) -> int:
        f = C.c_uint64(0)
        check(lib().gdsm_track_faults(self.handle, C.byref(f)), "gdsm_track_faults")
        return f.value

    def rearm(self):
        check(lib().gdsm_track_rearm(self.handle), "gdsm_track_rearm")

    def diff(self, ctx: "Context", cap: Optional[int] = None):
        """GPU diff of this interval's dirty pages -> (Runs, DeviceBuffer of page ids, count)."""
        n = len(self.dirty())
        runs = Runs(ctx, max(1, n), cap if cap is not None else max(64, n * MAX_RECORD))
        ids = ctx.buffer(max(4, 4 * n))
        cnt = C.c_uint64(0)
        check(lib().gdsm_track_diff(ctx.handle, self.handle, C.byref(runs.s), ids.ptr,
                                    C.byref(cnt)), "gdsm_track_diff")
        return runs, ids, cnt.value

    def close(self):
        if getattr(self, "handle", None):
            check(lib().gdsm_track_end(self.handle), "gdsm_track_end")
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def diff(mem1: bytes, mem2: bytes):
    """The reference diff() (gallocy/utils/diff.cpp:73-167): NW alignment -> (out1, out2)."""
    L = lib()
    o1, o2, n = C.c_void_p(), C.c_void_p(), C.c_size_t(0)
    check(L.gdsm_nw_diff(mem1, len(mem1), C.byref(o1), mem2, len(mem2), C.byref(o2), C.byref(n)), "diff")
    try:
        return C.string_at(o1, n.value), C.string_at(o2, n.value)
    finally:
        libc = C.CDLL(None)
        libc.free(o1)
        libc.free(o2)
