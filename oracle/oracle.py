"""ctypes wrapper of the C oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY: imported by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = Path(os.environ.get("GDSM_ORACLE_LIB") or HERE / "liboracle.so")
REF_DRIVER = HERE / "_ref" / "ref_nw_driver"
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-s", "-C", str(HERE), "oracle"], check=True)
        L = C.CDLL(str(LIB))
        vp, u64 = C.c_void_p, C.c_uint64
        L.or_hash3.restype = u64
        L.or_hash3.argtypes = [u64, u64, u64]
        L.or_gen_pages.argtypes = [vp, vp, vp, u64, u64, u64, u64, C.c_int, C.c_uint32]
        L.or_diff_pages.restype = u64
        L.or_diff_pages.argtypes = [vp, vp, vp, u64, vp, vp, u64]
        L.or_apply.argtypes = [vp, vp, u64, vp, vp]
        L.or_twin.argtypes = [vp, vp, vp, u64]
        L.or_nw_diff.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p,
                                 C.c_char_p, C.POINTER(C.c_size_t)]
        L.or_coh_init.argtypes = [vp, vp, u64, C.c_uint32]
        L.or_coherence.argtypes = [vp, vp, u64, C.c_uint32, vp, u64, vp]
        L.or_gen_events.argtypes = [vp, vp, u64, u64, u64, C.c_uint32, C.c_uint32]
        L.or_bench_diff_apply.argtypes = [u64, C.c_int, C.c_uint32, u64, C.c_double, C.c_int,
                                          C.POINTER(u64), C.POINTER(C.c_double),
                                          C.POINTER(C.c_int)]
        L.or_bench_coherence.argtypes = [C.c_void_p, C.c_void_p, u64, C.c_uint32, C.c_double,
                                         C.c_int, C.POINTER(u64), C.POINTER(C.c_double)]
        L.or_bench_mmult.argtypes = [vp, vp, u64, C.c_uint32, vp, vp, vp, u64, vp, vp, vp, vp,
                                     vp, vp, vp, vp, vp, u64, vp, C.POINTER(C.c_double),
                                     C.c_int]
        L.or_check_stream.restype = C.c_int64
        L.or_check_stream.argtypes = [vp, vp, u64, u64, u64, C.c_int, C.c_uint32, C.c_int]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def gen_pages(n, seed, mode=0, ppm=10000, first_page=0, replica=False, stride=1):
    twin = np.empty((n, 4096), np.uint8)
    cur = np.empty((n, 4096), np.uint8)
    rep = np.empty((n, 4096), np.uint8) if replica else None
    lib().or_gen_pages(_p(twin), _p(cur), _p(rep), first_page, stride, n, seed, mode, ppm)
    return (twin, cur, rep) if replica else (twin, cur)


def diff_pages(twin, cur, ids=None, cap=None):
    """Returns (rec_off uint64[n+1], data uint8[total])."""
    n = len(ids) if ids is not None else twin.shape[0]
    ids_a = None if ids is None else np.ascontiguousarray(ids, np.uint32)
    rec_off = np.empty(n + 1, np.uint64)
    if cap is None:
        cap = n * 10244
    data = np.empty(max(cap, 1), np.uint8)
    total = lib().or_diff_pages(_p(np.ascontiguousarray(twin)), _p(np.ascontiguousarray(cur)),
                                _p(ids_a), n, _p(rec_off), _p(data), cap)
    return rec_off, data[:min(total, cap)].copy()


def apply(target, rec_off, data, ids=None):
    n = len(rec_off) - 1
    ids_a = None if ids is None else np.ascontiguousarray(ids, np.uint32)
    d = np.ascontiguousarray(data, np.uint8)
    if d.size == 0:
        d = np.zeros(1, np.uint8)
    return lib().or_apply(_p(target), _p(ids_a), n, _p(np.ascontiguousarray(rec_off, np.uint64)), _p(d))


def nw_diff(a: bytes, b: bytes):
    n = len(a) + len(b) + 1
    o1, o2 = C.create_string_buffer(n), C.create_string_buffer(n)
    L = C.c_size_t(0)
    rc = lib().or_nw_diff(a, len(a), b, len(b), o1, o2, C.byref(L))
    assert rc == 0
    return o1.raw[:L.value], o2.raw[:L.value]


def coh_init(n_pages, n_nodes=8):
    st = np.empty(n_pages, np.uint32)
    fl = np.empty(n_pages, np.uint32)
    lib().or_coh_init(_p(st), _p(fl), n_pages, n_nodes)
    return st, fl


def coherence(state, faults, events, n_nodes=8):
    ev = np.ascontiguousarray(events, np.uint64)
    tot = np.zeros(10, np.uint64)
    rc = lib().or_coherence(_p(state), _p(faults), len(state), n_nodes,
                            _p(ev) if len(ev) else None, len(ev), _p(tot))
    return rc, {"invalidations": int(tot[0]), "transfers": int(tot[1]),
                "node_faults": [int(x) for x in tot[2:]]}


def gen_events(counts, seed, n_nodes=8, write_pct=20, first_page=0):
    counts = np.ascontiguousarray(counts, np.uint64)
    offs = np.zeros(len(counts) + 1, np.uint64)
    np.cumsum(counts, out=offs[1:])
    ev = np.empty(int(offs[-1]), np.uint64)
    lib().or_gen_events(_p(ev) if len(ev) else None, _p(offs), first_page, len(counts), seed, n_nodes, write_pct)
    return ev


def ref_available() -> bool:
    return REF_DRIVER.exists()


def ref_nw_batch(cases):
    """Runs the REFERENCE diff() (oracle/_ref) on [(a, b)] (no NUL bytes) -> [(out1, out2)]."""
    import struct
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        cin, cout = Path(d) / "in.bin", Path(d) / "out.bin"
        with open(cin, "wb") as f:
            for a, b in cases:
                f.write(struct.pack("<II", len(a), len(b)) + a + b)
        subprocess.run([str(REF_DRIVER), "run", str(cin), str(cout)], check=True)
        raw = cout.read_bytes()
    out, i = [], 0
    while i < len(raw):
        (L,) = struct.unpack_from("<I", raw, i)
        i += 4
        out.append((raw[i:i + L], raw[i + L:i + 2 * L]))
        i += 2 * L
    return out


def check_stream(rec_off, data, first, n, seed, mode, ppm, threads=16):
    """The stream (rec_off[n + 1], data) of the SPEC §6 workload's pages [first, first + n)
    against the oracle, record by record, on `threads` OpenMP threads (tests only). Returns -1
    when it matches everywhere, else the first mismatching page index."""
    ro = np.ascontiguousarray(rec_off, np.uint64)
    d = np.ascontiguousarray(data, np.uint8)
    assert len(ro) == n + 1
    rc = lib().or_check_stream(_p(ro), _p(d) if len(d) else None, first, n, seed, mode, ppm,
                               threads)
    if rc == -2:
        raise MemoryError("or_check_stream")
    return int(rc)


def bench_diff_apply(n, mode, ppm, seed, seconds, threads):
    """bench.py's CPU baseline: `threads` OpenMP threads, each repeating diff + apply passes
    over its own n-page sample for `seconds` (timed in C). Returns (pages, seconds, replicas ok)."""
    pages, dt, ok = C.c_uint64(), C.c_double(), C.c_int()
    rc = lib().or_bench_diff_apply(n, mode, ppm, seed, seconds, threads, C.byref(pages),
                                   C.byref(dt), C.byref(ok))
    if rc:
        raise OSError(-rc, "or_bench_diff_apply")
    return pages.value, dt.value, bool(ok.value)


def bench_mmult(state, faults, nodes, twin, cur, rep, plan, rowvals, retwin=False):
    """bench.py's config-5 CPU baseline: the whole round loop in C on one thread
    (or_bench_mmult). plan = dict of flat arrays events / ev_off / ids / home / ids_off / row_dst
    / row_src / row_off. retwin: no twin step before a round's writes; the round's stream is
    applied to the twin views after the diff instead (gdsm_release's re-twin, the dirty bytes
    only); twin must equal cur at the start. Returns (seconds, totals[10])."""
    a = {k: np.ascontiguousarray(v) for k, v in plan.items()}
    rv = np.ascontiguousarray(rowvals, np.uint8)
    tot = np.zeros(10, np.uint64)
    dt = C.c_double()
    rounds = len(a["ev_off"]) - 1
    rc = lib().or_bench_mmult(_p(state), _p(faults), len(state), nodes, _p(twin), _p(cur),
                              _p(rep), rounds, _p(a["events"]), _p(a["ev_off"]), _p(a["ids"]),
                              _p(a["home"]), _p(a["ids_off"]), _p(a["row_dst"]),
                              _p(a["row_src"]), _p(a["row_off"]), _p(rv), rv.shape[1], _p(tot),
                              C.byref(dt), 1 if retwin else 0)
    if rc:
        raise RuntimeError(f"or_bench_mmult: {rc}")
    return dt.value, tot


def bench_coherence(counts, events, seconds, threads, n_nodes=8):
    """bench.py's coherence CPU baseline: `threads` OpenMP threads, each folding the events of its
    own contiguous page range of the batch (page counts `counts`) for `seconds` (timed in C).
    Returns (events folded, seconds)."""
    counts = np.ascontiguousarray(counts, np.uint64)
    offs = np.zeros(len(counts) + 1, np.uint64)
    np.cumsum(counts, out=offs[1:])
    ev = np.ascontiguousarray(events, np.uint64)
    done, dt = C.c_uint64(), C.c_double()
    rc = lib().or_bench_coherence(_p(ev), _p(offs), len(counts), n_nodes, seconds, threads,
                                  C.byref(done), C.byref(dt))
    if rc:
        raise OSError(-rc, "or_bench_coherence")
    return done.value, dt.value


# ---------------------------------------------------------------- SPEC §5b (multi-GPU coherence)
def _access(w, d):
    """Node d's access to pages with state words w: 0 none, 1 read, 2 write (SPEC §5b)."""
    w = np.asarray(w, np.uint32)
    st = (w >> 16) & 3
    held = ((w >> d) & 1).astype(bool) & (st != 0)
    own = (st == 2) & (((w >> 8) & 0xFF) == d)
    return np.where(held, np.where(own, 2, 1), 0).astype(np.uint64)


def notices(pre, post, pages, n_nodes):
    """Per node d < n_nodes: the notices (u64, SPEC §5b packing) for the pages `pages` (global
    ids, ascending, unique) whose state words went from pre to post, sorted by page. Node d gets
    one iff its access changed or it is the old or new owner of a page whose owner changed."""
    pre = np.asarray(pre, np.uint32)
    post = np.asarray(post, np.uint32)
    pages = np.asarray(pages, np.uint64)
    ob, oa = (pre >> 8) & 0xFF, (post >> 8) & 0xFF
    out = []
    for d in range(n_nodes):
        ab, aa = _access(pre, d), _access(post, d)
        m = (ab != aa) | ((ob != oa) & ((ob == d) | (oa == d)))
        out.append((pages[m] | (ab[m] << np.uint64(32)) | (aa[m] << np.uint64(34))
                    | (ob[m].astype(np.uint64) << np.uint64(40))
                    | (oa[m].astype(np.uint64) << np.uint64(48))).astype(np.uint64))
    return out


def route_round(state, faults, stamped, n_nodes, total_pages):
    """The multi-GPU protocol of SPEC §5b restated sequentially: the nodes' stamped events of one
    batch merged by (page, seq), folded into the whole page table (state, faults updated in
    place), and the notices each node receives. Returns (rc, totals, notices per node)."""
    ev = np.sort(np.concatenate([np.asarray(s, np.uint64) for s in stamped]) if stamped
                 else np.zeros(0, np.uint64), kind="stable")
    plain = (((ev >> np.uint64(36)) << np.uint64(4)) | (ev & np.uint64(15))).astype(np.uint64)
    pages = np.unique((plain >> np.uint64(4)).astype(np.int64))
    pre = state[pages].copy()
    rc, tot = coherence(state, faults, plain, n_nodes=n_nodes)
    return rc, tot, notices(pre, state[pages], pages.astype(np.uint64), n_nodes)
