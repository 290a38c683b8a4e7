"""Regenerates the committed fixtures under tests/golden/. Run in the build container, where
/root/reference exists (the GPU box has no reference tree; the tests only READ these files).

  nw_ref.npz     inputs and outputs of the REFERENCE diff() (gallocy/utils/diff.cpp:73-167),
                 produced by oracle/_ref/ref_nw_driver compiled from the reference sources.
                 Cases: the three test_diff.cpp tests (13-16, 24-31, 38-57 shape), the SURVEY §8c
                 KATs, random lengths 0..1180 (its largest working size), substitution-only
                 equal-length pairs (the bridge to the page diff), shifted content.
  pages.npz      page diff vectors from the C oracle (docs/SPEC.md §3): edge-case pages and
                 seeded synthetic pages with their expected rec_off/data. PARITY UNPINNED by the
                 reference (it has no page diff); these pin the oracle against drift.
  c1_windows.npz BASELINE config 1 (64 x 4 KiB pages, SPEC §6 seed 1, 1 % word writes) cut into
                 256 windows of 1024 B (test/test_diff.cpp:38-57 shape, under the reference's
                 1180-B limit) after the byte remap tests/helpers.py:c1_remap (no NUL, no '-': the reference
                 returns NUL-terminated alignments with '-' gaps and no length, diff.h:9-11),
                 each window pair run through the REFERENCE diff() (oracle/_ref). Stored: the
                 alignment length, crc32 of both alignment strings, and the positions where
                 out1[i] != out2[i] (bit-packed). This pins the page diff / apply to the
                 reference itself wherever its alignment is gap-free.
  ref_windows.npz the same for more page sets (tests/helpers.py:REF_WINDOW_SETS): 64 pages of
                 BASELINE config 3's clustered workload, a dense set (40 % of the words
                 rewritten) and the SPEC edge pages of pages.npz; keys '<set>_<field>'. Windows
                 whose reference alignment has gaps keep only L and the crc32s.
  raw_windows.npz BASELINE's own bytes with no remap: the north-star generator's pages (SPEC §6
                 uniform 1 %, seed 2026; config 2's are its first 1M) in two ranges of 65 536
                 pages (the first and the last of the 16M), every 1024-B window whose bytes hold
                 neither NUL nor '-' (tests/helpers.py:RAW_RANGES), through the reference diff().
  ref_layout.npz zone offsets of test_mmult's objects (test/test_mmult.cpp:31-37, 152-154) as
                 the REFERENCE custom_malloc hands them out (libgallocy.cpp over
                 heaplayers/application.h:20-29, compiled in place into
                 oracle/_ref/ref_layout_driver) for NDIM 4, 64,
                 1000 and 1021, and the abort (---ENOMEM---, source.h:23-24) at NDIM 1022 with
                 the objects allocated before it.
  coherence.npz  a seeded event batch and its expected page table / totals from the C oracle
                 (SPEC §5, parity unpinned by the reference, which has no coherence logic).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle  # noqa: E402
from tests.helpers import (RAW_RANGES, REF_WINDOW_SETS, c1_windows, raw_range_pages,  # noqa: E402
                           raw_windows, window_pages)

OUT = Path(__file__).resolve().parent


def _nz(rng, n):
    # no NUL bytes: the reference returns NUL-terminated strings without a length (diff.h:9-11)
    return bytes(rng.integers(1, 256, n, dtype=np.uint8))


def nw_cases():
    rng = np.random.default_rng(20261015)
    cases = [(b"GGAATGG", b"ATG"), (b"FOO BOP BOOP", b"FOOO BOOP BOP"),
             (b"", b""), (b"", b"ABC"), (b"ABC", b""), (b"AB", b"BA"), (b"ABCD", b"BCDA"),
             (b"AAAA", b"AA"), (b"AA", b"AAAA"), (b"ACGT", b"TGCA"), (b"HELLO", b"YELLOW"),
             (b"0123456789", b"0123X56789")]
    # test_diff.cpp:38-57 shape: 512 random bytes, ~10 % substituted
    for _ in range(4):
        a = bytearray(_nz(rng, 512))
        b = bytearray(a)
        for i in range(512):
            if rng.integers(0, 10) == 1:
                b[i] = int(rng.integers(1, 256))
        cases.append((bytes(a), bytes(b)))
    # random lengths up to the reference's largest working size (1180)
    for n, m in [(1, 1), (7, 13), (64, 64), (100, 37), (255, 256), (600, 590), (1024, 1024),
                 (1180, 1180), (1180, 1)]:
        cases.append((_nz(rng, n), _nz(rng, m)))
    # substitution-only equal length, byte-diff structure like a page diff
    for n in (16, 64, 200, 777, 1024):
        a = bytearray(_nz(rng, n))
        b = bytearray(a)
        for _ in range(int(rng.integers(1, max(2, n // 20)))):
            o = int(rng.integers(0, n))
            ln = int(rng.integers(1, 9))
            for j in range(o, min(n, o + ln)):
                b[j] = (a[j] % 255) + 1 if rng.integers(0, 4) else a[j]
        cases.append((bytes(a), bytes(b)))
    # shifted content (memmove by one byte): where NW stops being a positional diff
    a = _nz(rng, 300)
    cases.append((a, a[:100] + a[101:151] + a[100:101] + a[151:]))
    return cases


def make_nw():
    cases = nw_cases()
    outs = oracle.ref_nw_batch(cases)
    lens = np.array([[len(a), len(b), len(o1)] for (a, b), (o1, o2) in zip(cases, outs)], np.int64)
    blob = b"".join(a + b + o1 + o2 for (a, b), (o1, o2) in zip(cases, outs))
    np.savez_compressed(OUT / "nw_ref.npz", lens=lens, blob=np.frombuffer(blob, np.uint8))
    print("nw_ref.npz", len(cases), "cases")


def edge_pages():
    rng = np.random.default_rng(7)
    base = rng.integers(0, 256, 4096, dtype=np.uint8)
    pages = []

    def var(fn):
        t = base.copy()
        c = base.copy()
        fn(c)
        pages.append((t, c))

    var(lambda c: None)                                # clean page
    var(lambda c: c.__setitem__(slice(None), c ^ 0xFF))  # every byte changed: one 4096-B run
    var(lambda c: c.__setitem__(slice(0, None, 2), c[0::2] ^ 1))  # alternating: 2048 runs
    var(lambda c: c.__setitem__(0, c[0] ^ 1))          # first byte
    var(lambda c: c.__setitem__(4095, c[4095] ^ 1))    # last byte
    var(lambda c: c.__setitem__(slice(15, 17), c[15:17] ^ 3))      # run across a 16-B chunk edge
    var(lambda c: c.__setitem__(slice(1000, 3000), c[1000:3000] ^ 0x5A))  # run over many chunks
    var(lambda c: c.__setitem__(slice(1023, 1025), c[1023:1025] ^ 9))  # across lanes' k wrap
    var(lambda c: c.__setitem__(slice(4095 - 16, 4096), c[4079:] ^ 1))  # tail run
    def sparse(c):
        idx = rng.choice(4096, 37, replace=False)
        c[idx] ^= rng.integers(1, 256, 37, dtype=np.uint8)
    var(sparse)
    def words(c):  # word writes where some bytes happen to be equal
        for w in rng.choice(512, 9, replace=False):
            x = rng.integers(0, 256, 8, dtype=np.uint8)
            x[rng.integers(0, 8)] = 0
            c[w * 8:w * 8 + 8] ^= x
    var(words)
    twin = np.stack([t for t, _ in pages])
    cur = np.stack([c for _, c in pages])
    return twin, cur


def make_pages():
    twin, cur = edge_pages()
    ro, data = oracle.diff_pages(twin, cur)
    t2, c2 = oracle.gen_pages(64, seed=1, mode=0, ppm=10000)  # config 1: 64 pages, 1 % words
    ro2, data2 = oracle.diff_pages(t2, c2)
    t3, c3 = oracle.gen_pages(16, seed=3, mode=1, ppm=100000, first_page=1 << 20)  # clustered
    ro3, data3 = oracle.diff_pages(t3, c3)
    np.savez_compressed(OUT / "pages.npz", edge_twin=twin, edge_cur=cur, edge_rec_off=ro,
                        edge_data=data, c1_rec_off=ro2, c1_data=data2, c1_cur_head=c2[:2],
                        cl_rec_off=ro3, cl_data=data3)
    print("pages.npz", twin.shape[0], "edge pages;", int(ro2[-1]), "B for config 1")


def _ref_windows(t, c, sel=None):
    """The pages cut into 1024-B windows (those listed in `sel`, else all), each pair aligned by
    the REFERENCE diff(): alignment length, crc32 of both strings, gap-free flag and (gap-free
    windows) the bit-packed positions where out1[i] != out2[i]."""
    import zlib
    tw, cw = t.reshape(-1, 1024), c.reshape(-1, 1024)
    if sel is not None:
        tw, cw = tw[sel], cw[sel]
    cases = [(tw[i].tobytes(), cw[i].tobytes()) for i in range(len(tw))]
    outs = oracle.ref_nw_batch(cases)
    L = np.array([len(o1) for o1, _ in outs], np.int64)
    crc = np.array([[zlib.crc32(o1), zlib.crc32(o2)] for o1, o2 in outs], np.uint32)
    mask = np.zeros((len(cases), 128), np.uint8)
    gapfree = np.zeros(len(cases), bool)
    for i, (o1, o2) in enumerate(outs):
        if len(o1) == 1024 and b"-" not in o1 + o2:
            gapfree[i] = True
            a, b = np.frombuffer(o1, np.uint8), np.frombuffer(o2, np.uint8)
            mask[i] = np.packbits(a != b)
    return {"L": L, "crc": crc, "gapfree": gapfree, "mask": mask}


def make_c1_windows():
    d = _ref_windows(*c1_windows())
    np.savez_compressed(OUT / "c1_windows.npz", **d)
    print("c1_windows.npz", len(d["L"]), "windows,", int(d["gapfree"].sum()), "gap-free")


def make_ref_windows():
    """ref_windows.npz: the page sets of tests/helpers.py:REF_WINDOW_SETS (config 3's clustered
    pages, a dense set, the SPEC edge pages) through the reference diff(), keys '<set>_<field>'."""
    golden = {"pages": np.load(OUT / "pages.npz")}
    out = {}
    for name in REF_WINDOW_SETS:
        d = _ref_windows(*window_pages(name, golden))
        out.update({f"{name}_{k}": v for k, v in d.items()})
        print(name, len(d["L"]), "windows,", int(d["gapfree"].sum()), "gap-free")
    np.savez_compressed(OUT / "ref_windows.npz", **out)


def make_raw_windows():
    """raw_windows.npz: BASELINE's own bytes, unremapped (tests/helpers.py:RAW_RANGES): every
    window of the two north-star page ranges that holds no 0x00 / 0x2D byte, through the
    reference diff(); keys 'r<i>_<field>' plus 'r<i>_win' (window index inside the range)."""
    out = {}
    for i, (first, n) in enumerate(RAW_RANGES):
        t, c = raw_range_pages(first, n)
        win = raw_windows(t, c)
        d = _ref_windows(t, c, win)
        out.update({f"r{i}_{k}": v for k, v in d.items()})
        out[f"r{i}_win"] = win.astype(np.int64)
        out[f"r{i}_range"] = np.array([first, n], np.int64)
        dirty = d["mask"].any(axis=1)
        print(f"range {first}+{n}:", len(win), "windows,", int(d["gapfree"].sum()), "gap-free,",
              int((dirty & d["gapfree"]).sum()), "gap-free with changes")
    np.savez_compressed(OUT / "raw_windows.npz", **out)


LAYOUT_DRIVER = ROOT / "oracle" / "_ref" / "ref_layout_driver"
LAYOUT_NDIMS = (4, 64, 1000, 1021)


def _layout_run(ndim):
    import subprocess
    r = subprocess.run([str(LAYOUT_DRIVER), str(ndim)], capture_output=True, text=True)
    rows = {"a": [], "b": [], "c": []}
    one = {}
    for ln in r.stdout.splitlines():
        f = ln.split()
        if len(f) == 3 and f[0].endswith("_row"):
            rows[f[0][0]].append(int(f[2]))
        elif len(f) == 2:
            one[f[0]] = int(f[1])
    return r, one, rows


def make_layout():
    if not LAYOUT_DRIVER.exists():
        raise SystemExit("oracle/_ref/ref_layout_driver missing: run `make -C oracle layout` first")
    out = {}
    for nd in LAYOUT_NDIMS:
        r, one, rows = _layout_run(nd)
        assert r.returncode == 0, r.stderr
        out[f"n{nd}_rp"] = np.array([one["a_rp"], one["b_rp"], one["c_rp"]], np.int64)
        out[f"n{nd}_rows"] = np.array([rows["a"], rows["b"], rows["c"]], np.int64)
        out[f"n{nd}_tail"] = np.array([one["threads"], one["args"], one["zone_used_min"]], np.int64)
    r, one, rows = _layout_run(1022)
    assert r.returncode != 0 and "---ENOMEM---" in r.stdout, (r.returncode, r.stdout[-200:])
    out["abort_1022"] = np.array([r.returncode, sum(len(v) for v in rows.values()) + len(one)],
                                 np.int64)
    np.savez_compressed(OUT / "ref_layout.npz", ndims=np.array(LAYOUT_NDIMS), **out)
    print("ref_layout.npz", LAYOUT_NDIMS, "abort at 1022 after", int(out["abort_1022"][1]),
          "objects, status", int(out["abort_1022"][0]))


def make_coherence():
    rng = np.random.default_rng(11)
    n_pages = 64
    counts = rng.integers(0, 40, n_pages).astype(np.uint64)
    counts[5] = 3000  # a hot page
    ev = oracle.gen_events(counts, seed=5, n_nodes=8, write_pct=20)
    st, fl = oracle.coh_init(n_pages, 8)
    rc, tot = oracle.coherence(st, fl, ev)
    assert rc == 0
    np.savez_compressed(OUT / "coherence.npz", counts=counts, events=ev, state=st, faults=fl,
                        totals=np.array([tot["invalidations"], tot["transfers"], *tot["node_faults"]],
                                        np.uint64))
    print("coherence.npz", len(ev), "events", tot)


if __name__ == "__main__":
    if not oracle.ref_available():
        raise SystemExit("oracle/_ref/ref_nw_driver missing: run `make -C oracle ref` here first")
    which = sys.argv[1:] or ["nw", "pages", "coherence", "c1_windows", "ref_windows", "layout",
                             "raw_windows"]
    for w in which:
        {"nw": make_nw, "pages": make_pages, "coherence": make_coherence,
         "c1_windows": make_c1_windows, "ref_windows": make_ref_windows,
         "raw_windows": make_raw_windows,
         "layout": make_layout}[w]()
