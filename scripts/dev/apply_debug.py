import sys; sys.path.insert(0, '.')
import numpy as np
import gallocy_amd as ga
from gallocy_amd.gdsm import HostRuns, Runs
from oracle import oracle

def rec(runs, fill):
    hdr = [o | (l << 16) for o, l in runs]
    pay = bytes((fill + i) & 255 for i in range(sum(l for _, l in runs)))
    pay += b"\0" * ((-len(pay)) % 4)
    return np.array([len(runs)] + hdr, "<u4").tobytes() + pay

cases = [
  [[(16, 8)]],
  [[(0, 4)]],
  [[(3, 2)]],
  [[(16, 8), (40, 8)]],
  [[(16, 8)], [(32, 8)]],
  [[(16, 8)], [(32, 8)], [(48, 8)], [(64, 8)], [(80, 8)]],
  [[(100, 40)]],
  [[(0, 4096)]],
]
for ci, recs in enumerate(cases):
    n = len(recs)
    data = b"".join(rec(r, 10 * (k + 1)) for k, r in enumerate(recs))
    ro = np.zeros(n + 1, np.uint64)
    ro[1:] = np.cumsum([len(rec(r, 0)) for r in recs])
    d = np.frombuffer(data, np.uint8).copy()
    base = np.zeros((n, 4096), np.uint8)
    want = base.copy(); assert oracle.apply(want, ro, d) == 0
    with ga.Context(n) as c:
        c.upload("replica", base)
        c.apply(Runs.from_host(c, HostRuns(ro, d)))
        try:
            c.sync(); err = None
        except Exception as e:
            err = e
        got = c.download("replica")
    bad = np.argwhere(got != want)
    print(ci, "err" if err else "ok", "mismatches", len(bad), bad[:6].tolist(), [ (int(got[i,j]), int(want[i,j])) for i,j in bad[:6]])

# config-1-like: 64 pages, 1 % word writes
for n, mode, ppm in [(64, 0, 10000), (8, 0, 10000), (16, 0, 10000), (4, 0, 10000), (64, 1, 100000)]:
    t, cur = oracle.gen_pages(n, seed=1, mode=mode, ppm=ppm)
    ro, d = oracle.diff_pages(t, cur)
    with ga.Context(n) as c:
        c.upload("replica", t)
        c.apply(Runs.from_host(c, HostRuns(ro, d)))
        c.sync()
        got = c.download("replica")
    badp = [p for p in range(n) if not np.array_equal(got[p], cur[p])]
    print("n", n, "mode", mode, "bad pages", badp[:20], len(badp))
    if badp:
        p = badp[0]
        idx = np.flatnonzero(got[p] != cur[p])
        print("  page", p, "runs", HostRuns(ro, d).runs(p)[:8] and [(o, l) for o, l, _ in HostRuns(ro, d).runs(p)], "bad bytes", idx[:20].tolist())
