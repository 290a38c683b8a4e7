"""In-process A/B of coherence pass-C variants (gdsm_tune "coh_variant") on BASELINE config 4
(16M pages, 8 nodes, 20 % writes; events per batch and page distribution from the command
line): per-stage times from HIP events; the batch totals and the final page table must agree
between variants (the page table is re-initialised before every batch).

    python scripts/dev/ab_coh.py [events] [zipf|uniform] [variants, e.g. 0,1]"""
import statistics
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402
from gallocy_amd.workloads import event_counts  # noqa: E402

n_ev = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
dist = sys.argv[2] if len(sys.argv) > 2 else "zipf"
VALUES = [int(v) for v in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["0"])]
pages = 16 << 20
ctx = ga.Context(pages, arenas=())
ev = ctx.gen_events(event_counts(pages, n_ev, dist, seed=2026), seed=2026, n_nodes=8, write_pct=20)
res = {v: [] for v in VALUES}
tot, tables = {}, {}
for r in range(4):
    for v in VALUES:
        assert gdsm.lib().gdsm_tune(b"coh_variant", v) == 0
        ctx.coh_init(8)
        ctx.prof_enable(True)
        try:
            t = ctx.coherence_batch(ev)
        except gdsm.GdsmError:
            if v < 2:
                raise
            t = None  # measurement-only variants (invalid output) may flag the batch
        p = ctx.prof_read()
        ctx.prof_enable(False)
        res[v].append({k: x[0] / x[1] for k, x in p.items() if x[1]})
        assert tot.setdefault(v, t) == t or v >= 2
        if r == 0:
            tables[v] = ctx.coh_download()
gdsm.lib().gdsm_tune(b"coh_variant", 0)
for v in VALUES:
    keys = res[v][0].keys()
    print(f"coh_variant={v}:", {k: round(statistics.median(d[k] for d in res[v][1:]), 4) for k in keys},
          flush=True)
ref = VALUES[0]
for v in VALUES[1:]:
    if v >= 2:  # measurement-only variants (-DGDSM_MEASURE build)
        continue
    assert tot[v] == tot[ref], (v, tot[v], tot[ref])
    assert all(np.array_equal(a, b) for a, b in zip(tables[v], tables[ref])), v
print("totals and page tables agree:", tot[ref]["invalidations"], tot[ref]["transfers"])
