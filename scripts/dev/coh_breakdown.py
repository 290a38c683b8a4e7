"""Config-4 fold time per measurement variant (a -DGDSM_MEASURE build, scripts/dev/build_measure.sh;
output invalid for 4-6): 2 = the fold, 4 = no walk, 5 = no look-back, 6 = no ordered look-back.
    GDSM_LIB=gallocy_amd/lib_x/libgdsm.so python scripts/dev/coh_breakdown.py [uniform|zipf]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd.workloads import event_counts  # noqa: E402

L = ga.gdsm.lib()
dist = sys.argv[1] if len(sys.argv) > 1 else "uniform"
n_pages, n_ev = 16 << 20, 1 << 30
counts = event_counts(n_pages, n_ev, dist, seed=3)
with ga.Context(n_pages, arenas=()) as c:
    ev = c.gen_events(counts, seed=3, n_nodes=8, write_pct=20)
    c.coh_init(8)
    tot = c.buffer(80)
    res = {}
    for r in range(3):
        for v in (2, 4, 5, 6):
            assert L.gdsm_tune(b"coh_variant", v) == 0
            L.gdsm_coherence_batch_async(c.handle, ev.ptr, ev.count, tot.ptr)
            c.sync()
            c.prof_enable(True)
            for _ in range(5):
                L.gdsm_coherence_batch_async(c.handle, ev.ptr, ev.count, tot.ptr)
            try:
                c.sync()
            except ga.gdsm.GdsmError:
                pass
            p = c.prof_read()
            c.prof_enable(False)
            res.setdefault(v, []).append(p["coh_fold"][0] / p["coh_fold"][1])
    L.gdsm_tune(b"coh_variant", 0)
    print(dist, {v: round(float(np.median(x)), 3) for v, x in sorted(res.items())}, flush=True)
