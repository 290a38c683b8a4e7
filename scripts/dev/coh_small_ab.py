"""Coherence batch time per variant at small batch sizes (kernel time from libgdsm's HIP events),
alternating variants: python scripts/dev/coh_small_ab.py [rounds]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd.workloads import event_counts  # noqa: E402

L = ga.gdsm.lib()
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for n_ev, n_pages in ((8192, 6011), (65536, 65536), (1 << 20, 1 << 18), (1 << 20, 16 << 20)):
    counts = event_counts(n_pages, n_ev, "uniform", seed=3)
    with ga.Context(n_pages, arenas=()) as c:
        ev = c.gen_events(counts, seed=3, n_nodes=8, write_pct=20)
        c.coh_init(8)
        tot = c.buffer(80)
        res = {}
        for r in range(rounds):
            for v in (2, 0, 1):
                assert L.gdsm_tune(b"coh_variant", v) == 0
                for _ in range(3):
                    L.gdsm_coherence_batch_async(c.handle, ev.ptr, ev.count, tot.ptr)
                c.sync()
                c.prof_enable(True)
                for _ in range(20):
                    L.gdsm_coherence_batch_async(c.handle, ev.ptr, ev.count, tot.ptr)
                c.sync()
                p = c.prof_read()
                c.prof_enable(False)
                res.setdefault(v, []).append(1e3 * p["coh_fold"][0] / p["coh_fold"][1])
        L.gdsm_tune(b"coh_variant", 0)
        print(f"events {ev.count} pages {n_pages}: " + ", ".join(
            f"v{v} {np.median(x):.2f} us" for v, x in sorted(res.items())), flush=True)
