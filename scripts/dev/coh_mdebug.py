"""Debug aid for a pass-C variant: runs many small random batches (random page-table states,
1..40 events over 1..3 pages) through the GPU and the oracle and saves the smallest batch whose
results differ to gpurun_out/coh_min.npz.

    python scripts/dev/coh_mdebug.py [variant] [trials]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402
from oracle import oracle  # noqa: E402

variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
assert gdsm.lib().gdsm_tune(b"coh_variant", variant) == 0
best = None
with ga.Context(4, arenas=()) as c:
    for t in range(trials):
        rng = np.random.default_rng(t)
        npg = int(rng.integers(1, 4))
        nev = int(rng.integers(1, 41)) if t < trials // 2 else int(rng.integers(1, 3000))
        pages = np.sort(rng.integers(0, npg, nev)).astype(np.uint64)
        ev = (pages << np.uint64(4)) | (rng.integers(0, 8, nev).astype(np.uint64) << np.uint64(1)) \
            | (rng.integers(0, 100, nev) < int(rng.choice([0, 30, 70, 100]))).astype(np.uint64)
        st = rng.choice(np.array([0, 0x20102, 0x10003, 0x60404, 0x2000F, 0x40000], np.uint32), 4)
        fl = np.zeros(4, np.uint32)
        c.coh_init(8)
        c.coh_upload(st, fl)
        tot = c.coherence_batch(ev)
        gst, gfl = c.coh_download()
        ost, ofl = st.copy(), fl.copy()
        rc, otot = oracle.coherence(ost, ofl, ev)
        if tot != otot or not np.array_equal(gst, ost) or not np.array_equal(gfl, ofl):
            if best is None or nev < len(best["events"]):
                best = dict(events=ev, st0=st, gst=gst, gfl=gfl, ost=ost, ofl=ofl,
                            gtot=np.array([tot["invalidations"], tot["transfers"], *tot["node_faults"]]),
                            otot=np.array([otot["invalidations"], otot["transfers"], *otot["node_faults"]]))
                print("trial", t, "events", nev, flush=True)
gdsm.lib().gdsm_tune(b"coh_variant", 0)
Path("gpurun_out").mkdir(exist_ok=True)
if best is not None:
    np.savez("gpurun_out/coh_min.npz", **best)
    print("smallest failing batch:", len(best["events"]), [hex(int(x)) for x in best["events"]][:40])
    print("state gpu", [hex(int(x)) for x in best["gst"]], "oracle", [hex(int(x)) for x in best["ost"]])
    print("faults gpu", best["gfl"].tolist(), "oracle", best["ofl"].tolist())
    print("totals gpu", best["gtot"].tolist(), "oracle", best["otot"].tolist())
else:
    print("all", trials, "batches agree")
