"""Small driver for rocprofv3 PMC passes over coherence pass C (not product code): one batch of
`events` Zipf/uniform events over 16M pages with the chosen pass-C variant, run twice."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402
from gallocy_amd.workloads import event_counts  # noqa: E402

n_ev = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 28
dist = sys.argv[2] if len(sys.argv) > 2 else "uniform"
var = int(sys.argv[3]) if len(sys.argv) > 3 else 0
pages = 16 << 20
ctx = ga.Context(pages, arenas=())
ev = ctx.gen_events(event_counts(pages, n_ev, dist, seed=2026), seed=2026, n_nodes=8, write_pct=20)
assert gdsm.lib().gdsm_tune(b"coh_variant", var) == 0
for _ in range(2):
    ctx.coh_init(8)
    ctx.coherence_batch(ev)
print("ok")
