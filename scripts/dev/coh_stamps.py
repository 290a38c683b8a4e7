"""Debug aid (needs a -DGDSM_COH_STAMPS build loaded with GDSM_LIB): average per-wave phase
durations of pass C (s_memtime ticks) on a config-4 batch."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402
from gallocy_amd.workloads import event_counts  # noqa: E402

n_ev = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
dist = sys.argv[2] if len(sys.argv) > 2 else "uniform"
pages = 16 << 20
L = gdsm.lib()
ctx = ga.Context(pages, arenas=())
ev = ctx.gen_events(event_counts(pages, n_ev, dist, seed=2026), seed=2026, n_nodes=8, write_pct=20)
assert L.gdsm_tune(b"coh_variant", int(sys.argv[3]) if len(sys.argv) > 3 else 0) == 0
for _ in range(2):
    ctx.coh_init(8)
    ctx.coherence_batch(ev)
buf = np.zeros(8192 * 4 * 8, np.uint64)
L.gdsm_debug_coh_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert L.gdsm_debug_coh_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(-1, 8).astype(np.int64)
nb = (n_ev + 2047) // 2048
used = st[: min(8192, (nb + 63) // 64) * 4]
used = used[used[:, 0] > 0]
d = np.diff(used, axis=1)
names = ["launch->P1", "P1", "P2+loader", "P3", "barrier", "carry", "walk", "P5+P6"]
print("waves sampled", len(used))
for i, nm in enumerate(names[1:]):
    print(f"{nm:12s} mean {d[:, i].mean():9.1f}  median {np.median(d[:, i]):9.1f}")
print("total", (used[:, 7] - used[:, 0]).mean())
