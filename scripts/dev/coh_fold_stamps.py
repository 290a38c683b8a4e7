"""Debug aid for the coherence fold kernel (needs the -DGDSM_COH_STAMPS build,
scripts/dev/build_stamps.sh, loaded with GDSM_LIB=gallocy_amd/lib_st/libgdsm.so): per-wave phase
durations (s_memtime ticks) of every 16th block on a config-4 batch, split by block kind.

    python scripts/dev/coh_fold_stamps.py [events] [zipf|uniform]"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402
from gallocy_amd.workloads import event_counts  # noqa: E402

n_ev = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
dist = sys.argv[2] if len(sys.argv) > 2 else "zipf"
pages = 16 << 20
L = gdsm.lib()
ctx = ga.Context(pages, arenas=())
ev = ctx.gen_events(event_counts(pages, n_ev, dist, seed=2026), seed=2026, n_nodes=8, write_pct=20)
assert L.gdsm_tune(b"coh_variant", 0) == 0
for _ in range(2):
    ctx.coh_init(8)
    ctx.coherence_batch(ev)
buf = np.zeros(8192 * 4 * 8, np.uint64)
L.gdsm_debug_coh_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert L.gdsm_debug_coh_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(-1, 8)
nb = n_ev // 2048
st = st[: nb // 16]
st = st[st[:, 4] > 0]
t = st[:, :5].astype(np.int64)
info = st[:, 5]
ordered = (info & 1).astype(bool)
heads = ((info >> 1) & 0x7F).astype(np.int64)
rounds = (info >> 16).astype(np.int64)
d = np.diff(t, axis=1)  # load, walk, look-back, tail
# the walk phase split: heads pass [1 -> 6], gathers landed [6 -> 7], walk proper [7 -> 2]
hp, ga, wk = st[:, 6].astype(np.int64) - t[:, 1], st[:, 7].astype(np.int64) - st[:, 6].astype(np.int64), t[:, 2] - st[:, 7].astype(np.int64)
print(f"walk phase split (means): heads pass {hp.mean():.0f}  gathers landed {ga.mean():.0f}  walk {wk.mean():.0f}")
start = t[:, 0] - t[:, 0].min()
print(f"{dist}: waves sampled {len(t)}, span {(t[:, 4].max() - t[:, 0].min())} ticks")
kinds = {
    "no head (hot interior/closing)": heads == 0,
    "1-8 head lanes": (heads >= 1) & (heads <= 8),
    "9-32 head lanes": (heads > 8) & (heads <= 32),
    "33-64 head lanes": heads > 32,
}
names = ["load", "walk", "look-back", "tail"]
for kn, m in list(kinds.items()) + [("ordered", ordered), ("all", np.ones(len(t), bool))]:
    if not m.any():
        continue
    parts = "  ".join(f"{nm} {d[m, i].mean():8.0f}" for i, nm in enumerate(names))
    print(f"{kn:32s} n={m.sum():6d}  {parts}  total {(t[m, 4] - t[m, 0]).mean():8.0f}  "
          f"rounds {rounds[m].mean():.2f} (max {rounds[m].max()})")
lb = d[:, 2]
for q in (50, 90, 99, 99.9):
    print(f"look-back p{q}: {np.percentile(lb, q):.0f}")
big = np.argsort(lb)[-8:]
for i in big:
    print("slow look-back: heads", heads[i], "ordered", ordered[i], "rounds", rounds[i], "ticks", lb[i])
