"""In-process A/B of the twin kernel geometries (gdsm_tune "twin_variant") on the north-star
pages: one allocation, variants alternating, median kernel time per variant."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402

n = 16 << 20
L = ga.gdsm.lib()
ctx = ga.Context(n, arenas=("twin", "current"))
ctx.gen_pages(seed=1, mode=ga.GEN_UNIFORM, ppm=10000, arenas=("twin", "current"))
res = {}
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    for v in (0, 1, 2, 3, 4):
        assert L.gdsm_tune(b"twin_variant", v) == 0
        ctx.twin()
        ctx.sync()
        ctx.prof_enable(True)
        for _ in range(5):
            ctx.twin()
        ctx.sync()
        p = ctx.prof_read()
        ctx.prof_enable(False)
        res.setdefault(v, []).append(p["twin"][0] / p["twin"][1])
L.gdsm_tune(b"twin_variant", 0)
assert ctx.diff(cap=1 << 20).total() == 0
for v, x in sorted(res.items()):
    print(f"v{v}: median {np.median(x):.3f} ms ({137.44 / np.median(x):.2f} TB/s) all {[round(t, 2) for t in x]}")
