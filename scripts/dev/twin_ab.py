"""In-process A/B of the twin kernel geometries on the north-star pages: one allocation, variants
alternating, median kernel time per variant. The round-4 measurement ran with a
gdsm_tune("twin_variant") knob (0 one page per wave step, 1 two pages + nontemporal loads, 2 two
pages + nontemporal loads and stores, 3 one page, both nontemporal, 4 four pages); the knob was
removed with the result, so this now times the kept kernel only."""
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
    for v in (0,):
        ctx.twin()
        ctx.sync()
        ctx.prof_enable(True)
        for _ in range(5):
            ctx.twin()
        ctx.sync()
        p = ctx.prof_read()
        ctx.prof_enable(False)
        res.setdefault(v, []).append(p["twin"][0] / p["twin"][1])
assert ctx.diff(cap=1 << 20).total() == 0
for v, x in sorted(res.items()):
    print(f"v{v}: median {np.median(x):.3f} ms ({137.44 / np.median(x):.2f} TB/s) all {[round(t, 2) for t in x]}")
