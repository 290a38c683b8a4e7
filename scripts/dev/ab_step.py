"""Per-kernel times of the config-2 step in one process (HIP events from libgdsm's profiler):
diff alone, apply alone (re-applying the same stream is idempotent), and the serial step
diff -> apply, so that the cost one kernel leaves to the next shows up.

    AB_MODE=clustered python scripts/dev/ab_step.py"""
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402

import os  # noqa: E402

CLUSTERED = os.environ.get("AB_MODE") == "clustered"  # config-3 density (442 B records)
n = 1 << 20
ctx = ga.Context(n)
if CLUSTERED:
    ctx.gen_pages(seed=77, mode=ga.GEN_CLUSTERED, ppm=100000)
else:
    ctx.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
runs = ga.Runs(ctx, n, cap=n * (1024 if CLUSTERED else 256))
ctx.diff(out=runs)
ctx.apply(runs)
ctx.sync()
REPS = 10


def measure(fn):
    fn()
    ctx.sync()
    ctx.prof_enable(True)
    for _ in range(REPS):
        fn()
    ctx.sync()
    p = ctx.prof_read()
    ctx.prof_enable(False)
    return {k: round(v[0] / v[1], 4) for k, v in p.items() if v[1]}


def step():
    ctx.diff(out=runs)
    ctx.apply(runs)


res = {}
for r in range(3):
    for name, fn in [("diff", lambda: ctx.diff(out=runs)), ("step", step)]:
        res.setdefault(name, []).append(measure(fn))
    res.setdefault("apply", []).append(measure(lambda: ctx.apply(runs)))
for name, lst in res.items():
    keys = lst[0].keys()
    print(name, {k: statistics.median(d[k] for d in lst) for k in keys}, flush=True)
