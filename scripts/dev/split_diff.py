"""Cost of splitting a rank's diff into one launch per destination (the N > 1 release shape):
2M pages (16M / 8 GPUs, 1 % words), one diff over all of them vs G diffs over contiguous
G-th slices (separate streams), per-step time from HIP events, same process.

    python scripts/dev/split_diff.py [pages] [G]"""
import statistics
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2 << 20
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ctx = ga.Context(n)
ctx.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
iota = ctx.ids(np.arange(n, dtype=np.uint32))
whole = ga.Runs(ctx, n, cap=n * 128)
per = n // G
parts = [ga.Runs(ctx, per, cap=per * 128) for _ in range(G)]


def one():
    ctx.diff(out=whole)


def split():
    for d in range(G):
        ctx.diff(iota.ptr + 4 * d * per, n=per, out=parts[d])


def split1():  # gdsm_diff_split: the same G streams from one launch
    ctx.diff_split([d * per for d in range(G + 1)], parts)


import time  # noqa: E402

res = {"one": [], "split": [], "split1": []}
wall = {"one": [], "split": [], "split1": []}
whole.total()  # the context learns the density (both shapes then take the same geometry)
for f in (one, split, split1):
    f()
    ctx.sync()
for r in range(5):
    for name, f in (("one", one), ("split", split), ("split1", split1)):
        ctx.sync()
        ctx.prof_enable(True)
        t0 = time.perf_counter()
        for _ in range(10):
            f()
        ctx.sync()
        wall[name].append((time.perf_counter() - t0) / 10 * 1e3)
        p = ctx.prof_read()
        ctx.prof_enable(False)
        res[name].append(p["diff"][0] / 10)
tot_one = whole.total()
tot_split = sum(x.total() for x in parts)
print(f"pages {n}, G {G}: one launch {statistics.median(res['one']):.4f} ms kernel / "
      f"{statistics.median(wall['one']):.4f} ms wall; {G} launches "
      f"{statistics.median(res['split']):.4f} ms kernels / {statistics.median(wall['split']):.4f} ms "
      f"wall; gdsm_diff_split {statistics.median(res['split1']):.4f} ms kernel / "
      f"{statistics.median(wall['split1']):.4f} ms wall per step; stream bytes {tot_one} vs "
      f"{tot_split}", flush=True)
