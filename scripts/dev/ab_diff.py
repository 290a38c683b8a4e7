"""In-process A/B of diff kernel variants (interleaved rounds, one device): per-launch time of
diff_pages_kernel from HIP events, for BASELINE config 2 (1M pages, 1 % word writes).

    python scripts/dev/ab_diff.py diff_variant 0,1,2

Every variant produces the same canonical stream; the totals are checked to agree."""
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402

KEY = sys.argv[1] if len(sys.argv) > 1 else "diff_variant"
VALUES = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1"])]
import os  # noqa: E402

ROUNDS, REPS = 6, 10
n = int(os.environ.get("AB_PAGES", 1 << 20))  # pages (default config 2's 1M)
ctx = ga.Context(n)

if os.environ.get("AB_MODE") == "clustered":  # config-3 density (442 B records)
    ctx.gen_pages(seed=77, mode=ga.GEN_CLUSTERED, ppm=100000)
else:
    ctx.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
runs = ga.Runs(ctx, n, cap=n * 1024)
total = None
res = {v: [] for v in VALUES}
full = {}
for r in range(ROUNDS):
    for v in VALUES:
        assert gdsm.lib().gdsm_tune(KEY.encode(), v) == 0
        ctx.diff(out=runs)
        ctx.sync()
        ctx.prof_enable(True)
        for _ in range(REPS):
            ctx.diff(out=runs)
        p = ctx.prof_read()
        ctx.prof_enable(False)
        res[v].append(p["diff"][0] / p["diff"][1])
        full.setdefault(v, []).append(sum(p[k][0] for k in ("diff",)) / REPS)
        if True:
            t = runs.total()
            assert total is None or t == total, (v, t, total)
            total = t
gdsm.lib().gdsm_tune(KEY.encode(), 0)
for v in VALUES:
    ms = res[v]
    gbs = (n * 8192 + (total or 0)) / (statistics.median(ms) * 1e-3) / 1e9
    print(f"{KEY}={v}: median {statistics.median(ms):.4f} ms  min {min(ms):.4f} ms  -> {gbs:.0f} GB/s"
          f"  (diff+scan+pack per call: {statistics.median(full[v]):.4f} ms)", flush=True)
