"""Apply kernel alone on one workload (re-applying the same stream is idempotent), for rocprofv3
PMC passes and same-box A/B of apply variants (gdsm_tune "apply_variant").

    APPLY_MODE=clustered APPLY_PAGES=2097152 APPLY_VARIANTS=0,1 python scripts/dev/apply_only.py"""
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402

mode = os.environ.get("APPLY_MODE", "clustered")
n = int(os.environ.get("APPLY_PAGES", 1 << 21))
reps = int(os.environ.get("APPLY_REPS", 10))
variants = [int(v) for v in os.environ.get("APPLY_VARIANTS", "0").split(",")]
ctx = ga.Context(n)
if mode == "clustered":
    ctx.gen_pages(seed=77, mode=ga.GEN_CLUSTERED, ppm=100000)
    cap = n * 1024
else:
    ctx.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
    cap = n * 128
runs = ga.Runs(ctx, n, cap=cap)
ctx.diff(out=runs)
ctx.sync()
total = runs.total()
L = gdsm.lib()
res = {}
for rnd in range(3):
    for v in variants:
        assert L.gdsm_tune(b"apply_variant", v) == 0
        ctx.apply(runs)
        ctx.sync()
        ctx.prof_enable(True)
        for _ in range(reps):
            ctx.apply(runs)
        ctx.sync()
        p = ctx.prof_read()
        ctx.prof_enable(False)
        res.setdefault(v, []).append(p["apply"][0] / p["apply"][1])
L.gdsm_tune(b"apply_variant", 0)
# correctness of the last variant: REPLICA == CURRENT
chk = ga.Runs(ctx, n, cap=1 << 20)
ws = ctx.buffer(L.gdsm_diff_workspace_bytes(n))
rc = L.gdsm_diff_raw(ctx.arena_ptr("replica"), ctx.arena_ptr("current"), None, n, chk.s.rec_off,
                     chk.s.data, chk.cap, ws.ptr, ws.nbytes, ctx.stream)
ok = rc == 0 and chk.total() == 0
for v, ts in res.items():
    ms = statistics.median(ts)
    print(f"apply_variant={v} {mode} n={n} stream={total} B: {ms:.4f} ms "
          f"({2 * total / ms / 1e9:.0f} GB/s of stream read + payload written, approx) "
          f"replica_ok={ok}", flush=True)
