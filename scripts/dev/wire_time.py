"""Times the diff wire format on BASELINE config 2 (1M pages, 1 % word writes): GPU diff ->
gdsm_wire_encode (frame + checksum + base64 on the GPU, text D2H) -> gdsm_wire_apply (text H2D,
base64 decode + verify + apply on the GPU), with per-kernel times from rocprofv3 if run under it."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    with ga.Context(n) as ctx:
        ctx.gen_pages(seed=2026, mode=ga.GEN_UNIFORM, ppm=10000)
        runs = ctx.diff()
        D = runs.total()
        text = ctx.wire_encode(runs)
        reps = 10
        t = time.perf_counter()
        for _ in range(reps):
            text = ctx.wire_encode(runs)
        te = (time.perf_counter() - t) / reps
        t = time.perf_counter()
        for _ in range(reps):
            ctx.wire_apply(text)
        ta = (time.perf_counter() - t) / reps
        ok = np.array_equal(ctx.download("replica", 0, 4096), ctx.download("current", 0, 4096))
        print(f"pages={n} stream={D} B text={len(text)} B encode={te * 1e3:.3f} ms "
              f"({len(text) / te / 1e9:.2f} GB/s text) apply={ta * 1e3:.3f} ms "
              f"({len(text) / ta / 1e9:.2f} GB/s text) replica_ok={ok}", flush=True)


if __name__ == "__main__":
    main()
