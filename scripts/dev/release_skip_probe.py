"""What bounds the chained release of a few dense pages? A -DGDSM_MEASURE build's kSkip variants
of the one-wave-per-workgroup chained kernel (output invalid), each timed by rocprofv3
--kernel-trace on m dense pages (doubles holding integers against zero twins, config 5's rows):
1 no home-apply stores, 2 no late-record stores, 4 no re-twin stores, 5 = 1 + 4, 8 no late path,
13 = 1 + 4 + 8, 16 no look-back, 32 no buffered-record copy, 61 all of them; 0 the product kernel.
TWIN is zeroed again by a copy kernel between launches; the case "clean" (CURRENT == TWIN) last.

    scripts/dev/build_measure.sh
    GDSM_LIB=gallocy_amd/lib_x/libgdsm.so rocprofv3 --kernel-trace -d DIR -o run -- \\
        python scripts/dev/release_skip_probe.py [m] [reps]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402

PAGE = 4096
SKIPS = (0, 1, 2, 4, 5, 8, 13, 16, 32, 61)


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    L = ga.gdsm.lib()
    ctx = ga.Context(64, arenas=("twin", "current", "replica"))
    zeros = np.zeros((64, PAGE), np.uint8)
    d_zero = ctx.buffer(64 * PAGE).upload(zeros)
    ctx.upload("twin", zeros)
    rng = np.random.default_rng(3)
    cur = rng.integers(1, 1 << 20, size=(m, PAGE // 8)).astype(np.float64).view(np.uint8)
    ids = ctx.ids(np.arange(m, dtype=np.uint32))
    out = ga.Runs(ctx, m, m * 10244)
    desc = ctx.buffer(24).upload(np.array([ctx.arena_ptr("twin"), d_zero.ptr, m * PAGE], np.uint64))
    for case in ("dense", "clean"):
        ctx.upload("current", cur.reshape(m, PAGE) if case == "dense" else zeros[:m])
        for k in (SKIPS if case == "dense" else (0,)):
            assert L.gdsm_tune(b"diff_skip", k) == 0, "needs the -DGDSM_MEASURE build (GDSM_LIB)"
            for _ in range(reps):
                L.gdsm_memcpy_batch(ctx.handle, desc.ptr, 1)
                ctx.release(ids, out=out, apply_to="replica", target_ids=ids)
            ctx.sync()
            print(case, k, flush=True)
    L.gdsm_tune(b"diff_skip", 0)
    ctx.close()


if __name__ == "__main__":
    main()
