"""Times the GPU NW (gdsm_nw_diff_batch) on batches of 4 KiB page pairs with sparse writes
(BASELINE config 1 shape) and prints one line per batch: ms, DP cells/s, per-kernel HIP events."""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, nargs="+", default=[64, 512])
    ap.add_argument("--len", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    rng = np.random.default_rng(1)
    L = _lib.load()
    with ga.Context(1, arenas=()) as ctx:
        for n in args.pairs:
            a = rng.integers(0, 256, (n, args.len), dtype=np.uint8)
            b = a.copy()
            w = rng.random((n, args.len // 8)) < 0.01
            b.reshape(n, -1, 8)[w] ^= 0x5A
            off = np.arange(n + 1, dtype=np.uint64) * args.len
            bufs = [ctx.buffer(x.nbytes).upload(x) for x in (a, off, b)]
            ob = 2 * n * args.len + n
            o1, o2, ol = ctx.buffer(ob), ctx.buffer(ob), ctx.buffer(8 * n)

            def run():
                _lib.check(L.gdsm_nw_diff_batch(ctx.handle, bufs[0].ptr, bufs[1].ptr, bufs[2].ptr,
                                                bufs[1].ptr, n, args.len, o1.ptr, o2.ptr, ol.ptr))
            run()
            ctx.prof_enable(True)
            ctx.prof_read()
            t = time.perf_counter()
            for _ in range(args.reps):
                run()
            dt = (time.perf_counter() - t) / args.reps
            p = ctx.prof_read()
            ctx.prof_enable(False)
            cells = n * (args.len + 1) ** 2
            fill = p["nw_fill"][0] / max(p["nw_fill"][1], 1)
            trace = p["nw_trace"][0] / max(p["nw_trace"][1], 1)
            print(f"pairs={n} len={args.len} wall={dt * 1e3:.3f} ms cells/s={cells / dt:.3e} "
                  f"fill={fill:.3f} ms trace={trace:.3f} ms "
                  f"fill_cells/s={cells / (fill * 1e-3):.3e}", flush=True)
            lens = ol.download(np.uint64, n)
            assert (lens == args.len).all(), lens[:8]  # substitution-only: gap-free
            for x in (*bufs, o1, o2, ol):
                x.free()


if __name__ == "__main__":
    main()
