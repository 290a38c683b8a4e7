"""NW stage times (fill, trace) of bench.py's nw workload, no result check: for measurement
builds selected with GDSM_LIB (e.g. variants that stop the trace after a phase).
    GDSM_LIB=gallocy_amd/<dir>/libgdsm.so python scripts/dev/nw_time.py [pairs] [steps]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ln = 4096
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (n, ln), dtype=np.uint8)
    b = a.copy()
    b.reshape(n, -1, 8)[rng.random((n, ln // 8)) < 0.01] ^= 0x5A
    off = np.arange(n + 1, dtype=np.uint64) * ln
    ctx = ga.Context(1, arenas=(), device=0)
    da, doff, db = (ctx.buffer(x.nbytes).upload(x) for x in (a, off, b))
    ob = 2 * n * ln + n
    o1, o2, ol = ctx.buffer(ob), ctx.buffer(ob), ctx.buffer(8 * n)
    L = _lib.load()

    def step():
        _lib.check(L.gdsm_nw_diff_batch(ctx.handle, da.ptr, doff.ptr, db.ptr, doff.ptr, n, ln,
                                        o1.ptr, o2.ptr, ol.ptr), "gdsm_nw_diff_batch")

    step()
    ctx.sync()
    ctx.prof_enable(True)
    ctx.prof_read()
    for _ in range(steps):
        step()
    ctx.sync()
    p = ctx.prof_read()
    print(_lib.LIB_PATH, {k: round(v[0] / v[1], 4) for k, v in p.items() if v[1]})
    ctx.close()


if __name__ == "__main__":
    main()
