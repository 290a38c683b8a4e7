"""Where does a short release's time go? (config 5: a round's release of ~12 dense pages, ~500 runs
each, was one diff_single_kernel<..., kSolo> launch of ~13 us, the round's critical path.)

Pages of doubles holding integers (C = A x B of test_mmult: two or three nonzero high bytes per
double, ~500 runs a page) against zero twins, m pages per launch, `reps` launches per case:
gdsm_diff, and gdsm_release applying to the home copy with re-twin (TWIN zeroed again by a
gdsm_memcpy_batch copy kernel between launches), under the launch forms named: `auto` (the
library's choice), `chain1` / `chain4` / `page` (the chained launch from one page up: one page
per one-wave workgroup / four pages per workgroup / a page per four-wave workgroup), `solo` (the
one-workgroup launch up to 16 pages, then automatic) and `prep` (one workgroup up to 16 pages,
then the grid behind its zeroing launch). m = 9 is the clean case (CURRENT == TWIN),
m = 11 the sparse one (one double a page). Run under rocprofv3 --kernel-trace and read with
scripts/dev/kstats.py (the cases differ by kernel, grid or workgroup size).

    rocprofv3 --kernel-trace -d DIR -o run -- python scripts/dev/solo_probe.py [reps] [forms]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402

PAGE = 4096
CASES = ((1, "dense"), (4, "dense"), (10, "dense"), (16, "dense"), (9, "clean"), (11, "sparse"),
         (20, "dense"), (32, "dense"), (64, "dense"), (200, "dense"), (512, "dense"),
         (1024, "dense"), (2048, "dense"))


def dense_pages(m, seed):
    rng = np.random.default_rng(seed)
    v = rng.integers(1, 1 << 20, size=(m, PAGE // 8)).astype(np.float64)
    return v.view(np.uint8).reshape(m, PAGE)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    forms = sys.argv[2].split(",") if len(sys.argv) > 2 else ["auto", "chain", "prep"]
    L = ga.gdsm.lib()
    n = 2048
    ctx = ga.Context(n, arenas=("twin", "current", "replica"))
    zeros = np.zeros((n, PAGE), np.uint8)
    d_zero = ctx.buffer(n * PAGE).upload(zeros)
    twin_ptr = ctx.arena_ptr("twin")
    for form in forms:
        L.gdsm_tune(b"diff_solo_max", 16 if form in ("prep", "solo") else 0)
        L.gdsm_tune(b"diff_chain", {"prep": 0, "chain1": 1, "chain4": 4, "page": 3,
                                     "solo": 2}.get(form, 2))
        for m, kind in CASES:
            if form != "auto" and m in (9, 11):
                continue
            ctx.upload("twin", zeros[:m])
            if kind == "dense":
                cur = dense_pages(m, m)
            elif kind == "clean":
                cur = np.zeros((m, PAGE), np.uint8)
            else:
                cur = np.zeros((m, PAGE), np.uint8)
                cur[:, 1000:1008] = dense_pages(m, 7)[:, :8]
            ctx.upload("current", cur)
            ids = ctx.ids(np.arange(m, dtype=np.uint32))
            out = ga.Runs(ctx, m, m * 10244)
            # TWIN zeroed again between releases by a copy kernel, as config 5's row writes are
            d_desc = ctx.buffer(24).upload(np.array([twin_ptr, d_zero.ptr, m * PAGE], np.uint64))
            for op in ("diff", "release"):
                for _ in range(reps):
                    if op == "diff":
                        ctx.diff(ids, out=out)
                    else:
                        ctx.release(ids, out=out, apply_to="replica", target_ids=ids)
                        L.gdsm_memcpy_batch(ctx.handle, d_desc.ptr, 1)
                ctx.sync()
            print(form, m, kind, out.total(), flush=True)
            out.free()
            ids.free()
            d_desc.free()
    L.gdsm_tune(b"diff_solo_max", 0)
    L.gdsm_tune(b"diff_chain", 2)
    ctx.close()


if __name__ == "__main__":
    main()
