"""Does where the arenas land in HBM move the twin kernel's time? (the twin of the
north-star pages ranges 0.67-0.76 of peak between processes on one box, ±0.1 ms inside one.)

In ONE process: a padding allocation of `shift` GiB, then a 16M-page TWIN + CURRENT arena pair
(128 GiB), the twin timed (HIP events, `reps` launches), the arenas and the padding freed; repeated
for several shifts and then the first shift again. Prints one JSON line per placement.

    python scripts/dev/placement_probe.py [pages] [reps]"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    holder = ga.Context(1, arenas=())
    for shift in (0, 1, 3, 7, 13, 29, 0, 3):
        pad = holder.buffer(shift << 30) if shift else None
        ctx = ga.Context(n, arenas=("twin", "current"))
        ctx.gen_pages(seed=1, arenas=("twin", "current"))
        ctx.twin()
        ctx.sync()
        times = []
        for _ in range(reps):
            ctx.prof_enable(True)
            ctx.twin()
            ctx.sync()
            p = ctx.prof_read()
            ctx.prof_enable(False)
            times.append(p["twin"][0] / p["twin"][1])
        print(json.dumps({"pad_gib": shift, "twin_ms": [round(t, 3) for t in times],
                          "min_ms": round(min(times), 3),
                          "frac_of_8TBs": round(8192 * n / (min(times) * 1e-3) / 8e12, 4)}),
              flush=True)
        ctx.close()
        if pad is not None:
            pad.free()
        time.sleep(0.5)
    holder.close()


if __name__ == "__main__":
    main()
