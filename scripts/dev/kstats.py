"""Per-kernel duration summary of a rocprofv3 --kernel-trace database, grouped by kernel name and
grid and workgroup size: count, mean, min and median in microseconds.

    python scripts/dev/kstats.py DIR/run_results.db [name-substring]"""
import sqlite3
import statistics
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    groups = {}
    for name, gx, wx, d in c.execute("select name, grid_x, workgroup_x, duration from kernels"):
        if pat in name:
            groups.setdefault((name, gx, wx), []).append(d / 1000)
    for (name, gx, wx), ds in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(ds):6d} grid={gx:7d} wg={wx:5d} mean={statistics.mean(ds):8.2f} min={min(ds):8.2f} "
              f"med={statistics.median(ds):8.2f}  {name[:110]}")


if __name__ == "__main__":
    main()
