"""Table of scripts/dev/solo_probe.py's rocprofv3 trace: median diff / release kernel time per form
and page count (dispatches in launch order, `reps` per case and operation).

    python scripts/dev/probe_table.py DIR/run_results.db REPS form[,form...]"""
import sqlite3
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from solo_probe import CASES  # noqa: E402


def main():
    db, reps, forms = sys.argv[1], int(sys.argv[2]), sys.argv[3].split(",")
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels where name like '%diff_single%' or "
                     "name like '%release_page%' order by start").fetchall()
    res, k = {}, 0
    for f in forms:
        for m, kind in CASES:
            if f != "auto" and m in (9, 11):
                continue
            for op in ("diff", "release"):
                res[(f, m, op)] = statistics.median(r[1] / 1000 for r in rows[k:k + reps])
                k += reps
    assert k == len(rows), (k, len(rows))
    print("m kind | " + " | ".join(f"{f} diff/rel" for f in forms))
    for m, kind in CASES:
        cells = []
        for f in forms:
            if (f, m, "diff") in res:
                cells.append(f"{res[(f, m, 'diff')]:.2f}/{res[(f, m, 'release')]:.2f}")
            else:
                cells.append("-")
        print(m, kind, "|", " | ".join(cells))
    prep = [r[1] / 1000 for r in c.execute("select name, duration from kernels where name like "
                                            "'%diff_prep%'")]
    if prep:
        print("zeroing launch median", round(statistics.median(prep), 2), len(prep))


if __name__ == "__main__":
    main()
