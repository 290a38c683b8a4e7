"""Host model of the checkpointed GPU NW (gdsm_nw.hip), lane for lane: the U = H + y + x fill of
one strip as 64 lanes x 4 rows with the rotating feed/bottom register, 128-step checkpoints and
stored bottom rows; the trace recomputing the 128-step region the path enters, with the record
window indexing of the kernel. Checks the algorithm (not the kernel) against the oracle:
    python scripts/dev/nw_ckpt_model.py [cases]
Garbage (not zeros) is fed to columns beyond n2 in the fill, as the kernel's LDS ring does.
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from oracle import oracle  # noqa: E402

ROWS, STRIP, BLK, CK = 8, 512, 16, 64
LANE = np.arange(64)


def step_blocks(n2):
    return (n2 + 63 + BLK - 1) // BLK


def run_block(st, R, b, t0, n2, rec):
    """One 16-step block; st = dict(a, left, diag, pass). Returns R (bottoms in lanes 48..63)."""
    nd = np.zeros((64, ROWS, BLK), bool)
    uu = np.zeros((64, ROWS, BLK), bool)
    for k in range(BLK):
        x = t0 + k - LANE + 1
        act = (x >= 1) & (x <= n2)
        bb = b[np.clip(x, 1, n2) - 1]
        up_in = np.concatenate(([R[0]], st["pass"][:-1]))
        R = np.roll(R, -1)  # lane l <- lane l+1, lane 63 <- lane 0 (consumed)
        up, dgv = up_in.copy(), st["diag"].copy()
        for r in range(ROWS):
            lf = st["left"][:, r].copy()
            d = dgv + 2 + (st["a"][:, r] == bb)
            mx = np.maximum(np.maximum(d, lf), up)
            nd[:, r, k] = d < mx
            uu[:, r, k] = lf < up
            dgv = lf
            up = mx
            st["left"][:, r] = np.where(act, mx, lf)
        st["diag"] = np.where(act, up_in, st["diag"])
        st["pass"] = up
        R = np.where(LANE == 63, up, R)
    if rec is not None:
        rec.append((nd, uu))
    return R


def fill(a, b, rng):
    n1, n2 = len(a), len(b)
    S = (n1 + STRIP - 1) // STRIP
    nblk = step_blocks(n2)
    ck, rows = {}, {}
    for s in range(S):
        y0 = s * STRIP + LANE * ROWS + 1
        st = {"a": np.stack([np.where(y0 + r <= n1, a[np.minimum(y0 + r, n1) - 1], 0)
                             for r in range(ROWS)], 1).astype(np.int64),
              "left": np.zeros((64, ROWS), np.int64), "diag": np.zeros(64, np.int64),
              "pass": np.zeros(64, np.int64)}
        row = np.zeros(n2 + 64, np.int64)
        for t0 in range(0, nblk * BLK, BLK):
            if t0 % CK == 0:
                ck[(s, t0 // CK)] = {k: v.copy() for k, v in st.items()}
            if t0 % 64 == 0:  # a phase: 64 feed words, one per lane
                x = t0 + 1 + LANE
                if s == 0:
                    R = np.zeros(64, np.int64)
                else:
                    prev = rows[s - 1]
                    R = np.where(x <= n2, prev[np.minimum(x, n2) - 1], rng.integers(0, 1 << 20, 64))
            R = run_block(st, R, b, t0, n2, None)
            for L in range(48, 64):
                xo = t0 + L - 110
                if 1 <= xo <= n2:
                    row[xo - 1] = R[L]
        rows[s] = row
    return ck, rows


def trace(a, b, ck, rows):
    n1, n2 = len(a), len(b)
    nblk = step_blocks(n2)
    y, x, moves = n1, n2, []
    rs, rq, lrec = -1, 0, None
    while y or x:
        if x == 0:
            code = 3
        elif y == 0:
            code = 2
        else:
            yy = y - 1
            s, lane, r = yy // STRIP, (yy // ROWS) & 63, yy % ROWS
            t = x - 1 + lane
            blk, k = t // BLK, t & (BLK - 1)
            if s != rs or blk < rq * (CK // BLK):
                rs, rq = s, blk // (CK // BLK)
                st = {kk: v.copy() for kk, v in ck[(s, rq)].items()}
                lrec = []
                for bi in range(CK // BLK):
                    t0 = rq * CK + bi * BLK
                    if t0 >= nblk * BLK:
                        break
                    if t0 % 64 == 0:
                        xf = t0 + 1 + LANE
                        R = np.zeros(64, np.int64) if s == 0 else \
                            np.where(xf <= n2, rows[s - 1][np.minimum(xf, n2) - 1], 0)
                    R = run_block(st, R, b, t0, n2, lrec)
            nd, uu = lrec[blk - rq * (CK // BLK)]
            code = 1 if not nd[lane, r, k] else (2 if not uu[lane, r, k] else 3)
        moves.append(code)
        y -= code != 2
        x -= code != 3
    o1, o2 = bytearray(), bytearray()
    yy, xx = 0, 0
    for c in reversed(moves):
        o1.append(a[yy] if c != 2 else ord("-"))
        o2.append(b[xx] if c != 3 else ord("-"))
        yy += c != 2
        xx += c != 3
    return bytes(o1), bytes(o2)


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    rng = np.random.default_rng(5)
    shapes = [(1, 1), (63, 64), (128, 65), (129, 66), (257, 300), (300, 257), (600, 130),
              (40, 700), (513, 513), (200, 193), (1000, 20), (20, 1000)]
    for i in range(cases):
        n1, n2 = shapes[i % len(shapes)]
        alpha = [2, 4, 256][i % 3]
        a = rng.integers(0, alpha, n1).astype(np.int64)
        b = rng.integers(0, alpha, n2).astype(np.int64)
        ck, rows = fill(a, b, rng)
        got = trace(a, b, ck, rows)
        want = oracle.nw_diff(bytes(a.astype(np.uint8)), bytes(b.astype(np.uint8)))
        ok = got == want
        print(i, n1, n2, alpha, "ok" if ok else "MISMATCH")
        if not ok:
            sys.exit(1)


if __name__ == "__main__" and (len(sys.argv) < 3 or sys.argv[2] != "spec"):
    main()


# ---- speculative strip-parallel trace (nw_trace_kernel v2) --------------------------------------
class Regions:
    """The trace's region cache for one walker: strip s, steps [rq*CK, rq*CK + CK)."""

    def __init__(self, a, b, ck, rows):
        self.a, self.b, self.ck, self.rows = a, b, ck, rows
        self.rs, self.rq, self.lrec = -1, 0, None

    def bits(self, y, x):
        n2 = len(self.b)
        nblk = step_blocks(n2)
        yy = y - 1
        s, lane, r = yy // STRIP, (yy // ROWS) & 63, yy % ROWS
        t = x - 1 + lane
        blk, k = t // BLK, t & (BLK - 1)
        if s != self.rs or blk < self.rq * (CK // BLK) or blk >= (self.rq + 1) * (CK // BLK):
            self.rs, self.rq = s, blk // (CK // BLK)
            st = {kk: v.copy() for kk, v in self.ck[(s, self.rq)].items()}
            self.lrec = []
            for bi in range(CK // BLK):
                t0 = self.rq * CK + bi * BLK
                if t0 >= nblk * BLK:
                    break
                if t0 % 64 == 0:
                    xf = t0 + 1 + LANE
                    R = np.zeros(64, np.int64) if s == 0 else \
                        np.where(xf <= n2, self.rows[s - 1][np.minimum(xf, n2) - 1], 0)
                R = run_block(st, R, self.b, t0, n2, self.lrec)
        nd, uu = self.lrec[blk - self.rq * (CK // BLK)]
        return 1 if not nd[lane, r, k] else (2 if not uu[lane, r, k] else 3)


def row_exit(v):
    lo, typ = v
    return lo - (typ == 1)


def walk_strip(reg, s, y, x, rec, spec=None, spec_hi=None):
    """Walk from (y, x) (y in strip s) until the path leaves the strip's top row; rec[y] =
    (lo, exit) per row (the row's entry column is the exit of row y + 1). With `spec` (the
    strip's recorded rows, whose row y was entered at spec_hi), stop at the first cell on that
    path (merge): the row keeps its record."""
    top = STRIP * s + 1
    while y >= top:
        if spec is not None and spec[y][0] <= x <= spec_hi:
            rec[y] = spec[y]
            return None  # merged: rows above are the spec path's
        code = 3 if x == 0 else reg.bits(y, x)
        if code == 2:
            x -= 1
            continue
        rec[y] = (x, code)
        if spec is not None:
            spec_hi = row_exit(spec[y])
        y -= 1
        x -= code == 1
    return y, x


def trace_spec(a, b, ck, rows):
    n1, n2 = len(a), len(b)
    rec = {}
    if n1:
        S = (n1 + STRIP - 1) // STRIP
        guess = {}
        # phase A: every strip from a guessed entry (exact for the last)
        for s in range(S - 1, -1, -1):
            ye = min(STRIP * (s + 1), n1)
            xg = n2 if s == S - 1 else (ye * n2 + n1 // 2) // n1
            guess[s] = xg
            walk_strip(Regions(a, b, ck, rows), s, ye, xg, rec)
        spec = dict(rec)
        # phase B: in order from the last strip, the real entry of each; re-walk on a mismatch
        reg = Regions(a, b, ck, rows)
        for s in range(S - 2, -1, -1):
            xe = row_exit(rec[STRIP * (s + 1) + 1])
            if xe != guess[s]:
                walk_strip(reg, s, STRIP * (s + 1), xe, rec, spec, guess[s])
    # phase C: output per row; row y's entry column is the exit of row y + 1 (n2 for row n1)
    hi = {y: (row_exit(rec[y + 1]) if y < n1 else n2) for y in range(n1 + 1)}
    o1, o2 = bytearray(), bytearray()
    for x in range(1, hi[0] + 1):
        o1.append(ord("-"))
        o2.append(b[x - 1])
    for y in range(1, n1 + 1):
        lo, typ = rec[y]
        o1.append(a[y - 1])
        o2.append(b[lo - 1] if typ == 1 else ord("-"))
        for x in range(lo + 1, hi[y] + 1):
            o1.append(ord("-"))
            o2.append(b[x - 1])
    return bytes(o1), bytes(o2)


def main_spec(cases=12):
    rng = np.random.default_rng(9)
    shapes = [(1, 1), (63, 64), (300, 257), (600, 130), (40, 700), (513, 513), (200, 193),
              (1000, 20), (20, 1000), (780, 800), (0, 5), (5, 0)]
    for i in range(cases):
        n1, n2 = shapes[i % len(shapes)]
        alpha = [2, 4, 256][i % 3]
        a = rng.integers(0, alpha, n1).astype(np.int64)
        b = rng.integers(0, alpha, n2).astype(np.int64)
        if i % 4 == 3 and n1 == n2:  # near-identical: the guesses hold
            b = a.copy()
            b[rng.integers(0, n2, 3)] ^= 1
        ck, rows = fill(a, b, rng) if n1 and n2 else ({}, {})
        got = trace_spec(a, b, ck, rows)
        want = oracle.nw_diff(bytes(a.astype(np.uint8)), bytes(b.astype(np.uint8)))
        print("spec", i, n1, n2, alpha, "ok" if got == want else "MISMATCH")
        if got != want:
            sys.exit(1)


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "spec":
    main_spec(int(sys.argv[1]))
