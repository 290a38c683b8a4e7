"""Host model of the streaming coherence fold (gdsm_coherence.hip, section S), lane for lane:
spans of `span` events walked as chunks of 64 by a segmented OR scan, the PROBE prefix, deferred
first segments, the per-span aggregates composed in order (the look-back's result). Checks the
algorithm (not the kernel) against the oracle fold on random batches:
    python scripts/dev/coh_stream_model.py [cases]
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from oracle import oracle  # noqa: E402

SF, PROBE, KCONST = 1 << 31, 1 << 28, 1 << 31


def s_state(v):
    base, R = v & 0x7FFFF, (v >> 20) & 0xFF
    flip = ((base >> 16) & 3) == 2 and (R & ~base & 0xFF)
    return (base | R) ^ (0x30000 if flip else 0)


def tcompose(a, b):
    R = b & 0xFF
    excl = ((a >> 16) & 3) == 2
    flip = (a & KCONST) and excl and (R & ~a & 0xFF)
    rr = (a | R) ^ (0x30000 if flip else 0)
    return b if (b & KCONST) else rr


def sor_scan(vals):
    out, acc = [], None
    for v in vals:
        acc = v if acc is None or (v & SF) else (acc | v)
        out.append(acc)
    return out


def run(state, faults, ev, span=4096, n_nodes=8):
    n_pages = len(state)
    pt = (state.astype(np.uint64) | (faults.astype(np.uint64) << np.uint64(32))).copy()
    n = len(ev)
    tot = np.zeros(10, np.int64)
    ns = (n + span - 1) // span
    aggs = []
    bad = False
    deferred = []  # per span: closures needing the incoming state
    for b in range(ns):
        lo, hi = b * span, min(n, (b + 1) * span)
        xprev = int(ev[lo - 1]) if lo else 0
        first_cont = lo > 0 and (int(ev[lo]) >> 4) == (xprev >> 4)
        carry = PROBE
        inv = xfer = 0
        F = np.zeros(8, np.int64)
        prefix_done, P8, pw, pw_node = False, 0, False, 0
        open_local, open_page, open_f0, open_cnt = False, int(ev[lo]) >> 4, 0, 0
        has_d, d_state, d_cnt, d_page = False, 0, 0, 0
        any_head = False
        pprev = xprev >> 4
        for c0 in range(lo, hi, 64):
            xs = [int(x) for x in ev[c0:min(hi, c0 + 64)]]
            L = len(xs)
            heads = []
            for i, x in enumerate(xs):
                p = x >> 4
                pp = pprev if i == 0 else xs[i - 1] >> 4
                first = c0 == 0 and i == 0
                h = first or p != pp
                if (x >> 32) or p >= n_pages or (not first and p < pp) or ((x >> 1) & 7) >= n_nodes:
                    bad = True
                heads.append(h)
            pprev = xs[-1] >> 4
            W = [int(pt[x >> 4]) if heads[i] and (x >> 4) < n_pages else 0 for i, x in enumerate(xs)]
            any_head |= any(heads)
            if c0 > lo and heads[0]:
                if open_local:
                    pt[open_page] = s_state(carry) | (((open_f0 + open_cnt) & 0xFFFFFFFF) << 32)
                else:
                    has_d, d_state, d_cnt, d_page = True, carry, open_cnt, open_page
            vs = []
            for i, x in enumerate(xs):
                nd, wr = (x >> 1) & 7, x & 1
                bit = 1 << nd
                wl = W[i] & 0x7FFFF
                v = (SF | 0x60000 | (nd << 8) | bit) if wr else ((SF | wl if heads[i] else 0) | (bit << 20))
                if i == 0 and not (v & SF):
                    v |= carry
                vs.append(v)
            incl = sor_scan(vs)
            M = []
            exs = []
            for i, x in enumerate(xs):
                nd, wr = (x >> 1) & 7, x & 1
                bit = 1 << nd
                ex = carry if i == 0 else incl[i - 1]
                exs.append(ex)
                sin = (SF | (W[i] & 0x7FFFF)) if heads[i] else ex
                exact = bool(sin & SF)
                st = s_state(sin)
                cs, own, excl = st & 0xFF, (st >> 8) & 0xFF, ((st >> 16) & 3) == 2
                fault_w = not (excl and own == nd)
                m = fault_w if wr else not ((cs >> nd) & 1)
                mm = (exact or not wr) and m
                wx = exact and wr
                if wx and fault_w:
                    inv += bin(cs & ~bit & 0xFF).count("1")
                if wx and own != nd:
                    xfer += 1
                if mm:
                    F[nd] += 1
                M.append(mm)
            if not prefix_done:
                for i, x in enumerate(xs):
                    if heads[i] or (x & 1):
                        P8 = (exs[i] >> 20) & 0xFF
                        pw = not heads[i]
                        pw_node = (x >> 1) & 7
                        prefix_done = True
                        break
            for i in range(L - 1):
                if heads[i + 1]:
                    hs = [k for k in range(i + 1) if heads[k]]
                    pg = xs[i] >> 4
                    if hs:
                        h = hs[-1]
                        cnt = sum(M[h:i + 1])
                        pt[pg] = s_state(incl[i]) | ((((W[h] >> 32) + cnt) & 0xFFFFFFFF) << 32)
                    else:
                        cnt = sum(M[:i + 1])
                        if open_local:
                            pt[pg] = s_state(incl[i]) | (((open_f0 + open_cnt + cnt) & 0xFFFFFFFF) << 32)
                        else:
                            has_d, d_state, d_cnt, d_page = True, incl[i], open_cnt + cnt, pg
            if any(heads):
                hl = max(k for k in range(L) if heads[k])
                open_local, open_page, open_f0 = True, xs[hl] >> 4, W[hl] >> 32
                open_cnt = sum(M[hl:])
            else:
                open_cnt += sum(M)
            carry = incl[-1]
        if not prefix_done:
            P8 = (carry >> 20) & 0xFF
        last_page = open_page
        next_head = hi >= n or (int(ev[hi]) >> 4) != last_page
        cont_first = False
        if next_head:
            if open_local:
                pt[last_page] = s_state(carry) | (((open_f0 + open_cnt) & 0xFFFFFFFF) << 32)
            else:
                has_d, d_state, d_cnt, d_page = True, carry, open_cnt, last_page
        elif open_local:
            pt[last_page] = np.uint64(int(pt[last_page]) + (open_cnt << 32) & 0xFFFFFFFFFFFFFFFF)
        else:
            cont_first = True
        agg = (KCONST | s_state(carry)) if (carry & SF) else ((carry >> 20) & 0xFF)
        cur = 0
        for a in aggs:
            cur = tcompose(cur, a)
        aggs.append(agg)
        dfc = 0
        if first_cont:
            if not (cur & KCONST):
                bad = True
            cs_in = cur & 0xFF
            minus = P8 & cs_in
            dfc -= bin(minus).count("1")
            for q in range(8):
                F[q] -= (minus >> q) & 1
            s1 = tcompose(cur, P8) & 0x7FFFF
            if pw:
                cs1, own1 = s1 & 0xFF, (s1 >> 8) & 0xFF
                f = not (((s1 >> 16) & 3) == 2 and own1 == pw_node)
                if f:
                    dfc += 1
                    F[pw_node] += 1
                    inv += bin(cs1 & ~(1 << pw_node) & 0xFF).count("1")
                if own1 != pw_node:
                    xfer += 1
            if has_d:
                word = s_state(d_state) if (d_state & SF) else (tcompose(cur, (d_state >> 20) & 0xFF) & 0x7FFFF)
                hiw = (int(pt[d_page]) >> 32) + d_cnt + dfc
                pt[d_page] = word | ((hiw & 0xFFFFFFFF) << 32)
            elif cont_first:
                hiw = (int(pt[last_page]) >> 32) + open_cnt + dfc
                pt[last_page] = (int(pt[last_page]) & 0xFFFFFFFF) | ((hiw & 0xFFFFFFFF) << 32)
        elif has_d:
            hiw = (int(pt[d_page]) >> 32) + d_cnt
            pt[d_page] = s_state(d_state) | ((hiw & 0xFFFFFFFF) << 32)
        tot += [inv, xfer, *F]
    return bad, pt, tot


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rng = np.random.default_rng(1)
    for k in range(cases):
        n_pages = int(rng.integers(1, 300))
        nn = int(rng.integers(1, 9))
        mode = k % 3
        if mode == 0:
            counts = rng.integers(0, 40, n_pages)
        elif mode == 1:
            counts = np.zeros(n_pages, np.int64)
            counts[rng.integers(0, n_pages, 3)] = rng.integers(1, 9000, 3)
            counts += rng.integers(0, 3, n_pages)
        else:
            counts = rng.zipf(1.5, n_pages).clip(0, 5000)
        ev = oracle.gen_events(counts.astype(np.uint64), seed=k, n_nodes=nn, write_pct=int(rng.integers(0, 60)))
        st = rng.integers(0, 1 << 19, n_pages).astype(np.uint32)
        fl = rng.integers(0, 1 << 32, n_pages, dtype=np.uint64).astype(np.uint32)
        span = int(rng.choice([64, 128, 256, 4096]))
        bad, pt, tot = run(st.copy(), fl.copy(), ev, span=span, n_nodes=nn)
        ost, ofl = st.copy(), fl.copy()
        rc, otot = oracle.coherence(ost, ofl, ev, n_nodes=nn)
        want = [otot["invalidations"], otot["transfers"], *otot["node_faults"]]
        ok = (not bad) and rc == 0 and tot.tolist() == want and \
            np.array_equal((pt & 0xFFFFFFFF).astype(np.uint32), ost) and \
            np.array_equal((pt >> np.uint64(32)).astype(np.uint32), ofl)
        print(k, len(ev), span, "ok" if ok else "MISMATCH", "" if ok else (tot.tolist(), want))
        if not ok:
            d = np.flatnonzero(((pt & 0xFFFFFFFF).astype(np.uint32) != ost) | ((pt >> np.uint64(32)).astype(np.uint32) != ofl))
            print("pages", d[:10], [(hex(int(pt[i])), hex(int(ost[i])), int(ofl[i])) for i in d[:3]])
            sys.exit(1)


if __name__ == "__main__":
    main()
