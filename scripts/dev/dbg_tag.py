import sys
sys.path.insert(0, "/root/repo")
import numpy as np
import gallocy_amd as ga
from gallocy_amd.gdsm import GdsmError
from oracle import oracle
offsets = [0, 1, 2, 31, 32, 33, 63, 64, 65, 1000, 1951, 1952, 1983, 1984, 1985, 2047]
counts = []
for o in offsets:
    counts += [o, 2048 * 2 + 17, 1, 0, 2048 - (o % 7) - 1, 3]
n = len(counts) + 8
cts = np.zeros(n, np.uint64); cts[:len(counts)] = counts
ev = oracle.gen_events(cts, seed=71, write_pct=0)
print("events", len(ev), "blocks", len(ev) / 2048)
starts = np.concatenate([[0], np.cumsum(cts)])
with ga.Context(n, arenas=()) as c:
    c.coh_init(8)
    ost, ofl = oracle.coh_init(n, 8)
    for it in range(2):
        try:
            c.coherence_batch(ev)
            print("ok", it)
        except GdsmError as e:
            print("err", it, e)
        oracle.coherence(ost, ofl, ev)
        st, fl = c.coh_download()
        print("tagged", np.flatnonzero(st & (1 << 30)))
        bad_st = np.flatnonzero(st != ost); bad_fl = np.flatnonzero(fl != ofl)
        print("state mismatches", bad_st[:10], "faults mismatches", bad_fl[:10])
        for p in list(bad_st[:4]) + list(bad_fl[:4]):
            print(" page", p, hex(st[p]), hex(ost[p]), fl[p], ofl[p], "events", starts[p], starts[p+1], "blocks", starts[p] // 2048, (starts[p+1]-1) // 2048)
    st, fl = c.coh_download()
    tagged = np.flatnonzero(st & (1 << 30))
    print("tagged pages", tagged[:20], len(tagged))
    for p in tagged[:10]:
        print(p, "events", starts[p], "..", starts[p + 1], "blocks", starts[p] // 2048, (starts[p + 1] - 1) // 2048)
