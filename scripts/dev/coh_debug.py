"""Prints the coherence verdicts of tiny malformed batches for every pass-C variant (debug aid)."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd import gdsm  # noqa: E402
from gallocy_amd.gdsm import GdsmError  # noqa: E402

for v in (0,):
    assert gdsm.lib().gdsm_tune(b"coh_variant", v) == 0
    with ga.Context(16, arenas=()) as c:
        for ev in ([5 << 4, 2 << 4], [99 << 4], [(99 << 4) | (3 << 1)], [(40 << 4) | 1],
                   [(3 << 4), (99 << 4)], [1 << 40]):
            c.coh_init(8)
            try:
                t = c.coherence_batch(np.array(ev, np.uint64))
                print(v, [hex(x) for x in ev], "accepted", t)
            except GdsmError as e:
                print(v, [hex(x) for x in ev], "rejected", e.errno)
