"""Config 5 end to end on the GPU: the test_mmult trace replayed through coherence batches and
twin/diff/apply propagation (gallocy_amd/replay.py). The home copies must equal the zone after
the whole multiplication, and the page table must equal the oracle's fold of the same events."""
import numpy as np
import pytest

from gallocy_amd.replay import MmultReplay
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ndim,nodes", [(64, 1), (64, 2), (96, 4), (64, 8), (257, 3),
                                        (1000, 1), (1000, 2), (1000, 4), (1000, 8)])
def test_mmult_replay_end_to_end(ndim, nodes):
    """NDIM = 1000 is BASELINE config 5's size (test/test_mmult.cpp:103-180 uses
    NDIM up to 1021 before the reference heap aborts)."""
    R = MmultReplay(ndim=ndim, nodes=nodes, seed=7)
    try:
        R.run()
        assert np.array_equal(R.home_copy(), R.final_image())
        st, fl = oracle.coh_init(R.Z, nodes)
        acc = np.zeros(10, np.int64)
        for r in range(R.T.rounds):
            rc, t = oracle.coherence(st, fl, R.T.round_events(r), n_nodes=nodes)
            assert rc == 0
            acc += [t["invalidations"], t["transfers"], *t["node_faults"]]
        assert R.totals.tolist() == acc.tolist()
        gst, gfl = R.pt.coh_download()
        assert np.array_equal(gst, st) and np.array_equal(gfl, fl)
    finally:
        R.close()
