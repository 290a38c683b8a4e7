"""Config 5 end to end on the GPU: the test_mmult trace replayed through coherence batches and
twin/diff/apply propagation (gallocy_amd/replay.py). The home copies must equal the zone after
the whole multiplication, and the page table must equal the oracle's fold of the same events."""
import numpy as np
import pytest

from gallocy_amd.replay import MmultReplay
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ndim,nodes,graph", [(64, 1, False), (64, 2, False), (96, 4, False),
                                              (64, 8, False), (257, 3, False), (1000, 1, False),
                                              (1000, 2, False), (1000, 4, False), (1000, 8, False),
                                              (96, 4, True), (1000, 4, True)])
def test_mmult_replay_end_to_end(ndim, nodes, graph):
    """NDIM = 1000 is BASELINE config 5's size (test/test_mmult.cpp:103-180 uses
    NDIM up to 1021 before the reference heap aborts). graph: every round recorded into one HIP
    graph (gdsm_capture_*) and replayed by one launch, or issued eagerly (the default)."""
    R = MmultReplay(ndim=ndim, nodes=nodes, seed=7)
    try:
        R.run(graph=graph)
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


def test_rank_replay_single_rank_rccl():
    """Config 5 with one process per DSM node (gallocy_amd.replay.MmultRankReplay), here the
    1-rank case on RCCL through gdsm_exchange: NDIM = 1000."""
    from gallocy_amd.replay import MmultRankReplay
    R = MmultRankReplay(0, 1, ndim=1000, seed=7)
    try:
        R.run()
        assert np.array_equal(R.home_block(), R.final_block())
        st, fl = oracle.coh_init(R.Z, 1)
        rc, t = oracle.coherence(st, fl, R.T.all_events(), n_nodes=1)
        assert rc == 0
        gst, gfl = R.pt.coh_download()
        assert np.array_equal(gst, st) and np.array_equal(gfl, fl)
        assert R.totals.tolist() == [t["invalidations"], t["transfers"], *t["node_faults"]]
    finally:
        R.close()


@pytest.mark.parametrize("ranks,ndim", [(2, 300), (4, 1000)])
def test_rank_replay_multi_rank_rehearsal_gloo(ranks, ndim):
    """MmultRankReplay with `ranks` processes sharing cuda:0, the exchange over gloo (RCCL cannot
    put two ranks on one GPU): every rank's home block equals the product zone, its page-table
    shard equals the oracle's fold of the whole trace on those pages, and the totals summed over
    ranks equal the oracle's (scripts/rank_replay.py)."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           str(root / "scripts" / "rank_replay.py"), "--ndim", str(ndim), "--transport", "gloo"]
    r = subprocess.run(cmd, cwd=root, env=dict(os.environ), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    assert lines[0]["ok"] is True, lines[0]
