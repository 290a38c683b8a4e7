"""BASELINE config 3 at its production shape through the multi-rank code path, on ONE GPU:
16M 4 KiB pages in all, clustered 10 % writes (SPEC §6 mode 1, 100 000 ppm), page-sharded over
8 ranks of 2M pages each, every release's per-home streams exchanged all-to-all. The 8 ranks are
threads of this process with their own contexts on cuda:0 (8 x 2M x 3 arenas = 192 GiB of HBM),
wired by libgdsm's loopback communicator: the peer loop, the whole-stream checks, the fixed
budgets, the agreement and the remote applies are the RCCL path's; only the move is a
device-to-device copy. Replaces the reference's per-peer fan-out of page updates
(gallocy/http/client.cpp:39-91; "copy over the latest contents", resources/NUTSHELL.md:59-69).

Layout as exchange.py: writer(p) = p mod G, home(p) = p // n."""
import json
import os
import time

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd import exchange
from oracle import oracle

from test_gpu_loopback import close_group, run_ranks

pytestmark = pytest.mark.gpu

G = 8
N_PER_RANK = 2 * 1024 * 1024      # 2M pages per rank, 16M in all
SEED, MODE, PPM = 2026, ga.GEN_CLUSTERED, 100000
CAP_PER_PAGE = 640                # clustered 10 %: 442 B of stream per page on average


@pytest.mark.timeout(600)
def test_config3_8_ranks_2M_clustered_pages_each():
    """Release 0 with exact sizes, calibrate(), then three pipelined fixed-budget releases with
    no host synchronisation, on all 8 ranks at once: no recovery, every home's REPLICA equals its
    pages' CURRENT (Shard.verify, on the device, against pages regenerated independently), and
    sampled home blocks equal the C oracle's regeneration of those pages on the host."""
    t0 = time.perf_counter()
    n = N_PER_RANK
    ctxs = [ga.Context(n) for _ in range(G)]
    comms, shards = [], []
    try:
        for r, ctx in enumerate(ctxs):
            ctx.gen_pages(seed=SEED, mode=MODE, ppm=PPM, first_global=r, stride=G,
                          arenas=("twin", "current"))
            ctx.gen_pages(seed=SEED, mode=MODE, ppm=PPM, first_global=r * n, stride=1,
                          arenas=("replica",))
        comms = exchange.Comm.loopback(ctxs)
        shards = [exchange.Shard(ctxs[r], r, G, n, CAP_PER_PAGE, transport="loopback",
                                 comm=comms[r]) for r in range(G)]
        for c in ctxs:
            c.sync()
        t_setup = time.perf_counter() - t0
        spans = [None] * G

        def rank(r):
            s = shards[r]
            a = time.perf_counter()
            s.run(1, pipelined=False)
            s.drain()
            s.calibrate()
            assert s.flags == exchange.XCHG_FIXED
            b = time.perf_counter()
            s.run(3, pipelined=True)
            s.drain()
            assert s.recoveries == 0
            spans[r] = (b - a, time.perf_counter() - b)
        run_ranks(G, rank)
        t_rel = time.perf_counter() - t0 - t_setup
        # every rank shipped its 7 remote streams and received 7
        assert all(s.sent_remote > 0 and s.received > s.sent_remote // 8 for s in shards)
        stream_bytes = sum(s.received for s in shards)
        assert all(shards[r].verify(SEED, MODE, PPM) for r in range(G))
        # host check: three 256-page blocks of every home (its first, a random, its last)
        rng = np.random.default_rng(3)
        for d, ctx in enumerate(ctxs):
            for j in (0, int(rng.integers(256, n - 512)), n - 256):
                got = ctx.download("replica", j, 256)
                _, want = oracle.gen_pages(256, SEED, MODE, PPM, first_page=d * n + j)
                assert np.array_equal(got, want), (d, j)
        wall = time.perf_counter() - t0
        rec = {"test": "config3_8_ranks_2M_clustered", "ranks": G, "pages_per_rank": n,
               "stream_bytes_per_release": stream_bytes, "recoveries": 0,
               "setup_s": round(t_setup, 2), "releases_s": round(t_rel, 2),
               "exact_release_s_max": round(max(x[0] for x in spans), 3),
               "fixed_releases_3_s_max": round(max(x[1] for x in spans), 3),
               "wall_s": round(wall, 2)}
        print(json.dumps(rec))
        out = os.environ.get("GDSM_EVIDENCE")
        if out:
            with open(out, "a") as f:
                f.write(json.dumps(rec) + "\n")
    finally:
        for s in shards:
            s.close()
        close_group(ctxs, comms)
