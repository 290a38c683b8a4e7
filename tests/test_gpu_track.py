"""Write-fault capture feeding the GPU path end to end: host writes -> SIGSEGV twin capture ->
gdsm_track_diff (pack, upload, diff on the GPU) -> gdsm_apply into a replica indexed by page id.
The diff stream must equal the oracle's on the same twin/current pages, and after each interval
the replica must equal the host region."""
import mmap

import numpy as np
import pytest

import gallocy_amd as ga
from oracle import oracle

pytestmark = pytest.mark.gpu


def _eq(got, ro, data):
    assert np.array_equal(got.rec_off, ro)
    assert np.array_equal(got.data, data)


def test_tracked_intervals_diff_and_apply_on_gpu():
    n = 600
    mm = mmap.mmap(-1, n * 4096)
    v = np.frombuffer(mm, np.uint8).reshape(n, 4096)
    rng = np.random.default_rng(11)
    v[:] = rng.integers(0, 256, v.shape, dtype=np.uint8)
    with ga.Context(n) as ctx, ga.Tracker(mm) as t:
        ctx.upload("replica", v.copy())
        pg = t.pages()
        for interval in range(3):
            for p in rng.choice(n, 60, replace=False):
                kind = rng.integers(0, 4)
                if kind == 0:    # a few words
                    for _ in range(rng.integers(1, 6)):
                        o = int(rng.integers(0, 512)) * 8
                        pg[p, o:o + 8] = rng.integers(0, 256, 8, dtype=np.uint8)
                elif kind == 1:  # one 64-B cluster
                    o = int(rng.integers(0, 64)) * 64
                    pg[p, o:o + 64] ^= 0x5A
                elif kind == 2:  # the whole page (> 64 dirty chunks)
                    pg[p] ^= 0xA5
                else:            # a write that changes nothing still makes the page dirty
                    pg[p, 10] = pg[p, 10]
            ids = t.dirty()
            runs, dids, k = t.diff(ctx)
            assert k == len(ids)
            ro, data = oracle.diff_pages(t.twin()[ids].copy(), pg[ids].copy())
            _eq(runs.to_host(), ro, data)
            ctx.apply(runs, "replica", dids)
            ctx.sync()
            assert np.array_equal(ctx.download("replica"), pg), interval
            t.rearm()
            assert t.dirty().size == 0
