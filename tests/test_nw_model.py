"""The GPU NW's algorithm on the host (scripts/dev/nw_ckpt_model.py, lane for lane: the U = H + y
+ x fill with the rotating feed/bottom register and checkpoints, the region recompute, and the
strip-parallel trace with its in-order check and merge) against the oracle NW (or_nw_diff <-
gallocy/utils/diff.cpp:73-167) on small ragged shapes. The kernels themselves are checked by
tests/test_gpu_nw.py."""
import importlib.util
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def model():
    spec = importlib.util.spec_from_file_location("nw_ckpt_model", ROOT / "scripts/dev/nw_ckpt_model.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("n1,n2,alpha,near", [(1, 1, 2, False), (63, 64, 4, False),
                                              (129, 66, 2, False), (600, 130, 256, False),
                                              (40, 700, 4, False), (520, 520, 4, True),
                                              (0, 5, 4, False), (5, 0, 4, False)])
def test_model_matches_oracle(model, n1, n2, alpha, near):
    rng = np.random.default_rng(n1 * 1000 + n2)
    a = rng.integers(0, alpha, n1).astype(np.int64)
    b = rng.integers(0, alpha, n2).astype(np.int64)
    if near:  # the guesses hold: no strip is walked again
        b = a.copy()
        b[rng.integers(0, n2, 3)] ^= 1
    ck, rows = model.fill(a, b, rng) if n1 and n2 else ({}, {})
    want = oracle.nw_diff(bytes(a.astype(np.uint8)), bytes(b.astype(np.uint8)))
    assert model.trace_spec(a, b, ck, rows) == want
    if n1 and n2:
        assert model.trace(a, b, ck, rows) == want
