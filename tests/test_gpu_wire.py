"""GPU diff wire format (gdsm_wire_encode / decode / apply, docs/SPEC.md §7) against the oracle
restatement (oracle/wire.py): the command text is byte-identical, decode returns the stream, the
follower apply reproduces CURRENT, and every malformed text is refused with nothing applied."""
import base64

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd.gdsm import GdsmError
from oracle import oracle, wire

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    with ga.Context(4096) as c:
        yield c


def _setup(ctx, seed, ppm=10000, mode=0):
    n = ctx.n_pages
    ctx.gen_pages(seed=seed, mode=mode, ppm=ppm)
    ctx.sync()
    return oracle.gen_pages(n, seed=seed, mode=mode, ppm=ppm)


def test_encode_matches_oracle_all_pages(ctx):
    twin, cur = _setup(ctx, 11)
    runs = ctx.diff()
    text = ctx.wire_encode(runs)
    ro, data = oracle.diff_pages(twin, cur)
    assert text == wire.encode(np.arange(ctx.n_pages, dtype=np.uint32), ro, data)
    runs.free()


@pytest.mark.parametrize("count", [1, 3, 1001])
def test_encode_listed_pages_and_apply(ctx, count):
    twin, cur = _setup(ctx, 20 + count, ppm=50000, mode=1)
    rng = np.random.default_rng(count)
    ids = np.sort(rng.choice(ctx.n_pages, count, replace=False)).astype(np.uint32)
    dids = ctx.ids(ids)
    runs = ctx.diff(dids)
    text = ctx.wire_encode(runs, dids)
    ro, data = oracle.diff_pages(twin, cur, ids=ids)
    assert text == wire.encode(ids, ro, data)
    # follower: replica holds the twin; try_apply the committed command
    ctx.upload("replica", twin)
    assert ctx.wire_apply(text) == count
    want = twin.copy()
    want[ids] = cur[ids]
    assert np.array_equal(ctx.download("replica"), want)
    # decode hands back the same stream
    i2, r2 = ctx.wire_decode(text, count, max(16, len(data)))
    h = r2.to_host()
    assert np.array_equal(h.rec_off, ro) and np.array_equal(h.data, data)
    assert np.array_equal(i2.download(np.uint32, count), ids)
    for x in (i2, r2, runs, dids):
        x.free()


def test_rejected_texts_apply_nothing(ctx):
    twin, cur = _setup(ctx, 31)
    ids = np.arange(0, 64, dtype=np.uint32)
    ro, data = oracle.diff_pages(twin, cur, ids=ids)
    good = wire.encode(ids, ro, data)
    f = base64.b64decode(good[6:])
    big = ids.copy()
    big[5] = ctx.n_pages  # outside the arena, checksum valid
    cases = [good[:-4], b"GDSM2" + good[5:], good[:100] + b"!" + good[101:],
             wire.PREFIX + base64.b64encode(f[:200] + bytes([f[200] ^ 0x10]) + f[201:]),
             wire.encode(big, ro, data), good[:6] + good[10:]]
    ctx.upload("replica", twin)
    for t in cases:
        with pytest.raises(GdsmError):
            ctx.wire_apply(t)
    assert np.array_equal(ctx.download("replica"), twin)
    assert ctx.wire_apply(good) == 64
    assert np.array_equal(ctx.download("replica")[:64], cur[:64])
