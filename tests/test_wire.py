"""Diff wire format (docs/SPEC.md §7) on the CPU: the oracle restatement round-trips diff streams
through the Raft append-entries JSON shape of consensus/client.cpp:133-142 and rejects what §7
rejects; libgdsm's gdsm_wire_size (host-only) agrees with it. Parity unpinned against the
reference (its log carries no diffs; try_apply is a stub, consensus/state.cpp:308-316)."""
import base64
import json

import numpy as np
import pytest

from oracle import oracle, wire


def _stream(n=64, seed=1, ppm=10000):
    twin, cur = oracle.gen_pages(n, seed=seed, mode=0, ppm=ppm)
    ro, data = oracle.diff_pages(twin, cur)
    return twin, cur, ro, data


def test_roundtrip_through_append_entries_json():
    twin, cur, ro, data = _stream()
    ids = np.arange(len(ro) - 1, dtype=np.uint32)
    text = wire.encode(ids, ro, data)
    assert b"\0" not in text
    s = text.decode("ascii")
    assert json.dumps(s) == '"' + s + '"'  # nothing for JSON to escape
    # gallocy::consensus::GallocyClient::send_append_entries payload (client.cpp:133-142)
    payload = json.dumps({"entries": [{"term": 3, "command": s}], "leader_commit": 0,
                          "previous_log_index": 0, "previous_log_term": 0, "term": 3})
    got = json.loads(payload)["entries"][0]["command"].encode()
    ids2, ro2, data2 = wire.decode(got)
    assert np.array_equal(ids2, ids) and np.array_equal(ro2, ro) and np.array_equal(data2, data)
    rep = twin.copy()
    oracle.apply(rep, ro2, data2, ids=ids2)
    assert np.array_equal(rep, cur)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 17])
def test_small_and_empty_streams(n):
    twin, cur, ro, data = _stream(max(n, 1), seed=5 + n)
    if n == 0:
        ro, data = np.zeros(1, np.uint64), np.zeros(0, np.uint8)
    ids = (np.arange(n, dtype=np.uint32) * 7 + 3)
    text = wire.encode(ids, ro[:n + 1], data)
    assert len(text) == 6 + 4 * -(-wire.frame_bytes(n, int(ro[n])) // 3)
    i2, r2, d2 = wire.decode(text)
    assert np.array_equal(i2, ids) and np.array_equal(r2, ro[:n + 1])


def _reframe(f: bytes) -> bytes:
    return wire.PREFIX + base64.b64encode(f)


def test_rejections():
    _, _, ro, data = _stream(8)
    ids = np.arange(8, dtype=np.uint32)
    text = wire.encode(ids, ro, data)
    f = base64.b64decode(text[6:])
    bad = [b"GDSM2:" + text[6:],                      # prefix
           text[:-1],                                  # length
           text[:50] + b"*" + text[51:],               # alphabet
           _reframe(f[:-8]),                           # frame length vs header
           _reframe(f[:40] + bytes([f[40] ^ 1]) + f[41:]),  # checksum
           _reframe(b"XDSM" + f[4:])]                  # magic
    for t in bad:
        with pytest.raises(ValueError):
            wire.decode(t)


def test_library_wire_size_matches_oracle():
    import gallocy_amd.gdsm as g
    for n, D in [(0, 0), (1, 0), (1, 12), (2, 40), (3, 4100), (1 << 20, 64_000_000)]:
        assert g.wire_size(n, D) == 6 + 4 * -(-wire.frame_bytes(n, D) // 3)
