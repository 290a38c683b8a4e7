"""TEST INFRASTRUCTURE (checker only; never imported by the product path).

Restatement of the diff wire format of docs/SPEC.md §7 in numpy + the standard base64 module:
a diff stream (SPEC §3) framed, checksummed and base64-encoded into the text of a gallocy Raft
log command (Command{string}, gallocy/include/gallocy/consensus/log.h:18-27; shipped as
{"term", "command"} entries of append-entries JSON, consensus/client.cpp:133-142). The reference
has no diff payload in its log (try_apply is a stub, consensus/state.cpp:308-316), so the format
is this build's and parity against the reference is unpinned; the GPU encoder/decoder must match
this restatement byte for byte.
"""
from __future__ import annotations

import base64

import numpy as np

PREFIX = b"GDSM1:"
MAGIC = 0x4D534447
PHI = np.uint64(0x9E3779B97F4A7C15)


def mix64(z: np.ndarray) -> np.ndarray:
    """SPEC §6 mixer (oracle/gdsm_oracle.c mix64), vectorised; wraps mod 2^64."""
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z


def frame_bytes(n: int, D: int) -> int:
    return 32 + 4 * ((n + 1) & ~1) + 8 * (n + 1) + ((D + 7) & ~7)


def checksum(frame: bytes) -> int:
    w = np.frombuffer(frame, "<u8").copy()
    w[3] = 0
    with np.errstate(over="ignore"):
        v = mix64(w + np.arange(len(w), dtype=np.uint64) * PHI)
    return int(v.sum(dtype=np.uint64))


def frame(ids: np.ndarray, rec_off: np.ndarray, data: np.ndarray) -> bytes:
    n = len(rec_off) - 1
    D = int(rec_off[-1])
    out = bytearray(frame_bytes(n, D))
    hdr = np.array([MAGIC | (1 << 32), n, D, 0], "<u8").tobytes()
    out[0:32] = hdr
    o = 32
    out[o:o + 4 * n] = np.asarray(ids, "<u4").tobytes()
    o += 4 * ((n + 1) & ~1)
    out[o:o + 8 * (n + 1)] = np.asarray(rec_off, "<u8").tobytes()
    o += 8 * (n + 1)
    out[o:o + D] = np.asarray(data[:D], np.uint8).tobytes()
    out[24:32] = np.array([checksum(bytes(out))], "<u8").tobytes()
    return bytes(out)


def encode(ids, rec_off, data) -> bytes:
    return PREFIX + base64.b64encode(frame(ids, rec_off, data))


def decode(text: bytes):
    """-> (ids, rec_off, data) or ValueError for anything SPEC §7 rejects (record-level checks
    excepted: those belong to apply)."""
    if not text.startswith(PREFIX):
        raise ValueError("prefix")
    body = text[len(PREFIX):]
    if len(body) % 4 or len(body) < 44:
        raise ValueError("length")
    f = base64.b64decode(body, validate=True)
    if len(f) % 8 or len(f) < 32:
        raise ValueError("frame length")
    h = np.frombuffer(f[:32], "<u8")
    if int(h[0]) != MAGIC | (1 << 32):
        raise ValueError("magic")
    n, D = int(h[1]), int(h[2])
    if D % 4 or frame_bytes(n, D) != len(f):
        raise ValueError("sizes")
    if checksum(f) != int(h[3]):
        raise ValueError("checksum")
    o = 32
    ids = np.frombuffer(f[o:o + 4 * n], "<u4").copy()
    o += 4 * ((n + 1) & ~1)
    rec_off = np.frombuffer(f[o:o + 8 * (n + 1)], "<u8").copy()
    o += 8 * (n + 1)
    data = np.frombuffer(f[o:o + D], np.uint8).copy()
    if rec_off[0] != 0 or rec_off[-1] != D or (rec_off % 4).any() or (np.diff(rec_off.astype(np.int64)) < 0).any():
        raise ValueError("rec_off")
    return ids, rec_off, data
