"""GPU Needleman-Wunsch (gdsm_nw_diff_batch, the legacy diff() on the GPU) against the reference's
own goldens, the vectors the reference produced (tests/golden/nw_ref.npz) and the C oracle
(or_nw_diff <- gallocy/utils/diff.cpp:73-167) on seeded random pairs. Bit-exact: the outputs are
bytes."""
import ctypes as C

import numpy as np
import pytest

import gallocy_amd as ga
from gallocy_amd import _lib
from gallocy_amd.gdsm import GdsmError
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    with ga.Context(1, arenas=()) as c:
        yield c


def _rand(rng, n, alphabet=256):
    return bytes(rng.integers(0, alphabet, n, dtype=np.uint8))


def test_reference_test_diff_goldens(ctx):
    # test/test_diff.cpp:13-16, 24-31 and the SURVEY §8c KATs, in one batch
    cases = [(b"GGAATGG", b"ATG", b"GGAATGG", b"---AT-G"),
             (b"FOO BOP BOOP", b"FOOO BOOP BOP", b"F-OO B-OP BOOP", b"FOOO BOOP B-OP"),
             (b"", b"", b"", b""), (b"", b"ABC", b"---", b"ABC"), (b"ABC", b"", b"ABC", b"---"),
             (b"AB", b"BA", b"AB", b"BA"), (b"ABCD", b"BCDA", b"ABCD-", b"-BCDA"),
             (b"AAAA", b"AA", b"AAAA", b"--AA"), (b"AA", b"AAAA", b"--AA", b"AAAA"),
             (b"ACGT", b"TGCA", b"ACGT", b"TGCA"), (b"HELLO", b"YELLOW", b"HELLO-", b"YELLOW"),
             (b"0123456789", b"0123X56789", b"0123456789", b"0123X56789")]
    got = ctx.nw_diff_batch([(a, b) for a, b, _, _ in cases])
    assert got == [(o1, o2) for _, _, o1, o2 in cases]


def test_reference_produced_vectors(ctx, golden):
    from tests.test_oracle import _nw_golden_cases
    cases = list(_nw_golden_cases(golden))
    assert len(cases) >= 31
    got = ctx.nw_diff_batch([(a, b) for a, b, _, _ in cases])
    assert got == [(o1, o2) for _, _, o1, o2 in cases]


# Shapes around every boundary of the kernel: strips (512 rows; 256 in the 4-row build), the
# 8-strip group whose last strip hands over through global memory (n1 > 4096), the lane pipeline
# (64 columns), the 16-step blocks, the 64-step phases and the regions the trace recomputes from
# checkpoints (a path through many regions: long and thin both ways).
SHAPES = [(1, 1), (1, 300), (300, 1), (63, 64), (64, 65), (255, 17), (256, 256), (257, 1000),
          (1000, 257), (700, 700), (4096, 33), (4097, 80), (8500, 40), (50, 5000),
          (128, 65), (129, 66), (200, 193), (3000, 2900), (16, 3000), (511, 100), (512, 512),
          (513, 70)]


@pytest.mark.parametrize("alphabet", [256, 4, 2])
def test_random_pairs_vs_oracle(ctx, alphabet):
    """Small alphabets make ties everywhere, which exercises diag > left > up."""
    rng = np.random.default_rng(100 + alphabet)
    pairs = [(_rand(rng, n1, alphabet), _rand(rng, n2, alphabet)) for n1, n2 in SHAPES]
    got = ctx.nw_diff_batch(pairs)
    for (a, b), g in zip(pairs, got):
        assert g == oracle.nw_diff(a, b), (len(a), len(b))


def test_pages_with_sparse_writes_and_shifts(ctx):
    """4 KiB pages (BASELINE config 1 shape): substitution-only edits (identity alignment), a
    memmove-shifted page and an insertion, which the run diff cannot express but NW can."""
    rng = np.random.default_rng(7)
    pairs = []
    for i in range(6):
        twin = bytearray(_rand(rng, 4096))
        cur = bytearray(twin)
        for off in rng.choice(512, 5, replace=False):
            cur[8 * off:8 * off + 8] = _rand(rng, 8)
        pairs.append((bytes(twin), bytes(cur)))
    base = _rand(rng, 4096)
    pairs.append((base, base[100:] + _rand(rng, 100)))
    pairs.append((base, base[:2000] + b"INSERTED" + base[2000:4088]))
    got = ctx.nw_diff_batch(pairs)
    for (a, b), g in zip(pairs, got):
        assert g == oracle.nw_diff(a, b)
    for (a, b), (o1, o2) in zip(pairs[:6], got[:6]):
        assert o1 == a and o2 == b  # equal-length substitutions align gap-free


def test_long_strings_read_b_from_global(ctx):
    """Beyond 48 KiB the fill reads b from global memory instead of LDS; the whole batch takes
    that kernel (max_len decides), short pairs included."""
    rng = np.random.default_rng(11)
    pairs = [(_rand(rng, 60, 4), _rand(rng, 50000, 4)), (_rand(rng, 50000, 4), _rand(rng, 70, 4)),
             (_rand(rng, 700, 4), _rand(rng, 650, 4))]
    got = ctx.nw_diff_batch(pairs)
    for (a, b), g in zip(pairs, got):
        assert g == oracle.nw_diff(a, b), (len(a), len(b))


def test_max_len_is_enforced(ctx):
    with pytest.raises(GdsmError):
        ctx.nw_diff_batch([(b"A" * 100, b"B" * 10)], max_len=64)


def test_legacy_diff_symbol_offloaded(ctx):
    """gdsm_set_diff_device routes the C++ `diff` symbol (diff.h:9-11) to the GPU."""
    lib = _lib.load()
    fn = getattr(lib, _lib.LEGACY_DIFF_SYMBOL)
    fn.restype = C.c_int
    fn.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p), C.c_char_p, C.c_size_t,
                   C.POINTER(C.c_void_p)]
    rng = np.random.default_rng(3)
    a, b = _rand(rng, 3000, 4), _rand(rng, 2900, 4)
    ga.set_diff_device(ctx, 0)
    try:
        r1, r2 = C.c_void_p(), C.c_void_p()
        assert fn(a, len(a), C.byref(r1), b, len(b), C.byref(r2)) == 0
        want = oracle.nw_diff(a, b)
        got = (C.string_at(r1, len(want[0])), C.string_at(r2, len(want[1])))
        assert C.string_at(r1) == want[0].split(b"\0")[0]  # NUL-terminated like the reference
        libc = C.CDLL(None)
        libc.free(r1)
        libc.free(r2)
        assert got == want
        assert ga.diff(a, b) == want  # gdsm_nw_diff takes the same route
    finally:
        ga.set_diff_device(None)


@pytest.mark.parametrize("name", ["c1", "cl", "dense", "edge"])
def test_page_windows_against_reference_alignments(ctx, golden, name):
    """The GPU NW on every 1024-B page window the REFERENCE diff() aligned for the page-diff pins
    (tests/golden/c1_windows.npz, ref_windows.npz; made by oracle/_ref): config 1's, config 3's
    clustered, a dense set and the SPEC edge pages. Every window — the ones whose reference
    alignment has gaps included — gives the reference's alignment length and the crc32 of both
    alignment strings."""
    import zlib

    from tests.helpers import c1_windows, window_pages
    if name == "c1":
        g = golden["c1_windows"]
        L, crc = g["L"], g["crc"]
        t, c = c1_windows()
    else:
        L, crc = golden["ref_windows"][name + "_L"], golden["ref_windows"][name + "_crc"]
        t, c = window_pages(name, golden)
    tw, cw = t.reshape(-1, 1024), c.reshape(-1, 1024)
    got = ctx.nw_diff_batch([(tw[i].tobytes(), cw[i].tobytes()) for i in range(len(tw))])
    for i, (o1, o2) in enumerate(got):
        assert len(o1) == L[i] and [zlib.crc32(o1), zlib.crc32(o2)] == crc[i].tolist(), (name, i)
