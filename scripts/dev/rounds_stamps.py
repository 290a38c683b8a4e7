"""Where a gdsm_rounds round's time goes (measurement only; needs the -DGDSM_ROUNDS_STAMPS build:
scripts/dev/build_variant.sh lib_st -DGDSM_ROUNDS_STAMPS, run with GDSM_LIB=gallocy_amd/lib_st/
libgdsm.so). Workgroup 0's s_memtime stamps per round (shader clock; us at 2.4 GHz): page data
[round start, copies done, barrier 1 done, release done] and page table [round start, fold done, span 0 published, span 0 looked back],
medians over the rounds.  Usage: rounds_stamps.py NODES"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from gallocy_amd import gdsm  # noqa: E402
from gallocy_amd.replay import MmultReplay  # noqa: E402

nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 1
L = gdsm.lib()
fn, fp = L.gdsm_debug_round_stamps, L.gdsm_debug_round_stamps_pt
fs = L.gdsm_debug_fold_spans
fn.argtypes = fp.argtypes = fs.argtypes = [C.c_void_p, C.c_size_t]
for rep in range(2):
    R = MmultReplay(ndim=1000, nodes=nodes, seed=0, driver="device")
    dt = R.run()
    st = np.zeros((2, 4096, 4), np.uint64)
    sp = np.zeros((2, 4096, 4), np.uint64)
    ss = np.zeros((1024, 32, 4), np.uint64)
    assert fn(st.ctypes.data, st.nbytes) == 0 and fp(sp.ctypes.data, sp.nbytes) == 0
    assert fs(ss.ctypes.data, ss.nbytes) == 0
    st[1] = sp[1]
    n = R.T.rounds
    R.close()
d = st[0, :n].astype(np.int64)
f = st[1, :n].astype(np.int64)
us = lambda x: round(float(np.median(x)) / 2400.0, 3)  # noqa: E731
print(f"nodes {nodes}: {n} rounds in {dt * 1e3:.3f} ms = {dt / n * 1e6:.2f} us per round")
print("page data: copies", us(d[:, 1] - d[:, 0]), "barrier 1", us(d[:, 2] - d[:, 1]),
      "release", us(d[:, 3] - d[:, 2]), "barrier 2", us(d[1:, 0] - d[:-1, 3]),
      "round", us(d[1:, 0] - d[:-1, 0]))
print("page table: fold", us(f[:, 1] - f[:, 0]), "barrier", us(f[1:, 0] - f[:-1, 1]),
      "round", us(f[1:, 0] - f[:-1, 0]))
print("  (one-workgroup LDS fold, GDSM_ROUNDS_LDS: staging + barrier", us(f[:, 2] - f[:, 0]),
      "walk", us(f[:, 3] - f[:, 2]), "totals + barrier", us(f[:, 1] - f[:, 3]), ")")
print("  span 0 of the fold: loads + gathers + scan", us(f[:, 2] - f[:, 0]),
      "look-back", us(f[:, 3] - f[:, 2]), "tail (corrections, totals)", us(f[:, 1] - f[:, 3]))
# every span of the fold against its round's start (workgroup 0's point 0): entry, published,
# looked back, exit (medians over the rounds that have the span)
nr = min(n, 1024)
f0 = f[:nr, 0][:, None]
s_ = ss[:nr].astype(np.int64)
print("fold spans (us after the round's start: entry / published / looked back / exit):")
for b in range(32):
    have = s_[:, b, 3] > f0[:, 0]
    if have.sum() < nr // 2:
        break
    row = [us((s_[have, b, k] - f0[have, 0])) for k in range(4)]
    print(f"  span {b:2d} ({int(have.sum())} rounds): {row}")
