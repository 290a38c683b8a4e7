"""bench.py's host-side pieces that need no GPU: the CPU baseline leg (the C oracle, one thread
and all-core, every sample's REPLICA checked equal to CURRENT inside the leg) and the diff-stream
payload count used for the roofline bytes."""
import numpy as np

import bench
from oracle import oracle


def test_cpu_baseline_single_and_all_core(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    out = bench.cpu_baseline(0, 10000, 7, 0.4)
    assert out["kind"] == "port" and out["unit"] == "pages/s"
    assert out["cores"] == min(2, len(__import__("os").sched_getaffinity(0)))
    assert out["value"] > 0 and out["single_thread"]["value"] > 0
    assert out["single_thread"]["cores"] == 1


def test_payload_bytes_matches_run_lengths():
    twin, cur = oracle.gen_pages(64, seed=3, mode=0, ppm=10000)
    ro, data = oracle.diff_pages(twin, cur)
    want = 0
    w = data.view("<u4")
    for i in range(64):
        a = int(ro[i]) // 4
        if ro[i + 1] > ro[i]:
            want += sum(int(h) >> 16 for h in w[a + 1:a + 1 + int(w[a])])
    assert bench.payload_bytes(ro, data) == want
    assert want == int(np.count_nonzero(twin != cur))  # runs cover exactly the changed bytes
