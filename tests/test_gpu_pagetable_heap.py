"""gdsm_hl::PageTableHeap release path on the GPU, from compiled C++ (tests/cpp/pagetable_heap.cpp
built in-tree by __graft_entry__.build()): two release intervals of a gallocy-style heap zone are
diffed on the GPU against their twins (gdsm_track_diff) and applied at a home REPLICA
(gdsm_apply); the replica must equal the zone after each release."""
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
DRIVER = Path(__file__).resolve().parents[1] / "tests" / "cpp" / "_build" / "pagetable_heap"


def test_pagetable_heap_release_and_apply_at_home():
    assert DRIVER.exists(), "build the test drivers first (__graft_entry__.build())"
    r = subprocess.run([str(DRIVER), "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.startswith("ok ")
