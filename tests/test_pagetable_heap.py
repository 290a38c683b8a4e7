"""gdsm_hl::PageTableHeap (include/gdsm_pagetable.h), the page-table heap layer gallocy reserves
but leaves as a logging stub (gallocy/include/gallocy/heaplayers/pagetableheap.h:12-29), inside a
gallocy-style layer stack SizeHeap<PageTableHeap<mmap zone source>> compiled in C++
(tests/cpp/pagetable_heap.cpp). CPU side: the allocator's own header writes and the program's
writes are exactly the dirty pages, twins hold the pre-interval contents, release re-arms."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
DRIVER = ROOT / "tests" / "cpp" / "_build" / "pagetable_heap"


def test_pagetable_heap_layer_tracks_the_zone():
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "cpp")], check=True, timeout=300)
    r = subprocess.run([str(DRIVER), "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok ")
