import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgdsm.so on cuda:0)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    g = ROOT / "tests" / "golden"
    return {k: np.load(g / f"{k}.npz") for k in ("nw_ref", "pages", "coherence", "c1_windows",
                                                   "ref_windows", "ref_layout",
                                                   "raw_windows")}
