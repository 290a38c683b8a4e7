"""Host-side workload shapes for the synthetic configs (BASELINE.json configs), SPEC §6."""
from __future__ import annotations

import numpy as np


def zipf_counts(n_pages: int, total: int, s: float = 0.8, seed: int = 0) -> np.ndarray:
    """Per-page event counts ~ multinomial(total, Zipf(s)) over a seeded page permutation."""
    rng = np.random.default_rng(seed)
    ranks = rng.permutation(n_pages).astype(np.float64) + 1.0
    w = ranks ** (-s)
    w /= w.sum()
    return rng.multinomial(total, w).astype(np.uint64)


def uniform_counts(n_pages: int, total: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.multinomial(total, np.full(n_pages, 1.0 / n_pages)).astype(np.uint64)


def event_counts(n_pages: int, total: int, dist: str = "zipf", seed: int = 0) -> np.ndarray:
    if dist == "zipf":
        return zipf_counts(n_pages, total, 0.8, seed)
    if dist == "uniform":
        return uniform_counts(n_pages, total, seed)
    raise ValueError(dist)
