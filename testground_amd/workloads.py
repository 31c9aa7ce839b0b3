"""Synthetic workload inputs of SURVEY.md 8(d) that are not reference plans.

config 5 (BASELINE.json configs[4]): a 1M-instance random-regular graph with heterogeneous per-instance
LinkShapes, flooded by publications with first-receipt dedup (tgsim_flood_* in include/tgsim.h).
"""
from __future__ import annotations

import numpy as np

from . import _abi as A

MS = 1_000_000


def random_regular_graph(n: int, degree: int = 8, seed: int = 5) -> tuple[np.ndarray, np.ndarray]:
    """Random `degree`-regular graph by the permutation model: degree/2 uniform permutations s_i,
    v adjacent to s_i(v) and s_i^-1(v). Self loops and repeated neighbours (O(degree^2) vertices, about 28 at degree 8, in
    expectation) are dropped, so the graph is simple and symmetric and all but a handful of vertices
    have exactly `degree` neighbours. Returns CSR (offsets[n+1] u32, neighbours u32); neighbours keep
    the generation order (the flood's seq slot)."""
    assert degree % 2 == 0 and n > degree
    rng = np.random.default_rng(seed)
    cols = []
    for _ in range(degree // 2):
        s = rng.permutation(n).astype(np.int64)
        inv = np.empty_like(s)
        inv[s] = np.arange(n)
        cols += [s, inv]
    nb = np.stack(cols, axis=1)                                   # [n, degree]
    keep = nb != np.arange(n)[:, None]
    order = np.argsort(nb, axis=1, kind="stable")
    srt = np.take_along_axis(nb, order, axis=1)
    dup_sorted = np.zeros_like(keep)
    dup_sorted[:, 1:] = srt[:, 1:] == srt[:, :-1]                  # later copies of a repeated neighbour
    dup = np.zeros_like(keep)
    np.put_along_axis(dup, order, dup_sorted, axis=1)
    keep &= ~dup
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum(keep.sum(axis=1))
    return off, nb[keep].astype(np.uint32)


def pubsub_shapes(n: int, seed: int = 5) -> list:
    """Per-instance LinkShapes of config 5: latency in {10, 50, 100, 200} ms, jitter uniform in
    [0, 20] ms (whole ms), loss in {0, 0.1, 1} %, bandwidth in {1, 10, 100} Mbit/s."""
    from .sim import make_shape
    rng = np.random.default_rng(seed + 1)
    lat = rng.choice([10, 50, 100, 200], n) * MS
    jit = rng.integers(0, 21, n) * MS
    loss = rng.choice([0.0, 0.1, 1.0], n)
    bw = rng.choice([1_000_000, 10_000_000, 100_000_000], n)
    return [make_shape(latency_ns=int(a), jitter_ns=int(b), bandwidth_bps=int(c), loss=float(d))
            for a, b, c, d in zip(lat, jit, bw, loss)]


def publishers(n: int, count: int, wave: int, seed: int = 5) -> np.ndarray:
    """`count` distinct publishing instances of one wave (1 % of the instances at config 5)."""
    rng = np.random.default_rng([seed, wave])
    return np.sort(rng.choice(n, count, replace=False)).astype(np.uint32)
