"""Synthetic workload inputs of SURVEY.md 8(d) that are not reference plans.

config 5 (BASELINE.json configs[4]): a 1M-instance random-regular graph with heterogeneous per-instance
LinkShapes, flooded by publications with first-receipt dedup (tgsim_flood_* in include/tgsim.h).
"""
from __future__ import annotations

import numpy as np

from . import _abi as A

MS = 1_000_000


def random_regular_graph(n: int, degree: int = 8, seed: int = 5) -> tuple[np.ndarray, np.ndarray]:
    """Random `degree`-regular simple graph by the configuration model:
    n * degree stubs paired uniformly at random, then every self loop and every repeated edge (about
    (d-1)/2 + (d-1)^2/4, ~16 at degree 8, in expectation) removed by a random switching with another
    edge: (a, b) + (c, d) -> (a, c) + (b, d), taken only when neither new edge is a loop or already
    present. Every vertex ends with exactly `degree` neighbours. Returns CSR (offsets[n+1] u32,
    neighbours u32); a vertex's neighbours are in edge order (the flood's seq slot)."""
    assert (n * degree) % 2 == 0 and n > degree
    rng = np.random.default_rng(seed)
    stubs = np.repeat(np.arange(n, dtype=np.int64), degree)
    rng.shuffle(stubs)
    u, v = stubs[0::2].copy(), stubs[1::2].copy()                 # edge e = (u[e], v[e])
    m = len(u)
    keys = np.minimum(u, v) * n + np.maximum(u, v)
    order = np.argsort(keys, kind="stable")
    sk = keys[order]
    bad = u == v
    rep = np.zeros(m, bool)
    rep[order[1:][sk[1:] == sk[:-1]]] = True                      # later copies of a repeated edge
    bad |= rep
    delta: dict[int, int] = {}                                    # edge multiset = sk + delta

    def key(a: int, b: int) -> int:
        return min(a, b) * n + max(a, b)

    def present(k: int) -> bool:
        base = int(np.searchsorted(sk, k, "right") - np.searchsorted(sk, k, "left"))
        return base + delta.get(k, 0) > 0

    for e1 in np.flatnonzero(bad).tolist():
        a, b = int(u[e1]), int(v[e1])
        while True:
            e2 = int(rng.integers(m))
            if e2 == e1 or bad[e2]:
                continue
            c, d = int(u[e2]), int(v[e2])
            if rng.integers(2):
                c, d = d, c
            if a == c or b == d:
                continue
            k1, k2 = key(a, c), key(b, d)
            if k1 == k2 or present(k1) or present(k2):
                continue
            break
        for k, dv in ((key(a, b), -1), (key(c, d), -1), (k1, 1), (k2, 1)):
            delta[k] = delta.get(k, 0) + dv
        u[e1], v[e1], u[e2], v[e2] = a, c, b, d
        bad[e1] = False
    src = np.concatenate([u, v])
    dst = np.concatenate([v, u])
    slot = np.concatenate([2 * np.arange(m), 2 * np.arange(m) + 1])
    o = np.lexsort((slot, src))
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum(np.bincount(src, minlength=n))
    return off, dst[o].astype(np.uint32)


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
