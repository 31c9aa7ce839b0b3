"""Compare a binding (HIP library or CPU oracle) against the committed golden fixtures
(tests/golden/, written by tests/golden/make_golden.py)."""
from __future__ import annotations

import json
import os

import numpy as np

from tests.golden import make_golden as G

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_scenarios():
    with open(os.path.join(HERE, "scenarios.json")) as f:
        meta = json.load(f)
    arrays = np.load(os.path.join(HERE, "scenarios.npz"))   # allow_pickle stays False
    return meta, arrays


def check_scenario(binding, name: str) -> int:
    meta, arrays = load_scenarios()
    spec = {s[0]: s for s in meta["scenarios"]}[name]
    _, driver, kw, _ = spec
    flat = G.flatten(G.run_scenario(binding, driver, kw), name, {})
    want = {k: v for k, v in meta["leaves"].items() if k == name or k.startswith(name + ".") or k.startswith(name + "[")}
    assert set(flat) == set(want), f"{name}: leaf sets differ: {sorted(set(flat) ^ set(want))[:5]}"
    for path, leaf in flat.items():
        w = want[path]
        if "array" in w:
            ref = arrays[w["array"]]
            assert isinstance(leaf, np.ndarray) and leaf.dtype == ref.dtype and leaf.shape == ref.shape, path
            if not np.array_equal(leaf, ref):
                bad = np.nonzero(leaf != ref)[0][:8]
                raise AssertionError(f"{path}: mismatch at {bad}: {leaf[bad]} vs {ref[bad]}")
        elif "sha256" in w:
            assert G.digest(leaf) == w["sha256"], f"{path}: digest differs (shape {leaf.shape} vs {w['shape']})"
        else:
            got = leaf if not isinstance(leaf, np.integer) else int(leaf)
            assert got == w["value"], f"{path}: {got} vs {w['value']}"
    return len(flat)


def check_plans(binding, keys=None) -> None:
    with open(os.path.join(HERE, "plans.json")) as f:
        meta = json.load(f)
    for p, c, n, prm in meta["cases"]:
        key = f"{p}/{c}/{n}"
        if keys is not None and key not in keys:
            continue
        got = json.loads(json.dumps(G.run_plan(binding, p, c, n, prm)))
        assert got == meta["results"][key], f"{key}: {got} != {meta['results'][key]}"
