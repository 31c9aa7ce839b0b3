#!/usr/bin/env python3
"""Regenerates the committed golden fixtures in tests/golden/ (run from the repo root, on CPU).

  philox_rocrand.json  Philox4x32-10 vectors from rocRAND's host engine
                       (/opt/rocm/include/rocrand/rocrand_philox4x32_10.h, ten_rounds), built from
                       philox_rocrand_kat.cpp with hipcc. Independent of the oracle and the kernels.
  scenarios.npz/.json  Every observable of the seeded scenarios in tests/scenarios.py, as produced
                       by the CPU oracle: full arrays for the small scenarios, SHA-256 digests of
                       each array for the large ones. The GPU must reproduce them bit for bit.
  plans.json           Outcomes of the workload descriptors (testground_amd/plans.py) on the oracle.

The reference ships no vectors for this path; these fixtures pin the oracle
against regressions and give the GPU tests a target that does not depend on building the oracle.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# (name, driver, kwargs, store full arrays?)
SCENARIOS = [
    ("random1", "run_random", dict(seed=1), True),
    ("random2_small_wheel", "run_random", dict(seed=2, cfg_kw=dict(wheel_slot_ns=3_000_000, wheel_slots=8)), True),
    ("heavy7", "run_heavy", dict(seed=7), False),
    ("sync3", "run_sync", dict(seed=3), True),
    ("storm300", "run_storm", dict(n_inst=300, rounds=4, seed=4), True),
    ("burst1", "run_burst", dict(seed=1), True),
]

PLAN_CASES = [
    ("network", "ping-pong", 2, {}),
    ("network", "traffic-allowed", 3, {}),
    ("network", "traffic-blocked", 3, {}),
    ("splitbrain", "drop", 30, {}),
    ("splitbrain", "reject", 30, {}),
    ("splitbrain", "accept", 30, {}),
    ("benchmarks", "barrier", 50, {"barrier_iterations": 2}),
    ("benchmarks", "storm", 20, {"conn_outgoing": 3, "conn_delay_ms": 1000, "data_size_kb": 16}),
]


def flatten(x, path, out):
    """Nested dict/list/tuple of arrays and scalars -> {path: leaf}."""
    if isinstance(x, dict):
        for k in sorted(x):
            flatten(x[k], f"{path}.{k}", out)
    elif isinstance(x, list) and x and all(isinstance(v, (int, np.integer)) for v in x):
        out[path] = [int(v) for v in x]          # a list of scalars is one leaf
    elif isinstance(x, (list, tuple)):
        for i, v in enumerate(x):
            flatten(v, f"{path}[{i}]", out)
    else:
        out[path] = x
    return out


def digest(a) -> str:
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.dtype.str.encode() + str(a.shape).encode() + a.tobytes()).hexdigest()


def run_scenario(binding, driver, kwargs):
    from tests import scenarios as S
    return getattr(S, driver)(binding, **kwargs)


def run_plan(binding, plan, case, n, params):
    from testground_amd import plans as P
    env = P.PlanEnv(n, seed=1, test_case=case, params=params, binding=binding)
    try:
        ok = P.PLANS[(plan, case)](env)
        res = {"ok": [bool(v) for v in ok], "failures": env.failures, "sim_now": env.sim.now,
               "stats": {k: v for k, v in env.sim.stats().items()
                         if k not in ("windows", "inflight", "tb_items", "extracted", "inserted")}}
        if hasattr(env, "rtts"):
            res["rtts"] = [[int(x) for x in r] for r in env.rtts]
        if hasattr(env, "probe_errors"):
            res["probe_errors"] = [int(x) for x in env.probe_errors]
            res["region"] = [int(x) for x in env.region]
        if hasattr(env, "barrier_times"):
            res["barrier_times"] = {k: [int(x) for x in v] for k, v in env.barrier_times.items()}
        if hasattr(env, "delivered_chunks"):
            res["delivered_chunks"] = env.delivered_chunks
        return res
    finally:
        env.close()


def make_philox():
    src = os.path.join(HERE, "philox_rocrand_kat.cpp")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "kat")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-o", exe, src])
        out = subprocess.check_output([exe]).decode()
    vec = json.loads(out)
    with open(os.path.join(HERE, "philox_rocrand.json"), "w") as f:
        json.dump(vec, f, indent=0)


def main():
    from oracle.pyoracle import oracle_binding
    ob = oracle_binding()
    if "--no-philox" not in sys.argv:
        make_philox()
    arrays, manifest = {}, {}
    for name, driver, kw, full in SCENARIOS:
        flat = flatten(run_scenario(ob, driver, kw), name, {})
        for path, leaf in flat.items():
            if isinstance(leaf, np.ndarray):
                if full:
                    key = f"a{len(arrays)}"
                    arrays[key] = leaf
                    manifest[path] = {"array": key}
                else:
                    manifest[path] = {"sha256": digest(leaf), "shape": list(leaf.shape), "dtype": leaf.dtype.str}
            else:
                manifest[path] = {"value": leaf if not isinstance(leaf, np.integer) else int(leaf)}
    np.savez_compressed(os.path.join(HERE, "scenarios.npz"), **arrays)
    with open(os.path.join(HERE, "scenarios.json"), "w") as f:
        json.dump({"scenarios": [[n, d, kw, full] for n, d, kw, full in SCENARIOS], "leaves": manifest}, f, indent=0)
    plans = {f"{p}/{c}/{n}": run_plan(ob, p, c, n, prm) for p, c, n, prm in PLAN_CASES}
    with open(os.path.join(HERE, "plans.json"), "w") as f:
        json.dump({"cases": PLAN_CASES, "results": plans}, f, indent=0)
    print(f"wrote {len(manifest)} scenario leaves ({len(arrays)} arrays), {len(plans)} plan results")


if __name__ == "__main__":
    main()
