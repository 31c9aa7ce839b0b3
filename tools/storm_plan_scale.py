#!/usr/bin/env python3
"""Host cost per window of the storm plan on the device reactor: the plan
(plans/benchmarks/storm.go through testground_amd.plans.storm, message mode) at several instance
counts with the same per-instance pattern, timing every window. Per window the host makes one
tgsim_advance and one tgsim_storm_react (a 16-B read); the GPU time of the window's kernels comes
from HIP events on the context stream (tgsim_profile_*), so host time = wall - GPU time.

    python tools/storm_plan_scale.py [--n 2000 20000 100000] [--out profiles/r04/storm_plan_scale.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from testground_amd import plans as P  # noqa: E402


def run(n: int, params: dict) -> dict:
    env = P.PlanEnv(n, seed=1, test_case="storm", params=params,
                    sim_kw=dict(max_msgs_per_window=max(1 << 18, 64 * n), max_records=max(1 << 20, 128 * n)))
    sim = env.sim
    sim.profile(None)
    base = sim.profile_read()
    walls = []
    orig_advance, orig_react = sim.advance, sim.storm_react

    def advance(t, *a, **k):
        walls.append(time.perf_counter())
        return orig_advance(t, *a, **k)
    sim.advance = advance
    t0 = time.perf_counter()
    ok = P.storm(env)
    wall = time.perf_counter() - t0
    prof = sim.profile_read()
    gpu_ms = sum(ms - base[k][0] for k, (ms, _) in prof.items())
    w = env.storm_windows
    per = np.diff(np.array(walls)) * 1e6 if len(walls) > 1 else np.zeros(1)
    res = {"instances": n, "ok": int(ok.sum()), "windows": w, "wall_s": wall,
           "wall_per_window_us": wall / max(w, 1) * 1e6, "gpu_per_window_us": gpu_ms * 1e3 / max(w, 1),
           "host_per_window_us": (wall - gpu_ms * 1e-3) / max(w, 1) * 1e6,
           "median_window_interval_us": float(np.median(per)), "p90_window_interval_us": float(np.percentile(per, 90)),
           "totals": env.storm_totals,
           "sim_end_s": sim.now / 1e9}
    env.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[2000, 20000, 100000])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    params = {"conn_outgoing": "5", "conn_delay_ms": "2000", "concurrent_dials": "10", "data_size_kb": "16"}
    rows = []
    for n in a.n:
        r = run(n, params)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump({"params": params, "rows": rows,
                   "note": "storm plan (message mode) on the device reactor; host time = wall - GPU kernel time"},
                  open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
