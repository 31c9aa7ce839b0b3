#!/usr/bin/env python3
"""Runs every registered workload descriptor once at a small size and prints the outcome.

    python tools/run_plans.py            # HIP library (needs a GPU)
    python tools/run_plans.py --oracle   # CPU oracle (test infrastructure)
"""
import os
import sys
import time
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from testground_amd import plans as P  # noqa: E402

CASES = [
    (("network", "ping-pong"), 2, {}),
    (("network", "traffic-allowed"), 3, {}),
    (("network", "traffic-blocked"), 3, {}),
    (("splitbrain", "drop"), 12, {}),
    (("splitbrain", "reject"), 12, {}),
    (("splitbrain", "accept"), 12, {}),
    (("benchmarks", "barrier"), 50, {"barrier_iterations": 2}),
    (("benchmarks", "storm"), 20, {"conn_outgoing": 3, "conn_delay_ms": 1000, "data_size_kb": 16}),
    (("benchmarks", "startup"), 10, {}),
    (("benchmarks", "netinit"), 10, {}),
    (("benchmarks", "netlinkshape"), 10, {}),
    (("benchmarks", "subtree"), 10, {"subtree_iterations": 100}),
    (("verify", "uses-data-network"), 4, {}),
    (("placebo", "ok"), 3, {}),
    (("placebo", "stall"), 3, {}),
    (("example", "sync"), 6, {}),
]


def main():
    binding = None
    if "--oracle" in sys.argv:
        from oracle.pyoracle import oracle_binding
        binding = oracle_binding()
    for key, n, params in CASES:
        t0 = time.time()
        env = P.PlanEnv(n, seed=1, test_case=key[1], params=params, binding=binding)
        try:
            ok = P.PLANS[key](env)
            extra = {k: getattr(env, k) for k in ("rtts", "probe_errors", "delivered_chunks") if hasattr(env, k)}
            print(key, "ok" if ok.all() else "FAIL", env.failures[:3], extra,
                  f"{time.time() - t0:.2f}s sim={env.sim.now / 1e6:.1f}ms", flush=True)
        except Exception:
            traceback.print_exc()
        finally:
            env.close()


if __name__ == "__main__":
    main()
