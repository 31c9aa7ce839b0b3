"""Address-exchange fan-out on the device (storm.go:232-255): N instances
publish one address each to one topic, then all N replay the whole topic — N^2 deliveries written
into per-subscriber inboxes by tgsim_sync_subscribe_device. Prints one JSON line per N with the
fill rate (deliveries/s) and the bytes the fill writes (4 B per delivery) against HBM peak.

    python tools/bench_topics.py --n 100000 --reps 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[100_000])
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from testground_amd.sim import SimConfig, Simulator
    dev = torch.device("cuda:0")
    for n in args.n:
        sim = Simulator(SimConfig(n_instances=n, max_states=16, data_prefix_len=16 if n < 65000 else 12))
        stream = torch.cuda.Stream(dev)  # the default stream's handle is 0, which set_stream reads as "own stream"
        torch.cuda.set_stream(stream)
        sim.set_stream(stream.cuda_stream)
        rng = np.random.default_rng(1)
        t = np.sort(rng.integers(0, 10**6, n))
        payloads = [b"/ip4/16.0.%d.%d/tcp/2000" % ((g + 2) >> 8 & 255, (g + 2) & 255) for g in range(n)]
        sim.publish(0, np.arange(n, dtype=np.uint32), t, payloads)
        subs = torch.zeros(n, dtype=torch.int32, device=dev)
        frm = subs + 1
        until = torch.full((n,), 1 << 62, dtype=torch.int64, device=dev)
        offs, _ = sim.subscribe_device(subs, frm, until, entries=False)
        total = int(offs[-1])
        ids = torch.empty(total, dtype=torch.int32, device=dev)
        lib, ctx = sim.lib, sim._ctx

        def run(with_entries: bool) -> None:
            rc = lib.sync_subscribe_device(ctx, n, subs.data_ptr(), frm.data_ptr(), until.data_ptr(), 0xFFFFFFFF,
                                           offs.data_ptr(), ids.data_ptr() if with_entries else None,
                                           total if with_entries else 0)
            assert rc == 0, rc

        res = {}
        for mode in (False, True):
            run(mode)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(args.reps):
                run(mode)
            b.record(stream)
            torch.cuda.synchronize()
            res[mode] = a.elapsed_time(b) / args.reps
        assert bool((ids.view(n, n)[:: max(1, n // 64)] == torch.arange(n, device=dev, dtype=torch.int32)).all())
        ms = res[True]
        print(json.dumps({"workload": "address_exchange_fanout", "n_instances": n, "deliveries": total,
                          "ms_counts_only": round(res[False], 4), "ms_fill": round(ms, 3),
                          "deliveries_per_s": total / (ms * 1e-3), "write_GBps": 4 * total / (ms * 1e-3) / 1e9,
                          "frac_hbm": 4 * total / (ms * 1e-3) / 8e12}), flush=True)
        del ids
        sim.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
