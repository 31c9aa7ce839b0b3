"""Per-shard kernel times of the sharded storm, in ONE process on one GPU: S
HIP contexts, one thread each, exchanging through the thread-group transport (as
tests/test_full_size.py::test_cfg4_storm_sharded_full runs them), against one context of N / S
instances (the same per-shard load without shards). With --shared-stream every context launches
on one HIP stream, so no shard's kernel runs beside another's and each kernel's duration (HIP
events here, or rocprofv3 --kernel-trace around this command) is its own.

    python3 tools/shard_profile.py --mode sharded --shards 2 [--shared-stream]
    python3 tools/shard_profile.py --mode single --instances 50000
Prints one JSON line: per kernel class the average launch time (us) and launches per round, per
shard (sharded) or for the one context (single); ms per round."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def run(sim, args, n_total, rounds, first):
    from testground_amd._abi import T_NOW
    spread, rtt = int(args.spread_ms * bench.MS), int(args.rtt_ms * bench.MS)
    for r in range(first, first + rounds):
        sim.gen_storm_round(r, T_NOW, args.fanout, args.size, spread, r)
        sim.advance_to_barrier(sim.barrier(r, n_total, T_NOW), rtt)


def profile_ctx(sim, args, n_total):
    run(sim, args, n_total, args.warmup, 0)
    sim.sync()
    sim.profile(None)
    base = sim.profile_read()
    t0 = time.perf_counter()
    run(sim, args, n_total, args.rounds, args.warmup)
    sim.sync()
    el = time.perf_counter() - t0
    prof = sim.profile_read()
    ks = {k: {"avg_us": round(1e3 * (ms - base[k][0]) / (n - base[k][1]), 2),
              "per_round": (n - base[k][1]) / args.rounds}
          for k, (ms, n) in prof.items() if n > base[k][1]}
    return {"kernels": ks, "ms_per_round": 1e3 * el / args.rounds, "lo": sim.lo, "hi": sim.hi}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", choices=("single", "sharded"), default="sharded")
    p.add_argument("--instances", type=int, default=100_000)
    p.add_argument("--shards", type=int, default=2)
    p.add_argument("--warmup", type=int, default=15)
    p.add_argument("--rounds", type=int, default=20)
    p.add_argument("--shared-stream", action="store_true")
    a = p.parse_args()
    args = argparse.Namespace(instances=a.instances, fanout=8, size=1024, spread_ms=10.0, rtt_ms=1.0, seed=4,
                              max_records=1 << 23, warmup=a.warmup, rounds=a.rounds, tcp=False)
    import numpy as np
    import torch
    from testground_amd.sim import Simulator
    torch.cuda.set_device(0)
    shapes = bench.storm_shapes(a.instances, args.seed)
    if a.mode == "single":
        sim = Simulator(bench.sim_config(args))
        sim.set_shapes(np.arange(a.instances), shapes)
        out = profile_ctx(sim, args, a.instances)
        sim.close()
        print(json.dumps({"mode": "single", "instances": a.instances, **out}), flush=True)
        return
    from testground_amd.exchange import ThreadGroup, run_threads
    S = a.shards
    g = ThreadGroup(S, device=True)
    shared = torch.cuda.Stream() if a.shared_stream else None
    res = [None] * S

    def shard(k):
        sim = Simulator(bench.sim_config(args, k, S, 0))
        if shared is not None:
            sim.set_stream(shared.cuda_stream)
        sim.set_transport(g.member(k))
        sim.set_shapes(np.arange(sim.lo, sim.hi), shapes[sim.lo:sim.hi])
        res[k] = profile_ctx(sim, args, a.instances)
        sim.close()

    run_threads([lambda k=k: shard(k) for k in range(S)])
    print(json.dumps({"mode": "sharded", "instances": a.instances, "shards": S, "shared_stream": a.shared_stream,
                      "per_shard": res}), flush=True)


if __name__ == "__main__":
    main()
