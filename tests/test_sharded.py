"""CPU: the N>1 path. Instances are sharded in contiguous ranges; each window the
sender shard shapes its copies and one all-to-all moves cross-shard records to the receiver shard.
The sharded run must equal the single-shard run bit for bit: per-shard statuses, the receiver
shard's deliveries and inbox offsets, and the summed counters.

  * in-process: 2 and 3 oracle shards exchanging through memmove;
  * multi-process: world_size 2 over torch.distributed gloo (the variable-size exchange of
    testground_amd/exchange.py, all_reduce MAX of the storm barrier release), the protocol bench.py
    runs over RCCL.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

from tests import scenarios as S
from testground_amd.sim import SimConfig, Simulator
from testground_amd.exchange import exchange as xchg


@pytest.mark.parametrize("world,seed", [(2, 1), (2, 5), (3, 2)])
def test_sharded_equals_single_in_process(oracle, world, seed):
    outs, srcs = S.run_random_sharded(lambda c: Simulator(c, binding=oracle), S.memmove_exchange, world, seed)
    S.assert_sharded_matches(outs, srcs, S.run_random(oracle, seed), world)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torch_view(addr, nbytes):
    import torch
    buf = (C.c_uint8 * nbytes).from_address(addr)
    return torch.from_numpy(np.frombuffer(buf, dtype=np.uint8))


def _worker(rank, world, port, seed, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        from oracle.pyoracle import oracle_binding
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ob = oracle_binding()

        def exchange(sims):  # the runner's variable-size exchange (testground_amd/exchange.py)
            s = sims[0]
            send, recv, nbytes = s.exchange_buffers()
            xchg(_torch_view(send, nbytes), _torch_view(recv, nbytes), nbytes // (world * 32), dist)

        outs, _ = S.run_random_sharded(lambda c: Simulator(c, binding=ob), exchange, world, seed, local=[rank])
        storm = _storm_rank(ob, rank, world, dist)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, outs[0], storm))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


def _storm_rank(binding, rank, world, dist, n=600, rounds=3):
    """bench.py's sharded storm step on one rank: generate, MAX-all-reduce the local release time,
    advance_begin(release + rtt), all-to-all, advance_end."""
    import torch
    from testground_amd.sim import make_shape
    sim = Simulator(SimConfig(n_instances=n, seed=4, shard_id=rank, n_shards=world, exchange_cap=1 << 14),
                    binding=binding)
    rng = np.random.default_rng(4)
    for g in range(n):
        sim.set_shape(g, make_shape(latency_ns=int(rng.integers(20, 101)) * S.MS, jitter_ns=5 * S.MS,
                                    bandwidth_bps=10_000_000, loss=0.5))
    res = []
    rel = C.c_int64()
    for r in range(rounds):
        sim.gen_storm_round(r, sim.now, 8, 1024, 10 * S.MS, r)
        sim._check(binding.cdll.tgo_storm_release(sim._ctx, C.byref(rel)))
        t = torch.tensor([rel.value], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sim.advance_begin(int(t.item()) + 1 * S.MS)
        send, recv, nbytes = sim.exchange_buffers()
        xchg(_torch_view(send, nbytes), _torch_view(recv, nbytes), nbytes // (world * 32), dist)
        sim.advance_end()
        res.append(dict(now=sim.now, status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    res.append(dict(stats=S.parity_stats(sim)))
    sim.close()
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gloo(oracle, world):
    import torch.multiprocessing as mp
    seed = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, outs, storm = q.get(timeout=240)
        assert outs != "ERR", storm
        got[rank] = (outs, storm)
    for p in procs:
        p.join(timeout=60)
    _, srcs = S.run_random_sharded(lambda c: Simulator(c, binding=oracle), S.memmove_exchange, world, seed)
    S.assert_sharded_matches([got[r][0] for r in range(world)], srcs, S.run_random(oracle, seed), world)
    # storm: shard deliveries concatenate to the single-shard inbox; counters sum
    single = S.run_storm(oracle, n_inst=600, rounds=3, seed=4)
    for r in range(3):
        cat = {f: np.concatenate([got[k][1][r]["deliv"][f] for k in range(world)]) for f in single[r]["deliv"]}
        S.assert_same(cat, single[r]["deliv"], f"storm round {r}")
        assert all(got[k][1][r]["now"] == single[r]["now"] for k in range(world))
    tot = {}
    for k in range(world):
        for name, v in got[k][1][-1]["stats"].items():
            tot[name] = tot.get(name, 0) + v
    assert tot == single[-1]["stats"]
