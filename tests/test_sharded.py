"""CPU: the N>1 path. Instances are sharded in contiguous ranges; each window the
sender shard shapes its copies and one all-to-all moves cross-shard records to the receiver shard.
The sharded run must equal the single-shard run bit for bit: per-shard statuses, the receiver
shard's deliveries and inbox offsets, and the summed counters.

  * in-process, caller-driven: 2 and 3 oracle shards exchanging through memmove between
    advance_begin and advance_end (the transport-less protocol of include/tgsim.h);
  * in-process, transport-driven: one thread per shard (testground_amd.exchange.ThreadGroup); every
    shard makes the single-shard calls (tgsim_advance, the storm's gen / barrier / advance_to_barrier)
    and the library runs the exchange, the storm batch's MAX all-reduce and the signal all-gather;
  * multi-process: world_size 2 and 3 over torch.distributed gloo (GlooTransport), the same calls -
    the protocol bench.py runs over the library's RCCL communicator on GPUs.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

from tests import scenarios as S
from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator


@pytest.mark.parametrize("world,seed", [(2, 1), (2, 5), (3, 2)])
def test_sharded_equals_single_in_process(oracle, world, seed):
    outs, srcs = S.run_random_sharded(lambda c: Simulator(c, binding=oracle), S.memmove_exchange, world, seed)
    S.assert_sharded_matches(outs, srcs, S.run_random(oracle, seed), world)


def _with_transport(binding, tr):
    def make(c):
        s = Simulator(c, binding=binding)
        s.set_transport(tr)
        return s
    return make


@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2)])
def test_sharded_transport_threads(oracle, world, seed):
    """tgsim_advance on every shard, the exchange inside the call (ThreadGroup transport)."""
    outs = S.sharded_threads(world, lambda k, tr: S.run_random_sharded(
        _with_transport(oracle, tr), None, world, seed, local=[k])[0][0])
    _, srcs = S.run_random_sharded(lambda c: Simulator(c, binding=oracle), S.memmove_exchange, world, seed)
    S.assert_sharded_matches(outs, srcs, S.run_random(oracle, seed), world)


@pytest.mark.parametrize("world", [2, 3])
def test_storm_transport_threads(oracle, world):
    """bench.py's storm step on every shard with the single-shard calls: the batch's first / last
    time is MAX-reduced and every shard holds the whole sync state, so the barrier resolves alike."""
    n, rounds = 600, 4
    outs = S.sharded_threads(world, lambda k, tr: S.run_storm(
        oracle, n_inst=n, rounds=rounds, cfg_kw=S.shard_cfg(world, k, exchange_cap=1 << 14),
        setup=lambda sim: sim.set_transport(tr)))
    S.assert_storm_sharded(outs, S.run_storm(oracle, n_inst=n, rounds=rounds), world, n)


def test_signal_gather_threads(oracle):
    """tgsim_sync_signal on a sharded run: each shard passes its own signals; sequence numbers and
    barrier releases equal those of the single-shard call with every signal."""
    world = 3
    rng = np.random.default_rng(8)
    batches = []
    for b in range(4):
        n = int(rng.integers(0, 400))
        batches.append((rng.integers(0, 4, n), rng.integers(0, 300, n), 1000 * b + rng.integers(0, 1000, n)))

    def shard(k, tr):
        sim = Simulator(SimConfig(n_instances=300, seed=1, shard_id=k, n_shards=world, max_states=16), binding=oracle)
        sim.set_transport(tr)
        lo, hi = S.shard_range(300, k, world)
        res = []
        for st, ins, t in batches:
            m = (ins >= lo) & (ins < hi)
            res.append((m, sim.signal(st[m], ins[m], t[m])))
            res.append(sim.poll(sim.barrier(1, 50, 0)))
        sim.close()
        return res

    outs = S.sharded_threads(world, shard)
    ref = Simulator(SimConfig(n_instances=300, seed=1, max_states=16), binding=oracle)
    for i, (st, ins, t) in enumerate(batches):
        seq = ref.signal(st, ins, t)
        for k in range(world):
            m, got = outs[k][2 * i]
            assert np.array_equal(got, seq[m])
        rel = ref.poll(ref.barrier(1, 50, 0))
        assert all(outs[k][2 * i + 1] == rel for k in range(world))
    ref.close()


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
        from testground_amd.exchange import GlooTransport
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ob = oracle_binding()
        tr = GlooTransport(dist)
        outs, _ = S.run_random_sharded(_with_transport(ob, tr), None, world, seed, local=[rank])
        storm = S.run_storm(ob, n_inst=600, rounds=3, cfg_kw=S.shard_cfg(world, rank, exchange_cap=1 << 14),
                            setup=lambda sim: sim.set_transport(tr))
        from tests.test_storm_plan import random_run
        reactor = random_run(ob, seed, shard=(rank, world, lambda ph: tr))  # the storm plan's reactor
        from tests.test_tcp import run_tcp_storm  # TCP mode: arrivals forwarded to the writers' shards
        tcp = run_tcp_storm(ob, n=400, rounds=4, acks=True, cfg_kw=S.shard_cfg(world, rank, exchange_cap=1 << 14),
                            setup=lambda sim: sim.set_transport(tr))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, outs[0], (storm, reactor, tcp)))
    except Exception:  # surface the failure in the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


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
    S.assert_storm_sharded([got[r][1][0] for r in range(world)], S.run_storm(oracle, n_inst=600, rounds=3), world, 600)
    from tests.test_storm_plan import assert_storm_shards_match, random_run
    assert_storm_shards_match([got[r][1][1] for r in range(world)], random_run(oracle, seed))
    from tests.test_tcp import combine_tcp_storm, run_tcp_storm
    a = combine_tcp_storm([got[r][1][2] for r in range(world)], world, 400, 4)
    b = run_tcp_storm(oracle, n=400, rounds=4, acks=True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]


def _failing_shard_run(binding, device=False, world=3):
    """World 3 over a thread group; two windows run normally, then shard 1 asks for a window that ends
    before its clock (ECAUSALITY) while the others enter the window's exchange. Every shard must
    return an error, within seconds, instead of waiting for shard 1."""
    import threading
    import time

    from testground_amd import _abi as A
    from testground_amd.exchange import ThreadGroup, run_threads
    MS = 1_000_000
    g = ThreadGroup(world, device=device, timeout=120.0)
    codes, elapsed = [None] * world, [None] * world
    start = threading.Barrier(world)

    def shard(k):
        sim = Simulator(SimConfig(n_instances=24, seed=1, shard_id=k, n_shards=world, exchange_cap=1 << 10,
                                  max_msgs_per_window=1 << 12, max_records=1 << 14), binding=binding)
        sim.set_transport(g.member(k))
        for w in range(2):
            src = np.arange(sim.lo, sim.hi, dtype=np.uint32)
            sim.enqueue(src, (src + 5) % 24, np.full(len(src), w), np.full(len(src), 100), np.full(len(src), w * MS))
            sim.advance((w + 1) * MS)
        start.wait()
        t0 = time.perf_counter()
        try:
            sim.advance(1 * MS if k == 1 else 3 * MS)   # shard 1: t_end before its clock
            codes[k] = A.OK
        except A.TgsimError as e:
            codes[k] = e.code
        elapsed[k] = time.perf_counter() - t0
        try:                                             # the context refuses sharded calls now
            sim.advance(4 * MS)
            after = A.OK
        except A.TgsimError as e:
            after = e.code
        sim.close()
        return after

    after = run_threads([lambda k=k: shard(k) for k in range(world)])
    return codes, elapsed, after


def test_shard_failure_aborts_peers(oracle):
    from testground_amd import _abi as A
    codes, elapsed, after = _failing_shard_run(oracle)
    assert codes[1] == A.ECAUSALITY
    assert codes[0] == A.EHIP and codes[2] == A.EHIP          # their exchange failed instead of waiting
    assert max(elapsed) < 10.0
    assert all(a == A.ESTATE for a in after)


@pytest.mark.gpu
def test_shard_failure_aborts_peers_hip(hip):
    from testground_amd import _abi as A
    codes, elapsed, after = _failing_shard_run(hip, device=True)
    assert codes[1] == A.ECAUSALITY and codes[0] == A.EHIP and codes[2] == A.EHIP
    assert max(elapsed) < 10.0 and all(a == A.ESTATE for a in after)


_RANK_PROBE = """
import json, os, sys
r = int(os.environ["RANK"])
print(json.dumps({k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
                 | {"argv": sys.argv[1:]}), flush=True)
sys.exit(int(os.environ.get("FAIL_RANK_CODE", "0")) if r == int(os.environ.get("FAIL_RANK", "-1")) else 0)
"""


def test_bench_spawns_its_own_ranks(tmp_path, capfd):
    """`python bench.py --gpus N` without torch.distributed.run starts the N ranks itself (VERDICT r4
    item 1): each child gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* and the parent's arguments;
    rank 0's output is forwarded; a failing rank makes the parent fail with its status."""
    import json
    import bench
    script = tmp_path / "probe.py"
    script.write_text(_RANK_PROBE)
    assert bench.spawn_ranks(3, argv=["--gpus", "3"], script=str(script)) == 0
    lines = [json.loads(x) for x in capfd.readouterr().out.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["RANK"] == "0" and lines[0]["WORLD_SIZE"] == "3"
    assert lines[0]["MASTER_ADDR"] == "127.0.0.1" and lines[0]["argv"] == ["--gpus", "3"]
    os.environ["FAIL_RANK"], os.environ["FAIL_RANK_CODE"] = "2", "7"
    try:
        assert bench.spawn_ranks(3, argv=[], script=str(script)) == 7
    finally:
        del os.environ["FAIL_RANK"], os.environ["FAIL_RANK_CODE"]


@pytest.mark.parametrize("n_msgs,ok", [(448, True), (512, True), (513, False)])
def test_skewed_exchange_bound_oracle(oracle, n_msgs, ok):
    """The per-peer exchange bound is the block's usable records (exchange_cap 513: 8 slices of 64 =
    512), whichever producers fill it: 512 records to one peer pass, 513 are ECAPACITY."""
    res = S.run_skewed_exchange(oracle, n_msgs)
    if ok:
        assert res[0][0] == "ok" and res[1][0] == "ok"
        assert len(res[1][1]["dst"]) == n_msgs
    else:
        assert res[0] == ("err", A.ECAPACITY)

