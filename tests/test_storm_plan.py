"""The storm plan reactor (tgsim_storm_*): plans/benchmarks/storm.go:117-190's dial
semaphore, DialTimeout, writesem and conn.Write blocking on a full send buffer, for every instance
on the device. Hand-computed answers on the oracle and the HIP library, the protocol (a reaction
after every window), randomised HIP-vs-oracle parity window by window, and the plan at 20k
instances on HIP against the oracle."""
import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd import plans as P
from testground_amd.network import int_to_ip
from testground_amd.sim import SimConfig, Simulator, make_rule, make_shape
from tests import scenarios as S

MS = 1_000_000
SEC = 1000 * MS
W = MS
NONE = np.iinfo(np.int64).min


def drive(sim, keep=True, max_windows=100_000):
    """Reactions after every window at the proposed ends until nothing is active. Returns the
    windows' observations (sorted statuses, deliveries, proposal, active count)."""
    out, ne, w = [], sim.now + W, 0
    while w < max_windows:
        sim.advance(ne)
        st, d = sim.status(), sim.deliveries()
        ne, act = sim.storm_react()
        if keep:
            out.append(dict(status=np.sort(st), deliv=d, ne=ne, act=act))
        w += 1
        if act == 0:
            return out, w
    raise AssertionError("the storm reactor did not finish")


def _hand_case(b):
    """2 instances x 2 connections, one semaphore slot, 2 chunks each, a one-chunk send buffer,
    zero-latency links, 1 ms windows. Dials: 0.0 (t_ready 0) and 1.1 (t_ready 0) SYN at 0; their
    peers answer at the SYN's arrival (0), the SYN-ACKs arrive at 0 in the window [1, 2) ms: OK at 0.
    The slots are free from 0: 0.1 (t_ready 0.5 ms) dials at max(0.5, 0, horizon 1) = 1 ms, 1.0
    (t_ready 2.3 ms) at 2.3 ms; their SYN-ACKs leave at max(arrival, horizon) = 2 and 2.3 ms and
    arrive in [3, 4) ms: OK at 2 and 2.3 ms. Writes from 4 ms: each instance's round writes chunk 0
    of both connections (the second taker blocks on nothing: the first released the slot), then the
    first connection, queued again, finds its buffer full and holds the slot; at 5 ms both buffers
    have drained and both write their last chunk."""
    s = Simulator(SimConfig(n_instances=2, seed=7), binding=b)
    dst = [1, 1, 0, 0]
    t_ready = [0, 500_000, 2_300_000, 0]
    s.storm_setup(dst, t_ready, outgoing=2, concurrent=1, data_bytes=8192, msg_window=1, window_ns=W)
    s.storm_start()
    dial_obs, _ = drive(s)
    res, t_done = s.storm_dials()
    assert res.tolist() == [A.PROBE_OK] * 4
    assert t_done.tolist() == [0, 2 * MS, 2_300_000, 0]
    assert s.now == 4 * MS
    s.storm_write_start(s.now)
    obs, w = drive(s)
    arr = [(int(a), int(b_), int(q) & 0x3FFFFFFF, int(t)) for o in obs
           for a, b_, q, t in zip(o["deliv"]["src"], o["deliv"]["dst"], o["deliv"]["seq"], o["deliv"]["t_deliver"])]
    # (src, dst, k * n_chunks + j, t): chunk 0 of both connections at 4 ms, chunk 1 at 5 ms
    assert sorted(arr) == sorted([(0, 1, 0, 4 * MS), (0, 1, 2, 4 * MS), (1, 0, 0, 4 * MS), (1, 0, 2, 4 * MS),
                                  (0, 1, 1, 5 * MS), (0, 1, 3, 5 * MS), (1, 0, 1, 5 * MS), (1, 0, 3, 5 * MS)])
    failed, t_last, tot = s.storm_results()
    assert not failed.any() and t_last.tolist() == [5 * MS, 5 * MS]
    assert tot["chunks_written"] == tot["chunks_delivered"] == 8 and tot["bytes_written"] == 4 * 8192
    assert tot["dials_ok"] == 4 and tot["conns_writing"] == 0 and w == 2
    s.storm_end()
    s.close()


def test_storm_hand_oracle(oracle):
    _hand_case(oracle)


@pytest.mark.gpu
def test_storm_hand_hip(hip):
    _hand_case(hip)


def _blocking_case(b):
    """writesem blocks: one instance, three connections, one slot, a one-chunk buffer, 2 ms latency
    (windows of 1 ms), 2 chunks each. At the write start connection 0 writes and queues again, 1
    writes, 2 writes, then 0 takes the slot and blocks holding it (buffer full): no one else can
    write until 0's chunk arrives at +2 ms; then 0 writes its last chunk and leaves, 1 takes the
    slot and writes (its chunk arrived too), 2 writes. So chunk 0 of all three leaves at the start
    t_w and chunk 1 of all three at the reaction after the window the first chunks arrive in."""
    s = Simulator(SimConfig(n_instances=2, seed=3), binding=b)
    s.set_shapes([0, 1], [make_shape(latency_ns=2 * MS)] * 2)
    s.storm_setup([1, 1, 1, 0, 0, 0], [0] * 6, outgoing=3, concurrent=1, data_bytes=2 * 4096, msg_window=1,
                  window_ns=W)
    s.storm_start()
    drive(s, keep=False)
    res, t_done = s.storm_dials()
    assert (res == A.PROBE_OK).all()
    t_w = s.now
    s.storm_write_start(t_w)
    obs, _ = drive(s)
    sent = sorted((int(t) - 2 * MS, int(q) & 0x3FFFFFFF) for o in obs
                  for q, t, src in zip(o["deliv"]["seq"], o["deliv"]["t_deliver"], o["deliv"]["src"]) if src == 0)
    # first chunks (j = 0: k * 2) at t_w; the arrivals at t_w + 2 ms fall in the window ending at
    # t_w + 3 ms, whose reaction writes the second chunks
    assert sent == [(t_w, 0), (t_w, 2), (t_w, 4), (t_w + 3 * MS, 1), (t_w + 3 * MS, 3), (t_w + 3 * MS, 5)]
    s.storm_end()
    s.close()


def test_storm_blocking_oracle(oracle):
    _blocking_case(oracle)


@pytest.mark.gpu
def test_storm_blocking_hip(hip):
    _blocking_case(hip)


def _failure_case(b):
    """A dial refused by the dialler's own route ends at its start (REFUSED), and so does every dial
    of a disabled instance (no route: UNREACHABLE); one to a disabled peer waits out the 30 s
    DialTimeout (the reactor jumps to the deadline + 1 ns). On the one-slot semaphore a dial queued
    behind a refused one starts at once, one behind a finished dial at max(its t_ready, the slot's
    release, the horizon)."""
    s = Simulator(SimConfig(n_instances=4, seed=1), binding=b)
    s.add_rules(0, [make_rule(int_to_ip(s.get_ip(1)) + "/32", A.FILTER_DROP)])
    s.set_enabled(2, False)
    s.storm_setup([1, 2, 2, 3, 0, 1, 1, 0], [0, 0, 1 * MS, 0, 0, 0, 0, 0], outgoing=2, concurrent=1,
                  data_bytes=4096, window_ns=W)
    s.storm_start()
    _, w = drive(s, keep=False)
    res, t_done = s.storm_dials()
    OK, RF, TO = A.PROBE_OK, A.PROBE_REFUSED, A.PROBE_TIMEOUT
    # instance 0: 0 -> 1 refused at 0 (its blackhole), then 0 -> 2 (peer down) from 0 to 30 s
    # instance 1: 1 -> 3 (t_ready 0) OK at 0, then 1 -> 2 at max(1 ms, 0, horizon 1 ms) to 30.001 s
    # instance 2 (disabled, no route): both dials refused at 0
    # instance 3: 3 -> 1 OK at 0; 3 -> 0 at max(0, 0, horizon 1 ms), answered at max(1 ms, 2 ms): OK at 2 ms
    assert res.tolist() == [RF, TO, TO, OK, RF, RF, OK, OK]
    assert t_done.tolist() == [0, 30 * SEC, 30 * SEC + 1 * MS, 0, 0, 0, 0, 2 * MS]
    assert w < 20
    with pytest.raises(A.TgsimError) as e:
        s.storm_write_start(s.now)       # a dial failed: "outgoing-dials-done" never releases
    assert e.value.code == A.ESTATE
    s.storm_end()
    s.close()


def test_storm_failures_oracle(oracle):
    _failure_case(oracle)


@pytest.mark.gpu
def test_storm_failures_hip(hip):
    _failure_case(hip)


def _protocol_case(b):
    s = Simulator(SimConfig(n_instances=4, seed=1), binding=b)
    with pytest.raises(A.TgsimError) as e:
        s.storm_react()
    assert e.value.code == A.ESTATE
    s.storm_setup([1, 2, 3, 0], [0, 0, 0, 0], outgoing=1, concurrent=1, data_bytes=4096, window_ns=W)
    s.storm_start()
    s.advance(W)
    for call in (lambda: s.enqueue([0], [1], [5], [64], [W]), lambda: s.advance(2 * W),
                 lambda: s.storm_write_start(W), lambda: s.probe_setup([0, 1], 66, 66, SEC, W)):
        with pytest.raises(A.TgsimError) as e:
            call()
        assert e.value.code == A.ESTATE
    s.storm_react()
    with pytest.raises(A.TgsimError) as e:
        s.storm_react()
    assert e.value.code == A.ESTATE
    s.storm_end()
    s.advance(2 * W)          # detached: windows no longer need a reaction
    s.close()


def test_storm_protocol_oracle(oracle):
    _protocol_case(oracle)


@pytest.mark.gpu
def test_storm_protocol_hip(hip):
    _protocol_case(hip)


def _foreign_case(b, foreign=True):
    """messages the host stages beside the reactor with the storm's tags - a SYN to a
    connection index past `outgoing`, a chunk id past every connection, a chunk not yet written, a
    chunk whose destination is not its connection's, a SYN-ACK past every connection - are not the
    storm's: they leave every table in range and every count unchanged (unshaped links, so they
    take nothing from the storm's packets either). Returns the dial and write results."""
    n, O = 8, 2
    s = Simulator(SimConfig(n_instances=n, seed=3), binding=b)
    src = np.repeat(np.arange(n), O)
    dst = (src + 1 + np.arange(len(src)) % 3) % n
    s.storm_setup(dst, np.zeros(len(src), np.int64), outgoing=O, concurrent=1, data_bytes=3 * 4096,
                  msg_window=1, window_ns=W)
    nchunks = 3

    def inject():
        if not foreign:
            return
        t = s.horizon
        g = np.array([0, 1, 2, 3, 4, 5], np.uint32)
        seq = np.array([A.STORM_SYN | O, A.STORM_DATA | (O * nchunks + 7), A.STORM_DATA | (nchunks - 1),
                        A.STORM_DATA | 0, A.STORM_SYNACK | (n * O + 3), A.STORM_DATA | 0x3FFFFFFF], np.uint32)
        d = (g + 1) % n
        d[3] = (g[3] + 5) % n      # not connection 3.0's destination
        s.enqueue(g, d, seq, np.full(len(g), 66, np.uint32), np.full(len(g), t, np.int64))

    def run():
        ne, w = s.now + W, 0
        while True:
            s.advance(ne)
            ne, act = s.storm_react()
            w += 1
            if act == 0:
                return w
            inject()

    s.storm_start()
    inject()
    wd = run()
    res, t_done = s.storm_dials()
    s.storm_write_start(s.now)
    inject()
    ww = run()
    failed, t_last, tot = s.storm_results()
    s.storm_end()
    s.close()
    return dict(wd=wd, res=res, t_done=t_done, ww=ww, failed=failed, t_last=t_last, tot=tot)


def _assert_foreign_ignored(b):
    a, ref = _foreign_case(b), _foreign_case(b, foreign=False)
    assert (a["res"] == A.PROBE_OK).all()
    for k in ("res", "t_done", "failed", "t_last"):
        assert np.array_equal(a[k], ref[k]), k
    assert a["tot"] == ref["tot"] and (a["wd"], a["ww"]) == (ref["wd"], ref["ww"])
    return a


def test_storm_foreign_messages_oracle(oracle):
    _assert_foreign_ignored(oracle)


@pytest.mark.gpu
def test_storm_foreign_messages_hip(hip, oracle):
    a, b = _assert_foreign_ignored(hip), _foreign_case(oracle)
    for k in ("res", "t_done", "failed", "t_last"):
        assert np.array_equal(a[k], b[k]), k
    assert a["tot"] == b["tot"]


def random_run(b, seed, n=60, keep=True, shard=None):
    """Shaped, lossy, duplicating links, a few blackhole / prohibit rules and a disabled instance:
    dials refused, timed out and OK; then (on a second context, lossless while it dials) the write
    phase with blocking writers and lost chunks. shard = (k, world, make_transport): shard k of a
    sharded run (configuration calls go to every shard; results are the shard's own)."""
    rng = np.random.default_rng(seed)
    out = {}
    for phase in ("dials", "writes"):
        kw = dict(shard_id=shard[0], n_shards=shard[1], exchange_cap=1 << 13) if shard else {}
        s = Simulator(SimConfig(n_instances=n, seed=seed, max_msgs_per_window=1 << 15, max_records=1 << 17, **kw),
                      binding=b)
        if shard:
            s.set_transport(shard[2](phase))
        kw = [dict(latency_ns=int(rng.integers(0, 4)) * MS, jitter_ns=int(rng.integers(0, 3)) * MS // 2,
                   loss=float(rng.choice([0.0, 0.0, 3.0])), duplicate=float(rng.choice([0.0, 5.0])),
                   bandwidth_bps=int(rng.choice([0, 0, 50_000_000]))) for _ in range(n)]
        lossless = [make_shape(**{**k, "loss": 0.0}) for k in kw]
        s.set_shapes(np.arange(n), [make_shape(**k) for k in kw] if phase == "dials" else lossless)
        O = int(rng.integers(1, 5))
        src = np.repeat(np.arange(n), O)
        dst = (src + rng.integers(1, n, len(src))) % n
        t_ready = rng.integers(0, 40, len(src)) * MS // 3
        if phase == "dials":
            ip = [int_to_ip(s.get_ip(g)) + "/32" for g in range(n)]
            for g in rng.choice(n, n // 6, replace=False):
                tgt = rng.choice(n, 4, replace=False)
                s.add_rules(int(g), [make_rule(ip[int(t)], int(rng.choice([A.FILTER_DROP, A.FILTER_REJECT])))
                                     for t in tgt if t != g])
            s.set_enabled(int(rng.integers(n)), False)
        s.storm_setup(dst, t_ready, outgoing=O, concurrent=int(rng.integers(1, 4)),
                      data_bytes=int(rng.integers(0, 9)) * 1500 + int(rng.integers(0, 3)) * 4096,
                      msg_window=int(rng.integers(1, 4)), dial_timeout_ns=int(rng.integers(30, 90)) * MS,
                      window_ns=W)
        s.storm_start()
        obs, w = drive(s, keep=keep)
        res, t_done = s.storm_dials()
        out[phase] = dict(obs=obs, w=w, res=res, t_done=t_done)
        if phase == "writes":
            assert (res == A.PROBE_OK).all()
            s.set_shapes(np.arange(n), [make_shape(**k) for k in kw])
            s.storm_write_start(s.now)
            obs, w = drive(s, keep=keep)
            failed, t_last, tot = s.storm_results()
            out["write_obs"], out["write_w"] = obs, w
            out["failed"], out["t_last"], out["totals"] = failed, t_last, tot
        out[phase + "_stats"] = S.parity_stats(s)
        s.storm_end()
        s.close()
    return out


def test_storm_random_oracle_properties(oracle):
    r = random_run(oracle, 1)
    res = r["dials"]["res"]
    assert {A.PROBE_OK, A.PROBE_REFUSED, A.PROBE_TIMEOUT} <= set(np.unique(res).tolist())
    tot = r["totals"]
    assert tot["chunks_written"] == tot["chunks_delivered"] + tot["chunks_failed"]
    assert tot["conns_writing"] == 0 and tot["dials_pending"] == 0
    assert tot["chunks_failed"] > 0 and r["failed"].any() and not r["failed"].all()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_storm_random_hip_matches_oracle(hip, oracle, seed):
    a, b = random_run(hip, seed), random_run(oracle, seed)
    for k in ("dials", "writes"):
        assert a[k]["w"] == b[k]["w"], f"{k}: window count"
        S.assert_same(a[k]["obs"], b[k]["obs"])
        assert np.array_equal(a[k]["res"], b[k]["res"]) and np.array_equal(a[k]["t_done"], b[k]["t_done"])
        assert a[k + "_stats"] == b[k + "_stats"]
    assert a["write_w"] == b["write_w"]
    S.assert_same(a["write_obs"], b["write_obs"])
    assert np.array_equal(a["failed"], b["failed"]) and np.array_equal(a["t_last"], b["t_last"])
    assert a["totals"] == b["totals"]


def sharded_random_run(b, seed, world, device=False):
    """random_run on `world` shards, one thread each over the thread-group transport (one group per
    phase: each phase is a fresh set of contexts)."""
    from testground_amd.exchange import ThreadGroup, run_threads
    groups = {ph: ThreadGroup(world, device=device) for ph in ("dials", "writes")}
    return run_threads([lambda k=k: random_run(b, seed, shard=(k, world, lambda ph, k=k: groups[ph].member(k)))
                        for k in range(world)])


def assert_storm_shards_match(outs, single):
    """The shards' observations against the single-context run: the same windows, proposals and
    active counts; statuses as one multiset; deliveries, dial outcomes and per-instance results
    concatenated in shard order; counters summed."""
    cat = lambda xs: np.concatenate(xs)
    for k in ("dials", "writes"):
        assert all(o[k]["w"] == single[k]["w"] for o in outs), f"{k}: window count"
        for w, ref in enumerate(single[k]["obs"]):
            obs = [o[k]["obs"][w] for o in outs]
            assert all((x["ne"], x["act"]) == (ref["ne"], ref["act"]) for x in obs), f"{k} window {w}: proposal"
            S.assert_same(np.sort(cat([x["status"] for x in obs])), ref["status"], f"{k} window {w} status")
            for f in ref["deliv"]:
                S.assert_same(cat([x["deliv"][f] for x in obs]), ref["deliv"][f], f"{k} window {w} deliv.{f}")
        assert np.array_equal(cat([o[k]["res"] for o in outs]), single[k]["res"])
        assert np.array_equal(cat([o[k]["t_done"] for o in outs]), single[k]["t_done"])
    assert all(o["write_w"] == single["write_w"] for o in outs)
    for w, ref in enumerate(single["write_obs"]):
        obs = [o["write_obs"][w] for o in outs]
        assert all((x["ne"], x["act"]) == (ref["ne"], ref["act"]) for x in obs), f"write window {w}: proposal"
        S.assert_same(np.sort(cat([x["status"] for x in obs])), ref["status"], f"write window {w} status")
        for f in ref["deliv"]:
            S.assert_same(cat([x["deliv"][f] for x in obs]), ref["deliv"][f], f"write window {w} deliv.{f}")
    assert np.array_equal(cat([o["failed"] for o in outs]), single["failed"])
    assert np.array_equal(cat([o["t_last"] for o in outs]), single["t_last"])
    for k in single["totals"]:
        assert sum(o["totals"][k] for o in outs) == single["totals"][k], k
    for ph in ("dials_stats", "writes_stats"):
        for k in single[ph]:
            assert sum(o[ph][k] for o in outs) == single[ph][k], (ph, k)


@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2), (4, 3)])
def test_storm_sharded_threads_oracle(oracle, world, seed):
    """The storm reactor sharded: every instance's dials and writes on its own
    shard, SYNs and requests reach the peer's shard through the window's exchange, the listener's
    answers and chunk arrivals reach the dialer's shard as notices, the proposal is collective -
    equal to the single context window by window."""
    assert_storm_shards_match(sharded_random_run(oracle, seed, world), random_run(oracle, seed))


@pytest.mark.gpu
@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2), (4, 3)])
def test_storm_sharded_threads_hip(hip, oracle, world, seed):
    """The sharded reactor on the device: `world` HIP contexts on one GPU (thread-group transport,
    device buffers) equal the single oracle context window by window."""
    assert_storm_shards_match(sharded_random_run(hip, seed, world, device=True), random_run(oracle, seed))


def storm_reactor_run(b, n, shard=None, outgoing=5, delay_ms=2000, limit=3, size=8 * 1024):
    """The storm plan's reactor calls (plans.storm at conn_outgoing 5, conn_delay_ms 2000,
    concurrent_dials 3, data_size_kb 8, message mode): dials until none is active, the write phase
    from the last dial's end, writes until none is active. shard = (k, world, transport)."""
    rng = np.random.default_rng(0)
    src = np.repeat(np.arange(n), outgoing)
    dst = (src + rng.integers(1, n, len(src))) % n
    t_ready = rng.integers(0, delay_ms, len(src)) * MS
    kw = dict(shard_id=shard[0], n_shards=shard[1], exchange_cap=1 << 16) if shard else {}
    s = Simulator(SimConfig(n_instances=n, seed=1, max_msgs_per_window=max(1 << 18, 64 * n),
                            max_records=max(1 << 20, 128 * n), **kw), binding=b)
    if shard:
        s.set_transport(shard[2])
    s.storm_setup(dst, t_ready, outgoing=outgoing, concurrent=limit, data_bytes=size, window_ns=W)
    s.storm_start()
    props = []

    def windows():
        ne = s.now + W
        while True:
            s.advance(ne)
            ne, act = s.storm_react()
            props.append((ne, act))
            if act == 0:
                return

    windows()
    res, t_done = s.storm_dials()
    s.storm_write_start(s.now)
    windows()
    failed, t_last, tot = s.storm_results()
    out = dict(props=props, res=res, t_done=t_done, failed=failed, t_last=t_last, tot=tot, now=s.now,
               stats=S.parity_stats(s))
    s.storm_end()
    s.close()
    return out


def assert_reactor_shards_match(outs, single):
    assert all(o["props"] == single["props"] and o["now"] == single["now"] for o in outs)
    for k in ("res", "t_done", "failed", "t_last"):
        assert np.array_equal(np.concatenate([o[k] for o in outs]), single[k]), k
    for k in single["tot"]:
        assert sum(o["tot"][k] for o in outs) == single["tot"][k], k
    for k in single["stats"]:
        assert sum(o["stats"][k] for o in outs) == single["stats"][k], k


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_storm_reactor_20k_sharded_hip(hip, oracle, world):
    """the storm plan's reactor at 20k instances as 2 and 4 HIP contexts on one GPU
    (thread-group transport) equals the single HIP context, which equals the oracle."""
    from testground_amd.exchange import ThreadGroup, run_threads
    single = storm_reactor_run(hip, 20_000)
    assert (single["res"] == A.PROBE_OK).all() and single["tot"]["chunks_delivered"] == 20_000 * 5 * 2
    if world == 2:
        ref = storm_reactor_run(oracle, 20_000)
        assert single["props"] == ref["props"] and single["tot"] == ref["tot"] and single["stats"] == ref["stats"]
        for k in ("res", "t_done", "failed", "t_last"):
            assert np.array_equal(single[k], ref[k]), k
    g = ThreadGroup(world, device=True)
    outs = run_threads([lambda k=k: storm_reactor_run(hip, 20_000, shard=(k, world, g.member(k)))
                        for k in range(world)])
    assert_reactor_shards_match(outs, single)


def test_storm_reactor_sharded_threads_oracle(oracle):
    """The same on the oracle at 2,000 instances over 3 shards."""
    from testground_amd.exchange import ThreadGroup, run_threads
    single = storm_reactor_run(oracle, 2000)
    g = ThreadGroup(3)
    outs = run_threads([lambda k=k: storm_reactor_run(oracle, 2000, shard=(k, 3, g.member(k))) for k in range(3)])
    assert_reactor_shards_match(outs, single)


def storm_plan_run(b, n, params, seed=1):
    env = P.PlanEnv(n, seed=seed, test_case="storm", params=params, binding=b,
                    sim_kw=dict(max_msgs_per_window=max(1 << 18, 64 * n), max_records=max(1 << 20, 128 * n)))
    ok = P.storm(env)
    r = dict(ok=ok, failures=list(env.failures), now=env.sim.now, totals=getattr(env, "storm_totals", None),
             windows=env.storm_windows, stats={k: v for k, v in env.sim.stats().items() if k != "windows"})
    env.close()
    return r


@pytest.mark.gpu
def test_storm_plan_20k_hip_matches_oracle(hip, oracle):
    """the storm plan at 20k instances (5 dials each, 8 KiB per connection, dials
    spread over 2 s) on the device reactor, equal to the oracle."""
    params = {"conn_outgoing": "5", "conn_delay_ms": "2000", "concurrent_dials": "3", "data_size_kb": "8"}
    a = storm_plan_run(hip, 20_000, params)
    b = storm_plan_run(oracle, 20_000, params)
    assert a["ok"].all() and np.array_equal(a["ok"], b["ok"])
    for k in ("now", "totals", "windows", "stats"):
        assert a[k] == b[k], k
    assert a["totals"]["chunks_delivered"] == 20_000 * 5 * 2


def _big_signal_batch(b, n=150_000):
    """A signal batch larger than the device's batch (the storm's N * outgoing "outgoing-dials-done"
    signals): cut in (t, instance) order into device batches, every state's sequence numbers are those
    one batch gives, and a barrier on the last one releases at the last signal."""
    rng = np.random.default_rng(9)
    s = Simulator(SimConfig(n_instances=40_000, seed=1, max_states=8), binding=b)
    inst = rng.integers(0, 40_000, n).astype(np.uint32)
    t = rng.integers(0, 5_000, n) * 1000
    st = rng.integers(0, 3, n).astype(np.uint32)
    seq = s.signal(st, inst, t)
    w = s.barrier(2, int((st == 2).sum()), 0)
    rel = s.poll(w)
    s.close()
    return seq, rel


def test_big_signal_batch_oracle(oracle):
    seq, rel = _big_signal_batch(oracle)
    assert rel >= 0 and len(np.unique(seq)) < len(seq)


@pytest.mark.gpu
def test_big_signal_batch_hip_matches_oracle(hip, oracle):
    a, b = _big_signal_batch(hip), _big_signal_batch(oracle)
    assert np.array_equal(a[0], b[0]) and a[1] == b[1]


# ---- TCP mode: connections, the SYN a bare segment, the socket buffer 2 x cwnd ----------------------

def drive_tcp(sim, keep=True, max_windows=100_000):
    """As drive, with the TCP reaction (ACK clock, timers) before the storm's."""
    out, ne, w = [], sim.now + W, 0
    while w < max_windows:
        sim.advance(ne)
        st, d = sim.status(), sim.deliveries()
        sim.tcp_react()
        ne, act = sim.storm_react()
        if keep:
            out.append(dict(status=np.sort(st), deliv=d, ne=ne, act=act))
        w += 1
        if act == 0:
            return out, w
    raise AssertionError("the storm reactor did not finish")


def _tcp_hand_case(b):
    """2 instances x 1 connection, zero latency, 1 ms windows, 3 chunks of 4 KiB (3 segments each).
    The SYN leaves at 0 and arrives at 0; its ACK leaves then (a late send from the reaction) and
    is delivered in the window [1, 2) ms, so both dials end at that window's end, 2 ms. From the write start at 2 ms
    a connection writes one chunk per reaction while 2 x cwnd (IW10) covers the unACKed segments:
    chunk 0 at 2 ms, 1 at 3 ms, 2 at 4 ms, each delivered in the window it is sent in; every write
    settles DELIVERED and the last conn.Write returned at 4 ms."""
    s = Simulator(SimConfig(n_instances=2, seed=11), binding=b)
    s.tcp_enable(acks=True, rto_ns=200 * MS)
    s.storm_setup([1, 0], [0, 0], outgoing=1, concurrent=1, data_bytes=3 * 4096, window_ns=W)
    s.storm_start()
    drive_tcp(s, keep=False)
    res, t_done = s.storm_dials()
    assert res.tolist() == [A.PROBE_OK] * 2 and t_done.tolist() == [2 * MS, 2 * MS]
    assert s.now == 2 * MS
    s.storm_write_start(s.now)
    obs, w = drive_tcp(s)
    data = sorted((int(sq) >> 4, int(t)) for o in obs
                  for sq, t, src in zip(o["deliv"]["seq"], o["deliv"]["t_deliver"], o["deliv"]["src"])
                  if not (int(sq) & A.TCP_ACK_BIT) and src == 0)
    # instance 0's segments: SYN = its first reserved segment, then 3 per chunk
    assert [t for _, t in data] == [2 * MS] * 3 + [3 * MS] * 3 + [4 * MS] * 3
    failed, t_last, tot = s.storm_results()
    assert not failed.any() and t_last.tolist() == [4 * MS, 4 * MS]
    assert tot["chunks_written"] == tot["chunks_delivered"] == 6 and tot["chunks_failed"] == 0 and w == 3
    st = s.tcp_stats()
    assert st["writes"] == 8 and st["delivered"] == 8 and st["retransmissions"] == 0
    s.storm_end()
    # the reactor's connections stay closed to host writes (their queues end where the
    # reactor left them); a new connection takes writes
    with pytest.raises(A.TgsimError) as e:
        s.tcp_write([0], [100], [s.now])
    assert e.value.code == A.ESTATE
    (c,) = s.tcp_connect([0], [1])
    s.tcp_write([c], [100], [s.now])
    s.close()


def test_storm_tcp_hand_oracle(oracle):
    _tcp_hand_case(oracle)


@pytest.mark.gpu
def test_storm_tcp_hand_hip(hip):
    _tcp_hand_case(hip)


def _tcp_dial_timeout_case(b):
    """in TCP mode a dial also ends at net.DialTimeout (storm.go:144), not only when its
    SYN write gives up (16 attempts from a 20 ms RTO: hours). 3 instances x 2 connections, one dial
    slot, zero latency, 1 ms windows, DialTimeout 50 ms; instance 1's link drops everything, so its
    SYNs and its ACKs are lost. 0.0 -> 1 and 1.0 -> 0 time out at 50 ms (seen after the window
    ending at 51 ms); their second dials start at 51 ms: 0.1 -> 2 is ACKed in [52, 53) ms, OK at
    53 ms; 1.1 -> 2 times out at 101 ms. 2.0 -> 0 is OK at 2 ms (the hand case's timing), 2.1 -> 1
    starts at 2 ms and times out at 52 ms. Each timed-out SYN write fails at its deadline."""
    s = Simulator(SimConfig(n_instances=3, seed=5), binding=b)
    s.tcp_enable(acks=True, rto_ns=20 * MS, max_attempts=16)
    s.set_shapes([1], [make_shape(loss=100.0)])
    s.storm_setup([1, 2, 0, 2, 0, 1], [0] * 6, outgoing=2, concurrent=1, data_bytes=4096,
                  dial_timeout_ns=50 * MS, window_ns=W)
    s.storm_start()
    _, w = drive_tcp(s, keep=False)
    res, t_done = s.storm_dials()
    T, OK = A.PROBE_TIMEOUT, A.PROBE_OK
    assert res.tolist() == [T, OK, T, T, OK, T]
    assert t_done.tolist() == [50 * MS, 53 * MS, 50 * MS, 101 * MS, 2 * MS, 52 * MS]
    assert w == 102 and s.now == 102 * MS  # 1.1 resolved after the window ending at 102 ms
    st = s.tcp_stats()
    s.storm_end()
    s.close()
    return res, t_done, st


def test_storm_tcp_dial_timeout_oracle(oracle):
    _tcp_dial_timeout_case(oracle)


@pytest.mark.gpu
def test_storm_tcp_dial_timeout_hip(hip, oracle):
    a, b = _tcp_dial_timeout_case(hip), _tcp_dial_timeout_case(oracle)
    assert a[2] == b[2]


def random_tcp_run(b, seed, n=40, keep=True, restart=()):
    """TCP storm on shaped, lossy, duplicating, corrupting links: SYN and data retransmissions, the
    Reno window's collapses, writes blocked on the socket buffer; window by window. restart: window
    counts after whose reactions the run is snapshotted and restored into a fresh context."""
    rng = np.random.default_rng(seed)
    cfg = SimConfig(n_instances=n, seed=seed, max_msgs_per_window=1 << 15, max_records=1 << 17)
    enable = dict(acks=True, rto_ns=30 * MS, max_attempts=6, max_writes=1 << 16, max_segments=1 << 18)
    s = Simulator(cfg, binding=b)
    s.tcp_enable(**enable)
    s.set_shapes(np.arange(n), [make_shape(latency_ns=int(rng.integers(1, 4)) * MS, jitter_ns=int(rng.integers(0, 2)) * MS // 2,
                                           loss=float(rng.choice([0.0, 2.0])), duplicate=float(rng.choice([0.0, 5.0])),
                                           corrupt=float(rng.choice([0.0, 1.0])),
                                           bandwidth_bps=int(rng.choice([0, 100_000_000]))) for _ in range(n)])
    O = int(rng.integers(1, 4))
    src = np.repeat(np.arange(n), O)
    dst = (src + rng.integers(1, n, len(src))) % n
    t_ready = rng.integers(0, 30, len(src)) * MS // 2
    setup = dict(outgoing=O, concurrent=int(rng.integers(1, 3)),
                 data_bytes=int(rng.integers(1, 6)) * 4096 + int(rng.integers(0, 2)) * 1000, window_ns=W)
    s.storm_setup(dst, t_ready, **setup)
    s.storm_start()
    windows = [0]

    def drive(s):
        out, ne, w = [], s.now + W, 0
        while True:
            s.advance(ne)
            st, d = s.status(), s.deliveries()
            s.tcp_react()
            ne, act = s.storm_react()
            if keep:
                out.append(dict(status=np.sort(st), deliv=d, ne=ne, act=act))
            w += 1
            windows[0] += 1
            if act == 0:
                return out, w, s
            if windows[0] in restart:
                image = s.snapshot()
                s.close()
                s = Simulator(cfg, binding=b)
                s.tcp_enable(**enable)
                s.storm_setup(dst, t_ready, **setup)
                s.restore(image)

    dial_obs, dial_w, s = drive(s)
    res, t_done = s.storm_dials()
    out = dict(dial_obs=dial_obs, dial_w=dial_w, res=res, t_done=t_done)
    if (res == A.PROBE_OK).all():
        s.storm_write_start(s.now)
        out["write_obs"], out["write_w"], s = drive(s)
        out["failed"], out["t_last"], out["totals"] = s.storm_results()
    out["tcp"] = s.tcp_stats()
    out["stats"] = S.parity_stats(s)
    s.storm_end()
    s.close()
    return out


def test_storm_tcp_random_oracle(oracle):
    r = random_tcp_run(oracle, 1)
    assert "totals" in r and r["tcp"]["retransmissions"] > 0
    tot = r["totals"]
    assert tot["chunks_written"] == tot["chunks_delivered"] + tot["chunks_failed"] and tot["conns_writing"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,restart", [(1, ()), (2, ()), (3, ()), (1, (3, 9, 20, 31))],
                         ids=["1", "2", "3", "1-resumed"])
def test_storm_tcp_random_hip_matches_oracle(hip, oracle, seed, restart):
    """(1-resumed: the TCP storm reactor snapshotted and restored four times; tgsim_snapshot)"""
    a, b = random_tcp_run(hip, seed, restart=restart), random_tcp_run(oracle, seed)
    assert a["dial_w"] == b["dial_w"]
    S.assert_same(a["dial_obs"], b["dial_obs"])
    assert np.array_equal(a["res"], b["res"]) and np.array_equal(a["t_done"], b["t_done"])
    assert ("totals" in a) == ("totals" in b)
    if "totals" in a:
        assert a["write_w"] == b["write_w"]
        S.assert_same(a["write_obs"], b["write_obs"])
        assert np.array_equal(a["failed"], b["failed"]) and np.array_equal(a["t_last"], b["t_last"])
        assert a["totals"] == b["totals"]
    assert a["tcp"] == b["tcp"] and a["stats"] == b["stats"]
