"""Checkpoint / resume (tgsim_snapshot / tgsim_restore): a run that is snapshotted at a
window boundary, destroyed and restored into a fresh context continues exactly as the uninterrupted
run - which the oracle's uninterrupted run pins (every window's statuses, deliveries and inbox
offsets, the counters, sync sequence numbers and barrier releases). The checkpoints fall before
mid-run reconfigurations, inside queue-limit bursts with late sends, between storm rounds with
wheel records in flight, and between signal batches with open barriers."""
import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator, make_shape

from . import scenarios as S

MS = 1_000_000


def restarter(binding, at):
    """restart hook: after window `at`, snapshot, destroy, restore into a new context."""
    def f(w, sim):
        if w not in at:
            return sim
        image = sim.snapshot()
        cfg = sim.cfg
        sim.close()
        fresh = Simulator(cfg, binding=binding)
        fresh.restore(image)
        return fresh
    return f


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_random_resumed_matches_oracle(hip, oracle, seed):
    a = S.run_random(hip, seed, windows=8, restart=restarter(hip, {1, 3}))
    b = S.run_random(oracle, seed, windows=8)
    S.assert_same(a, b)


@pytest.mark.gpu
def test_burst_resumed_matches_oracle(hip, oracle):
    """queue-limit bursts and late sends at the reaction horizon across the checkpoint"""
    a = S.run_burst(hip, 1, restart=restarter(hip, {1, 5}))
    b = S.run_burst(oracle, 1)
    S.assert_same(a, b)


@pytest.mark.gpu
def test_storm_resumed_matches_oracle(hip, oracle):
    a = S.run_storm(hip, n_inst=2000, rounds=10, restart=restarter(hip, {3, 6}))
    b = S.run_storm(oracle, n_inst=2000, rounds=10)
    S.assert_same(a, b)


@pytest.mark.gpu
def test_sync_resumed_matches_oracle(hip, oracle):
    a = S.run_sync(hip, 5, restart=restarter(hip, {1, 3}))
    b = S.run_sync(oracle, 5)
    assert len(a) == len(b)
    for (ka, va), (kb, vb) in zip(a, b):
        assert ka == kb and np.array_equal(np.asarray(va), np.asarray(vb)), ka


@pytest.mark.gpu
def test_snapshot_refusals(hip):
    s = Simulator(SimConfig(n_instances=8, seed=1), binding=hip)
    s.set_shape(0, make_shape(latency_ns=5 * MS))
    s.advance(1 * MS)
    s.probe_setup([0, 1], 66, 66, 60_000 * MS, 100_000)
    s.probe_start(s.now)
    s.advance(2 * MS)
    with pytest.raises(A.TgsimError) as e:     # a probe reaction owed: not a window boundary
        s.snapshot()
    assert e.value.code == A.ESTATE
    s.close()
    s = Simulator(SimConfig(n_instances=8, seed=1), binding=hip)
    s.set_shape(0, make_shape(latency_ns=5 * MS))
    s.enqueue([0], [1], [0], [100], [0])
    s.advance(1 * MS)
    image = s.snapshot()
    other = Simulator(SimConfig(n_instances=9, seed=1), binding=hip)
    with pytest.raises(A.TgsimError) as e:     # another configuration
        other.restore(image)
    assert e.value.code == A.EINVAL
    same = Simulator(SimConfig(n_instances=8, seed=1), binding=hip)
    with pytest.raises(A.TgsimError) as e:     # truncated image: refused, the context unchanged
        same.restore(image[:-8])
    assert e.value.code == A.EINVAL
    old = bytearray(image)                     # an image of an older layout (version 01): named as such
    old[6:8] = b"01"
    with pytest.raises(A.TgsimError) as e:
        same.restore(bytes(old))
    assert e.value.code == A.EINVAL and "version 01" in str(e.value)
    same.enqueue([2], [3], [0], [10], [0])
    same.advance(1 * MS)
    assert same.deliveries()["dst"].tolist() == [3]
    same.restore(image)                        # the in-flight copy of 0 -> 1 arrives at 5 ms
    assert same.now == 1 * MS
    same.advance(10 * MS)
    d = same.deliveries()
    assert d["src"].tolist() == [0] and d["t_deliver"].tolist() == [5 * MS]
    s.tcp_enable()
    image2 = s.snapshot()                      # TCP mode is captured too: its image restores only
    with pytest.raises(A.TgsimError) as e:     # into a context with the same TCP configuration
        same.restore(image2)
    assert e.value.code == A.EINVAL
    for x in (s, other, same):
        x.close()


def _staged_run(b, restore_at=None):
    """Host and device-generated staging across the checkpoint: each window's messages are staged
    (and, at restore_at, snapshotted with them staged) before the window runs."""
    rng = np.random.default_rng(7)
    n = 64
    sim = Simulator(SimConfig(n_instances=n, seed=7), binding=b)
    for g in range(n):
        sim.set_shape(g, make_shape(latency_ns=int(rng.integers(1, 30)) * MS, jitter_ns=2 * MS, duplicate=10.0,
                                    bandwidth_bps=int(rng.choice([0, 1_000_000]))))
    out, t = [], 0
    for w in range(6):
        k = 400
        sim.enqueue(rng.integers(0, n, k), rng.integers(0, n, k), np.arange(k) + w * k, rng.choice([100, 1500], k),
                    t + rng.integers(0, 10 * MS, k))
        if restore_at is not None and w in restore_at:  # the window's messages are staged
            image = sim.snapshot()
            cfg = sim.cfg
            sim.close()
            sim = Simulator(cfg, binding=b)
            sim.restore(image)
        t += 10 * MS
        sim.advance(t)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    t += 200 * MS
    sim.advance(t)
    out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=S.parity_stats(sim)))
    sim.close()
    return out


@pytest.mark.gpu
def test_staged_resumed_matches_oracle(hip, oracle):
    """a snapshot with the next window's messages staged (round 6: captured, no longer refused)"""
    S.assert_same(_staged_run(hip, restore_at={1, 4}), _staged_run(oracle))


@pytest.mark.gpu
def test_flood_resumed_matches_oracle(hip, oracle):
    """a flood checkpointed after its reactions (the forwards staged, publications in flight) and
    restored into a context with the same graph; a context without it refuses the image"""
    a = S.run_flood(hip, n_inst=1500, waves=3, restart={2, 6})
    b = S.run_flood(oracle, n_inst=1500, waves=3)
    S.assert_same(a[:-1], b[:-1])
    assert a[-1]["stats"] == b[-1]["stats"] and a[-1]["tot"] == b[-1]["tot"]


@pytest.mark.gpu
def test_flood_image_needs_the_graph(hip):
    from testground_amd import workloads as W
    cfg = SimConfig(n_instances=200, seed=5)
    s = Simulator(cfg, binding=hip)
    off, nbr = W.random_regular_graph(200, 4, 5)
    s.flood_set_graph(off, nbr, 4)
    s.flood_publish([3], [0], 0, 100)
    s.advance(10 * MS)
    s.flood_react(100)
    image = s.snapshot()
    for setup in (None, (W.random_regular_graph(200, 4, 6), 4), ((off, nbr), 8)):
        f = Simulator(cfg, binding=hip)
        if setup:
            f.flood_set_graph(*setup[0], setup[1])
        with pytest.raises(A.TgsimError) as e:
            f.restore(image)
        assert e.value.code == A.EINVAL
        f.close()
    s.close()


def _probe_run(b, restore_at=()):
    """splitbrain-style probes (tests/test_probe.py) checkpointed between reactions"""
    from testground_amd.network import int_to_ip
    from testground_amd.sim import make_rule
    rng = np.random.default_rng(3)
    n, W = 30, 100_000
    cfg = SimConfig(n_instances=n, seed=3, max_msgs_per_window=1 << 14, max_records=1 << 16)
    sim = Simulator(cfg, binding=b)
    sim.set_shapes(np.arange(n), [make_shape(latency_ns=int(rng.integers(0, 3)) * MS, loss=float(rng.choice([0.0, 5.0])))
                                  for _ in range(n)])
    ip = [int_to_ip(sim.get_ip(g)) + "/32" for g in range(n)]
    for g in rng.choice(n, n // 4, replace=False):
        sim.add_rules(int(g), [make_rule(ip[int(t)], A.FILTER_DROP) for t in rng.choice(n, 4, replace=False) if t != g])
    order = rng.permutation(n)
    args = (order, 66, 66, 80 * MS, W)
    sim.probe_setup(*args)
    sim.probe_start(0)
    out, ne, w = [], W, 0
    while w < 100_000:
        sim.advance(ne)
        st, d = sim.status(), sim.deliveries()
        ne, act = sim.probe_react()
        out.append(dict(status=np.sort(st), deliv=d, ne=ne, act=act))
        w += 1
        if act == 0:
            break
        if w in restore_at:  # the next requests and replies are staged
            image = sim.snapshot()
            sim.close()
            sim = Simulator(cfg, binding=b)
            sim.probe_setup(*args)
            sim.restore(image)
    res, t_done = sim.probe_results()
    stats = S.parity_stats(sim)
    sim.close()
    return out, res, t_done, stats


@pytest.mark.gpu
def test_probes_resumed_matches_oracle(hip, oracle):
    a = _probe_run(hip, restore_at={3, 10, 40})
    b = _probe_run(oracle)
    assert len(a[0]) == len(b[0]) > 40
    S.assert_same(a[0], b[0])
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3]


def _storm_reactor_run(b, seed, restore_at=()):
    """the storm plan reactor (dial semaphore, DialTimeout, writesem, send buffers) checkpointed
    between reactions in both phases; a restoring context repeats tgsim_storm_setup first"""
    rng = np.random.default_rng(seed)
    n = 40
    cfg = SimConfig(n_instances=n, seed=seed, max_msgs_per_window=1 << 15, max_records=1 << 17)
    kw = [dict(latency_ns=int(rng.integers(0, 4)) * MS, jitter_ns=int(rng.integers(0, 3)) * MS // 2,
               loss=float(rng.choice([0.0, 0.0, 3.0])), duplicate=float(rng.choice([0.0, 5.0])),
               bandwidth_bps=int(rng.choice([0, 0, 50_000_000]))) for _ in range(n)]
    shapes = [make_shape(**k) for k in kw]
    lossless = [make_shape(**{**k, "loss": 0.0}) for k in kw]  # every dial succeeds; the writes lose chunks
    O = 3
    src = np.repeat(np.arange(n), O)
    dst = (src + rng.integers(1, n, len(src))) % n
    t_ready = rng.integers(0, 40, len(src)) * MS // 3
    args = dict(outgoing=O, concurrent=2, data_bytes=5 * 1500 + 4096, msg_window=2, dial_timeout_ns=60 * MS,
                window_ns=MS)
    sim = Simulator(cfg, binding=b)
    sim.set_shapes(np.arange(n), lossless)
    sim.storm_setup(dst, t_ready, **args)
    sim.storm_start()
    out, w = [], 0
    for phase in ("dials", "writes"):
        if phase == "writes":
            sim.set_shapes(np.arange(n), shapes)
            sim.storm_write_start(sim.now)
        ne = sim.now + MS
        while True:
            sim.advance(ne)
            st, d = sim.status(), sim.deliveries()
            ne, act = sim.storm_react()
            out.append(dict(status=np.sort(st), deliv=d, ne=ne, act=act))
            w += 1
            if act == 0:
                break
            if w in restore_at:
                image = sim.snapshot()
                sim.close()
                sim = Simulator(cfg, binding=b)
                sim.storm_setup(dst, t_ready, **args)
                sim.restore(image)
    res, t_done = sim.storm_dials()
    failed, t_last, tot = sim.storm_results()
    stats = S.parity_stats(sim)
    sim.storm_end()
    sim.close()
    return out, res, t_done, failed, t_last, tot, stats


@pytest.mark.gpu
def test_storm_reactor_resumed_matches_oracle(hip, oracle):
    a = _storm_reactor_run(hip, 2, restore_at={2, 5, 9, 14, 20})
    b = _storm_reactor_run(oracle, 2)
    assert len(a[0]) == len(b[0]) > 20
    S.assert_same(a[0], b[0])
    for x, y in zip(a[1:5], b[1:5]):
        assert np.array_equal(x, y)
    assert a[5] == b[5] and a[6] == b[6]


@pytest.mark.gpu
@pytest.mark.parametrize("acks", [False, True])
def test_tcp_random_resumed_matches_oracle(hip, oracle, acks):
    """TCP mode across checkpoints: writes, segments, retransmission lists, the acks-mode timer ring"""
    from tests import test_tcp as T
    w = 120 if acks else 60
    T._same(T.run_random(hip, 2, acks=acks, windows=w, restart={5, 17, 40}),
            T.run_random(oracle, 2, acks=acks, windows=w))


@pytest.mark.gpu
def test_tcp_storm_resumed_matches_oracle(hip, oracle):
    from tests import test_tcp as T
    a = T.run_tcp_storm(hip, n=300, rounds=5, acks=True, restart={1, 3})
    b = T.run_tcp_storm(oracle, n=300, rounds=5, acks=True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]


@pytest.mark.gpu
def test_tcp_connections_resumed_matches_oracle(hip, oracle):
    """connections (Reno windows, queued writes, loss episodes) across checkpoints; the restoring
    context opens the same connections first"""
    from tests import test_tcp_conn as T
    a, b = T.random_conn_run(hip, 2, restart={20, 55, 90}), T.random_conn_run(oracle, 2)
    S.assert_same(a["deliv"], b["deliv"])
    assert np.array_equal(a["writes"][0], b["writes"][0]) and np.array_equal(a["writes"][1], b["writes"][1])
    for k in a["conns"]:
        assert np.array_equal(a["conns"][k], b["conns"][k]), k
    assert a["stats"] == b["stats"] and a["tcp"] == b["tcp"]
