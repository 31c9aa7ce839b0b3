"""Sequential probes (tgsim_probe_*): plans/splitbrain/main.go:153-175 probes its
peers one httpclient.Get at a time, each with a one-minute timeout. Hand-computed answers on the
oracle and the HIP library, randomised HIP-vs-oracle parity (every window's statuses, deliveries,
outcomes and end times)."""
import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd.network import int_to_ip
from testground_amd.sim import SimConfig, Simulator, make_rule, make_shape
from tests import scenarios as S

MS = 1_000_000
SEC = 1000 * MS
W = 100_000          # 100 us reaction windows


def drive(sim, order, t0=0, req=66, rep=66, timeout=60 * SEC, window=W, max_windows=200_000, keep=True):
    """probe_setup + start, then window after window at the proposed end until no instance probes."""
    sim.probe_setup(order, req, rep, timeout, window)
    sim.probe_start(t0)
    out, ne, w = [], t0 + window, 0
    while w < max_windows:
        sim.advance(ne)
        st, d = sim.status(), sim.deliveries()
        ne, act = sim.probe_react()
        if keep:
            out.append(dict(status=np.sort(st), deliv=d, ne=ne, act=act))
        w += 1
        if act == 0:
            break
    res, t_done = sim.probe_results()
    return out, res, t_done, w


def _hand_case(b):
    """0 drops its route to 1 (blackhole), 2 rejects 3 (prohibit): 0 -> 1 and 2 -> 3 end REFUSED at
    once; 1 -> 0 and 3 -> 2 reach the peer, whose reply its own route discards, so they end at the
    one-minute deadline; every other probe takes a request and a reply, one window each."""
    n = 5
    s = Simulator(SimConfig(n_instances=n, seed=3), binding=b)
    ip = [int_to_ip(s.get_ip(g)) + "/32" for g in range(n)]
    s.add_rules(0, [make_rule(ip[1], A.FILTER_DROP)])
    s.add_rules(2, [make_rule(ip[3], A.FILTER_REJECT)])
    _, res, t_done, w = drive(s, np.arange(n))
    OK, RF, TO = A.PROBE_OK, A.PROBE_REFUSED, A.PROBE_TIMEOUT
    assert res.tolist() == [[0, RF, OK, OK, OK],
                            [TO, 0, OK, OK, OK],
                            [OK, OK, 0, RF, OK],
                            [OK, OK, TO, 0, OK],
                            [OK, OK, OK, OK, 0]]
    # a reply leaves at max(request arrival, horizon) and the next request at max(reply arrival,
    # horizon): with zero latency every hop after the first costs one window W. Instance 4: four
    # probes end at 0, 2W, 4W, 6W; instance 0's refusal ends at once, then three probes: 5W
    assert t_done[4] == 6 * W and t_done[0] == 5 * W and t_done[2] == 5 * W
    # 1's first probe waits out the deadline (60 s after t = 0; the window jumps to it: end + 1 ns),
    # then three probes end at +1, +1 + 2W, +1 + 4W
    assert t_done[1] == 60 * SEC + 1 + 4 * W
    assert w < 40
    s.close()


def test_probe_hand_oracle(oracle):
    _hand_case(oracle)


@pytest.mark.gpu
def test_probe_hand_hip(hip):
    _hand_case(hip)


def _random_run(b, seed, n=40, keep=True, shard=None):
    """shard = (k, world, transport): shard k of a sharded run (configuration calls to every shard;
    results are the shard's own probers)."""
    rng = np.random.default_rng(seed)
    kw = dict(shard_id=shard[0], n_shards=shard[1], exchange_cap=1 << 12) if shard else {}
    s = Simulator(SimConfig(n_instances=n, seed=seed, max_msgs_per_window=1 << 14, max_records=1 << 16, **kw),
                  binding=b)
    if shard:
        s.set_transport(shard[2])
    shapes = [make_shape(latency_ns=int(rng.integers(0, 3)) * MS, jitter_ns=int(rng.integers(0, 2)) * MS // 2,
                         loss=float(rng.choice([0.0, 0.0, 5.0])), duplicate=float(rng.choice([0.0, 10.0])))
              for _ in range(n)]
    s.set_shapes(np.arange(n), shapes)
    ip = [int_to_ip(s.get_ip(g)) + "/32" for g in range(n)]
    for g in rng.choice(n, n // 4, replace=False):
        tgt = rng.choice(n, 5, replace=False)
        s.add_rules(int(g), [make_rule(ip[int(t)], int(rng.choice([A.FILTER_DROP, A.FILTER_REJECT]))) for t in tgt if t != g])
    s.set_enabled(int(rng.integers(n)), False)
    order = rng.permutation(n)
    out, res, t_done, w = drive(s, order, t0=3 * MS, timeout=int(rng.integers(20, 200)) * MS, window=W, keep=keep)
    stats = S.parity_stats(s)
    s.close()
    return out, res, t_done, w, stats, order


def test_probe_random_oracle_properties(oracle):
    out, res, t_done, w, _, order = _random_run(oracle, 1)
    assert out[-1]["act"] == 0 and np.all(t_done >= 3 * MS)
    n = len(res)
    assert np.all(res[order, np.arange(n)] == A.PROBE_NONE)     # nobody probes itself
    assert np.count_nonzero(res) == n * (n - 1)                # every other probe ended
    assert set(np.unique(res)) <= {0, A.PROBE_OK, A.PROBE_REFUSED, A.PROBE_TIMEOUT}


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_probe_random_hip_matches_oracle(hip, oracle, seed):
    a = _random_run(hip, seed)
    b = _random_run(oracle, seed)
    assert a[3] == b[3], "window count"
    S.assert_same(a[0], b[0])
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[4] == b[4]


def _sharded_random_run(b, seed, world, device=False):
    from testground_amd.exchange import ThreadGroup, run_threads
    g = ThreadGroup(world, device=device)
    return run_threads([lambda k=k: _random_run(b, seed, shard=(k, world, g.member(k))) for k in range(world)])


def _assert_probe_shards_match(outs, single):
    """Per window: the same proposal and active count on every shard; statuses as one multiset,
    deliveries concatenated in shard order; outcomes and end times concatenated; counters summed."""
    out1, res1, td1, w1, st1, _ = single
    assert all(o[3] == w1 for o in outs), "window count"
    for w, ref in enumerate(out1):
        obs = [o[0][w] for o in outs]
        assert all((x["ne"], x["act"]) == (ref["ne"], ref["act"]) for x in obs), f"window {w}: proposal"
        S.assert_same(np.sort(np.concatenate([x["status"] for x in obs])), ref["status"], f"window {w} status")
        for f in ref["deliv"]:
            S.assert_same(np.concatenate([x["deliv"][f] for x in obs]), ref["deliv"][f], f"window {w} deliv.{f}")
    assert np.array_equal(np.concatenate([o[1] for o in outs]), res1)
    assert np.array_equal(np.concatenate([o[2] for o in outs]), td1)
    for k in st1:
        assert sum(o[4][k] for o in outs) == st1[k], k


@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2), (4, 3)])
def test_probe_sharded_threads_oracle(oracle, world, seed):
    """The probes sharded: every prober on its own shard, a request reaching its
    peer's shard through the window's exchange, the peer's answer reaching the prober's shard as a
    notice, the proposal collective - equal to the single context window by window."""
    _assert_probe_shards_match(_sharded_random_run(oracle, seed, world), _random_run(oracle, seed))


@pytest.mark.gpu
@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2), (4, 3)])
def test_probe_sharded_threads_hip(hip, oracle, world, seed):
    _assert_probe_shards_match(_sharded_random_run(hip, seed, world, device=True), _random_run(oracle, seed))


def test_probe_errors(oracle):
    s = Simulator(SimConfig(n_instances=4, seed=1), binding=oracle)
    with pytest.raises(A.TgsimError) as e:
        s.probe_react()
    assert e.value.code == A.ESTATE
    with pytest.raises(A.TgsimError) as e:
        s.probe_setup([0, 9], 66, 66, SEC, W)
    assert e.value.code == A.EINVAL
    s.probe_setup(np.arange(4), 66, 66, SEC, W)
    with pytest.raises(A.TgsimError) as e:
        s.tcp_enable()
    assert e.value.code == A.ESTATE
    s.close()


def _deadline_case(b):
    """a request that arrives within one window of its deadline. 0 -> 1 has 1 ms of
    latency and the probes a 1.05 ms timeout: 0's request arrives at 1.0 ms, in the window
    [1.0, 1.1) ms, and 1 answers it at 1.0 ms over its zero-latency link. The reaction after that
    window sees the deadline (1.05 ms) already behind the window end, but the reply it just staged
    can still beat it: the decision waits a window, and the reply's arrival at 1.0 ms makes the probe
    OK. 1's probe of 0 crosses the slow link on the way back and ends OK at 1.0 ms as well."""
    s = Simulator(SimConfig(n_instances=2, seed=5), binding=b)
    s.set_shapes([0], [make_shape(latency_ns=1 * MS)])
    _, res, t_done, _ = drive(s, np.arange(2), timeout=1 * MS + 50_000)
    assert res.tolist() == [[0, A.PROBE_OK], [A.PROBE_OK, 0]]
    assert t_done.tolist() == [1 * MS, 1 * MS]
    s.close()


def test_probe_deadline_within_a_window_oracle(oracle):
    _deadline_case(oracle)


@pytest.mark.gpu
def test_probe_deadline_within_a_window_hip(hip):
    _deadline_case(hip)


def _react_owed_case(b):
    """after a window, the probe reaction owns the window's staged rows and deliveries.
    Staging, a probe start or the next window before tgsim_probe_react is refused (ESTATE), and so
    is a second reaction without a window in between."""
    s = Simulator(SimConfig(n_instances=4, seed=1), binding=b)
    s.probe_setup(np.arange(4), 66, 66, SEC, W)
    s.probe_start(0)
    s.advance(W)
    for call in (lambda: s.enqueue([0], [1], [77], [64], [W]), lambda: s.probe_start(W),
                 lambda: s.advance(2 * W), lambda: s.gen_storm_round(0, W, 2, 64, 0, 1)):
        with pytest.raises(A.TgsimError) as e:
            call()
        assert e.value.code == A.ESTATE
    ne, act = s.probe_react()
    assert act > 0 and ne == 2 * W
    with pytest.raises(A.TgsimError) as e:
        s.probe_react()
    assert e.value.code == A.ESTATE
    s.enqueue([0], [1], [77], [64], [W])   # now allowed
    s.advance(ne)
    s.probe_react()
    s.close()


def test_probe_react_owed_oracle(oracle):
    _react_owed_case(oracle)


@pytest.mark.gpu
def test_probe_react_owed_hip(hip):
    _react_owed_case(hip)


def _late_request_case(b):
    """prober 0's first request (to 1) is slower than the timeout (150 ms latency, 100 ms
    timeout): the probe times out at 100 ms and the second request (to 2) leaves at 100 ms over a
    60 ms link (the shape changed meanwhile). Both requests arrive in the window [150, 200) ms, the
    first at 150, the second at 160. The reply answers the second request: it must leave at its own
    request's arrival (160), not at the earlier arrival of the first (150), so the probe ends OK at
    160 ms (the reply's zero-latency arrival), not 150."""
    s = Simulator(SimConfig(n_instances=3, seed=1), binding=b)
    s.set_shape(0, make_shape(latency_ns=150 * MS))
    s.probe_setup(np.arange(3), 66, 66, 100 * MS, 50 * MS)
    s.probe_start(0)
    ne, out, changed = 50 * MS, [], False
    for _ in range(100):
        s.advance(ne)
        out.append(dict(status=np.sort(s.status()), deliv=s.deliveries()))
        ne, act = s.probe_react()
        if not changed and s.now >= 150 * MS:
            s.set_shape(0, make_shape(latency_ns=60 * MS))
            changed = True
        if act == 0:
            break
    res, t_done = s.probe_results()
    s.close()
    assert res[0].tolist() == [0, A.PROBE_TIMEOUT, A.PROBE_OK]
    assert t_done[0] == 160 * MS
    return out, res, t_done


def test_probe_late_request_reply_time_oracle(oracle):
    _late_request_case(oracle)


@pytest.mark.gpu
def test_probe_late_request_reply_time_hip(hip, oracle):
    S.assert_same(_late_request_case(hip), _late_request_case(oracle))
