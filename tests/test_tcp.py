"""TCP mode (tgsim_tcp_*): writes segmented into MSS
packets over the per-packet path, lost / corrupted segments retransmitted with exponential backoff
from the RTO, refused routes failing the write, in-order delivery per connection. Hand-computed
answers run on the oracle (CPU) and the HIP library (GPU); randomised runs compare the two bit for
bit (deliveries, per-packet statuses as a multiset — the device releases retransmissions in
arbitrary order —, write outcomes, counters). Parity unpinned against real TCP: there is no packet
capture of the reference's plans to compare with."""
import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd import tcp as T
from testground_amd.sim import SimConfig, Simulator, make_rule, make_shape
from tests import scenarios as S

MS = 1_000_000


def sim(b, n=4, **kw):
    kw.setdefault("max_msgs_per_window", 1 << 14)
    kw.setdefault("max_records", 1 << 16)
    s = Simulator(SimConfig(n_instances=n, seed=kw.pop("seed", 3), **kw), binding=b)
    return s


def window(s, t_end):
    s.advance(t_end)
    d = s.deliveries()
    s.tcp_react()
    return d


def case_segmentation(b):
    s = sim(b)
    s.tcp_enable()
    s.tcp_send([0, 1], [1, 2], [0, 0], [4096, 0], [5, 6])
    d = window(s, 1 * MS)
    # 4096 B = 1448 + 1448 + 1200, each + 52 B of headers; a 0-byte write is one bare segment
    assert sorted(zip(d["seq"].tolist(), d["size"].tolist())) == [(0, 1500), (16, 1500), (32, 1252), (48, 52)]
    st, t = s.tcp_writes()
    assert list(st) == [A.TCP_DELIVERED] * 2 and list(t) == [5, 6]
    assert s.tcp_stats()["segments"] == 4 and s.tcp_stats()["retransmissions"] == 0
    with pytest.raises(A.TgsimError) as e:
        s.enqueue([0], [1], [9], [1], [2 * MS])   # TCP mode: all traffic is TCP
    assert e.value.code == A.ESTATE
    s.close()


def case_loss_backoff_and_timeout(b):
    s = sim(b)
    s.tcp_enable(max_attempts=3)
    s.set_shape(0, make_shape(loss=100.0))
    s.tcp_send([0, 2], [1, 1], [0, 0], [100, 100], [1 * MS, 1 * MS])
    for k in range(1, 1500, 50):                 # 50 ms windows up to 1.5 s
        window(s, k * MS + 50 * MS)
        if k == 151:                              # sender 2 loses everything from 0.2 s on
            s.set_shape(2, make_shape(loss=100.0))
    st, t = s.tcp_writes()
    # sender 0: attempts at 1, 201, 601 ms all lost; the third failure times out at 601 + 800 ms
    assert st[0] == A.TCP_TIMEOUT and t[0] == 1401 * MS
    assert st[1] == A.TCP_DELIVERED and t[1] == 1 * MS
    stats = s.tcp_stats()
    assert stats["retransmissions"] == 2 and stats["failed"] == 1 and stats["delivered"] == 1
    assert stats["packets"] == 2 + 2
    s.close()


def case_retransmission_recovers(b):
    s = sim(b)
    s.tcp_enable()
    s.set_shape(0, make_shape(loss=100.0))
    s.tcp_send([0], [1], [0], [10], [3 * MS])
    window(s, 10 * MS)
    s.set_shape(0, make_shape(latency_ns=7 * MS))  # the link heals before the 200 ms timer fires
    for k in range(1, 30):
        window(s, 10 * MS + k * 10 * MS)
    st, t = s.tcp_writes()
    assert st[0] == A.TCP_DELIVERED and t[0] == 3 * MS + 200 * MS + 7 * MS
    s.close()


def case_corruption_waits_for_the_copy(b):
    """Every copy corrupted: the retransmission leaves at max(t + RTO, the corrupted copy's
    arrival) - a 300 ms path is slower than the 200 ms RTO."""
    s = sim(b)
    s.tcp_enable(max_attempts=2)
    s.set_shape(0, make_shape(latency_ns=300 * MS, corrupt=100.0))
    s.tcp_send([0], [1], [0], [64], [0])
    for k in range(1, 120):
        window(s, k * 10 * MS)
    st, t = s.tcp_writes()
    # attempt 0 at 0 arrives corrupted at 300 ms -> attempt 1 at 300 ms, corrupted at 600 ms;
    # attempt 1 was the last: timeout at max(300 + 400, 600) = 700 ms
    assert st[0] == A.TCP_TIMEOUT and t[0] == 700 * MS
    s.close()


def case_duplicates_and_refusal(b):
    s = sim(b, n=8)
    s.tcp_enable()
    s.set_shape(0, make_shape(duplicate=100.0, latency_ns=2 * MS))
    from testground_amd.network import int_to_ip
    s.add_rules(3, [make_rule(int_to_ip(s.get_ip(4)) + "/32", A.FILTER_REJECT)])
    s.tcp_send([0, 3, 3], [1, 4, 5], [0, 0, 0], [3000, 10, 10], [0, 1, 2])
    window(s, 10 * MS)
    st, t = s.tcp_writes()
    assert list(st) == [A.TCP_DELIVERED, A.TCP_REFUSED, A.TCP_DELIVERED] and list(t) == [2 * MS, 1, 2]
    assert s.tcp_stats()["retransmissions"] == 0
    s.close()


CASES = [case_segmentation, case_loss_backoff_and_timeout, case_retransmission_recovers,
         case_corruption_waits_for_the_copy, case_duplicates_and_refusal]


# ---- acks = 1: ACK packets on the reverse path, retransmission timers (tgsim.h) ------------------

def _run_windows(s, until_ms, step_ms=10):
    """10 ms windows up to until_ms; every window's deliveries, concatenated."""
    out = []
    for k in range(step_ms, until_ms + 1, step_ms):
        d = window(s, k * MS)
        out.append(d)
    return {key: np.concatenate([d[key] for d in out]) for key in out[0]}


def case_ack_clean(b):
    """The data arrives at 10 ms; its ACK leaves then (a late send from the reaction after that
    window) and arrives at 20 ms, before the 200 ms timer: nothing is retransmitted."""
    s = sim(b)
    s.tcp_enable(acks=True)
    for g in range(4):
        s.set_shape(g, make_shape(latency_ns=10 * MS))
    s.tcp_send([0], [1], [0], [100], [0])
    d = _run_windows(s, 400)
    acks = (d["seq"] & A.TCP_ACK_BIT) != 0
    assert d["t_deliver"][~acks].tolist() == [10 * MS] and d["t_deliver"][acks].tolist() == [20 * MS]
    assert d["src"][acks].tolist() == [1] and d["dst"][acks].tolist() == [0]
    assert d["size"][acks].tolist() == [52]
    st, t = s.tcp_writes()
    assert st[0] == A.TCP_DELIVERED and t[0] == 10 * MS
    assert s.tcp_stats()["retransmissions"] == 0 and s.tcp_stats()["packets"] == 1
    s.close()


def case_ack_lost_spurious(b):
    """Every ACK is lost (the receiver's link drops everything): the sender retransmits at 200 and
    600 ms although the data arrived at 10 ms, then gives up at 1400 ms; the write stays delivered."""
    s = sim(b)
    s.tcp_enable(acks=True, max_attempts=3)
    s.set_shape(0, make_shape(latency_ns=10 * MS))
    s.set_shape(1, make_shape(loss=100.0))
    s.tcp_send([0], [1], [0], [100], [0])
    d = _run_windows(s, 1600)
    data = (d["seq"] & A.TCP_ACK_BIT) == 0
    assert d["t_deliver"][data].tolist() == [10 * MS, 210 * MS, 610 * MS]
    assert (d["seq"][data] & 15).tolist() == [0, 1, 2]
    st, t = s.tcp_writes()
    assert st[0] == A.TCP_DELIVERED and t[0] == 10 * MS
    stats = s.tcp_stats()
    assert stats["retransmissions"] == 2 and stats["failed"] == 0 and stats["packets"] == 3
    s.close()


def case_ack_data_lost(b):
    """The first attempt is lost; the timer resends it at 200 ms once the link has healed."""
    s = sim(b)
    s.tcp_enable(acks=True)
    s.set_shape(0, make_shape(loss=100.0))
    s.set_shape(1, make_shape(latency_ns=10 * MS))
    s.tcp_send([0], [1], [0], [100], [0])
    window(s, 10 * MS)
    s.set_shape(0, make_shape(latency_ns=10 * MS))
    _run_windows(s, 400)
    st, t = s.tcp_writes()
    assert st[0] == A.TCP_DELIVERED and t[0] == 210 * MS
    assert s.tcp_stats()["retransmissions"] == 1
    s.close()


def case_ack_slow_path(b):
    """A 300 ms data path is slower than the 200 ms timer: a spurious retransmission leaves at 200 ms
    (arriving at 500 ms); the original's ACK (sent at 300, arriving at 305 ms) stops the next timer."""
    s = sim(b)
    s.tcp_enable(acks=True)
    s.set_shape(0, make_shape(latency_ns=300 * MS))
    s.set_shape(1, make_shape(latency_ns=5 * MS))
    s.tcp_send([0], [1], [0], [100], [0])
    d = _run_windows(s, 1000)
    data = (d["seq"] & A.TCP_ACK_BIT) == 0
    assert d["t_deliver"][data].tolist() == [300 * MS, 500 * MS]
    assert sorted(d["t_deliver"][~data].tolist()) == [305 * MS, 505 * MS]
    st, t = s.tcp_writes()
    assert st[0] == A.TCP_DELIVERED and t[0] == 300 * MS
    assert s.tcp_stats()["retransmissions"] == 1
    s.close()


def case_ack_timeout_before_data(b):
    """max_attempts = 1 and a 300 ms path: the only timer fires at 200 ms, before the data arrives -
    the write fails (TIMEOUT at 200 ms) and the later arrival does not revive it."""
    s = sim(b)
    s.tcp_enable(acks=True, max_attempts=1)
    s.set_shape(0, make_shape(latency_ns=300 * MS))
    s.tcp_send([0], [1], [0], [100], [0])
    _run_windows(s, 500)
    st, t = s.tcp_writes()
    assert st[0] == A.TCP_TIMEOUT and t[0] == 200 * MS
    s.close()


ACK_CASES = [case_ack_clean, case_ack_lost_spurious, case_ack_data_lost, case_ack_slow_path,
             case_ack_timeout_before_data]


@pytest.mark.parametrize("case", CASES, ids=[c.__name__[5:] for c in CASES])
def test_tcp_oracle(oracle, case):
    case(oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c.__name__[5:] for c in CASES])
def test_tcp_hip(hip, case):
    case(hip)


@pytest.mark.parametrize("case", ACK_CASES, ids=[c.__name__[5:] for c in ACK_CASES])
def test_tcp_ack_oracle(oracle, case):
    case(oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ACK_CASES, ids=[c.__name__[5:] for c in ACK_CASES])
def test_tcp_ack_hip(hip, case):
    case(hip)


def test_in_order_view():
    # connection 0->1: write b (seq 1) arrives before write a (seq 0) is retransmitted
    src, dst, seq, ts = [0, 0, 0, 2], [1, 1, 1, 1], [0, 1, 2, 0], [0, 0, 0, 0]
    st = [T.DELIVERED, T.DELIVERED, T.PENDING, T.TIMEOUT]
    td = [205, 10, 0, 900]
    s2, t2 = T.in_order(src, dst, seq, ts, st, td)
    assert list(s2) == [T.DELIVERED, T.DELIVERED, T.PENDING, T.TIMEOUT]
    assert list(t2) == [205, 205, T.NEVER, 900]
    s3, t3 = T.in_order([0, 0], [1, 1], [0, 1], [0, 0], [T.REFUSED, T.DELIVERED], [3, 50])
    assert list(s3) == [T.REFUSED, T.REFUSED] and list(t3) == [3, 3]   # the reset fails what follows


def run_random(b, seed, n=300, windows=60, window_ns=10 * MS, wait=True, acks=False, restart=()):
    """Lossy, corrupting, duplicating, reordering links with jitter and rate limits; writes of 0 to
    9000 B over the first 30 windows. Per window: deliveries and the statuses as a sorted multiset;
    at the end the write outcomes and counters. restart: windows after whose reaction the run is
    snapshotted and restored into a fresh context (checkpoint / resume)."""
    rng = np.random.default_rng(seed)
    cfg = SimConfig(n_instances=n, seed=seed, max_msgs_per_window=1 << 16, max_records=1 << 18)
    s = Simulator(cfg, binding=b)
    enable = dict(max_attempts=int(rng.integers(3, 8)), rto_ns=int(rng.integers(20, 80)) * MS, acks=acks)
    s.tcp_enable(**enable)
    for g in range(n):
        s.set_shape(g, make_shape(latency_ns=int(rng.integers(1, 60)) * MS, jitter_ns=int(rng.integers(0, 5)) * MS,
                                  bandwidth_bps=int(rng.choice([0, 2_000_000, 20_000_000])),
                                  loss=float(rng.choice([0, 2, 10])), corrupt=float(rng.choice([0, 3])),
                                  duplicate=float(rng.choice([0, 5])), reorder=float(rng.choice([0, 10]))))
    out, t = [], 0
    for w in range(windows):
        if w < 30:
            k = int(rng.integers(0, 80))
            src = rng.integers(0, n, k)
            s.tcp_send(src, (src + rng.integers(1, n, k)) % n, rng.integers(0, 1 << 20, k),
                       rng.integers(0, 9000, k), t + rng.integers(0, window_ns, k))
        t += window_ns
        s.advance(t)
        st = s.status()
        d = s.deliveries()
        s.tcp_react(wait=wait)
        out.append(dict(deliv=d, status=np.sort(st)))
        if w in restart:
            image = s.snapshot()
            s.close()
            s = Simulator(cfg, binding=b)
            s.tcp_enable(**enable)
            s.restore(image)
    ws, wt = s.tcp_writes()
    out.append(dict(writes=(ws, wt), stats=s.tcp_stats()))
    s.close()
    return out


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a[:-1], b[:-1]):
        for k in x["deliv"]:
            assert np.array_equal(x["deliv"][k], y["deliv"][k]), k
        assert np.array_equal(x["status"], y["status"])
    assert np.array_equal(a[-1]["writes"][0], b[-1]["writes"][0])
    assert np.array_equal(a[-1]["writes"][1], b[-1]["writes"][1])
    assert a[-1]["stats"] == b[-1]["stats"]


def test_tcp_random_oracle_properties(oracle):
    out = run_random(oracle, 1)
    ws, wt = out[-1]["writes"]
    st = out[-1]["stats"]
    assert st["retransmissions"] > 0 and st["delivered"] > 0.8 * st["writes"]
    assert np.all(wt[ws != A.TCP_PENDING] >= 0)
    assert st["packets"] == st["segments"] + sum(np.count_nonzero(x["status"] >= 0) for x in out[:-1]) - st["segments"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tcp_random_hip_matches_oracle(hip, oracle, seed):
    _same(run_random(hip, seed), run_random(oracle, seed))


def test_tcp_random_acks_oracle_properties(oracle):
    """acks mode on the lossy links: every write ends (delivered or timed out), ACKs travel the
    reverse path (deliveries with the ACK bit, header-sized), and retransmissions happen."""
    out = run_random(oracle, 1, acks=True, windows=120)
    ws, wt = out[-1]["writes"]
    st = out[-1]["stats"]
    acks = np.concatenate([(x["deliv"]["seq"] & A.TCP_ACK_BIT) != 0 for x in out[:-1]])
    sizes = np.concatenate([x["deliv"]["size"] for x in out[:-1]])
    assert acks.any() and np.all(sizes[acks] == 52)
    assert st["retransmissions"] > 0 and st["delivered"] > 0.8 * st["writes"]
    assert np.all(ws != A.TCP_PENDING) and np.all(wt[ws != A.TCP_PENDING] >= 0)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_tcp_random_acks_hip_matches_oracle(hip, oracle, seed):
    _same(run_random(hip, seed, acks=True, windows=120), run_random(oracle, seed, acks=True, windows=120))


@pytest.mark.gpu
def test_tcp_random_async_reaction_matches_oracle(hip, oracle):
    """Reactions queued without a read-back (the host's pending bounds grow until a snapshot is
    read): the same windows, statuses and outcomes as the oracle's synchronous reactions."""
    _same(run_random(hip, 2, wait=False), run_random(oracle, 2))


def _pingpong_tcp(binding):
    """plans/network/pingpong.go over TCP mode: the reference's RTT windows hold ([200, 215] ms at
    100 ms egress latency, [20, 35] ms at 10 ms) - the plan's data is 1-byte writes on one
    connection, so segmentation adds only the 52 header bytes."""
    from testground_amd import plans as P
    env = P.PlanEnv(2, seed=1, params={"transport": "tcp", "tcp_acks": "false"}, binding=binding)
    ok = P.pingpong(env)
    rtts = getattr(env, "rtts", [])
    stats = env.sim.tcp_stats()
    env.close()
    return ok, rtts, stats


def test_pingpong_over_tcp_oracle(oracle):
    ok, rtts, stats = _pingpong_tcp(oracle)
    assert ok.all() and len(rtts) == 2 and stats["writes"] > 0 and stats["retransmissions"] == 0


@pytest.mark.gpu
def test_pingpong_over_tcp_hip(hip, oracle):
    a, b = _pingpong_tcp(hip), _pingpong_tcp(oracle)
    assert a[0].all() and [list(x) for x in a[1]] == [list(x) for x in b[1]] and a[2] == b[2]


def _lossy_rpc(binding):
    """Request / reply over a 30 %-loss link in TCP mode: every exchange completes (the lost
    segments are retransmitted after 200 ms, 400 ms, ...), and the RTTs fall on the retransmission
    grid - base RTT + k * 200 ms - instead of being lost as in the message-level model."""
    from testground_amd import plans as P
    from testground_amd.network import MS as NMS
    env = P.PlanEnv(8, seed=2, params={"transport": "tcp", "tcp_acks": "false"}, binding=binding)
    for g in range(8):
        env.sim.set_shape(g, make_shape(latency_ns=5 * MS, loss=30.0))
    src = np.arange(8)
    ok, rtt = env.rpc(src, (src + 1) % 8, 100, 100, env.sim.now, 10_000 * NMS)
    env.close()
    return ok, rtt


def test_lossy_rpc_over_tcp_oracle(oracle):
    ok, rtt = _lossy_rpc(oracle)
    assert ok.all()
    extra = (rtt - 10 * MS) % (200 * MS)
    assert np.all(rtt >= 10 * MS) and np.all((extra <= 1 * MS) | (extra >= 199 * MS))
    assert rtt.max() >= 210 * MS   # some exchange needed a retransmission


@pytest.mark.gpu
def test_lossy_rpc_over_tcp_hip(hip, oracle):
    a, b = _lossy_rpc(hip), _lossy_rpc(oracle)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def run_tcp_storm(b, seed=4, n=400, rounds=6, wait=True, acks=False, rto_ns=30 * MS, cfg_kw=None, setup=None,
                  restart=()):
    """The storm plan over TCP mode (plans/benchmarks/storm.go dials and writes 1 KiB per peer):
    tgsim_tcp_gen_storm_round generates each round as writes on the device, SignalAndWait ends
    the window, and the reaction recovers the 10 % lost segments. Drained afterwards. Sharded
    (cfg_kw shard_id / n_shards, setup attaching a transport): the same calls on every shard, each
    collective; a shard reports its own writers' writes (each round's block of its instances) and
    its own counters."""
    rng = np.random.default_rng(seed)
    # a window stages the round's writes, the ACKs of every intact data copy of the last window
    # (retransmitted ones included) and the fired timers: with a 30 ms RTO nearly every segment is
    # retransmitted once, spuriously
    per_window = max(1 << 16, 5 * n * 8)
    cfg = SimConfig(n_instances=n, seed=seed, max_msgs_per_window=per_window, max_records=max(1 << 18, 16 * n * 8),
                    max_states=64, data_prefix_len=12, **(cfg_kw or {}))
    s = Simulator(cfg, binding=b)
    if setup is not None:
        setup(s)
    enable = dict(max_attempts=5, rto_ns=rto_ns, acks=acks, max_writes=rounds * n * 8, max_segments=rounds * n * 8)
    s.tcp_enable(**enable)
    for g in range(n):
        s.set_shape(g, make_shape(latency_ns=int(rng.integers(5, 21)) * MS, jitter_ns=2 * MS, loss=10.0,
                                  bandwidth_bps=10_000_000))
    for r in range(rounds):
        s.tcp_gen_storm_round(r, A.T_NOW, 8, 1024, 5 * MS, r)
        w = s.barrier(r, n, A.T_NOW)
        s.advance_to_barrier(w, 1 * MS)
        s.tcp_react(wait=wait)
        if r in restart:
            image = s.snapshot()
            s.close()
            s = Simulator(cfg, binding=b)
            if setup is not None:
                setup(s)
            s.tcp_enable(**enable)
            s.restore(image)
    for _ in range(40):
        s.advance(s.now + 20 * MS, wait=wait)
        s.tcp_react(wait=wait)
    st, t = s.tcp_writes()
    out = (st, t, s.tcp_stats(), s.stats()["delivered"])
    s.close()
    return out


def test_tcp_storm_oracle(oracle):
    st, t, stats, _ = run_tcp_storm(oracle)
    assert stats["writes"] == 6 * 400 * 8 and stats["retransmissions"] > 0.05 * stats["writes"]
    assert np.all(st != A.TCP_PENDING) and (st == A.TCP_DELIVERED).mean() > 0.99


def test_tcp_storm_acks_oracle(oracle):
    st, t, stats, _ = run_tcp_storm(oracle, acks=True)
    assert stats["writes"] == 6 * 400 * 8 and stats["retransmissions"] > 0.05 * stats["writes"]
    assert np.all(st != A.TCP_PENDING) and (st == A.TCP_DELIVERED).mean() > 0.99


@pytest.mark.gpu
@pytest.mark.parametrize("wait", [True, False], ids=["sync", "async"])
def test_tcp_storm_acks_hip_matches_oracle(hip, oracle, wait):
    a, b = run_tcp_storm(hip, wait=wait, acks=True), run_tcp_storm(oracle, acks=True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]


@pytest.mark.gpu
@pytest.mark.parametrize("wait", [True, False], ids=["sync", "async"])
def test_tcp_storm_hip_matches_oracle(hip, oracle, wait):
    """async: every window and reaction queued without a host read-back (bench.py --tcp's loop)."""
    a, b = run_tcp_storm(hip, wait=wait), run_tcp_storm(oracle)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]


@pytest.mark.gpu
def test_tcp_acks_staged_overflow_reports_capacity(hip):
    """acks mode stages the last reaction's ACKs and the fired timers behind the device-side staged
    count, which the host cannot see: a window whose data + ACKs exceed max_msgs_per_window must end
    in ECAPACITY with the count held at the capacity (the netem pass reads it), not read past the
    staged arrays. 400 instances x fanout 8 = 3200 writes per round plus ~3200 ACKs > 4096."""
    s = Simulator(SimConfig(n_instances=400, seed=4, max_msgs_per_window=4096, max_records=1 << 18,
                            max_states=64), binding=hip)
    s.tcp_enable(max_attempts=5, rto_ns=30 * MS, acks=True)
    for g in range(400):
        s.set_shape(g, make_shape(latency_ns=5 * MS, bandwidth_bps=10_000_000))
    with pytest.raises(A.TgsimError) as e:
        for r in range(4):
            s.tcp_gen_storm_round(r, A.T_NOW, 8, 1024, 5 * MS, r)
            s.advance_to_barrier(s.barrier(r, 400, A.T_NOW), 1 * MS)
            s.tcp_react()
        s.sync()
    assert e.value.code == A.ECAPACITY
    s.close()


@pytest.mark.gpu
def test_tcp_storm_acks_full_size(hip, oracle):
    """config 4's 100k instances over TCP with ACKs (bench.py --tcp --tcp-acks's mode; its queued
    reactions): 3.2 M writes, their ACKs and the retransmissions of 10 % loss (Linux's 200 ms RTO:
    no spurious ones at these RTTs), bit-exact vs the oracle."""
    a = run_tcp_storm(hip, n=100_000, rounds=4, wait=False, acks=True, rto_ns=200 * MS)
    b = run_tcp_storm(oracle, n=100_000, rounds=4, acks=True, rto_ns=200 * MS)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]
    assert a[2]["retransmissions"] > 0.05 * a[2]["writes"] and (a[0] == A.TCP_DELIVERED).mean() > 0.99


def tcp_storm_sharded(b, world, device=False, exchange_cap=1 << 14, **kw):
    """run_tcp_storm over `world` shards (one thread each, ThreadGroup transport), recombined into the
    single run's form: every round's writes in instance order (shard k owns instances [lo, hi)), the
    counters summed."""
    outs = S.sharded_threads(world, lambda k, tr: run_tcp_storm(
        b, cfg_kw=S.shard_cfg(world, k, exchange_cap=exchange_cap), setup=lambda sim: sim.set_transport(tr), **kw),
        device=device)
    return combine_tcp_storm(outs, world, kw.get("n", 400), kw.get("rounds", 6))


def combine_tcp_storm(outs, world, n, rounds):
    """Per-shard run_tcp_storm outputs -> the single run's form."""
    per_round = lambda k: (S.shard_range(n, k, world)[1] - S.shard_range(n, k, world)[0]) * 8
    st = np.concatenate([outs[k][0].reshape(rounds, per_round(k)) for k in range(world)], axis=1).ravel()
    t = np.concatenate([outs[k][1].reshape(rounds, per_round(k)) for k in range(world)], axis=1).ravel()
    stats = {f: sum(o[2][f] for o in outs) for f in outs[0][2]}
    return st, t, stats, sum(o[3] for o in outs)


@pytest.mark.parametrize("world,acks", [(2, False), (3, False), (2, True), (3, True)])
def test_tcp_storm_sharded_oracle(oracle, world, acks):
    """TCP mode sharded. A data copy is settled on its writer's shard (forwarded
    there after the window through the exchange blocks), its ACK leaves from the receiver's shard:
    the sharded oracle run equals the single one (write outcomes and times, counters)."""
    a = tcp_storm_sharded(oracle, world, acks=acks)
    b = run_tcp_storm(oracle, acks=acks)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]
    assert b[2]["retransmissions"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("world,acks", [(2, False), (4, False), (2, True), (4, True)])
def test_tcp_storm_sharded_hip(hip, oracle, world, acks):
    """The same on HIP shards on one GPU (thread transport): equal to the single HIP context and the
    oracle, with the reactions queued without a read-back (bench.py --tcp's loop)."""
    a = tcp_storm_sharded(hip, world, device=True, acks=acks, wait=False)
    b = run_tcp_storm(oracle, acks=acks)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3]
