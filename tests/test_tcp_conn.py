"""TCP connections (tgsim_tcp_connect / _write): a per-connection Reno window over
the acks = 1 path, so a connection's writes are ACK-clocked (plans/benchmarks/
storm.go:158-183 writes 4 KiB chunks into one connection). Hand-computed slow start, congestion
avoidance after a timeout, reset connections; randomised HIP-vs-oracle parity."""
import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator, make_rule, make_shape
from testground_amd.network import int_to_ip
from tests import scenarios as S

MS = 1_000_000
MSS = 1448


def sim(b, n=4, **kw):
    kw.setdefault("max_msgs_per_window", 1 << 14)
    kw.setdefault("max_records", 1 << 16)
    s = Simulator(SimConfig(n_instances=n, seed=kw.pop("seed", 3), **kw), binding=b)
    s.tcp_enable(acks=True)
    return s


def run(s, t_end, step=1 * MS, writes=None):
    """1 ms windows up to t_end; returns per-window deliveries; writes: {t: [(conn, size)]}."""
    out, t = [], s.now
    while t < t_end:
        for (tw, items) in sorted((writes or {}).items()):
            if t <= tw < t + step:
                s.tcp_write([c for c, _ in items], [z for _, z in items], [tw] * len(items))
        s.advance(t + step)
        d = s.deliveries()
        s.tcp_react()
        out.append((t, d))
        t += step
    return out


def data_arrivals(out, src):
    """times at which data segments of sender src arrived, with counts"""
    got = {}
    for _, d in out:
        m = (d["src"] == src) & ((d["seq"] & A.TCP_ACK_BIT) == 0)
        for t in d["t_deliver"][m].tolist():
            got[t] = got.get(t, 0) + 1
    return sorted(got.items())


def case_slow_start(b):
    """100 segments on one connection, 10 ms each way: IW10 at 0; every ACK round (a data arrival
    at 10 ms + k*20 ms, its ACK leaving as it arrives and back 10 ms later, where the segments it
    lets out leave) doubles the window: 10, 20, 40, then the last 30 - 20 ms rounds, one RTT each."""
    s = sim(b)
    s.set_shapes([0, 1], [make_shape(latency_ns=10 * MS)] * 2)
    c = s.tcp_connect([0], [1])
    assert list(c) == [0]
    out = run(s, 100 * MS, writes={0: [(0, 100 * MSS)]})
    assert data_arrivals(out, 0) == [(10 * MS, 10), (30 * MS, 20), (50 * MS, 40), (70 * MS, 30)]
    st, t = s.tcp_writes()
    assert list(st) == [A.TCP_DELIVERED] and list(t) == [70 * MS]
    cs = s.tcp_conns()
    assert cs["acked"].tolist() == [100] and cs["cwnd"].tolist() == [110]
    assert cs["flight"].tolist() == [0] and cs["queued"].tolist() == [0]
    s.close()


def case_timeout_then_congestion_avoidance(b):
    """The first 10 segments are lost (the link drops everything until 300 ms). The 200 ms timeout
    starts a loss episode: ssthresh 5, cwnd 1, all 10 marked lost and only the oldest resent (lost
    again); its 600 ms timeout is the same episode (ssthresh stays 5) and its third attempt gets
    through (610 ms). Every 20 ms ACK round then resends under cwnd: 2 (cwnd 2), 4 (4), then cwnd 5
    in congestion avoidance: the last 3 lost ones and 2 new (670 ms), 6 (690 ms), the last 2 (710 ms)."""
    s = sim(b)
    s.set_shapes([0, 1], [make_shape(latency_ns=10 * MS, loss=100.0), make_shape(latency_ns=10 * MS)])
    s.tcp_connect([0], [1])
    out = run(s, 300 * MS, writes={0: [(0, 20 * MSS)]})
    s.set_shape(0, make_shape(latency_ns=10 * MS))
    out += run(s, 750 * MS)
    assert data_arrivals(out, 0) == [(610 * MS, 1), (630 * MS, 2), (650 * MS, 4), (670 * MS, 5), (690 * MS, 6),
                                     (710 * MS, 2)]
    st, t = s.tcp_writes()
    assert list(st) == [A.TCP_DELIVERED] and list(t) == [710 * MS]
    cs = s.tcp_conns()
    assert cs["cwnd"].tolist() == [7] and cs["acked"].tolist() == [20]
    assert cs["flight"].tolist() == [0] and cs["queued"].tolist() == [0]
    assert s.tcp_stats()["retransmissions"] == 11
    s.close()


def case_loss_recovery_under_cwnd(b):
    """DESIGN.md 2.11b's hand case: 10 segments lost once (the link drops everything until 100 ms).
    The 200 ms timeout marks all 10 lost; they are resent 1, 2, 4, 3 per 20 ms ACK round (cwnd 1,
    2, 4, then 5 = ssthresh), not all at once."""
    s = sim(b)
    s.set_shapes([0, 1], [make_shape(latency_ns=10 * MS, loss=100.0), make_shape(latency_ns=10 * MS)])
    s.tcp_connect([0], [1])
    out = run(s, 100 * MS, writes={0: [(0, 10 * MSS)]})
    s.set_shape(0, make_shape(latency_ns=10 * MS))
    out += run(s, 300 * MS)
    assert data_arrivals(out, 0) == [(210 * MS, 1), (230 * MS, 2), (250 * MS, 4), (270 * MS, 3)]
    st, t = s.tcp_writes()
    assert list(st) == [A.TCP_DELIVERED] and list(t) == [270 * MS]
    cs = s.tcp_conns()
    assert cs["cwnd"].tolist() == [6] and cs["acked"].tolist() == [10] and cs["flight"].tolist() == [0]
    assert s.tcp_stats()["retransmissions"] == 10
    s.close()


def case_fast_retransmit(b):
    """One mid-flight loss is recovered in about one RTT, not one RTO. Ten 1-segment writes leave
    at 0..9 ms (10 ms each way); the sender's link drops everything during [3, 4) ms, so segment 3
    alone is lost. The ACKs of 4, 5 and 6 (arriving at 24, 25, 26 ms) are three duplicate ACKs: at
    26 ms segment 3 is resent (ssthresh = max(flight 4 / 2, 2) = 2, cwnd 2) and arrives at 36 ms -
    the 200 ms timer would have resent it at 203 ms. cwnd then grows in congestion avoidance to 3."""
    s = sim(b)
    s.set_shapes([0, 1], [make_shape(latency_ns=10 * MS)] * 2)
    s.tcp_connect([0], [1])
    writes = {i * MS: [(0, MSS)] for i in range(10)}
    out = run(s, 3 * MS, writes=writes)
    s.set_shape(0, make_shape(latency_ns=10 * MS, loss=100.0))
    out += run(s, 4 * MS, writes=writes)
    s.set_shape(0, make_shape(latency_ns=10 * MS))
    out += run(s, 100 * MS, writes=writes)
    assert data_arrivals(out, 0) == [((i + 10) * MS, 1) for i in (0, 1, 2, 4, 5, 6, 7, 8, 9)] + [(36 * MS, 1)]
    retx = [(t, d["seq"][(d["src"] == 0)].tolist()) for t, d in out if np.any((d["src"] == 0) & ((d["seq"] & 15) != 0))]
    assert retx == [(36 * MS, [(3 << 4) | 1])]        # the resent attempt, delivered in the window [36, 37) ms
    st, t = s.tcp_writes()
    assert list(st) == [A.TCP_DELIVERED] * 10 and list(t) == [(i + 10) * MS if i != 3 else 36 * MS for i in range(10)]
    cs = s.tcp_conns()
    assert cs["cwnd"].tolist() == [3] and cs["acked"].tolist() == [10] and cs["flight"].tolist() == [0]
    assert s.tcp_stats()["retransmissions"] == 1
    s.close()


def case_queued_writes_and_reset(b):
    """Two connections from one sender; the second meets a prohibit route: its first segment is
    refused and the connection resets, failing its queued writes; the first is unaffected and its
    writes complete in order."""
    s = sim(b)
    ip = int_to_ip(s.get_ip(2)) + "/32"
    s.add_rules(0, [make_rule(ip, A.FILTER_REJECT)])
    c = s.tcp_connect([0, 0], [1, 2])
    out = run(s, 20 * MS, writes={0: [(c[0], 30 * MSS), (c[1], 30 * MSS), (c[0], 1000), (c[1], 1000)]})
    st, t = s.tcp_writes()
    assert list(st) == [A.TCP_DELIVERED, A.TCP_REFUSED, A.TCP_DELIVERED, A.TCP_REFUSED]
    assert t[1] == 0 and t[3] == 1 * MS                 # refused at once / at the reset's window end
    cs = s.tcp_conns()
    assert cs["acked"].tolist() == [31, 0] and cs["queued"].tolist() == [0, 0]
    s.close()


def case_errors(b):
    s = Simulator(SimConfig(n_instances=4, seed=1), binding=b)
    s.tcp_enable()                                       # acks = 0: no ACK clock
    with pytest.raises(A.TgsimError) as e:
        s.tcp_connect([0], [1])
    assert e.value.code == A.ESTATE
    s.close()
    s = sim(b)
    s.tcp_connect([0], [1])
    with pytest.raises(A.TgsimError) as e:
        s.tcp_send([0], [1], [0], [10], [0])             # one interface per context
    assert e.value.code == A.ESTATE
    with pytest.raises(A.TgsimError) as e:
        s.tcp_write([5], [10], [0])
    assert e.value.code == A.EINVAL
    s.close()


CASES = [case_slow_start, case_timeout_then_congestion_avoidance, case_loss_recovery_under_cwnd, case_fast_retransmit,
         case_queued_writes_and_reset,
         case_errors]


@pytest.mark.parametrize("case", CASES, ids=lambda f: f.__name__)
def test_conn_oracle(oracle, case):
    case(oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda f: f.__name__)
def test_conn_hip(hip, case):
    case(hip)


def random_conn_run(b, seed, n=16, windows=160, restart=()):
    """Connections between random pairs (some twice), lossy / duplicating / corrupting links of a
    few ms, writes of 1 B .. 40 segments arriving over the first 60 windows, a prohibit route."""
    rng = np.random.default_rng(seed)
    s = sim(b, n=n, seed=seed, max_msgs_per_window=1 << 15, max_records=1 << 17)
    s.set_shapes(np.arange(n), [make_shape(latency_ns=int(rng.integers(1, 6)) * MS, jitter_ns=int(rng.integers(0, 2)) * MS,
                                           loss=float(rng.choice([0.0, 2.0, 10.0])), duplicate=float(rng.choice([0.0, 5.0])),
                                           corrupt=float(rng.choice([0.0, 3.0]))) for _ in range(n)])
    s.add_rules(3, [make_rule(int_to_ip(s.get_ip(7)) + "/32", A.FILTER_REJECT)])
    src = rng.integers(0, n, 24)
    dst = (src + rng.integers(1, n, 24)) % n
    src[0], dst[0] = 3, 7
    conns = s.tcp_connect(src, dst)
    writes = {}
    for w in range(60):
        k = int(rng.integers(0, 4))
        if k:
            t = w * MS + int(rng.integers(0, MS))
            writes[t] = [(int(rng.choice(conns)), int(rng.integers(1, 40 * MSS))) for _ in range(k)]
    if restart:  # checkpoint / resume: after the windows ending at the given ms, a fresh context
        cfg = s.cfg
        out = []
        for stop in sorted(restart) + [windows]:
            out += run(s, stop * MS, writes=writes)
            if stop == windows:
                break
            image = s.snapshot()
            s.close()
            s = Simulator(cfg, binding=b)
            s.tcp_enable(acks=True)
            s.tcp_connect(src, dst)
            s.restore(image)
    else:
        out = run(s, windows * MS, writes=writes)
    st, t = s.tcp_writes()
    res = dict(deliv=[d for _, d in out], status=None, writes=(st, t), conns=s.tcp_conns(), stats=S.parity_stats(s),
               tcp=s.tcp_stats())
    s.close()
    return res


def test_conn_random_oracle_properties(oracle):
    r = random_conn_run(oracle, 1)
    st, _ = r["writes"]
    # Reno at 10 % loss holds cwnd near 1.22 / sqrt(p) ~ 4 segments (fast retransmit halves it at
    # every hole), so some writes are still queued behind their connection's window at 160 ms
    assert np.count_nonzero(st == A.TCP_DELIVERED) > 0.5 * len(st)
    cs = r["conns"]
    assert np.all(cs["cwnd"] >= 1) and cs["acked"].sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_conn_random_hip_matches_oracle(hip, oracle, seed):
    a, b = random_conn_run(hip, seed), random_conn_run(oracle, seed)
    S.assert_same(a["deliv"], b["deliv"])
    assert np.array_equal(a["writes"][0], b["writes"][0]) and np.array_equal(a["writes"][1], b["writes"][1])
    for k in a["conns"]:
        assert np.array_equal(a["conns"][k], b["conns"][k]), k
    assert a["stats"] == b["stats"]
