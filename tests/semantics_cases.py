"""Hand-computed known answers for the pinned semantics. Each case takes a
binding and asserts; tests/test_semantics.py runs them on the CPU oracle, tests/test_gpu_parity.py
on the HIP library."""
from __future__ import annotations

import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator, make_rule, make_shape

MS = 1_000_000


def sim(binding, n=4, **kw):
    kw.setdefault("max_msgs_per_window", 1 << 14)
    kw.setdefault("max_records", 1 << 16)
    return Simulator(SimConfig(n_instances=n, seed=kw.pop("seed", 7), **kw), binding=binding)


def one_window(s, src, dst, size, t, t_end, seq=None):
    src = np.atleast_1d(src)
    n = len(src)
    seq = np.arange(n) if seq is None else seq
    s.enqueue(src, np.broadcast_to(dst, (n,)), seq, np.broadcast_to(size, (n,)), np.broadcast_to(t, (n,)))
    s.advance(t_end)
    return s.status(), s.deliveries()


def case_unshaped_delivers_at_send_time(b):
    s = sim(b)
    st, d = one_window(s, [0, 1, 2], [1, 2, 3], 100, [5, 6, 7], 10)
    assert list(st) == [A.ST_QUEUED] * 3
    assert list(d["t_deliver"]) == [5, 6, 7] and list(d["dst"]) == [1, 2, 3]
    assert list(s.inbox_offsets()) == [0, 0, 1, 2, 3]
    s.close()


def case_latency(b):
    s = sim(b)
    s.set_shape(0, make_shape(latency_ns=20 * MS))
    st, d = one_window(s, 0, 1, 10, 1000, 10 * MS)
    assert list(st) == [A.ST_QUEUED] and len(d["t_deliver"]) == 0
    s.advance(30 * MS)
    d = s.deliveries()
    assert list(d["t_deliver"]) == [1000 + 20 * MS]
    s.close()


def case_loss_all_and_none(b):
    s = sim(b)
    s.set_shape(0, make_shape(loss=100.0))
    st, d = one_window(s, [0] * 50 + [1] * 50, 2, 10, 0, 1 * MS)
    assert list(st[:50]) == [A.ST_LOST] * 50 and list(st[50:]) == [A.ST_QUEUED] * 50
    assert len(d["src"]) == 50 and set(d["src"]) == {1}
    stats = s.stats()
    assert stats["lost"] == 50 and stats["delivered"] == 50
    s.close()


def case_duplicate_all(b):
    s = sim(b)
    s.set_shape(0, make_shape(duplicate=100.0))
    st, d = one_window(s, [0] * 10, 1, 10, 100, 1 * MS)
    assert all(x == A.ST_QUEUED | A.ST_FLAG_DUP for x in st)
    assert len(d["seq"]) == 20
    # inbox order (dst, t, src, seq, clone first): each seq appears twice, clone first
    assert list(d["seq"]) == [k for k in range(10) for _ in range(2)]
    assert list(d["flags"] & A.F_CLONE) == [1, 0] * 10
    s.close()


def case_duplicate_and_loss_cancel(b):
    s = sim(b)
    s.set_shape(0, make_shape(duplicate=100.0, loss=100.0))
    st, d = one_window(s, [0] * 10, 1, 10, 100, 1 * MS)
    # netem_enqueue [EXT]: count = 1 + dup - loss = 1 -> the original alone goes out, no clone
    assert all((x & 0x0F) == A.ST_QUEUED and x & A.ST_FLAG_DUP_CANCEL and not x & A.ST_FLAG_DUP for x in st)
    assert list(d["seq"]) == list(range(10)) and not np.any(d["flags"] & A.F_CLONE)
    s.close()


def case_jitter_bounds(b):
    s = sim(b, n=8, seed=11)
    senders = [0, 2, 3, 4]    # 1000 each: a full netem queue, nothing tail-dropped (limit 1000)
    for g in senders:
        s.set_shape(g, make_shape(latency_ns=50 * MS, jitter_ns=10 * MS))
    n = 4000
    one_window(s, np.repeat(senders, n // 4), 1, 10, 0, 1 * MS)
    s.advance(100 * MS)
    delay = s.deliveries()["t_deliver"]
    assert len(delay) == n
    assert delay.min() >= 40 * MS and delay.max() < 60 * MS
    # uniform: mean within 4 standard errors of 50 ms (parity unpinned vs real netem: DESIGN.md 3)
    assert abs(delay.mean() - 50 * MS) < 4 * (20 * MS / np.sqrt(12)) / np.sqrt(n)
    s.close()


def case_token_bucket_spacing(b):
    """8 Mbit/s = 1e6 B/s; HTB burst = rate/HZ + 1600 B -> tau ~ 1.6 ms. 1000-B messages all at t:
    GCRA departures e, e, e+0.4ms, e+1.4ms, ... (spacing = cost = 1 ms after the burst)."""
    s = sim(b)
    s.set_shape(0, make_shape(bandwidth_bps=8_000_000))
    _, d0 = one_window(s, np.zeros(10, np.int64), 1, 1000, 0, 1)
    s.advance(20 * MS)
    d = np.concatenate([d0["t_deliver"], s.deliveries()["t_deliver"]])
    assert len(d) == 10 and d[0] == 0 and d[1] == 0 and len(d0["t_deliver"]) == 2
    gaps = np.diff(d[2:])
    assert np.all(np.abs(gaps - 1_000_000) <= 1), gaps
    assert abs(d[2] - 400_000) <= 1_000
    s.close()


def case_reorder_and_corrupt(b):
    s = sim(b)
    s.set_shape(0, make_shape(latency_ns=10 * MS, reorder=100.0, corrupt=100.0))
    one_window(s, np.zeros(5, np.int64), 1, 64, 7, 1 * MS)
    d = s.deliveries()
    assert list(d["t_deliver"]) == [7] * 5                       # reordered: sent without delay
    assert np.all(d["flags"] & A.F_REORDERED) and np.all(d["flags"] & A.F_CORRUPT)
    assert np.all(d["corrupt_off"] < 64)
    s.close()


def case_rules_longest_prefix(b):
    s = sim(b, n=8)
    ip = [s.get_ip(g) for g in range(8)]
    from testground_amd.network import int_to_ip
    net24 = int_to_ip(ip[3] & 0xFFFFFF00) + "/24"
    s.add_rules(0, [make_rule(net24, A.FILTER_DROP), make_rule(int_to_ip(ip[3]) + "/32", A.FILTER_REJECT)])
    st, _ = one_window(s, [0, 0, 1], [3, 4, 3], 10, 0, 1 * MS)
    # the data network's connected /16 loses to the /24 and /32 rules (longest prefix wins)
    assert list(st) == [A.ST_REJECTED, A.ST_DROPPED, A.ST_QUEUED]
    s.add_rules(0, [make_rule(int_to_ip(ip[3]) + "/32", A.FILTER_ACCEPT)])   # deletes only the /32
    st, _ = one_window(s, [0], [3], 10, 1 * MS, 2 * MS, seq=[10])
    assert list(st) == [A.ST_DROPPED]
    s.add_rules(0, [make_rule(net24, A.FILTER_ACCEPT)])
    st, _ = one_window(s, [0], [3], 10, 2 * MS, 3 * MS, seq=[11])
    assert list(st) == [A.ST_QUEUED]
    with pytest.raises(A.TgsimError) as e:
        s.add_rules(0, [make_rule(int_to_ip(ip[3]) + "/24", A.FILTER_DROP)])   # host bits set
    assert e.value.code == A.EINVAL
    s.close()


def case_rules_batch_order(b):
    """AddRules applies a batch in order (link.go:187-217): the last rule for a prefix wins within
    the batch (Drop then Accept deletes, Accept then Reject installs), and the first invalid rule
    stops the batch with the earlier rules applied."""
    s = sim(b, n=8)
    from testground_amd.network import int_to_ip
    ip = [int_to_ip(s.get_ip(g)) + "/32" for g in range(8)]
    s.add_rules(0, [make_rule(ip[1], A.FILTER_DROP), make_rule(ip[2], A.FILTER_ACCEPT), make_rule(ip[1], A.FILTER_ACCEPT),
                    make_rule(ip[2], A.FILTER_REJECT), make_rule(ip[3], A.FILTER_REJECT), make_rule(ip[3], A.FILTER_DROP)])
    st, _ = one_window(s, [0, 0, 0, 0], [1, 2, 3, 4], 10, 0, 1 * MS)
    assert list(st) == [A.ST_QUEUED, A.ST_REJECTED, A.ST_DROPPED, A.ST_QUEUED]
    with pytest.raises(A.TgsimError) as e:
        s.add_rules(0, [make_rule(ip[4], A.FILTER_DROP), make_rule(ip[5], 7), make_rule(ip[6], A.FILTER_DROP)])
    assert e.value.code == A.EINVAL
    st, _ = one_window(s, [0, 0, 0], [4, 5, 6], 10, 1 * MS, 2 * MS, seq=[4, 5, 6])
    assert list(st) == [A.ST_DROPPED, A.ST_QUEUED, A.ST_QUEUED]
    s.close()


def case_policy_and_external(b):
    s = sim(b)
    s.set_policy(1, A.POLICY_ALLOW_ALL)
    st, _ = one_window(s, [0, 1], A.DST_EXTERNAL, 10, 0, 1 * MS)
    assert list(st) == [A.ST_UNREACHABLE, A.ST_EXTERNAL]
    stats = s.stats()
    assert stats["external"] == 1 and stats["unreachable"] == 1 and stats["delivered"] == 0
    s.close()


def case_enable_and_ip_change(b):
    s = sim(b)
    s.set_enabled(2, False)
    st, _ = one_window(s, [0, 2, 1], [2, 0, 0], 10, 0, 1 * MS)
    # receiver down: DEST_DOWN; sender down: no data route and external routing denied
    assert list(st) == [A.ST_DEST_DOWN, A.ST_UNREACHABLE, A.ST_QUEUED]
    old = s.get_ip(3)
    s.set_enabled(3, True, ip=old + 100)          # docker_network.go:77-88: disconnect + reconnect
    assert s.get_ip(3) == old + 100
    s.set_enabled(2, True)
    st, d = one_window(s, [0, 2], [3, 0], 10, 1 * MS, 2 * MS, seq=[5, 6])
    assert list(st) == [A.ST_QUEUED, A.ST_QUEUED] and len(d["src"]) == 2
    with pytest.raises(A.TgsimError):
        s.set_enabled(1, True, ip=old + 100)     # address in use
    s.close()


def case_apply_order_docker_vs_k8s(b):
    """docker_network.go:51-148 applies the routing policy first, even to a disconnect; K8sNetwork
    (k8s_network.go:50-61, :166-174) returns after a disconnect and applies the policy last, so a
    failing AddRules leaves it as it was. External routes leave through the control network and do
    not need the data link (route.go:68-100)."""
    from testground_amd.network import Config, IPNet, LinkRule, LinkShape, FilterAction
    s = sim(b)
    off = Config(network="default", enable=False, routing_policy="allow_all")
    s.configure(0, off, "docker")
    s.configure(1, off, "k8s")
    st, _ = one_window(s, [0, 1], A.DST_EXTERNAL, 10, 0, 1 * MS)
    assert list(st) == [A.ST_EXTERNAL, A.ST_UNREACHABLE]
    bad = Config(network="default", enable=True, routing_policy="allow_all",
                 rules=[LinkRule(IPNet.parse("16.0.0.5/24"), LinkShape(filter=FilterAction.Drop))])  # host bits
    for g, order in ((2, "docker"), (3, "k8s")):
        with pytest.raises(A.TgsimError) as e:
            s.configure(g, bad, order)
        assert e.value.code == A.EINVAL
    st, _ = one_window(s, [2, 3, 0, 1], [A.DST_EXTERNAL, A.DST_EXTERNAL, 3, 3], 10, 1 * MS, 2 * MS, seq=[1, 1, 2, 2])
    # docker: policy applied before the failing AddRules; k8s: never reached. Disabled senders 0/1
    # have no data route, whatever their policy says about external traffic.
    assert list(st) == [A.ST_EXTERNAL, A.ST_UNREACHABLE, A.ST_UNREACHABLE, A.ST_UNREACHABLE]
    on = Config(network="default", enable=True, routing_policy="allow_all", default=LinkShape(latency=3 * MS))
    s.configure(1, on, "k8s")
    st, _ = one_window(s, [1, 1], [2, A.DST_EXTERNAL], 10, 2 * MS, 3 * MS, seq=[3, 4])
    assert list(st) == [A.ST_QUEUED, A.ST_EXTERNAL]
    s.advance(10 * MS)
    assert list(s.deliveries()["t_deliver"]) == [5 * MS]
    with pytest.raises(A.TgsimError) as e:
        s.configure(1, Config(network="other", enable=True), "k8s")
    assert e.value.code == A.EUNSUPPORTED_NETWORK
    s.close()


def case_loopback(b):
    s = sim(b)
    s.set_shape(0, make_shape(latency_ns=10 * MS, loss=100.0))
    st, d = one_window(s, [0], [0], 10, 3, 1 * MS)
    assert list(st) == [A.ST_LOCAL] and list(d["t_deliver"]) == [3] and d["flags"][0] & A.F_LOCAL
    s.close()


def case_reaction_horizon(b):
    s = sim(b)
    s.advance(10 * MS)
    s.advance(20 * MS)
    assert s.horizon == 10 * MS and s.now == 20 * MS
    with pytest.raises(A.TgsimError) as e:
        s.enqueue([0], [1], [0], [1], [10 * MS - 1])
    assert e.value.code == A.ECAUSALITY
    # a reaction at a time inside the last window is admissible and delivered late, at its own time
    st, d = one_window(s, [0], [1], 10, 15 * MS, 30 * MS, seq=[1])
    assert list(st) == [A.ST_QUEUED] and list(d["t_deliver"]) == [15 * MS]
    s.close()


def case_staged_after_window_end(b):
    """A staged message sent at/after the window end is refused before anything changes: the
    context stays usable and the message goes out with the next window that covers it."""
    s = sim(b)
    s.enqueue([0], [1], [0], [1], [5 * MS])
    with pytest.raises(A.TgsimError) as e:
        s.advance(5 * MS)
    assert e.value.code == A.ECAUSALITY
    assert s.now == 0
    s.advance(6 * MS)
    st, d = s.status(), s.deliveries()
    assert list(st) == [A.ST_QUEUED] and list(d["t_deliver"]) == [5 * MS]
    st, _ = one_window(s, [1], [2], 1, 6 * MS, 7 * MS)
    assert list(st) == [A.ST_QUEUED]
    s.close()


def case_sync_sequence_and_barrier(b):
    s = sim(b, n=4, max_states=16)
    seq = s.signal([0, 0, 0, 1], [3, 1, 2, 0], [50, 50, 40, 10])
    assert list(seq) == [3, 2, 1, 1]          # (t, instance) order within a state
    w = s.barrier(0, 3, 20)
    assert s.poll(w) == 50                    # released by the third signal
    w2 = s.barrier(0, 5, 20)
    assert s.poll(w2) == -1
    s.signal([0, 0], [9, 8], [60, 70])
    assert s.poll(w2) == 70 and s.count(0) == 5
    assert s.poll(s.barrier(1, 0, 33)) == 33  # target 0: immediate
    assert s.poll(s.barrier(1, 1, 5)) == 10   # released at max(t_wait, signal time)
    with pytest.raises(A.TgsimError) as e:
        s.signal([0], [1], [65])              # goes back in time for state 0
    assert e.value.code == A.ECAUSALITY
    s.close()


def case_queue_limit_burst(b):
    """netem limit 1000 [EXT netlink default; link.go:169-179 sets none]: a burst of 1500 at one
    instant fills the queue with the first 1000 in enqueue order (t_send, seq); 500 tail-drops."""
    s = sim(b)
    s.set_shape(0, make_shape(latency_ns=10 * MS))
    st, d = one_window(s, np.zeros(1500, np.int64), 1, 10, 0, 1 * MS, seq=np.arange(1500)[::-1].copy())
    # seq runs backwards in enqueue index: the queue takes the 1000 smallest seq (indices 500..1499)
    assert list(st[500:]) == [A.ST_QUEUED] * 1000 and list(st[:500]) == [A.ST_OVERLIMIT | A.ST_FLAG_OVERLIMIT] * 500
    s.advance(20 * MS)
    d = s.deliveries()
    assert len(d["seq"]) == 1000 and set(d["seq"]) == set(range(1000))
    assert s.stats()["overlimit"] == 500
    s.close()


def case_queue_limit_spans_windows(b):
    """Copies queued in earlier windows count until they depart; a copy departing at exactly t has
    left the queue for an enqueue at t (occupancy over [enqueue, departure))."""
    s = sim(b)
    s.set_shape(0, make_shape(latency_ns=10 * MS))
    st, _ = one_window(s, np.zeros(1000, np.int64), 1, 10, 0, 5 * MS)
    assert list(st) == [A.ST_QUEUED] * 1000
    t = np.array([10 * MS - 1] * 10 + [10 * MS] * 10 + [10 * MS + 1] * 10)
    st, d = one_window(s, np.zeros(30, np.int64), 1, 10, t, 20 * MS, seq=np.arange(1000, 1030))
    assert list(st) == [A.ST_OVERLIMIT | A.ST_FLAG_OVERLIMIT] * 10 + [A.ST_QUEUED] * 20
    assert len(d["seq"]) == 1000 and s.stats()["overlimit"] == 10
    s.close()


def case_queue_limit_duplicates(b):
    """The clone is enqueued first (through the root qdisc) and counts for the original's check."""
    s = sim(b)
    s.set_shape(0, make_shape(latency_ns=10 * MS, duplicate=100.0))
    st, _ = one_window(s, np.zeros(600, np.int64), 1, 10, 0, 1 * MS)
    full = A.ST_OVERLIMIT | A.ST_FLAG_DUP | A.ST_FLAG_CLONE_LOST | A.ST_FLAG_OVERLIMIT
    assert list(st) == [A.ST_QUEUED | A.ST_FLAG_DUP] * 500 + [full] * 100
    s.close()
    s = sim(b)
    s.set_shape(0, make_shape(latency_ns=10 * MS))
    one_window(s, np.zeros(999, np.int64), 1, 10, 0, 1 * MS)
    s.set_shape(0, make_shape(latency_ns=10 * MS, duplicate=100.0))
    st, _ = one_window(s, [0, 0], 1, 10, 1 * MS, 2 * MS, seq=[999, 1000])
    # 999 queued: the clone takes the last place, the original is tail-dropped; then both dropped
    assert list(st) == [A.ST_QUEUED | A.ST_FLAG_DUP | A.ST_FLAG_OVERLIMIT, full]
    s.close()


def case_queue_limit_token_bucket(b):
    """A limited sender's copies stay queued until the HTB lets them go: the queue admits exactly
    as many new copies as have departed (departure <= t) by the time they arrive."""
    s = sim(b)
    s.set_shape(0, make_shape(bandwidth_bps=8_000_000))   # 1000-B copies: 1 ms each
    st, d0 = one_window(s, np.zeros(1200, np.int64), 1, 1000, 0, 400 * MS)
    assert list(st) == [A.ST_QUEUED] * 1000 + [A.ST_OVERLIMIT | A.ST_FLAG_OVERLIMIT] * 200
    st, d1 = one_window(s, np.zeros(700, np.int64), 1, 1000, 500 * MS, 501 * MS, seq=np.arange(1200, 1900))
    departed = int(np.count_nonzero(d0["t_deliver"] <= 500 * MS)) + int(np.count_nonzero(d1["t_deliver"] <= 500 * MS))
    assert 490 < departed < 510
    assert int(np.count_nonzero(st == A.ST_QUEUED)) == departed
    assert list(st[departed:]) == [A.ST_OVERLIMIT | A.ST_FLAG_OVERLIMIT] * (700 - departed)
    s.close()


def case_seed_determinism(b):
    def run(seed):
        s = sim(b, seed=seed)
        s.set_shape(0, make_shape(latency_ns=1 * MS, jitter_ns=1 * MS, loss=30.0))
        st, _ = one_window(s, np.zeros(200, np.int64), 1, 10, 0, 1 * MS)
        s.advance(10 * MS)
        out = st.copy(), s.deliveries()["t_deliver"].copy()
        s.close()
        return out
    a, a2, c = run(1), run(1), run(2)
    assert np.array_equal(a[0], a2[0]) and np.array_equal(a[1], a2[1])
    assert not np.array_equal(a[0], c[0])


CASES = [v for k, v in sorted(globals().items()) if k.startswith("case_")]
