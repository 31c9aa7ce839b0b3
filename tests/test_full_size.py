"""Parity at BASELINE.json's full sizes on the HIP library.

The oracle cannot replay 1e8-message runs in seconds, so the full-size runs are checked three ways:

* sender restriction: all shaping state is sender-egress (pkg/sidecar/link.go:33-34, :155-217), so
  the fate of a sender's messages depends on that sender's messages only. The oracle replays a
  subset of senders over the whole run; the HIP run's statuses and deliveries filtered to those
  senders must equal it bit for bit (delivery order (dst, t, src, seq) survives the filter);
* size-independent properties over every message: conservation (deliveries = queued copies),
  uniqueness of (src, seq), delay bounds of the shape, inbox order, the routing truth table;
* the 100k storm (config 4), whose barrier couples all senders, is replayed whole by the oracle
  for its first rounds.
"""
import ctypes as C

import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator, make_shape
from tests import scenarios as S

pytestmark = pytest.mark.gpu
MS = 1_000_000


def _filter(d: dict, keep: np.ndarray) -> dict:
    return {k: v[keep] for k, v in d.items()}


def _assert_inbox_order(d: dict) -> None:
    """Deliveries of one window are ordered by (dst, t_deliver, src, seq, clone first)."""
    if len(d["dst"]) < 2:
        return
    key = np.lexsort((d["seq"], d["src"], d["t_deliver"], d["dst"]))
    assert np.array_equal(key, np.arange(len(key))), "inbox order broken"


# ---- config 2: 1k instances all-to-all, 4 KiB, jitter + loss, 100 rounds ------------------------

def _a2a_send_time(src: np.ndarray, seq: np.ndarray, t0: int) -> np.ndarray:
    """t_send uniform in [t0, t0 + 1 ms), a pure function of (src, seq) so deliveries can be
    checked against it without keeping the rounds' inputs."""
    h = (src.astype(np.uint64) * np.uint64(2654435761) + seq.astype(np.uint64) * np.uint64(40503)) & np.uint64(0xFFFFFFFF)
    return t0 + (h % np.uint64(MS)).astype(np.int64)


def _run_a2a(binding, n: int, rounds: int, senders=None, on_window=None):
    """plans/benchmarks storm shape (storm.go:23: 4 KiB writes) as all-to-all rounds of 10 ms."""
    sim = Simulator(SimConfig(n_instances=n, seed=2, max_msgs_per_window=1 << 20, max_records=1 << 22),
                    binding=binding)
    sim.set_shapes(np.arange(n), [make_shape(latency_ns=50 * MS, jitter_ns=10 * MS, loss=1.0)] * n)
    snd = np.arange(n, dtype=np.uint32) if senders is None else np.asarray(senders, np.uint32)
    out = []
    for r in range(rounds + 8):                   # 8 trailing windows drain the in-flight copies
        t0 = r * 10 * MS
        if r < rounds:
            src = np.repeat(snd, n - 1)
            off = np.tile(np.arange(1, n, dtype=np.uint32), len(snd))
            dst = (src + off) % np.uint32(n)
            seq = np.uint32(r * n) + dst
            t = _a2a_send_time(src, seq, t0)
            sim.enqueue(src, dst, seq, np.full(len(src), 4096, np.uint32), t)
        sim.advance(t0 + 10 * MS)
        st = sim.status() if r < rounds else np.zeros(0, np.uint8)
        d = sim.deliveries()
        out.append((st, d) if on_window is None else on_window(r, st, d))
        if r % 20 == 0:
            print(f"  a2a {binding.name} window {r}", flush=True)
    sim.close()
    return out


def test_cfg2_all_to_all_full(hip, oracle, n=1000, rounds=100):
    subset = np.unique(np.array([0, 1, 2, n // 2, n - 2, n - 1] + list(range(37, n, 61)), np.uint32))
    in_subset = np.zeros(n, bool)
    in_subset[subset] = True
    tot = dict(sent=0, queued=0, lost=0, over=0, delivered=0)
    seen = []

    def check(r, st, d):
        _assert_inbox_order(d)
        tot["delivered"] += len(d["dst"])
        if len(st):
            assert len(st) == n * (n - 1)
            tot["sent"] += len(st)
            tot["queued"] += int(np.count_nonzero(st == A.ST_QUEUED))
            tot["lost"] += int(np.count_nonzero(st == A.ST_LOST))
            tot["over"] += int(np.count_nonzero(st == (A.ST_OVERLIMIT | A.ST_FLAG_OVERLIMIT)))
        if len(d["dst"]):
            # delay = latency + U[-jitter, jitter) (sch_netem tabledist), never below 40 ms
            r_send = (d["seq"] // n).astype(np.int64)
            ts = _a2a_send_time(d["src"], d["seq"], r_send * 10 * MS)
            delay = d["t_deliver"] - ts
            assert delay.min() >= 40 * MS and delay.max() < 60 * MS
            assert np.all(d["size"] == 4096) and np.all(d["flags"] == 0)
            seen.append((d["src"].astype(np.uint64) << np.uint64(32)) | d["seq"].astype(np.uint64))
        ks = in_subset[d["src"]]
        kst = in_subset[np.repeat(np.arange(n), n - 1)] if len(st) else np.zeros(0, bool)
        return st[kst], _filter(d, ks)

    gpu = _run_a2a(hip, n, rounds, on_window=check)
    ids = np.concatenate(seen)
    assert len(np.unique(ids)) == len(ids) == tot["delivered"]       # every copy delivered once
    assert tot["sent"] == n * (n - 1) * rounds
    assert tot["queued"] + tot["lost"] + tot["over"] == tot["sent"] and tot["delivered"] == tot["queued"]
    # netem's 1000-packet queue: 999 sends per 1 ms burst every 10 ms at 50 +- 10 ms
    # latency keep ~5 bursts queued per sender, so about 4 in 5 copies are tail-dropped
    assert 0.7 < tot["over"] / tot["sent"] < 0.9, tot
    p = 42949672 / 2 ** 32                                              # Percentage2u32(1 %)
    sd = np.sqrt(p * (1 - p) / tot["sent"])
    assert abs(tot["lost"] / tot["sent"] - p) < 6 * sd
    ref = _run_a2a(oracle, n, rounds, senders=subset)
    for w, ((gs, gd), (os_, od)) in enumerate(zip(gpu, ref)):
        assert np.array_equal(gs, os_), f"window {w}: statuses differ"
        S.assert_same(gd, od, f"window {w}")


# ---- config 3: 10k instances, splitbrain /32 rules, all-pairs probes --------------------------

def _rule_block(sim: Simulator, targets: np.ndarray, action: int):
    arr = (A.LinkRule * len(targets))()
    for i, g in enumerate(targets):
        arr[i].subnet_ip = sim.get_ip(int(g))
        arr[i].prefix_len = 32
        arr[i].shape.filter = action
    return arr


def _run_splitbrain(binding, n: int, senders: np.ndarray, chunk: int, on_window=None):
    """plans/splitbrain/main.go:60-186 at config 3 size: region = g % 3, region-A senders hold a
    /32 rule toward every region-B address; the action goes Drop -> Reject -> Accept; each phase
    sends one all-pairs round of 64 B probes, the senders g in [c*chunk, (c+1)*chunk) in window c
    of the phase (a run restricted to `senders` keeps the same windows). Every sender also fetches
    an external address each window it sends (plans/network/traffic.go:46-52), and the routing
    policy of every instance flips AllowAll <-> DenyAll every 5 windows (BASELINE config 3)."""
    sim = Simulator(SimConfig(n_instances=n, seed=3, max_msgs_per_window=1 << 24, max_records=1 << 25),
                    binding=binding)
    sim.set_shapes(np.arange(n), [make_shape(latency_ns=10 * MS)] * n)
    region = np.arange(n) % 3
    a_ids, b_ids = np.nonzero(region == 0)[0], np.nonzero(region == 1)[0]
    senders = np.asarray(senders)
    out, t0, w = [], 0, 0
    policy = A.POLICY_DENY_ALL
    for phase, action in enumerate((A.FILTER_DROP, A.FILTER_REJECT, A.FILTER_ACCEPT)):
        rules = _rule_block(sim, b_ids, action)
        for g in a_ids:
            sim._check(sim.lib.add_rules(sim._ctx, int(g), rules, len(b_ids)))
        print(f"  splitbrain {binding.name} phase {phase}: rules installed", flush=True)
        for c0 in range(0, n, chunk):
            if w % 5 == 0:
                policy = A.POLICY_ALLOW_ALL if policy == A.POLICY_DENY_ALL else A.POLICY_DENY_ALL
                for g in range(n):
                    sim.set_policy(g, policy)
            snd = senders[(senders >= c0) & (senders < c0 + chunk)].astype(np.uint32)
            src = np.repeat(snd, n)
            dst = (src + np.tile(np.arange(1, n + 1, dtype=np.uint32), len(snd))) % np.uint32(n)
            ext = dst == src                       # the n-th probe of each sender: the external fetch
            dst[ext] = A.DST_EXTERNAL
            seq = np.where(ext, np.uint32(3 * n + phase), np.uint32(phase * n) + dst)
            sim.enqueue(src, dst, seq, np.full(len(src), 64, np.uint32), np.full(len(src), t0, np.int64))
            t0 += 10 * MS
            sim.advance(t0)
            st, d = sim.status(), sim.deliveries()
            out.append((src, dst, st, d) if on_window is None else on_window(w, phase, policy, src, dst, st, d))
            w += 1
    t0 += 10 * MS
    sim.advance(t0)
    d = sim.deliveries()
    e = np.zeros(0, np.uint32)
    out.append((e, e, np.zeros(0, np.uint8), d) if on_window is None else on_window(w, 3, policy, e, e, np.zeros(0, np.uint8), d))
    sim.close()
    return out


def _splitbrain_want(n, phase, policy, src, dst):
    """Statuses the pinned semantics give one window of probes: the truth table of
    plans/splitbrain/main.go:50-58 (region = g % 3), the policy for the external fetch
    (route.go:102-117), and netem's 1000-packet queue: a sender's routable probes enter it in seq
    (= destination) order, all at one instant, so the first 1000 are queued and the rest dropped."""
    region = np.arange(n) % 3
    expect_blocked = {0: A.ST_DROPPED, 1: A.ST_REJECTED, 2: None}
    want = np.full(len(src), A.ST_QUEUED, np.uint8)
    ext = dst == A.DST_EXTERNAL
    want[ext] = A.ST_EXTERNAL if policy == A.POLICY_ALLOW_ALL else A.ST_UNREACHABLE
    dd = np.where(ext, 0, dst)
    blocked = ~ext & (region[src] == 0) & (region[dd] == 1)
    if expect_blocked[phase] is not None:
        want[blocked] = expect_blocked[phase]
    else:
        blocked[:] = False
    q = np.nonzero(~ext & ~blocked)[0]
    order = q[np.lexsort((dst[q], src[q]))]
    first = np.r_[True, src[order][1:] != src[order][:-1]]
    start = np.maximum.accumulate(np.where(first, np.arange(len(order)), 0))
    rank = np.arange(len(order)) - start
    want[order[rank >= A.NETEM_LIMIT]] = A.ST_OVERLIMIT | A.ST_FLAG_OVERLIMIT
    return want


def _splitbrain_descriptor(binding, n, case):
    """plans/splitbrain as the reference runs it (testground_amd.plans.splitbrain): sequential
    probes, one-minute timeouts, the 300 s plan context."""
    from testground_amd import plans as P
    env = P.PlanEnv(n, seed=3, test_case=case, binding=binding,
                    sim_kw=dict(max_msgs_per_window=1 << 16, max_records=1 << 18))
    ok = P.PLANS[("splitbrain", case)](env)
    res = dict(ok=ok, outcome=env.probe_outcome, done=env.probe_done, region=env.region,
               windows=env.probe_windows, unexpected=env.probe_unexpected, errors=env.probe_errors,
               stats={k: v for k, v in env.sim.stats().items() if k not in ("windows", "inflight")},
               testcomplete=env.testcomplete)
    env.close()
    return res


def _check_splitbrain_truth(r, n, case):
    from testground_amd import plans as P
    region = r["region"]
    assert list(region) == [(g + 1) % 3 for g in range(n)]
    assert not r["unexpected"].any() and r["stats"]["overlimit"] == 0
    out = r["outcome"]
    a, b = np.flatnonzero(region == 0), np.flatnonzero(region == 1)
    probed = ~np.eye(n, dtype=bool)               # topic order = instance order (seq = g + 1)
    if case == "accept":
        assert np.all(out[probed] == A.PROBE_OK)
        # zero latency, lock step: n - 1 probes of two one-window hops each, from t0 on
        assert len(np.unique(r["done"])) == 1 and r["ok"].all()
    else:
        assert np.all(out[np.ix_(a, b)] == A.PROBE_REFUSED) and np.all(out[np.ix_(b, a)] == A.PROBE_TIMEOUT)
        other = probed.copy()
        other[np.ix_(a, b)] = other[np.ix_(b, a)] = False
        assert np.all(out[other] == A.PROBE_OK)
        # region B waits out one minute per region-A peer: far past the plan's 300 s context
        assert r["done"][b].min() > len(a) * P.PROBE_TIMEOUT_NS and not r["ok"].any()


@pytest.mark.timeout(900)
def test_cfg3_splitbrain_full(hip, oracle, n=10_000):
    """BASELINE config 3 as the reference plan generates it: 10k instances,
    region = seq % 3, every node GETs every other node one at a time (plans/splitbrain/main.go:
    153-175) - 1e8 probes, 2e8 messages over 2e4 windows. HIP and the oracle agree on every probe's
    outcome, every node's end time, the window count and the counters."""
    gpu = _splitbrain_descriptor(hip, n, "accept")
    _check_splitbrain_truth(gpu, n, "accept")
    ref = _splitbrain_descriptor(oracle, n, "accept")
    assert gpu["windows"] == ref["windows"]
    assert np.array_equal(gpu["outcome"], ref["outcome"]) and np.array_equal(gpu["done"], ref["done"])
    assert gpu["stats"] == ref["stats"] and gpu["testcomplete"] == ref["testcomplete"]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("case", ["drop", "reject"])
def test_cfg3_splitbrain_blocked_full(hip, oracle, case, n=10_000):
    """drop / reject at 10k on HIP (3.3k /32 rules on each of 3.3k region-A nodes; region B's
    probes of region A wait out one-minute timeouts, so the run covers ~56 simulated hours in
    ~5e4 windows): the truth table of main.go:50-58 probe by probe; at 2k, bit-exact vs the oracle."""
    gpu = _splitbrain_descriptor(hip, n, case)
    _check_splitbrain_truth(gpu, n, case)
    m = 2000
    g2, o2 = _splitbrain_descriptor(hip, m, case), _splitbrain_descriptor(oracle, m, case)
    _check_splitbrain_truth(g2, m, case)
    assert g2["windows"] == o2["windows"] and g2["stats"] == o2["stats"]
    assert np.array_equal(g2["outcome"], o2["outcome"]) and np.array_equal(g2["done"], o2["done"])


def test_cfg3_all_at_once_stress(hip, oracle, n=10_000, chunk=1000):
    """STRESS TEST, not the reference's traffic: SURVEY.md 8(d)'s synthetic config 3 - every node
    fires all its probes at one instant (the reference plan sends one GET at a time: see
    test_cfg3_splitbrain_full) through 1.1e7 /32 rules, policy flips and 10 ms links, so the netem
    queue limit tail-drops all but 1000 per sender."""
    subset = np.unique(np.array([0, 1, 2, 3, 4, 5, n // 3, 2 * n // 3, n - 3, n - 2, n - 1, 1500, 4001], np.uint32))
    in_subset = np.zeros(n, bool)
    in_subset[subset] = True
    tot = dict(queued=0, delivered=0, probes=0)

    def check(w, phase, policy, src, dst, st, d):
        _assert_inbox_order(d)
        if len(d["dst"]):
            assert np.all(d["t_deliver"] == w * 10 * MS)
        tot["delivered"] += len(d["dst"])
        if len(st):
            tot["probes"] += len(st)
            assert np.array_equal(st, _splitbrain_want(n, phase, policy, src, dst)), f"window {w}: statuses"
            tot["queued"] += int(np.count_nonzero(st == A.ST_QUEUED))
        return st[in_subset[src]], _filter(d, in_subset[d["src"]])

    gpu = _run_splitbrain(hip, n, np.arange(n), chunk, on_window=check)
    assert tot["probes"] == 3 * n * n
    assert tot["delivered"] == tot["queued"] == 3 * n * A.NETEM_LIMIT
    # the oracle replays the subset's senders in the same windows: statuses and deliveries (all
    # seven fields, t_deliver included) bit-exact per window
    ref = _run_splitbrain(oracle, n, subset, chunk)
    assert len(ref) == len(gpu)
    for w, ((gs, gd), (_, _, os_, od)) in enumerate(zip(gpu, ref)):
        assert np.array_equal(gs, os_), f"window {w}: statuses"
        S.assert_same(gd, od, f"window {w}")


# ---- config 4: the 100k-instance storm, replayed whole ------------------------------------------

def test_cfg4_storm_full(hip, oracle, n=100_000, rounds=8):
    kw = dict(max_records=1 << 23, data_prefix_len=12)
    a = S.run_storm(hip, n_inst=n, rounds=rounds, cfg_kw=kw)
    b = S.run_storm(oracle, n_inst=n, rounds=rounds, cfg_kw=kw)
    S.assert_same(a, b)
    assert sum(len(x["deliv"]["dst"]) for x in a[:-1]) > n * 8


def _bench_storm_cfg(n: int, k: int, world: int) -> dict:
    """bench.sim_config's context for shard k of `world` (the test proves the
    bench's own peer blocks, 1.25 x N x 8 / S^2 + 4096 records, not a roomier capacity)."""
    import argparse
    import dataclasses
    import bench
    a = argparse.Namespace(instances=n, fanout=8, seed=4, max_records=1 << 23, tcp=False, tcp_acks=False)
    c = dataclasses.asdict(bench.sim_config(a, k, world))
    for f in ("n_instances", "seed", "device"):
        c.pop(f)
    return c


def test_cfg4_storm_sharded_full(hip, n=100_000, rounds=10, world=8):
    """config 4 as bench.py shards it: the 100k storm over 8 HIP contexts (one thread each, one GPU,
    the exchange and the barrier's all-reduce through the transport), each built by bench.sim_config
    (its exchange blocks of 19.7k records at 8 shards), equals the single-context run bit for bit
    (which test_cfg4_storm_full pins to the oracle), with no ECAPACITY over the rounds."""
    kw = dict(max_records=1 << 23, data_prefix_len=12)
    single = S.run_storm(hip, n_inst=n, rounds=rounds, cfg_kw=kw)
    assert _bench_storm_cfg(n, 0, world)["exchange_cap"] == int(1.25 * n * 8 / world ** 2) + 4096
    outs = S.sharded_threads(world, lambda k, tr: S.run_storm(
        hip, n_inst=n, rounds=rounds, cfg_kw=_bench_storm_cfg(n, k, world),
        setup=lambda sim: sim.set_transport(tr)), device=True)
    S.assert_storm_sharded(outs, single, world, n)
    assert sum(len(x["deliv"]["dst"]) for x in single[:-1]) > n * 8
