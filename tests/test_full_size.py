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
    tot = dict(sent=0, queued=0, lost=0, delivered=0)
    seen = []

    def check(r, st, d):
        _assert_inbox_order(d)
        tot["delivered"] += len(d["dst"])
        if len(st):
            assert len(st) == n * (n - 1)
            tot["sent"] += len(st)
            tot["queued"] += int(np.count_nonzero(st == A.ST_QUEUED))
            tot["lost"] += int(np.count_nonzero(st == A.ST_LOST))
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
    assert tot["queued"] + tot["lost"] == tot["sent"] and tot["delivered"] == tot["queued"]
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
    sends one all-pairs round of 64 B probes, `chunk` senders per window."""
    sim = Simulator(SimConfig(n_instances=n, seed=3, max_msgs_per_window=1 << 24, max_records=1 << 25),
                    binding=binding)
    sim.set_shapes(np.arange(n), [make_shape(latency_ns=10 * MS)] * n)
    region = np.arange(n) % 3
    a_ids, b_ids = np.nonzero(region == 0)[0], np.nonzero(region == 1)[0]
    out, t0, w = [], 0, 0
    for phase, action in enumerate((A.FILTER_DROP, A.FILTER_REJECT, A.FILTER_ACCEPT)):
        rules = _rule_block(sim, b_ids, action)
        for g in a_ids:
            sim._check(sim.lib.add_rules(sim._ctx, int(g), rules, len(b_ids)))
        print(f"  splitbrain {binding.name} phase {phase}: rules installed", flush=True)
        for c0 in range(0, len(senders), chunk):
            snd = senders[c0:c0 + chunk].astype(np.uint32)
            src = np.repeat(snd, n - 1)
            dst = (src + np.tile(np.arange(1, n, dtype=np.uint32), len(snd))) % np.uint32(n)
            seq = np.uint32(phase * n) + dst
            sim.enqueue(src, dst, seq, np.full(len(src), 64, np.uint32), np.full(len(src), t0, np.int64))
            t0 += 10 * MS
            sim.advance(t0)
            st, d = sim.status(), sim.deliveries()
            out.append((src, dst, st, d) if on_window is None else on_window(w, phase, src, dst, st, d))
            w += 1
    t0 += 10 * MS
    sim.advance(t0)
    d = sim.deliveries()
    e = np.zeros(0, np.uint32)
    out.append((e, e, np.zeros(0, np.uint8), d) if on_window is None else on_window(w, 3, e, e, np.zeros(0, np.uint8), d))
    sim.close()
    return out


def test_cfg3_splitbrain_full(hip, oracle, n=10_000, chunk=1000):
    region = np.arange(n) % 3
    subset = np.unique(np.array([0, 1, 2, 3, 4, 5, n // 3, 2 * n // 3, n - 3, n - 2, n - 1], np.uint32))
    in_subset = np.zeros(n, bool)
    in_subset[subset] = True
    expect_blocked = {0: A.ST_DROPPED, 1: A.ST_REJECTED, 2: None}
    tot = dict(queued=0, delivered=0, probes=0)

    def check(w, phase, src, dst, st, d):
        _assert_inbox_order(d)
        if len(d["dst"]):
            assert np.all(d["t_deliver"] == w * 10 * MS)
        tot["delivered"] += len(d["dst"])
        if len(st):
            tot["probes"] += len(st)
            blocked = (region[src] == 0) & (region[dst] == 1)          # splitbrain/main.go:50-58
            want = np.full(len(st), A.ST_QUEUED, np.uint8)
            if expect_blocked[phase] is not None:
                want[blocked] = expect_blocked[phase]
            assert np.array_equal(st, want), f"window {w}: routing truth table"
            tot["queued"] += int(np.count_nonzero(st == A.ST_QUEUED))
        ks = in_subset[src]
        return st[ks], _filter(d, in_subset[d["src"]])

    gpu = _run_splitbrain(hip, n, np.arange(n), chunk, on_window=check)
    per_phase = -(-n // chunk)
    assert tot["probes"] == 3 * n * (n - 1)
    assert tot["delivered"] == tot["queued"]
    ref = _run_splitbrain(oracle, n, subset, len(subset))
    # the oracle sends every subset sender in one window per phase; gather the GPU's per phase
    gpu_by_phase = [[], [], []]
    for i, x in enumerate(gpu[:-1]):
        gpu_by_phase[i // per_phase].append(x)
    for phase in range(3):
        gs = np.concatenate([x[0] for x in gpu_by_phase[phase]])
        assert np.array_equal(gs, ref[phase][2]), f"phase {phase}: statuses"
    # deliveries: the GPU delivers window w's probes in window w+1; compare per phase, sorted
    def cat(ds):
        keys = ("t_deliver", "src", "dst", "seq", "size", "flags", "corrupt_off")
        return {k: np.concatenate([x[k] for x in ds]) for k in keys}
    gd = cat([gpu[i][1] for i in range(1, len(gpu))])
    od = cat([ref[i][3] for i in range(1, len(ref))])
    for dd in (gd, od):
        o = np.lexsort((dd["seq"], dd["dst"], dd["src"]))
        for k in dd:
            dd[k] = dd[k][o]
    for k in ("src", "dst", "seq", "size", "flags", "corrupt_off"):
        assert np.array_equal(gd[k], od[k]), k


# ---- config 4: the 100k-instance storm, replayed whole ------------------------------------------

def test_cfg4_storm_full(hip, oracle, n=100_000, rounds=8):
    kw = dict(max_records=1 << 23, data_prefix_len=12)
    a = S.run_storm(hip, n_inst=n, rounds=rounds, cfg_kw=kw)
    b = S.run_storm(oracle, n_inst=n, rounds=rounds, cfg_kw=kw)
    S.assert_same(a, b)
    assert sum(len(x["deliv"]["dst"]) for x in a[:-1]) > n * 8
