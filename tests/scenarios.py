"""Seeded scenario drivers shared by the parity tests: the same calls are made on the HIP simulator
and on the CPU oracle, and every observable (statuses, deliveries, inbox offsets, stats, sync
sequence numbers and barrier releases) is collected for bit-exact comparison."""
from __future__ import annotations

import numpy as np

from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator, make_rule, make_shape, int_to_ip

MS = 1_000_000


STRUCTURAL_STATS = ("windows", "inflight", "tb_items", "extracted", "inserted")


def parity_stats(sim):
    """Counters that are part of the semantics (the rest describe implementation structure)."""
    return {k: v for k, v in sim.stats().items() if k not in STRUCTURAL_STATS}


def random_shape(rng, *, allow_bw=True):
    lat = int(rng.choice([0, 1_000, 999_999, 5 * MS, 20 * MS, 100 * MS]))
    jit = int(rng.choice([0, 0, 3 * MS, 10 * MS, 150 * MS]))
    bw = int(rng.choice([0, 0, 1 << 20, 10_000_000, 800_000])) if allow_bw else 0
    loss = float(rng.choice([0, 0, 1.0, 20.0, 100.0]))
    dup = float(rng.choice([0, 0, 5.0, 50.0]))
    cor = float(rng.choice([0, 0, 10.0]))
    reo = float(rng.choice([0, 0, 25.0]))
    return make_shape(latency_ns=lat, jitter_ns=jit, bandwidth_bps=bw, loss=loss, duplicate=dup,
                      corrupt=cor, reorder=reo)


def run_random(binding, seed: int, n_inst: int = 24, windows: int = 6, msgs_per_window: int = 300,
               window_ns: int = 40 * MS, rules: bool = True, cfg_kw=None, restart=None):
    """restart(w, sim) -> sim, after window w (checkpoint / resume tests)."""
    rng = np.random.default_rng(seed)
    cfg = SimConfig(n_instances=n_inst, seed=1000 + seed, **(cfg_kw or {}))
    sim = Simulator(cfg, binding=binding)
    out = []
    seqc = np.zeros(n_inst, np.int64)
    for g in range(n_inst):
        sim.set_shape(g, random_shape(rng))
        if rng.random() < 0.3:
            sim.set_policy(g, A.POLICY_ALLOW_ALL)
    if rules:
        for g in rng.choice(n_inst, size=n_inst // 3, replace=False):
            rl = []
            for _ in range(int(rng.integers(1, 6))):
                tgt = int(rng.integers(0, n_inst))
                ip = sim.get_ip(tgt)
                plen = int(rng.choice([32, 32, 30, 24, 16, 0]))
                mask = (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF if plen else 0
                f = int(rng.choice([A.FILTER_DROP, A.FILTER_REJECT, A.FILTER_ACCEPT]))
                rl.append(make_rule(f"{int_to_ip(ip & mask)}/{plen}", f))
            sim.add_rules(int(g), rl)
    t0 = 0
    for w in range(windows):
        if w == windows // 2:  # mid-run reconfiguration: shapes, an IP change, a disabled link
            for g in rng.choice(n_inst, size=4, replace=False):
                sim.set_shape(int(g), random_shape(rng))
            g = int(rng.integers(0, n_inst))
            sim.set_enabled(g, True, ip=sim.get_ip(g) + 1000)
            sim.set_enabled(int((g + 3) % n_inst), False)
        n = msgs_per_window
        src = rng.integers(0, n_inst, n)
        dst = rng.integers(0, n_inst, n)
        dst[rng.random(n) < 0.03] = A.DST_EXTERNAL
        loc = rng.random(n) < 0.02
        dst[loc] = src[loc]
        seq = np.zeros(n, np.int64)
        for i in range(n):
            seq[i] = seqc[src[i]]
            seqc[src[i]] += 1
        size = rng.choice([0, 1, 64, 1024, 4096, 65536], n)
        t = t0 + np.sort(rng.integers(0, window_ns, n))
        if rng.random() < 0.5:  # ties in send time
            t[: n // 4] = t0
        sim.enqueue(src, dst, seq, size, t)
        t0 += window_ns
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
        if restart is not None:
            sim = restart(w, sim)
    # drain
    for w in range(3):
        t0 += 10 * window_ns
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def run_limit_switch(binding, seed: int, n_inst: int = 32, windows: int = 8, window_ns: int = 10 * MS):
    """Bandwidth limits switched on and off mid-run with copies in flight. A context whose senders
    have never been limited skips the token-bucket stage (Dev::ever_limited): windows 0-1 run
    without any limit, windows 2-3 limit a quarter of the senders (their copies then sit in the wheel
    and in A), and from window 4 on the limits are gone again while those copies are still in flight
    (the stage must keep running for them)."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, seed=3000 + seed), binding=binding)
    base = [make_shape(latency_ns=int(rng.integers(5, 36)) * MS, jitter_ns=int(rng.choice([0, 2 * MS])),
                       loss=float(rng.choice([0.0, 5.0]))) for _ in range(n_inst)]
    for g in range(n_inst):
        sim.set_shape(g, base[g])
    limited = rng.choice(n_inst, size=n_inst // 4, replace=False)
    out, seqc, t0 = [], np.zeros(n_inst, np.int64), 0
    for w in range(windows):
        if w in (2, 4):
            for g in limited:
                sh = base[int(g)]
                sim.set_shape(int(g), make_shape(latency_ns=sh.latency_ns, jitter_ns=sh.jitter_ns,
                                                 loss=sh.loss, bandwidth_bps=800_000 if w == 2 else 0))
        n = 200
        src = rng.integers(0, n_inst, n)
        dst = (src + rng.integers(1, n_inst, n)) % n_inst
        seq = np.zeros(n, np.int64)
        for i in range(n):
            seq[i] = seqc[src[i]]
            seqc[src[i]] += 1
        t = t0 + np.sort(rng.integers(0, window_ns, n))
        sim.enqueue(src, dst, seq, rng.choice([64, 1000, 4000], n), t)
        t0 += window_ns
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    for w in range(4):
        t0 += 20 * window_ns
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def run_heavy(binding, seed: int, n_inst: int = 64):
    """One sender with a long backlog (token-bucket segment > LDS tile) and one receiver with a large
    inbox (delivery segment > LDS tile): exercises the merge-path large-segment paths. With more
    instances than one fused bucket holds, the heavy bucket takes the global form next to normal
    buckets (the segment boundary between them is written by the oversized one)."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, seed=seed), binding=binding)
    for g in range(n_inst):
        sim.set_shape(g, make_shape(latency_ns=10 * MS, jitter_ns=int(rng.choice([0, 5 * MS])),
                                    bandwidth_bps=int(rng.choice([0, 100_000_000])), duplicate=2.0))
    out = []
    t0 = 0
    for w in range(3):
        n = 9000
        src = np.where(rng.random(n) < 0.6, 0, rng.integers(1, n_inst, n))
        dst = np.where(rng.random(n) < 0.6, 5, rng.integers(0, n_inst, n))
        dst[dst == src] = (dst[dst == src] + 1) % n_inst
        seq = np.arange(n) + w * n
        size = rng.choice([100, 1500], n)
        t = t0 + np.sort(rng.integers(0, 20 * MS, n))
        t[:500] = t0
        sim.enqueue(src, dst, seq, size, t)
        t0 += 20 * MS
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    t0 += 5_000 * MS
    sim.advance(t0)
    out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def run_many_large(binding, seed: int, n_inst: int = 64, n: int = 40_000):
    """Several long backlogs and large inboxes in the same window (k_rest's task-parallel path: every
    chunk of every large segment sorted by its own task, every element ranked by its own thread):
    four heavy senders (~8k copies each: four chunks) and two heavy receivers (~16k deliveries:
    eight chunks, so the rank search covers more than one group of four chunks)."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, seed=seed), binding=binding)
    for g in range(n_inst):
        sim.set_shape(g, make_shape(latency_ns=int(rng.choice([0, 2 * MS])), jitter_ns=int(rng.choice([0, 3 * MS])),
                                    bandwidth_bps=int(rng.choice([0, 0, 0, 1_000_000_000])), duplicate=1.0))
    out = []
    t0 = 0
    for w in range(3):
        src = np.where(rng.random(n) < 0.8, rng.integers(0, 4, n), rng.integers(4, n_inst, n))
        dst = np.where(rng.random(n) < 0.8, rng.integers(5, 7, n), rng.integers(0, n_inst, n))
        dst[dst == src] = (dst[dst == src] + 9) % n_inst
        seq = np.arange(n) + w * n
        t = t0 + rng.integers(0, 20 * MS, n)
        t[: n // 10] = t0 + 7 * MS  # ties on the primary key, broken by (src, seq, clone)
        sim.enqueue(src, dst, seq, rng.choice([64, 1500], n), t)
        t0 += 20 * MS
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    t0 += 200 * MS
    sim.advance(t0)
    out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def run_whole_inbox(binding, seed: int, n_inst: int = 4000, counters=None):
    """Long inboxes of up to 10240 deliveries are sorted by one workgroup in LDS when their keys
    pack into 32 bits (whole_sort); the others go back to the chunk and rank tasks.
    Window 0: two ~5k inboxes whose deliveries share one arrival time (duplicates: clone ties) next
    to a 12k inbox (tasks); window 1: arrivals spread over 1 us (packed key of ~25 bits); window 2:
    90 % of arrivals at one instant, the rest over 60 us (a bucket over its mate bound: tasks);
    window 3: arrivals over 20 ms (key wider than 32 bits: tasks). counters (HIP): the kernel
    counters after each window."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, seed=seed, max_msgs_per_window=1 << 16), binding=binding)
    for g in range(n_inst):
        sim.set_shape(g, make_shape(latency_ns=MS, duplicate=30.0))
    snd = np.arange(3, n_inst, dtype=np.int64)
    out = []
    t0 = 0
    sent = np.zeros(n_inst, np.int64)

    def window(src, dst, t, span):
        nonlocal t0
        # per-sender sequence numbers (one (src, seq) per message): narrow seq ranges per inbox
        order = np.argsort(src, kind="stable")
        s_sorted = src[order]
        first = np.r_[0, np.flatnonzero(np.diff(s_sorted)) + 1]
        occ = np.empty(len(src), np.int64)
        occ[order] = np.arange(len(src)) - np.repeat(first, np.diff(np.r_[first, len(src)]))
        seq = sent[src] + occ
        np.add.at(sent, src, 1)
        sim.enqueue(src, dst, seq, rng.choice([64, 1500], len(src)), t)
        t0 += span
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
        if counters is not None:
            counters.append(sim.kernel_counters())

    # the window's sends: every sender to 0 and 1; 12k to 2 (three per sender)
    src = np.concatenate([snd, snd, np.repeat(snd, 3)])
    dst = np.concatenate([np.zeros_like(snd), np.ones_like(snd), np.full(3 * len(snd), 2)])
    window(src, dst, np.full(len(src), t0), 5 * MS)
    src = rng.permutation(np.concatenate([snd, snd[::2]]))
    window(src, np.zeros_like(src), t0 + rng.integers(0, 1000, len(src)), 5 * MS)
    src = rng.permutation(snd)
    t = np.where(rng.random(len(src)) < 0.9, t0, t0 + rng.integers(0, 60_000, len(src)))
    window(src, np.ones_like(src), t, 5 * MS)
    window(src, np.zeros_like(src), t0 + rng.integers(0, 20 * MS, len(src)), 25 * MS)
    t0 += 100 * MS
    sim.advance(t0)
    out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def run_bucket_overflow(binding, seed: int, n_inst: int = 4096, per_sender: int = 80, windows: int = 3,
                        counters=None):
    """More items per fused bucket than it holds (kBktCap) on both group-bys: 4096 instances (24
    keys per bucket), every sender 80 messages a window to random receivers, every sender
    bandwidth-limited - ~1900 items per bucket, so most buckets take the global form and their keys
    go to k_rest in spans of several keys (kMediumSpans). counters (HIP): kernel counters per window."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, seed=seed, max_msgs_per_window=1 << 20, max_records=1 << 21),
                    binding=binding)
    for g in range(n_inst):
        sim.set_shape(g, make_shape(latency_ns=int(rng.choice([1, 2, 3])) * MS, jitter_ns=int(rng.choice([0, 2 * MS])),
                                    bandwidth_bps=int(rng.choice([50_000_000, 400_000_000])), duplicate=5.0,
                                    loss=1.0))
    out = []
    t0 = 0
    for w in range(windows):
        n = n_inst * per_sender
        src = np.repeat(np.arange(n_inst), per_sender)
        dst = rng.integers(0, n_inst, n)
        dst[dst == src] = (dst[dst == src] + 1) % n_inst
        seq = np.tile(np.arange(per_sender), n_inst) + w * per_sender
        t = t0 + rng.integers(0, 4 * MS, n)
        sim.enqueue(src, dst, seq, rng.choice([100, 1000], n), t)
        t0 += 4 * MS
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
        if counters is not None:
            counters.append(sim.kernel_counters())
    t0 += 50 * MS
    sim.advance(t0)
    out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def run_rest_hint(binding, seed: int, n_inst: int = 512, pattern=(1, 1, 0, 1, 0, 0, 1, 1), heavy: int = 4,
                  burst: int = 700, counters=None):
    """Token-bucket windows that do and do not leave long senders to k_rest<TB>, in runs: a window
    whose `pattern` entry is 1 has `heavy` bandwidth-limited senders send `burst` messages each (a key
    run past kBktRankMax in their bucket), every other sender 3. With a sync after every window, a
    busy window after a quiet one runs k_rest<TB> inside the window end's first launch
    (k_rest_local_hist, busy roles by ticket), one after a busy one in a launch of its own (the host
    hint), and a quiet one after a busy one resets the hint - every form against the oracle."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, seed=seed, max_msgs_per_window=1 << 16, max_records=1 << 19),
                    binding=binding)
    # no duplicates and heavy senders that drain within the window: a burst stays under netem's
    # 1000-packet limit, so the queue-limit lane (k_shape_seq) never takes it from the token bucket
    hv = rng.choice(n_inst, heavy, replace=False)
    for g in range(n_inst):
        bw = 4_000_000_000 if g in hv else int(rng.choice([20_000_000, 200_000_000]))
        sim.set_shape(g, make_shape(latency_ns=int(rng.choice([0, 1])) * MS, jitter_ns=int(rng.choice([0, MS // 2])),
                                    bandwidth_bps=bw, loss=1.0))
    out = []
    t0 = 0
    for w, busy in enumerate(pattern):
        per = np.full(n_inst, 3)
        if busy:
            per[hv] = burst
        src = np.repeat(np.arange(n_inst), per)
        n = len(src)
        dst = rng.integers(0, n_inst, n)
        dst[dst == src] = (dst[dst == src] + 1) % n_inst
        seq = np.concatenate([np.arange(k) for k in per]) + w * burst
        t = t0 + rng.integers(0, 2 * MS, n)
        sim.enqueue(src, dst, seq, rng.choice([200, 1200], n), t)
        t0 += 4 * MS
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
        if counters is not None:
            counters.append(sim.kernel_counters())
    t0 += 200 * MS
    sim.advance(t0)
    out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def run_burst(binding, seed: int, n_inst: int = 10, windows: int = 5, per_sender: int = 1400,
              window_ns: int = 4 * MS, restart=None):
    """Senders whose bursts overrun netem's 1000-packet queue under every kind of
    shape: jitter, a saturated token bucket, duplicates + loss, reorder + corrupt, correlated
    duplicates, zero delay; late sends (t_send before the window start, at the reaction horizon);
    queues that stay full across windows and then drain."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, seed=2000 + seed, max_msgs_per_window=1 << 16,
                              max_records=1 << 18), binding=binding)
    shapes = [
        make_shape(latency_ns=10 * MS, jitter_ns=3 * MS),
        make_shape(latency_ns=2 * MS, bandwidth_bps=100_000_000),
        make_shape(latency_ns=5 * MS, duplicate=30.0, loss=5.0),
        make_shape(latency_ns=1 * MS, jitter_ns=1 * MS, reorder=20.0, corrupt=10.0, bandwidth_bps=400_000_000),
        make_shape(latency_ns=8 * MS, duplicate=20.0, duplicate_corr=50.0, reorder=10.0, reorder_corr=30.0),
        make_shape(),
    ]
    for g, shp in enumerate(shapes):
        sim.set_shape(g, shp)
    heavy = np.arange(len(shapes))
    seqc = np.zeros(n_inst, np.int64)
    out, t0 = [], 0
    for w in range(windows + 4):
        src, ts = [], []
        if w < windows:
            for g in heavy:
                k = per_sender if (w + g) % 3 else per_sender // 4
                t = t0 + np.sort(rng.integers(0, window_ns // 2, k))
                t[: k // 4] = t0
                src.append(np.full(k, g)); ts.append(t)
            light = rng.integers(len(shapes), n_inst, 50)
            src.append(light); ts.append(t0 + rng.integers(0, window_ns, 50))
            if w > 0:   # reactions at the horizon: sent before this window's start
                late = rng.integers(0, len(shapes), 120)
                src.append(late); ts.append(t0 - rng.integers(1, window_ns, 120))
        src = np.concatenate(src) if src else np.zeros(0, np.int64)
        ts = np.concatenate(ts) if ts else np.zeros(0, np.int64)
        n = len(src)
        dst = (src + rng.integers(1, n_inst, n)) % n_inst
        seq = np.zeros(n, np.int64)
        for i in range(n):
            seq[i] = seqc[src[i]]
            seqc[src[i]] += 1
        size = rng.choice([64, 1000, 1500], n)
        if n:
            sim.enqueue(src, dst, seq, size, ts)
        t0 += window_ns if w < windows else 60 * MS
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
        if restart is not None:
            sim = restart(w, sim)
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def run_wide(binding, seed: int, n_inst: int = 16, windows: int = 5, window_ns: int = 8 * MS, counters=None):
    """The queue-limit lane's whole-sender closed form (k_shape_seq_wide) and each of
    its ways back to the chunked lane: senders of <= 1024 deferred messages whose copies all outlive
    the window's last enqueue (40-60 ms of netem against a 1 ms send spread) fill their 1000-packet
    queues over a few windows; one sender repeats (t_send, seq) pairs (the exact sort), one spreads
    its sends over more than 2^22 ns (the unpacked sort), one sends more than 1024 messages, one has
    a token bucket, one a delay shorter than its send spread (the closed form does not hold), and
    late sends at the horizon come in between."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, seed=3000 + seed, max_msgs_per_window=1 << 16,
                              max_records=1 << 18), binding=binding)
    big = make_shape(latency_ns=50 * MS, jitter_ns=10 * MS, duplicate=10.0, loss=2.0, corrupt=1.0)
    shapes = [big, big, big, big,                                  # closed form (packed sort)
              make_shape(latency_ns=50 * MS, jitter_ns=10 * MS),   # repeated (t_send, seq): exact sort
              make_shape(latency_ns=80 * MS),                      # sends spread over 6 ms: unpacked sort
              make_shape(latency_ns=50 * MS, jitter_ns=5 * MS),    # > 1024 messages: chunked lane
              make_shape(latency_ns=50 * MS, bandwidth_bps=1_000_000_000),   # token bucket: chunked lane
              make_shape(latency_ns=200 * 1000, jitter_ns=100 * 1000)]       # short delay: no closed form
    for g, shp in enumerate(shapes):
        sim.set_shape(g, shp)
    seqc = np.zeros(n_inst, np.int64)

    def seqs_for(src):
        q = np.zeros(len(src), np.int64)
        for i, g in enumerate(src):
            q[i] = seqc[g]
            seqc[g] += 1
        return q

    out, t0 = [], 0
    for w in range(windows + 40):
        src, ts, seqs = [], [], []
        if w < windows:
            for g in range(len(shapes)):
                k = 1100 if g == 6 else int(rng.integers(600, 1000))
                spread = 6 * MS if g == 5 else MS
                t = t0 + rng.integers(0, spread, k)
                q = seqc[g] + np.arange(k)
                seqc[g] += k
                if g == 4:  # every tenth message repeats its predecessor's (t_send, seq)
                    m = len(t[1::10])
                    t[1::10] = t[0:-1:10][:m]
                    q[1::10] = q[0:-1:10][:m]
                src.append(np.full(k, g)); ts.append(t); seqs.append(q)
            light = rng.integers(len(shapes), n_inst, 40)
            src.append(light); ts.append(t0 + rng.integers(0, window_ns, 40)); seqs.append(seqs_for(light))
            if w > 0:   # reactions at the horizon
                late = rng.integers(0, len(shapes), 60)
                src.append(late); ts.append(t0 - rng.integers(1, window_ns, 60)); seqs.append(seqs_for(late))
        src = np.concatenate(src) if src else np.zeros(0, np.int64)
        ts = np.concatenate(ts) if ts else np.zeros(0, np.int64)
        seq = np.concatenate(seqs) if seqs else np.zeros(0, np.int64)
        n = len(src)
        dst = (src + rng.integers(1, n_inst, n)) % n_inst
        # a repeated (t_send, seq) pair draws the same netem fate; another receiver keeps the two
        # deliveries apart (at one receiver their inbox order would be a tie of every key)
        for i in range(1, n):
            if src[i] == 4 and src[i - 1] == 4 and ts[i] == ts[i - 1] and seq[i] == seq[i - 1] and dst[i] == dst[i - 1]:
                dst[i] = (dst[i] + 1) % n_inst if (dst[i] + 1) % n_inst != 4 else (dst[i] + 2) % n_inst
        size = rng.choice([64, 1000, 1500], n)
        if n:
            sim.enqueue(src, dst, seq, size, ts)
        t0 += window_ns if w < windows else 5 * MS
        sim.advance(t0)
        out.append(dict(status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
    out.append(dict(stats=parity_stats(sim)))
    if counters is not None:  # HIP only: which lane decided the deferred messages
        counters.update(sim.kernel_counters())
    sim.close()
    return out


def run_sync(binding, seed: int, restart=None):
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=8, seed=seed, max_states=64), binding=binding)
    res = []
    waiters = []
    t = 0
    for b in range(6):
        n = int(rng.integers(1, 3000))
        states = rng.integers(0, 5, n)
        inst = rng.integers(0, 5000, n)
        ts = t + rng.integers(0, 1000, n)
        ts[rng.random(n) < 0.3] = t  # ties -> broken by instance
        seq = sim.signal(states, inst, ts)
        res.append(("seq", seq.copy()))
        for _ in range(3):
            waiters.append(sim.barrier(int(rng.integers(0, 5)), int(rng.integers(0, 4000)), int(t + rng.integers(0, 2000))))
        res.append(("rel", [sim.poll(w) for w in waiters]))
        res.append(("cnt", [sim.count(s) for s in range(6)]))
        t += 1000
        if restart is not None:
            sim = restart(b, sim)
    sim.close()
    return res


def run_storm(binding, n_inst=2000, rounds=12, fanout=8, seed=4, cfg_kw=None, setup=None, restart=None,
              t_now=False, size_of=None, between=None):
    """The storm step of bench.py. Sharded (cfg_kw shard_id / n_shards, setup attaching a
    transport): the same calls on every shard, each collective; a shard reports its own senders'
    statuses and its own receivers' deliveries. t_now: rounds start at the device clock
    (TGSIM_T_NOW, bench.py's loop: the library may generate the next round speculatively);
    size_of(r): the round's message size; between(r, sim): calls made before round r's generation."""
    sim = Simulator(SimConfig(n_instances=n_inst, seed=seed, **(cfg_kw or {})), binding=binding)
    if setup is not None:
        setup(sim)
    rng = np.random.default_rng(seed)
    for g in range(n_inst):
        sim.set_shape(g, make_shape(latency_ns=int(rng.integers(20, 101)) * MS, jitter_ns=5 * MS,
                                    bandwidth_bps=10_000_000, loss=0.5))
    out = []
    for r in range(rounds):
        if between is not None:
            between(r, sim)
        t0 = A.T_NOW if t_now else sim.now
        sim.gen_storm_round(r, t0, fanout, size_of(r) if size_of else 1024, 10 * MS, r)
        w = sim.barrier(r, n_inst, t0)
        sim.advance_to_barrier(w, 1 * MS)
        out.append(dict(now=sim.now, status=sim.status(), deliv=sim.deliveries(), inbox=sim.inbox_offsets()))
        if restart is not None:
            sim = restart(r, sim)
    out.append(dict(stats=parity_stats(sim)))
    sim.close()
    return out


def assert_same(a, b, path="out"):
    if isinstance(a, dict):
        assert set(a) == set(b), f"{path}: keys {set(a)} vs {set(b)}"
        for k in a:
            assert_same(a[k], b[k], f"{path}.{k}")
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b), f"{path}: len {len(a)} vs {len(b)}"
        for i, (x, y) in enumerate(zip(a, b)):
            assert_same(x, y, f"{path}[{i}]")
    elif isinstance(a, np.ndarray):
        assert a.shape == b.shape, f"{path}: shape {a.shape} vs {b.shape}"
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0][:10]
            raise AssertionError(f"{path}: mismatch at {bad}: {a[bad]} vs {b[bad]}")
    else:
        assert a == b, f"{path}: {a} vs {b}"


# ---- sharded runs: contiguous instance ranges per shard, one exchange per window --

def shard_range(n, k, s):
    return (k * n) // s, ((k + 1) * n) // s


def run_random_sharded(make_sim, exchange, world: int, seed: int, n_inst: int = 24, windows: int = 6,
                       msgs_per_window: int = 300, window_ns: int = 40 * MS, local=None, exchange_cap: int = 4096):
    """run_random's workload split over `world` shards. make_sim(cfg) -> Simulator of one shard;
    exchange(sims) moves every shard's send blocks to the peers' receive blocks (an all-to-all)
    between advance_begin and advance_end; exchange=None: the shards carry a transport and each
    calls tgsim_advance (collective: one shard per thread or process, local=[k]).
    local: the shard ids this process runs (default all; one per rank in a multi-process run).
    Returns (per-shard observables in run_random's structure, per-window global sender arrays)."""
    rng = np.random.default_rng(seed)
    local = list(range(world)) if local is None else list(local)
    sims = [make_sim(SimConfig(n_instances=n_inst, seed=1000 + seed, shard_id=k, n_shards=world,
                               exchange_cap=exchange_cap)) for k in local]
    outs = [[] for _ in local]
    srcs = []
    seqc = np.zeros(n_inst, np.int64)
    for g in range(n_inst):
        shp = random_shape(rng)
        allow = rng.random() < 0.3
        for s in sims:   # configuration calls go to every shard (replicated tables, owner keeps state)
            s.set_shape(g, shp)
            if allow:
                s.set_policy(g, A.POLICY_ALLOW_ALL)
    for g in rng.choice(n_inst, size=n_inst // 3, replace=False):
        rl = []
        for _ in range(int(rng.integers(1, 6))):
            tgt = int(rng.integers(0, n_inst))
            ip = sims[0].get_ip(tgt)
            plen = int(rng.choice([32, 32, 30, 24, 16, 0]))
            mask = (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF if plen else 0
            f = int(rng.choice([A.FILTER_DROP, A.FILTER_REJECT, A.FILTER_ACCEPT]))
            rl.append(make_rule(f"{int_to_ip(ip & mask)}/{plen}", f))
        for s in sims:
            s.add_rules(int(g), rl)
    t0 = 0

    def window(t_end):
        if exchange is None:
            for s in sims:
                s.advance(t_end)
        else:
            for s in sims:
                s.advance_begin(t_end)
            exchange(sims)
            for s in sims:
                s.advance_end()
        for i, s in enumerate(sims):
            outs[i].append(dict(status=s.status(), deliv=s.deliveries(), inbox=s.inbox_offsets()))

    for w in range(windows):
        if w == windows // 2:
            for g in rng.choice(n_inst, size=4, replace=False):
                shp = random_shape(rng)
                for s in sims:
                    s.set_shape(int(g), shp)
            g = int(rng.integers(0, n_inst))
            ip = sims[0].get_ip(g) + 1000
            for s in sims:
                s.set_enabled(g, True, ip=ip)
                s.set_enabled(int((g + 3) % n_inst), False)
        n = msgs_per_window
        src = rng.integers(0, n_inst, n)
        dst = rng.integers(0, n_inst, n)
        dst[rng.random(n) < 0.03] = A.DST_EXTERNAL
        loc = rng.random(n) < 0.02
        dst[loc] = src[loc]
        seq = np.zeros(n, np.int64)
        for i in range(n):
            seq[i] = seqc[src[i]]
            seqc[src[i]] += 1
        size = rng.choice([0, 1, 64, 1024, 4096, 65536], n)
        t = t0 + np.sort(rng.integers(0, window_ns, n))
        if rng.random() < 0.5:
            t[: n // 4] = t0
        for k, s in zip(local, sims):
            lo, hi = shard_range(n_inst, k, world)
            m = (src >= lo) & (src < hi)
            s.enqueue(src[m], dst[m], seq[m], size[m], t[m])
        srcs.append(src)
        t0 += window_ns
        window(t0)
    for w in range(3):
        t0 += 10 * window_ns
        srcs.append(np.zeros(0, np.int64))
        window(t0)
    for i, s in enumerate(sims):
        outs[i].append(dict(stats=parity_stats(s)))
        s.close()
    return outs, srcs


def split_single(single, srcs, world: int, n_inst: int = 24):
    """Single-shard run_random output -> what each shard of a sharded run must report: statuses of
    its senders (enqueue order), deliveries to its receivers (global inbox order restricted), its
    local inbox offsets. Statistics are compared as sums over shards."""
    per = []
    for k in range(world):
        lo, hi = shard_range(n_inst, k, world)
        wins = []
        for x, src in zip(single[:-1], srcs):
            m_src = (src >= lo) & (src < hi)
            d = x["deliv"]
            m = (d["dst"] >= lo) & (d["dst"] < hi)
            dk = {f: v[m] for f, v in d.items()}
            counts = np.bincount(dk["dst"] - lo, minlength=hi - lo) if len(dk["dst"]) else np.zeros(hi - lo, np.int64)
            inbox = np.r_[0, np.cumsum(counts)].astype(np.uint32)
            wins.append(dict(status=x["status"][m_src], deliv=dk, inbox=inbox))
        per.append(wins)
    return per


def assert_sharded_matches(outs, srcs, single, world: int, n_inst: int = 24):
    want = split_single(single, srcs, world, n_inst)
    for k in range(world):
        assert_same(outs[k][:-1], want[k], f"shard{k}")
    tot = {}
    for k in range(world):
        for name, v in outs[k][-1]["stats"].items():
            tot[name] = tot.get(name, 0) + v
    assert tot == single[-1]["stats"], (tot, single[-1]["stats"])


def memmove_exchange(sims):
    """In-process all-to-all over host buffers (the oracle's): block p of shard q's send buffer ->
    block q of shard p's receive buffer."""
    import ctypes as C
    S = len(sims)
    bufs = [s.exchange_buffers() for s in sims]
    blk = bufs[0][2] // S
    for q in range(S):
        for p in range(S):
            C.memmove(bufs[p][1] + q * blk, bufs[q][0] + p * blk, blk)


# ---- config 5: flood with first-receipt dedup over a random-regular graph -----------------------

def run_flood(binding, n_inst=3000, pubs_per_wave=3, waves=2, wave_gap_windows=4, window_ns=10 * MS, size=512,
              seed=5, degree=8, shapes=None, keep=True, on_window=None, cfg_kw=None, max_windows=2000,
              windows=None, setup=None, count=True, restart=()):
    """Waves of publications flooding the graph; every window: advance, read the deliveries, then
    tgsim_flood_react stages the first-receipt forwards for the next window. Returns per-window
    observables (keep=True) and the totals. windows: run exactly that many windows (a sharded run
    driven through a transport, whose shards cannot see the global end condition); setup(sim)
    attaches that transport. count=False: the reaction stays asynchronous (no forward counts; give
    `windows`). restart: windows after whose reaction the run is snapshotted and restored into a
    fresh context with the same graph (checkpoint / resume)."""
    from testground_amd import workloads as W
    assert count or windows is not None
    kw = dict(max_msgs_per_window=1 << 20, max_records=1 << 22, data_prefix_len=12)
    kw.update(cfg_kw or {})
    sim = Simulator(SimConfig(n_instances=n_inst, seed=seed, **kw), binding=binding)
    if setup is not None:
        setup(sim)
    sim.set_shapes(np.arange(n_inst), shapes if shapes is not None else W.pubsub_shapes(n_inst, seed))
    off, nbr = W.random_regular_graph(n_inst, degree, seed)
    sim.flood_set_graph(off, nbr, pubs_per_wave * waves)
    out, tot = [], dict(delivered=0, forwarded=0, windows=0)
    t, w, fwd = 0, 0, 0
    while w < (windows if windows is not None else max_windows):
        if w % wave_gap_windows == 0 and w // wave_gap_windows < waves:
            wave = w // wave_gap_windows
            pubs = W.publishers(n_inst, pubs_per_wave, wave, seed)
            sim.flood_publish(pubs, np.arange(pubs_per_wave) + wave * pubs_per_wave, t, size)
        elif windows is None and fwd == 0 and sim.stats()["inflight"] == 0 and w // wave_gap_windows >= waves:
            break
        t += window_ns
        sim.advance(t, wait=count)
        d = sim.deliveries()
        fwd = sim.flood_react(size, count=count)
        tot["delivered"] += len(d["dst"])
        tot["forwarded"] += fwd or 0
        if on_window is not None:
            on_window(w, d, fwd)
        if keep:
            out.append(dict(status=sim.status(), deliv=d, inbox=sim.inbox_offsets(), fwd=fwd))
        if w in restart:
            image = sim.snapshot()
            cfg = sim.cfg
            sim.close()
            sim = Simulator(cfg, binding=binding)
            if setup is not None:
                setup(sim)
            sim.flood_set_graph(off, nbr, pubs_per_wave * waves)
            sim.restore(image)
        w += 1
    tot["windows"] = w
    out.append(dict(stats=parity_stats(sim), tot=tot))
    sim.close()
    return out


def run_flood_sharded(make_sim, exchange, world: int, n_inst=900, pubs_per_wave=3, waves=2, wave_gap_windows=4,
                      window_ns=10 * MS, size=512, seed=5, degree=8, shapes=None, max_windows=2000):
    """run_flood over `world` shards of one process (every shard gets the same configuration calls;
    the owner keeps state). Each window: advance_begin on every shard, exchange, advance_end, react.
    Returns per window the shards' deliveries concatenated in shard order (= the single run's global
    inbox order, shards owning contiguous receivers) and the summed forward count, plus the summed
    statistics."""
    from testground_amd import workloads as W
    sims = [make_sim(SimConfig(n_instances=n_inst, seed=seed, shard_id=k, n_shards=world, exchange_cap=1 << 15,
                               max_msgs_per_window=1 << 20, max_records=1 << 22, data_prefix_len=12))
            for k in range(world)]
    shapes = shapes if shapes is not None else W.pubsub_shapes(n_inst, seed)
    off, nbr = W.random_regular_graph(n_inst, degree, seed)
    for s in sims:
        s.set_shapes(np.arange(n_inst), shapes)
        s.flood_set_graph(off, nbr, pubs_per_wave * waves)
    out = []
    t, w, fwd = 0, 0, 0
    while w < max_windows:
        if w % wave_gap_windows == 0 and w // wave_gap_windows < waves:
            wave = w // wave_gap_windows
            pubs = W.publishers(n_inst, pubs_per_wave, wave, seed)
            for s in sims:
                s.flood_publish(pubs, np.arange(pubs_per_wave) + wave * pubs_per_wave, t, size)
        elif fwd == 0 and sum(s.stats()["inflight"] for s in sims) == 0 and w // wave_gap_windows >= waves:
            break
        t += window_ns
        for s in sims:
            s.advance_begin(t)
        exchange(sims)
        for s in sims:
            s.advance_end()
        ds = [s.deliveries() for s in sims]
        fwd = sum(s.flood_react(size) for s in sims)
        out.append(dict(deliv={k: np.concatenate([d[k] for d in ds]) for k in ds[0]}, fwd=fwd))
        w += 1
    tot = {}
    for s in sims:
        for name, v in parity_stats(s).items():
            tot[name] = tot.get(name, 0) + v
        s.close()
    out.append(dict(stats=tot))
    return out


def flood_single_view(single):
    """run_flood output in run_flood_sharded's structure."""
    return [dict(deliv=x["deliv"], fwd=x["fwd"]) for x in single[:-1]] + [dict(stats=single[-1]["stats"])]


# ---- sharded runs driven through a transport (tgsim_set_transport): one shard per thread -----------

def sharded_threads(world: int, fn, device: bool = False):
    """fn(k, member_transport) for every shard k, each on its own thread with a ThreadGroup member
    (host buffers, or device buffers on one GPU); returns the results in shard order."""
    from testground_amd.exchange import ThreadGroup, run_threads
    g = ThreadGroup(world, device=device)
    return run_threads([lambda k=k: fn(k, g.member(k)) for k in range(world)])


def run_skewed_exchange(binding, n_msgs: int, device: bool = False, exchange_cap: int = 513):
    """one sender of shard 0 sends an unshaped (zero-delay) burst of n_msgs to shard 1's
    receivers in one window, so one or two workgroups of the netem pass append every record to one
    peer - far more than a slice's (exchange_cap - 1) / 8. Returns per shard ("ok", statuses or
    deliveries) or ("err", code)."""
    from testground_amd.exchange import ThreadGroup, run_threads
    g = ThreadGroup(2, device=device, timeout=120.0)

    def shard(k):
        sim = Simulator(SimConfig(n_instances=16, seed=7, shard_id=k, n_shards=2, exchange_cap=exchange_cap),
                        binding=binding)
        sim.set_transport(g.member(k))
        try:
            if k == 0:
                i = np.arange(n_msgs, dtype=np.int64)
                sim.enqueue(np.zeros(n_msgs, np.int64), 8 + i % 8, i, np.full(n_msgs, 100), np.zeros(n_msgs, np.int64))
            sim.advance(1 * MS)
            return ("ok", sim.status() if k == 0 else sim.deliveries())
        except A.TgsimError as e:
            return ("err", e.code)
        finally:
            sim.close()
    return run_threads([lambda k=k: shard(k) for k in range(2)])


def shard_cfg(world: int, k: int, **kw):
    return dict(shard_id=k, n_shards=world, **kw)


def assert_storm_sharded(outs, single, world: int, n: int):
    """Per-shard storm outputs (run_storm on every shard) against the single-shard run: the shards'
    statuses (their own senders, generator order) and deliveries (their own receivers, inbox order)
    concatenate to the single run's, inbox offsets are the single run's slice, clocks agree and the
    counters sum."""
    for r in range(len(single) - 1):
        for f in single[r]["deliv"]:
            cat = np.concatenate([outs[k][r]["deliv"][f] for k in range(world)])
            assert_same(cat, single[r]["deliv"][f], f"round {r} deliv.{f}")
        assert_same(np.concatenate([outs[k][r]["status"] for k in range(world)]), single[r]["status"],
                    f"round {r} status")
        for k in range(world):
            lo, hi = shard_range(n, k, world)
            inbox = single[r]["inbox"][lo:hi + 1] - single[r]["inbox"][lo]
            assert_same(outs[k][r]["inbox"], inbox, f"round {r} shard {k} inbox")
            assert outs[k][r]["now"] == single[r]["now"]
    tot = {}
    for k in range(world):
        for name, v in outs[k][-1]["stats"].items():
            tot[name] = tot.get(name, 0) + v
    assert tot == single[-1]["stats"], (tot, single[-1]["stats"])


def combine_flood_shards(outs):
    """Per-shard run_flood outputs -> run_flood_sharded's structure (deliveries concatenated in
    shard order, forwards and counters summed)."""
    world = len(outs)
    res = []
    for w in range(len(outs[0]) - 1):
        d = {f: np.concatenate([outs[k][w]["deliv"][f] for k in range(world)]) for f in outs[0][w]["deliv"]}
        res.append(dict(deliv=d, fwd=sum(outs[k][w]["fwd"] for k in range(world))))
    tot = {}
    for k in range(world):
        for name, v in outs[k][-1]["stats"].items():
            tot[name] = tot.get(name, 0) + v
    res.append(dict(stats=tot))
    return res
