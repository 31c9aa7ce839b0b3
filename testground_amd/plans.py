"""Workload descriptors: the reference's test plans restated as message patterns over simulated
instances (hard part 6). A plan here is a function ``plan(env) -> ok[]`` that returns
the per-instance outcome, written against the same client calls the Go plan makes
(``env.sync``: sync.Client, ``env.net``: network.Client) so it can be read beside the original.

Messages are the units the simulator shapes. A TCP segment is modelled as one message of
``payload + TCP_OVERHEAD`` bytes; there is no retransmission, so a lost segment fails the exchange
it belongs to (packet/TCP-level modelling is SURVEY.md 8(f) rank 4).

Registered plans (``PLANS[(plan, case)]``):
  network/ping-pong           plans/network/pingpong.go:16-201
  network/traffic-allowed     plans/network/traffic.go:16-72 (AllowAll)
  network/traffic-blocked     plans/network/traffic.go:16-72 (DenyAll)
  splitbrain/{drop,reject,accept}   plans/splitbrain/main.go:41-186
  benchmarks/storm            plans/benchmarks/storm.go:31-197
  benchmarks/barrier          plans/benchmarks/benchmarks.go:90-145
  benchmarks/{startup,netinit,netlinkshape,subtree}   plans/benchmarks/benchmarks.go:20-86, 148-270
  verify/uses-data-network    plans/verify/main.go:43-130
  placebo/{ok,panic,stall}    plans/placebo/main.go:17-40
  example/{sync,failure,panic} plans/example/{sync,failure,panic}.go
"""
from __future__ import annotations

import math

import numpy as np

from . import _abi as A
from .network import (MS, SECOND, AllowAll, Config, DenyAll, FilterAction, IPNet, LinkRule, LinkShape, RuleList,
                      int_to_ip)
from .sidecar import NetClient, Sidecar
from .sim import SimConfig, Simulator
from .sync import SyncService

TCP_OVERHEAD = 66          # Ethernet 14 + IPv4 20 + TCP 20 + timestamp option 12 bytes per segment
TCP_CHUNK = 4 * 1024       # storm.go:23 write size
NEVER = np.iinfo(np.int64).max


class RunParams(dict):
    """A run's test parameters; names whose value differs between groups raise when read (the
    descriptors are written for one value per run; runtime.RunEnv in the reference is per instance)."""

    def __init__(self, values: dict, ambiguous=()):
        super().__init__(values)
        self.ambiguous = frozenset(ambiguous)

    def get(self, name, default=None):
        if name in self.ambiguous:
            raise ValueError(f"test parameter {name!r} differs between groups; the workload descriptor "
                             f"takes one value per run")
        return super().get(name, default)

    def __getitem__(self, name):
        return self.get(name) if name in self else super().__getitem__(name)


class PlanEnv:
    """One simulated run: simulator + sync service + sidecars + network clients, and a message
    layer that stages sends when their time falls in the next window and records, per message,
    its status and first arrival time."""

    def __init__(self, n_instances: int, seed: int = 1, test_case: str = "", params: dict | None = None,
                 binding=None, window_ns: int = 1 * MS, sim_kw: dict | None = None):
        self.n = int(n_instances)
        self.test_case = test_case
        self.params = params if isinstance(params, RunParams) else RunParams(params or {})
        self.window_ns = int(window_ns)
        # reaction latency of a request/reply hop on an unshaped link (a local HTTP round trip over a
        # bridge is ~100 us): the window of the sequential probes while messages are in flight
        self.probe_window_ns = int(self.params.get("probe_window_ns", 100_000))
        # plans give instances their own sync states (splitbrain's "reconfigured<host>" callbacks)
        # a /16 data network holds 65,534 instances (pkg/runner/common.go:28-40); larger runs get a
        # wider simulated prefix with the same CIDR semantics (hard part 7)
        kw = dict(max_msgs_per_window=1 << 18, max_records=1 << 20, max_states=max(1024, 2 * self.n + 256),
                  max_waiters=max(1 << 16, 4 * self.n), data_prefix_len=16 if self.n <= 65534 else 8)
        kw.update(sim_kw or {})
        self.sim = Simulator(SimConfig(n_instances=self.n, seed=seed, **kw), binding=binding)
        self.sync = SyncService(self.sim)
        # sidecar_wire (a test parameter): configs travel as JSON on the network:<hostname> topics
        wire = self.params.get("sidecar_wire", "false") == "true"
        self.sidecar = Sidecar(self.sim, self.sync, self.n, track_configs=self.n <= 4096, wire=wire)
        self.net = NetClient(self.sidecar)
        self._seq = np.zeros(self.n, np.int64)
        self._pend = []                       # (t, src, dst, seq, size) arrays not yet staged
        self._st_keys, self._st_vals = [], []  # status log
        self._ar_keys, self._ar_vals = [], []  # arrival log (first arrival per key after compaction)
        self.failures: list[str] = []
        # transport "tcp" (a test parameter): application data goes through TCP mode (DESIGN.md
        # 2.11); a step then reports the writes that completed, at their last segment's arrival
        self.tcp = self.params.get("transport", "message") == "tcp"
        if self.tcp:
            # tcp_acks (default true): ACK packets, timers and the connections' Reno windows
            # (DESIGN.md 2.11b); "false" keeps the per-write model without a reverse path
            self.tcp_acks = self.params.get("tcp_acks", "true") == "true"
            self.sim.tcp_enable(acks=self.tcp_acks)
            self._tw_keys = []                     # write id -> key, in send order
            self._tw_first = 0                     # writes before it have all been reported
            self._tw_seen = np.zeros(0, bool)      # writes [_tw_first, ...) already reported
        self.sidecar.initialize(0)

    def close(self):
        self.sim.close()

    # ---- parameters (runtime.RunEnv.IntParam & co.) ---------------------------------------------
    def int_param(self, name: str, default=None) -> int:
        v = self.params.get(name, default)
        if v is None:
            raise KeyError(f"missing test parameter {name!r}")
        return int(v)

    # ---- messages ---------------------------------------------------------------------------
    @staticmethod
    def key(src, seq):
        return (np.asarray(src, np.uint64) << np.uint64(32)) | np.asarray(seq, np.uint64)

    def send(self, src, dst, size, t) -> np.ndarray:
        """Queue messages src[i] -> dst[i] of size[i] bytes at time t[i]; returns their keys."""
        src = np.atleast_1d(np.asarray(src, np.int64))
        n = len(src)
        dst = np.broadcast_to(np.asarray(dst, np.int64), (n,)).copy()
        size = np.broadcast_to(np.asarray(size, np.int64), (n,)).copy()
        t = np.broadcast_to(np.asarray(t, np.int64), (n,)).copy()
        if n == 0:
            return np.zeros(0, np.uint64)
        if t.min() < self.sim.horizon:
            raise A.TgsimError(A.ECAUSALITY, "send before the reaction horizon")
        order = np.argsort(src, kind="stable")
        s_sorted = src[order]
        first = np.r_[0, np.flatnonzero(np.diff(s_sorted)) + 1]
        run_start = np.repeat(first, np.diff(np.r_[first, n]))
        rank = np.arange(n) - run_start
        seq = np.empty(n, np.int64)
        seq[order] = self._seq[s_sorted] + rank
        np.add.at(self._seq, src, 1)
        self._pend.append((t, src, dst, seq, size))
        return self.key(src, seq)

    def step(self, t_end: int | None = None) -> dict:
        """Run one window [now, t_end) (default: one window_ns). Returns its deliveries."""
        t_end = self.sim.now + self.window_ns if t_end is None else int(t_end)
        if self._pend:
            t = np.concatenate([p[0] for p in self._pend])
            cols = [np.concatenate([p[k] for p in self._pend]) for k in range(1, 5)]
            due = t < t_end
            keep = ~due
            self._pend = [(t[keep], *[c[keep] for c in cols])] if keep.any() else []
            if due.any():
                src, dst, seq, size = (c[due] for c in cols)
                if self.tcp:
                    self.sim.tcp_send(src, dst, seq, size, t[due])
                    self._tw_keys.append(self.key(src, seq))
                else:
                    self.sim.enqueue(src, dst, seq, size, t[due])
                staged_keys = self.key(src, seq)
            else:
                staged_keys = np.zeros(0, np.uint64)
        else:
            staged_keys = np.zeros(0, np.uint64)
        if self.tcp:
            return self._step_tcp(t_end)
        self.sim.advance(t_end)
        if len(staged_keys):
            self._st_keys.append(staged_keys)
            self._st_vals.append(self.sim.status())
        d = self.sim.deliveries()
        if len(d["t_deliver"]):
            self._ar_keys.append(self.key(d["src"], d["seq"]))
            self._ar_vals.append(d["t_deliver"])
        return d

    def _step_tcp(self, t_end: int) -> dict:
        """One window in TCP mode: the writes that completed in it as deliveries (src, dst, seq =
        the write's key, t_deliver = its last segment's arrival); failed writes enter the status
        log (TIMEOUT as LOST, REFUSED as REJECTED). Only writes from the first unsettled one on are
        read back (not the whole table every window)."""
        self.sim.advance(t_end)
        self.sim.tcp_react()
        # _tw_keys holds the keys of writes _tw_first, _tw_first + 1, ... (the settled prefix is dropped)
        keys = np.concatenate(self._tw_keys) if self._tw_keys else np.zeros(0, np.uint64)
        st, t = self.sim.tcp_writes_range(self._tw_first, len(keys))
        seen = np.r_[self._tw_seen, np.zeros(len(st) - len(self._tw_seen), bool)]
        new = (st != A.TCP_PENDING) & ~seen
        seen |= new
        settled = int(np.argmin(seen)) if not seen.all() else len(seen)
        self._tw_keys = [keys[settled:]] if settled < len(keys) else []
        self._tw_first += settled
        self._tw_seen = seen[settled:]
        self.tcp_settled_keys = keys[new]
        ok = new & (st == A.TCP_DELIVERED)
        bad = new & (st != A.TCP_DELIVERED)
        if bad.any():
            self._st_keys.append(keys[bad])
            self._st_vals.append(np.where(st[bad] == A.TCP_TIMEOUT, A.ST_LOST, A.ST_REJECTED).astype(np.uint8))
        if ok.any():
            self._ar_keys.append(keys[ok])
            self._ar_vals.append(t[ok])
        order = np.argsort(t[ok], kind="stable")
        k = keys[ok][order]
        return {"src": (k >> np.uint64(32)).astype(np.uint32), "seq": (k & np.uint64(0xFFFFFFFF)).astype(np.uint32),
                "t_deliver": t[ok][order]}

    def _compact(self, keys, vals, first_min: bool):
        if len(keys) > 1 or (keys and first_min):
            k = np.concatenate(keys)
            v = np.concatenate(vals)
            o = np.lexsort((v, k)) if first_min else np.argsort(k, kind="stable")
            k, v = k[o], v[o]
            u = np.r_[True, k[1:] != k[:-1]]
            keys[:] = [k[u]]
            vals[:] = [v[u]]
        return (keys[0], vals[0]) if keys else (np.zeros(0, np.uint64), np.zeros(0, np.int64))

    def status_of(self, keys) -> np.ndarray:
        """Status byte of each message, or 0xFF if it has not been processed yet."""
        k, v = self._compact(self._st_keys, self._st_vals, False)
        return _lookup(k, v, keys, 0xFF).astype(np.int64)

    def arrival_of(self, keys) -> np.ndarray:
        """First arrival time of each message, or NEVER."""
        k, v = self._compact(self._ar_keys, self._ar_vals, True)
        return _lookup(k, v, keys, NEVER)

    def wait(self, keys, timeout_ns: int) -> np.ndarray:
        """Step windows until every message has arrived or failed (or the timeout). Returns
        arrival times (NEVER for failures)."""
        keys = np.asarray(keys, np.uint64)
        deadline = self.sim.now + int(timeout_ns)
        while True:
            arr = self.arrival_of(keys)
            st = self.status_of(keys)
            failed = (st != 0xFF) & ((st & 0x0F) != A.ST_QUEUED) & ((st & 0x0F) != A.ST_LOCAL)
            if np.all((arr != NEVER) | failed) or self.sim.now >= deadline:
                return arr
            self.step()

    def advance_to(self, t: int) -> None:
        """Let simulated time pass until t (time.Sleep), window by window while traffic is in flight."""
        while self.sim.now < t:
            idle = not self._pend and self.sim.stats()["inflight"] == 0
            self.step(t if idle else min(t, self.sim.now + self.window_ns))

    def rpc(self, src, dst, req_size, rep_size, t, timeout_ns) -> tuple[np.ndarray, np.ndarray]:
        """Request src->dst at t; dst answers at the request's first arrival (in the window right
        after it, at the arrival time: the reaction horizon allows it). Returns (ok, rtt)."""
        src = np.atleast_1d(np.asarray(src, np.int64))
        n = len(src)
        dst = np.broadcast_to(np.asarray(dst, np.int64), (n,))
        t = np.broadcast_to(np.asarray(t, np.int64), (n,))
        req = self.send(src, dst, req_size, t)
        deadline = int(t.max()) + int(timeout_ns) if n else self.sim.now
        o_req = np.argsort(req)
        req_sorted = req[o_req]
        rep = np.zeros(n, np.uint64)
        answered = np.zeros(n, bool)
        while n:
            d = self.step()
            if len(d["t_deliver"]):
                k = self.key(d["src"], d["seq"])
                i = np.minimum(np.searchsorted(req_sorted, k), n - 1)
                hit = req_sorted[i] == k
                idx = o_req[i[hit]]
                at = d["t_deliver"][hit]
                idx, first = np.unique(idx, return_index=True)   # duplicates: first copy only
                at = at[first]
                new = ~answered[idx]
                if new.any():
                    j = idx[new]
                    rep[j] = self.send(dst[j], src[j], rep_size, at[new])
                    answered[j] = True
            st_req = self.status_of(req)
            req_failed = (st_req != 0xFF) & ~np.isin(st_req & 0x0F, (A.ST_QUEUED, A.ST_LOCAL))
            arr = np.where(answered, self.arrival_of(rep), NEVER)
            st_rep = np.where(answered, self.status_of(rep), 0xFF)
            rep_failed = (st_rep != 0xFF) & ~np.isin(st_rep & 0x0F, (A.ST_QUEUED, A.ST_LOCAL))
            if np.all((arr != NEVER) | req_failed | rep_failed) or self.sim.now >= deadline:
                break
        if not n:
            return np.zeros(0, bool), np.zeros(0, np.int64)
        ok = arr != NEVER
        return ok, np.where(ok, arr - t, -1)

    def tcp_write(self, conn, sizes, t, src, dst) -> np.ndarray:
        """Writes on TCP connections (transport=tcp) at t; returns their keys
        (src, seq) - tracked like sent messages: arrival = the write's delivery, a failure enters
        the status log."""
        src = np.atleast_1d(np.asarray(src, np.int64))
        n = len(src)
        order = np.argsort(src, kind="stable")
        s_sorted = src[order]
        first = np.r_[0, np.flatnonzero(np.diff(s_sorted)) + 1] if n else np.zeros(0, np.int64)
        rank = np.arange(n) - np.repeat(first, np.diff(np.r_[first, n])) if n else np.zeros(0, np.int64)
        seq = np.empty(n, np.int64)
        seq[order] = self._seq[s_sorted] + rank
        np.add.at(self._seq, src, 1)
        keys = self.key(src, seq)
        self.sim.tcp_write(conn, sizes, t)
        self._tw_keys.append(keys)
        return keys

    def probe(self, order, req_size: int, rep_size: int, timeout_ns: int, t0: int, window_ns: int | None = None):
        """Every instance probes order[...] (itself excluded) one request/reply at a time, the next
        probe leaving when the previous one ended (tgsim_probe_*): the sequential
        httpclient.Get loop of plans/splitbrain/main.go:159-175. Windows follow the device's
        proposal (window_ns while traffic is in flight, a jump to the next deadline when idle).
        Returns (outcome[instance, position in order], t_done[instance])."""
        window = int(window_ns or self.probe_window_ns)
        self.advance_to(t0)
        self.sim.probe_setup(order, req_size, rep_size, timeout_ns, window)
        self.sim.probe_start(t0)
        ne = max(int(t0), self.sim.now) + window
        self.probe_windows = 0
        while True:
            self.sim.advance(ne)
            self.probe_windows += 1
            ne, active = self.sim.probe_react()
            if active == 0:
                break
        return self.sim.probe_results()

    def fail(self, msg: str) -> None:
        self.failures.append(msg)


def _lookup(k, v, q, missing):
    q = np.asarray(q, np.uint64)
    out = np.full(len(q), missing, dtype=v.dtype if len(v) else np.int64)
    if len(k):
        i = np.searchsorted(k, q)
        i = np.minimum(i, len(k) - 1)
        hit = k[i] == q
        out[hit] = v[i[hit]]
    return out


# ============================================================================================
# plans/network
# ============================================================================================

def pingpong(env: PlanEnv) -> np.ndarray:
    """plans/network/pingpong.go:16-201: two instances, 100 ms egress latency + 1 Mibit/s each,
    1-byte ping-pong RTT must be in [200, 215] ms; then 10 ms latency, RTT in [20, 35] ms."""
    if env.n != 2:
        raise ValueError("ping-pong needs exactly two instances (pingpong.go:100)")
    t = env.net.wait_network_initialized(0)
    # each instance owns its Config (pingpong.go:29-41 runs in two processes)
    configs = [Config(network="default", enable=True, default=LinkShape(latency=100 * MS, bandwidth=1 << 20),
                      callback_state="network-configured", routing_policy=DenyAll) for _ in range(2)]
    rel = [env.net.configure_network(g, configs[g], t) for g in range(2)]
    t = max(rel)
    seq, t = env.sync.signal_and_wait("ip-allocation", [0, 1], t, 2)
    # pingpong.go:57-66: ip = subnet.a.b.(seq>>8 + 1).(seq & 255)
    base = env.net.get_data_network_ip(0) & 0xFFFF0000
    rel = []
    for g in range(2):
        s = int(seq[g])
        configs[g].callback_state = "ip-changed"
        configs[g].ipv4 = IPNet(base | ((((s >> 8) + 1) & 255) << 8) | (s & 255), 15)
        rel.append(env.net.configure_network(g, configs[g], t))
    t = max(rel)
    _, t = env.sync.signal_and_wait("listening", [0, 1], t, 2)
    env.sync.publish("peers", [0, 1], t, [int_to_ip(env.net.get_data_network_ip(g)) for g in range(2)])
    _, t = env.sync.signal_and_wait("got-other-addrs", [0, 1], t, 2)
    env.advance_to(t)
    # TCP connect from seq 2 to seq 1: SYN / SYN-ACK (+ ACK piggybacked on the first write)
    dialer = int(np.flatnonzero(seq == 2)[0])
    ok, _ = env.rpc([dialer], [1 - dialer], TCP_OVERHEAD, TCP_OVERHEAD, env.sim.now, 30 * SECOND)
    if not ok[0]:
        env.fail("dial failed")
        return np.zeros(2, bool)
    ok = np.ones(2, bool)
    for test, lo, hi in (("200", 200 * MS, 215 * MS), ("10", 20 * MS, 35 * MS)):
        if test == "10":
            for c in configs:
                c.default.latency = 10 * MS
                c.callback_state = "latency-reduced"
            rel = [env.net.configure_network(g, configs[g], env.sim.now) for g in range(2)]
            env.advance_to(max(rel))
        rtt = _pingpong_round(env, seq)
        for g in range(2):
            if not lo <= rtt[g] <= hi:
                env.fail(f"instance {g}: expected an RTT between {lo} and {hi}, got {rtt[g]}")
                ok[g] = False
        env.rtts = getattr(env, "rtts", []) + [rtt]
        _, t = env.sync.signal_and_wait("ping-pong-" + test, [0, 1], env.sim.now, 2)
        env.advance_to(t)
    return ok


def _pingpong_round(env: PlanEnv, seq) -> np.ndarray:
    """pingpong.go:116-173 over one connection: both write a 0 byte and read the peer's (start);
    write own id; read the peer's id and echo it; read own id back (end). Returns end - start."""
    sz = TCP_OVERHEAD + 1
    now = env.sim.now
    k = env.send([0, 1], [1, 0], sz, [now, now])
    arr = env.wait(k, 10 * SECOND)             # arr[0]: 0 -> 1 arrives at 1; arr[1]: at 0
    start = np.array([arr[1], arr[0]])         # instance g starts after reading the peer's 0
    kid = env.send([0, 1], [1, 0], sz, start)  # write my id
    a_id = env.wait(kid, 10 * SECOND)          # a_id[0] = my id (0) at 1, a_id[1] = 1's id at 0
    got_peer_id = np.array([a_id[1], a_id[0]])
    echo_t = np.maximum(got_peer_id, start)    # read their id (after my own write), write it back
    kecho = env.send([0, 1], [1, 0], sz, echo_t)
    a_echo = env.wait(kecho, 10 * SECOND)      # a_echo[0] = echo of 1's id, arrives at 1
    back = np.array([a_echo[1], a_echo[0]])
    end = np.maximum(back, echo_t)             # read my id after echoing theirs
    if np.any(end == NEVER):
        env.fail("ping-pong message lost")
        return np.full(2, -1, np.int64)
    return end - start


def traffic(policy):
    """plans/network/traffic.go:16-72: an HTTP GET to a host outside the data network must fail
    under DenyAll and succeed under AllowAll."""
    def plan(env: PlanEnv) -> np.ndarray:
        t = env.net.wait_network_initialized(0)
        cfg = Config(network="default", enable=True, callback_state="network-configured-with-policy",
                     routing_policy=policy)
        t = max(env.net.configure_network(g, cfg, t) for g in range(env.n))
        env.advance_to(t)
        k = env.send(np.arange(env.n), A.DST_EXTERNAL, TCP_OVERHEAD, env.sim.now)
        env.step()
        st = env.status_of(k) & 0x0F
        reached = st == A.ST_EXTERNAL
        ok = ~reached if policy == DenyAll else reached
        for g in np.flatnonzero(~ok):
            env.fail(f"instance {g}: external request {'succeeded' if reached[g] else 'failed'} under {policy.value}")
        return ok
    return plan


# ============================================================================================
# plans/splitbrain
# ============================================================================================

REGION_A, REGION_B, REGION_C = 0, 1, 2


def expect_errors(test_case: str, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """plans/splitbrain/main.go:50-58, vectorised."""
    if test_case == "accept":
        return np.zeros(np.broadcast(a, b).shape, bool)
    return ((a == REGION_A) & (b == REGION_B)) | ((a == REGION_B) & (b == REGION_A))


SPLITBRAIN_CTX_NS = 300 * SECOND     # context.WithTimeout(..., 300*time.Second), main.go:64
PROBE_TIMEOUT_NS = 60 * SECOND       # http.Client{Timeout: time.Minute}, main.go:153-155


def splitbrain(action: FilterAction):
    """plans/splitbrain/main.go:60-186: region = SignalEntry("region-select") % 3; every node
    publishes itself on "nodes" and lists the others in topic order; region A installs a /32 rule
    with `action` toward every region-B node; SignalAndWait("nodeRoundup"); time.Sleep(10 s); then
    each node GETs every other node ONE AT A TIME in that order (main.go:159-175), each GET with a
    one-minute timeout; SignalAndWait("testcomplete") under the plan's 300 s context (main.go:64).

    A probe is a request and its reply (device sequential probes): it fails at once
    when the prober's own route refuses it (A -> B: blackhole / prohibit make connect() fail
    immediately) and at the one-minute deadline when the peer's reply is dropped by the peer's
    routes (B -> A: the SYN-ACK meets A's rule). Failures are expected exactly between A and B
    (expectErrors, main.go:50-58); an unexpected one fails the prober. The "testcomplete" barrier
    releases when the slowest prober is done; a release past the 300 s context is an error for every
    instance - which is what the reference does once region B waits out enough one-minute timeouts
    (>= 5 region-A nodes). env.probe_unexpected / env.probe_errors keep the probe truth table."""
    def plan(env: PlanEnv) -> np.ndarray:
        n = env.n
        t = env.net.wait_network_initialized(0)
        seq = env.sync.signal_entry("region-select", np.arange(n), t)
        region = (seq.astype(np.int64) % 3)
        ips = np.array([env.net.get_data_network_ip(g) for g in range(n)], np.int64)
        pos = env.sync.publish("nodes", np.arange(n), t, list(zip(region.tolist(), ips.tolist())))
        order = np.argsort(pos, kind="stable")                 # instances in topic order
        b_ips = ips[order][region[order] == REGION_B]          # main.go:118: nodes in topic order
        rules = RuleList(LinkRule(IPNet(int(ip), 32), LinkShape(filter=action)) for ip in b_ips)
        for a in np.flatnonzero(region == REGION_A):
            cfg = Config(network="default", enable=True, callback_state=f"reconfigured{a}", callback_target=1,
                         rules=rules)
            env.net.configure_network(int(a), cfg, t)
        _, t = env.sync.signal_and_wait("nodeRoundup", np.arange(n), t, n)
        t_probe = t + 10 * SECOND                               # time.Sleep(10 * time.Second), main.go:145
        outcome, t_done = env.probe(order, TCP_OVERHEAD, TCP_OVERHEAD, PROBE_TIMEOUT_NS, t_probe)
        peer = np.broadcast_to(order, outcome.shape)
        me = np.broadcast_to(np.arange(n)[:, None], outcome.shape)
        probed = peer != me
        errs = probed & (outcome != A.PROBE_OK)
        unexpected = errs & ~expect_errors(env.test_case, region[me], region[peer])
        env.probe_outcome = outcome
        env.probe_errors = errs.sum(axis=1)
        env.probe_unexpected = unexpected.sum(axis=1)
        env.probe_done = t_done
        env.region = region
        ok = env.probe_unexpected == 0
        for g in np.flatnonzero(~ok):
            env.fail(f"instance {g} (region {region[g]}): {env.probe_unexpected[g]} unexpected probe failures")
        _, t_all = env.sync.signal_and_wait("testcomplete", np.arange(n), t_done, n)
        env.testcomplete = t_all
        if t_all > SPLITBRAIN_CTX_NS:
            env.fail(f"testcomplete released at {t_all / SECOND:.1f} s, after the plan's 300 s context "
                     f"(main.go:64): context deadline exceeded")
            ok[:] = False
        env.advance_to(max(env.sim.now, t_all))
        return ok
    return plan


# ============================================================================================
# plans/benchmarks
# ============================================================================================

STORM_DIAL_TIMEOUT_NS = 30 * SECOND   # net.DialTimeout("tcp", addr, 30*time.Second), storm.go:144
STORM_CTX_NS = 3000 * SECOND          # context.WithTimeout(..., 3000*time.Second), storm.go:32
STORM_MSG_WINDOW = 10                 # message mode: writes a connection keeps in flight (IW10's segments)


def storm(env: PlanEnv) -> np.ndarray:
    """plans/benchmarks/storm.go:31-197: every instance dials `conn_outgoing` random peers, each
    after U[0, conn_delay_ms) ms and under a semaphore of `concurrent_dials` (storm.go:141-152:
    DialTimeout 30 s); every dialler signals "outgoing-dials-done" (target N * conn_outgoing) and,
    once it releases, writes data_size_kb KiB into its connection in 4 KiB chunks, each conn.Write
    under a second semaphore of `concurrent_dials` (writesem, storm.go:158-183); conn.Write returns
    when the chunk fits the socket's buffer, so a full buffer blocks its writer - holding its
    writesem slot. Then SignalAndWait("done writing", N).

    transport=message: a chunk is one message; a connection keeps at most STORM_MSG_WINDOW in
    flight (a chunk leaves the buffer at its arrival: message mode has no ACKs), and a lost chunk
    fails its instance. transport=tcp: connections with the Reno window (tgsim_tcp_connect,
    DESIGN.md 2.11b), the SYN a bare segment whose ACK completes the dial; the buffer holds
    2 * cwnd segments (Linux autotunes sk_sndbuf to about twice the window, tcp_sndbuf_expand
    [EXT]) and drains as ACKs arrive; a write fails on a timeout or a reset. A failed dial never
    signals, so "outgoing-dials-done" cannot release and the run fails at its 3000 s context, as
    in the reference."""
    n = env.n
    outgoing = env.int_param("conn_outgoing", 5)
    delay_ms = env.int_param("conn_delay_ms", 30000)
    limit = max(1, env.int_param("concurrent_dials", 10))
    size = env.int_param("data_size_kb", 128) * 1024
    rng = np.random.default_rng(env.int_param("seed", 0))
    t = env.net.wait_network_initialized(0)
    _, t = env.sync.signal_and_wait("listening", np.arange(n), t, n)
    _, t = env.sync.signal_and_wait("got-other-addrs", np.arange(n), t, n)
    env.advance_to(t)
    src = np.repeat(np.arange(n), outgoing)
    off = rng.integers(1, n, len(src)) if n > 1 else np.zeros(len(src), np.int64)
    dst = (src + off) % n                                           # rand.Intn over the other nodes
    t_ready = env.sim.now + rng.integers(0, max(delay_ms, 1), len(src)) * MS
    env.bytes_sent = 0
    if env.tcp and not env.tcp_acks:
        raise ValueError("storm over TCP writes into connections: it needs tcp_acks = true (the ACK clock)")
    return _storm_device(env, dst, t_ready, outgoing, limit, size)


def _storm_windows(env: PlanEnv, t_first: int, deadline: int) -> bool:
    """Windows at the storm reactor's proposed ends until no connection is active; False if
    simulated time passed the deadline first. Host work per window is O(1): one window and one
    reaction, whose proposal and active count are the only values read back."""
    ne = t_first + env.window_ns
    while True:
        env.sim.advance(ne)
        env.storm_windows += 1
        if env.tcp:
            env.sim.tcp_react(wait=False)   # segments, ACKs, timers and the windows' ACK clock
        ne, act = env.sim.storm_react()
        if act == 0:
            return True
        if env.sim.now > deadline:
            return False


def _storm_device(env: PlanEnv, dst, t_ready, outgoing: int, limit: int, size: int) -> np.ndarray:
    """The storm on the device reactor (tgsim_storm_*): dials under `sem` with
    DialTimeout (storm.go:141-152), SignalAndWait("outgoing-dials-done", N * outgoing) (:156), then
    4 KiB conn.Writes under `writesem` (:158-183), each connection's send buffer holding
    STORM_MSG_WINDOW chunks (message mode) or 2 x cwnd segments (TCP mode: connections, the SYN a
    bare segment whose ACK completes the dial); SignalAndWait("done writing", N) at each instance's
    last write (:190)."""
    n, sim = env.n, env.sim
    env.storm_windows = 0
    sim.storm_setup(dst, t_ready, outgoing=outgoing, concurrent=limit, data_bytes=size, chunk_bytes=TCP_CHUNK,
                    header_bytes=TCP_OVERHEAD, syn_bytes=TCP_OVERHEAD, msg_window=STORM_MSG_WINDOW,
                    dial_timeout_ns=STORM_DIAL_TIMEOUT_NS, window_ns=env.window_ns)
    try:
        sim.storm_start()
        _storm_windows(env, sim.now, STORM_CTX_NS)
        res, t_dial = sim.storm_dials()
        ok = res == A.PROBE_OK
        env.dials_ok = int(ok.sum())
        env.bytes_sent = 0
        if not ok.all():
            src = np.repeat(np.arange(n), outgoing)
            for i in np.flatnonzero(~ok)[:5]:
                env.fail(f"instance {src[i]}: couldnt dial {dst[i]}")
            env.fail("outgoing-dials-done never released (a failed dial does not signal): context deadline exceeded")
            return np.zeros(n, bool)
        _, t_b = env.sync.signal_and_wait("outgoing-dials-done", np.repeat(np.arange(n), outgoing), t_dial,
                                          n * outgoing)
        t_w = max(int(t_b), sim.now)
        sim.storm_write_start(t_w)
        if not _storm_windows(env, t_w, STORM_CTX_NS):
            env.fail("writes still blocked at the 3000 s context")
            return np.zeros(n, bool)
        failed, t_last, tot = sim.storm_results()
    finally:
        sim.storm_end()
    env.bytes_sent = int(tot["bytes_written"])
    env.delivered_chunks = int(tot["chunks_delivered"])
    env.storm_totals = tot
    # wg.Wait(): the last conn.Write of each instance returned; then SignalAndWait("done writing", N)
    t_last = np.where(t_last == np.iinfo(np.int64).min, int(t_b), t_last)
    env.sync.signal_and_wait("done writing", np.arange(n), t_last, n)
    env.overlimit = int(sim.stats()["overlimit"])
    return ~failed


def barrier_bench(env: PlanEnv) -> np.ndarray:
    """plans/benchmarks/benchmarks.go:90-145: for each iteration and percentage p in the Go float
    loop 0.2, 0.4, ... <= 1.0: SignalAndWait(ready, N), then SignalAndWait(test, max(1, floor(N p)))."""
    n = env.n
    iterations = env.int_param("barrier_iterations", 10)
    t = env.net.wait_network_initialized(0)
    tests = []
    p = 0.2
    while p <= 1.0:        # the same IEEE-754 accumulation as the Go loop
        tests.append((f"barrier_time_{int(p * 100)}_percent", p))
        p += 0.2
    env.barrier_times = {}
    everyone = np.arange(n)
    for i in range(1, iterations + 1):
        for name, p in tests:
            _, t = env.sync.signal_and_wait(f"ready_{i}_{name}", everyone, t, n)
            target = int(math.floor(n * p)) or 1
            _, rel = env.sync.signal_and_wait(f"test_{i}_{name}", everyone, t, target)
            env.barrier_times.setdefault(name, []).append(rel - t)
            t = rel
    return np.ones(n, bool)


def startup(env: PlanEnv) -> np.ndarray:
    """plans/benchmarks/benchmarks.go:20-24 (StartTimeBench): records the time since the run
    started; simulated instances start at time 0."""
    env.time_to_start = np.zeros(env.n, np.int64)
    return np.ones(env.n, bool)


def netinit(env: PlanEnv) -> np.ndarray:
    """benchmarks.go:29-48 (NetworkInitBench): the time until the sidecars' network-initialized
    barrier releases."""
    t = env.net.wait_network_initialized(0)
    env.time_to_network_init = np.full(env.n, t, np.int64)
    return np.ones(env.n, bool)


def netlinkshape(env: PlanEnv) -> np.ndarray:
    """benchmarks.go:51-86 (NetworkLinkShapeBench): every instance sends its sidecar
    Config{Network: "default", Default: {Latency: 250 ms}, CallbackState: callback-<random>,
    CallbackTarget: 1} and waits for its own callback. Enable is left at its zero value, so the
    sidecar disconnects the data link (docker_network.go:65-88) - as the reference plan does."""
    n = env.n
    t = env.net.wait_network_initialized(0)
    rng = np.random.default_rng(env.int_param("seed", 0))
    rel = np.empty(n, np.int64)
    for g in range(n):
        cfg = Config(network="default", default=LinkShape(latency=250 * MS),
                     callback_state=f"callback-{int(rng.integers(0, 1 << 62))}", callback_target=1)
        rel[g] = env.net.configure_network(g, cfg, t)
    env.time_to_shape_network = rel - t
    return rel >= 0


def subtree(env: PlanEnv) -> np.ndarray:
    """benchmarks.go:148-270 (SubtreeBench): every instance publishes its run id on "instances";
    the one with sequence number 1 publishes `subtree_iterations` items on each of the topics
    subtree_time_<size>_bytes (size 64 .. 4096, doubling), signals "handoff" and waits on "end"
    for the whole group; the others wait for "handoff", read `subtree_iterations` items of every
    topic, compare each with the published value and signal "end". The published value is the
    reference's `string(make([]byte, 0, size))` after rand.Read: zero bytes are read into a
    zero-length slice, so every item is the empty string."""
    n = env.n
    iterations = env.int_param("subtree_iterations", 2000)
    t = env.net.wait_network_initialized(0)
    seq = env.sync.publish("instances", np.arange(n), t, ["run"] * n)
    pub = int(np.flatnonzero(seq == 1)[0])
    sizes = []
    s = 64
    while s <= 4 * 1024:
        sizes.append(s)
        s <<= 1
    data = ""
    for size in sizes:
        env.sync.publish(f"subtree_time_{size}_bytes", np.full(iterations, pub), t, [data] * iterations)
    env.sync.signal_entry("handoff", [pub], t)
    ok = np.ones(n, bool)
    receivers = np.flatnonzero(np.arange(n) != pub)
    if len(receivers):
        t_h = env.sync.barrier("handoff", 1, t)
        for size in sizes:
            items = env.sync.subscribe(f"subtree_time_{size}_bytes", until_t=t_h)
            if len(items) < iterations or any(x != data for x in items[:iterations]):
                ok[receivers] = False
                env.fail(f"subtree_time_{size}_bytes: received unexpected value")
        env.sync.signal_entry("end", receivers, t_h)
    _, t_end = env.sync.signal_and_wait("end", [pub], t, n)
    if t_end < 0:
        ok[pub] = False
        env.fail("end never released")
    return ok


# ============================================================================================
# plans/placebo (the engine's own integration plan: outcome reporting)
# ============================================================================================

class PlanPanic(Exception):
    """A test case that panics: every instance of the run reports a CrashEvent (sdk-go runtime)."""


def placebo_ok(env: PlanEnv) -> np.ndarray:
    """plans/placebo/main.go:23-27: bind a sync client and return."""
    return np.ones(env.n, bool)


def placebo_panic(env: PlanEnv) -> np.ndarray:
    """plans/placebo/main.go:29-33: panic(errors.New("this is an intentional panic"))."""
    raise PlanPanic("this is an intentional panic")


def placebo_stall(env: PlanEnv) -> np.ndarray:
    """plans/placebo/main.go:35-40: sleep 24 hours, then return. Simulated time costs nothing while
    nothing is in flight: the run ends 24 simulated hours later (a wall-clock run timeout, the
    reference runners' way out of it, never fires)."""
    env.advance_to(24 * 3600 * SECOND)
    return np.ones(env.n, bool)


# ============================================================================================
# plans/example (the SDK's demonstration plan)
# ============================================================================================

def example_sync(env: PlanEnv) -> np.ndarray:
    """plans/example/sync.go:20-80 (ExampleSync): every instance signals "enrolled" at start; the
    one with sequence number 1 leads: it waits on Barrier("ready", N - 1), sleeps 1 + 5 s and
    signals "released"; each follower sleeps U{0..4} s, signals "ready" and waits on
    Barrier("released", 1). env.released = each follower's release time."""
    n = env.n
    rng = np.random.default_rng(env.int_param("seed", 0))
    seq = env.sync.signal_entry("enrolled", np.arange(n), 0)
    leader = int(np.flatnonzero(seq == 1)[0])
    followers = np.flatnonzero(np.arange(n) != leader)
    t_ready = rng.integers(0, 5, len(followers)) * SECOND
    if len(followers):
        env.sync.signal_entry("ready", followers, t_ready)
    t_all = env.sync.barrier("ready", len(followers), 0)
    ok = np.ones(n, bool)
    if t_all < 0:
        env.fail("the followers never became ready")
        return np.zeros(n, bool)
    env.sync.signal_entry("released", [leader], t_all + 6 * SECOND)
    env.released = np.array([env.sync.barrier("released", 1, int(t)) for t in t_ready], np.int64)
    ok[followers] = env.released >= 0
    return ok


def example_failure(env: PlanEnv) -> np.ndarray:
    """plans/example/failure.go:11-14: returns errors.New("intentional oops")."""
    env.fail("intentional oops")
    return np.zeros(env.n, bool)


def example_panic(env: PlanEnv) -> np.ndarray:
    """plans/example/panic.go:12: panic("intentional panic")."""
    raise PlanPanic("intentional panic")


# ============================================================================================
# plans/verify
# ============================================================================================

def _is_control_net(addr: str) -> bool:
    """verify/main.go:33-35: the local:docker and cluster:k8s control networks"""
    return addr.startswith("192.18.") or addr.startswith("100.96.")


def verify_uses_data_network(env: PlanEnv) -> np.ndarray:
    """plans/verify/main.go:43-130 (UsesDataNetwork): SignalAndWait("ready", N); the instance with
    sequence number 1 (targetmode) publishes the addresses of its control interface (eth0, on
    192.18.0.0/16) and its data interface (eth1) and "endOfNetworks" on topic "addrs", then signals
    "target-ready"; every other instance waits for it and pings each address 10 times, 500 ms
    apart with a 1 s timeout: the control address must lose 100 % of the pings, the data address
    0 % (:103-106). SignalAndWait("finished", N). A simulated instance routes only its data
    network (and, under AllowAll, the default route out of it), so a control address is outside
    everything it can reach."""
    n = env.n
    t = env.net.wait_network_initialized(0)
    seq, t = env.sync.signal_and_wait("ready", np.arange(n), t, n)
    target = int(np.flatnonzero(seq == 1)[0])
    data_ip = env.net.get_data_network_ip(target)
    addrs = [f"192.18.{(target >> 8) & 255}.{(target & 255) or 1}/16",
             f"{int_to_ip(data_ip)}/{env.sim.cfg.data_prefix_len}", "endOfNetworks"]
    env.sync.publish("addrs", [target] * len(addrs), t, addrs)
    env.sync.signal_entry("target-ready", [target], t)
    ok = np.ones(n, bool)
    pingers = np.flatnonzero(np.arange(n) != target)
    env.packet_loss = {}
    t_ready = env.sync.barrier("target-ready", 1, t)
    if len(pingers):
        env.advance_to(t_ready)
        for a in env.sync.subscribe("addrs", until_t=t_ready):
            if a == "endOfNetworks":
                break
            ip = a.split("/")[0]
            dst = target if ip == int_to_ip(data_ip) else A.DST_EXTERNAL
            t0 = env.sim.now
            src = np.repeat(pingers, 10)
            t_ping = t0 + np.tile(np.arange(10) * 500 * MS, len(pingers))
            got, _ = env.rpc(src, dst, 84, 84, t_ping, 1 * SECOND)     # ICMP echo: 56 B + 8 + 20
            loss = 100.0 * (1.0 - got.reshape(len(pingers), 10).mean(axis=1))
            env.packet_loss[a] = loss
            bad = loss != 100.0 if _is_control_net(ip) else loss > 0.0
            for g in pingers[bad]:
                env.fail(f"instance {g}: " + ("control network is accessible; it should not be" if _is_control_net(ip)
                                              else "data network is not accessible; it should be"))
            ok[pingers[bad]] = False
    _, t_fin = env.sync.signal_and_wait("finished", np.arange(n), max(env.sim.now, t_ready), n)
    return ok & (t_fin >= 0)


PLANS = {
    ("network", "ping-pong"): pingpong,
    ("network", "traffic-allowed"): traffic(AllowAll),
    ("network", "traffic-blocked"): traffic(DenyAll),
    ("splitbrain", "drop"): splitbrain(FilterAction.Drop),
    ("splitbrain", "reject"): splitbrain(FilterAction.Reject),
    ("splitbrain", "accept"): splitbrain(FilterAction.Accept),
    ("benchmarks", "storm"): storm,
    ("benchmarks", "barrier"): barrier_bench,
    ("benchmarks", "startup"): startup,
    ("benchmarks", "netinit"): netinit,
    ("benchmarks", "netlinkshape"): netlinkshape,
    ("benchmarks", "subtree"): subtree,
    ("verify", "uses-data-network"): verify_uses_data_network,
    ("placebo", "ok"): placebo_ok,
    ("placebo", "panic"): placebo_panic,
    ("placebo", "stall"): placebo_stall,
    ("example", "sync"): example_sync,
    ("example", "failure"): example_failure,
    ("example", "panic"): example_panic,
}
