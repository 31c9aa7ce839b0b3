"""CPU: the reference's own known answers for this path, through the host-side mirrors of its
interfaces (sidecar.Network, network.Client, sync.Client, api.Runner) over the CPU oracle.

  pkg/sidecar/sidecar_test.go:19-93   initial config, empty-callback error, config pass-through
  plans/network/pingpong.go:185,195   RTT in [200, 215] ms at 100 ms/side, [20, 35] ms at 10 ms
  plans/network/traffic.go:46-52      external traffic blocked under DenyAll, allowed under AllowAll
  plans/splitbrain/main.go:50-58      errors exactly between regions A and B unless "accept"
  plans/benchmarks/benchmarks.go      barrier ladder (Go float loop 0.2 .. 1.0)
  plans/benchmarks/storm.go           every dial and write completes without shaping
"""
import io
import tarfile

import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd import plans as P
from testground_amd.network import MS, Config, LinkShape
from testground_amd.runner import LocalMI355XRunner, RunGroup, RunInput
from testground_amd.sidecar import ERR_NO_CALLBACK, NET_INIT_STATE


def env_for(oracle, n, case="", params=None, **kw):
    return P.PlanEnv(n, seed=1, test_case=case, params=params, binding=oracle, **kw)


# ---- pkg/sidecar/sidecar_test.go ---------------------------------------------------------------

def test_network_initialize(oracle):
    """TestNetworkInitialize: the handler configures the network once at init, and
    WaitNetworkInitialized returns once every sidecar signalled network-initialized."""
    env = env_for(oracle, 1)
    env.net.wait_network_initialized(0)
    assert len(env.sidecar.network(0).configured) == 1
    assert env.sync.count(NET_INIT_STATE) == 1
    assert env.sidecar.network(0).list_active() == ["default"]
    env.close()


def test_network_configured_fails_misconfigured(oracle):
    """TestNetworkConfiguredFailsMisconfigured: a Config without CallbackState is refused with the
    SDK's message."""
    env = env_for(oracle, 1)
    with pytest.raises(ValueError, match="^" + ERR_NO_CALLBACK + "$"):
        env.net.configure_network(0, Config(), 0)
    env.close()


def test_network_configured_passes_config_unmodified(oracle):
    """TestNetworkConfigured: the sidecar passes the config on to the backing network unmodified
    and the plan's barrier releases once the sidecar signalled the callback state."""
    env = env_for(oracle, 1)
    cfg = Config(network="default", enable=True, callback_state="reconfigured",
                 default=LinkShape(latency=3600 * 10 ** 9))
    rel = env.net.configure_network(0, cfg, 5)
    assert rel == 5
    net = env.sidecar.network(0)
    assert len(net.configured) == 2
    assert net.active["default"] == cfg and net.active["default"] is not cfg
    env.close()


def test_unsupported_network(oracle):
    env = env_for(oracle, 1)
    with pytest.raises(A.TgsimError) as e:
        env.net.configure_network(0, Config(network="other", enable=True, callback_state="x"), 0)
    assert e.value.code == A.EUNSUPPORTED_NETWORK and "unsupported network: other" in str(e.value)
    env.close()


def test_callback_target_defaults_to_all_instances(oracle):
    env = env_for(oracle, 3)
    cfg = Config(network="default", enable=True, callback_state="cb")
    assert env.net.configure_network(0, cfg, 10) == -1        # 1 of 3 sidecars signalled
    assert env.net.configure_network(1, cfg, 20) == -1
    assert env.net.configure_network(2, cfg, 30) == 30        # the third releases everyone
    cfg1 = Config(network="default", enable=True, callback_state="cb1", callback_target=1)
    assert env.net.configure_network(0, cfg1, 40) == 40
    env.close()


# ---- plans ---------------------------------------------------------------------------------------

def test_pingpong_rtt_windows(oracle):
    env = env_for(oracle, 2)
    ok = P.pingpong(env)
    assert ok.all(), env.failures
    rtt100, rtt10 = env.rtts
    assert all(200 * MS <= r <= 215 * MS for r in rtt100)
    assert all(20 * MS <= r <= 35 * MS for r in rtt10)
    ips = sorted(env.net.get_data_network_ip(g) & 0xFFFF for g in range(2))
    assert ips == [0x0101, 0x0102]      # pingpong.go:57-60: x.y.(seq>>8 + 1).seq for seq 1, 2
    env.close()


def test_pingpong_fails_outside_window_with_more_latency(oracle, monkeypatch):
    """The RTT check is live: 120 ms per side breaks the [200, 215] ms window."""
    env = env_for(oracle, 2)
    orig = P.Config

    def patched(**kw):
        c = orig(**kw)
        if c.default.latency == 100 * MS:
            c.default.latency = 120 * MS
        return c
    monkeypatch.setattr(P, "Config", patched)
    ok = P.pingpong(env)
    assert not ok.all() and any("expected an RTT" in f for f in env.failures)
    env.close()


@pytest.mark.parametrize("case,expect_ok", [("traffic-allowed", True), ("traffic-blocked", True)])
def test_routing_policy(oracle, case, expect_ok):
    env = env_for(oracle, 3)
    ok = P.PLANS[("network", case)](env)
    assert ok.all() == expect_ok, env.failures
    env.close()


@pytest.mark.parametrize("n", [12, 30])
@pytest.mark.parametrize("case", ["drop", "reject", "accept"])
def test_splitbrain_truth_table(oracle, case, n):
    """main.go:50-58 over sequential probes: errors exactly between regions A and B. B -> A probes
    wait out the one-minute timeout (A's rule drops the reply), so with 10 region-A nodes (n = 30)
    region B is still probing when the plan's 300 s context expires (main.go:64) and every
    SignalAndWait("testcomplete") fails, as in the reference; with 4 (n = 12) it finishes."""
    env = env_for(oracle, n, case)
    ok = P.PLANS[("splitbrain", case)](env)
    region = env.region
    assert list(region) == [(g + 1) % 3 for g in range(n)]   # seq = g + 1 (ties broken by instance)
    na, nb = (region == 0).sum(), (region == 1).sum()
    want = np.zeros(n, np.int64)
    if case != "accept":
        want[region == 0] = nb
        want[region == 1] = na
    assert np.array_equal(env.probe_errors, want)
    assert not env.probe_unexpected.any()
    out, order = env.probe_outcome, np.argsort(np.arange(n))   # topic order = instance order here
    if case != "accept":
        a, b = np.flatnonzero(region == 0), np.flatnonzero(region == 1)
        assert np.all(out[np.ix_(a, b)] == A.PROBE_REFUSED)      # A's own route refuses: immediate
        assert np.all(out[np.ix_(b, a)] == A.PROBE_TIMEOUT)      # A drops the reply: one minute
    slow = 10 * 60 * P.SECOND if case != "accept" else 0
    if case == "accept" or n == 12:
        assert ok.all(), env.failures
        assert env.testcomplete < P.SPLITBRAIN_CTX_NS
    else:
        assert not ok.any() and any("context deadline exceeded" in f for f in env.failures)
        assert env.testcomplete > slow
    env.close()


def test_splitbrain_accept_1200(oracle):
    """splitbrain accept at 1,200 instances passes (sequential probes; the all-at-once
    descriptor of round 2 tail-dropped 437,800 probes at this size)."""
    n = 1200
    env = env_for(oracle, n, "accept")
    ok = P.PLANS[("splitbrain", "accept")](env)
    assert ok.all(), env.failures[:3]
    assert np.all(env.probe_outcome.sum(axis=1) == n - 1)       # n - 1 probes OK per node
    assert env.sim.stats()["overlimit"] == 0
    env.close()


def test_barrier_bench(oracle):
    env = env_for(oracle, 50, params={"barrier_iterations": 3})
    ok = P.barrier_bench(env)
    assert ok.all()
    # the Go float loop yields 0.2, 0.4, 0.6000000000000001, 0.8, 1.0
    assert sorted(env.barrier_times) == sorted(f"barrier_time_{p}_percent" for p in (20, 40, 60, 80, 100))
    assert all(len(v) == 3 for v in env.barrier_times.values())
    env.close()


def test_benchmark_small_cases(oracle):
    """benchmarks.go:20-86 / 148-270: startup, netinit, netlinkshape, subtree"""
    env = env_for(oracle, 6, "startup")
    assert P.startup(env).all() and env.time_to_start.max() == 0
    env.close()
    env = env_for(oracle, 6, "netinit")
    assert P.netinit(env).all()
    env.close()
    env = env_for(oracle, 6, "netlinkshape", params={"seed": "3"})
    assert P.netlinkshape(env).all() and np.all(env.time_to_shape_network >= 0)
    # Enable stays false in the plan's config: the sidecar disconnects every data link
    assert not any(env.sidecar.network(g).list_active() for g in range(6))
    env.close()
    env = env_for(oracle, 5, "subtree", params={"subtree_iterations": "50"})
    assert P.subtree(env).all() and not env.failures
    assert env.sync.count("end") == 5 and env.sync.count("handoff") == 1
    assert len(env.sync.subscribe("subtree_time_4096_bytes")) == 50
    env.close()


def test_verify_uses_data_network(oracle):
    """plans/verify/main.go:103-106: pings to the target's control address lose 100 %, to its data
    address 0 %"""
    env = env_for(oracle, 4, "uses-data-network")
    ok = P.verify_uses_data_network(env)
    assert ok.all() and not env.failures
    (ctl, c_loss), (dat, d_loss) = env.packet_loss.items()
    assert ctl.startswith("192.18.") and np.all(c_loss == 100.0)
    assert dat.startswith("16.0.") and np.all(d_loss == 0.0)
    env.close()


STORM_TOML = {"conn_count": "10", "conn_outgoing": "10", "conn_delay_ms": "30000", "concurrent_dials": "2",
              "data_size_kb": "1024"}   # plans/benchmarks/compositions/storm.toml:18-23 (50 instances)


def storm_toml_run(binding, transport, n=50):
    env = env_for(binding, n, "storm", params=dict(STORM_TOML, transport=transport))
    ok = P.storm(env)
    # "windows" is the oracle's own bookkeeping (the HIP library ends windows on the device and does
    # not count them); the plan-level window counts are compared through the plan's own state
    stats = {k: v for k, v in env.sim.stats().items() if k != "windows"}
    res = dict(ok=ok, failures=list(env.failures), stats=stats, now=env.sim.now, chunks=env.delivered_chunks,
               dials=env.dials_ok, bytes=env.bytes_sent)
    if transport == "tcp":
        res["tcp"] = env.sim.tcp_stats()
    env.close()
    return res


@pytest.mark.parametrize("transport", ["message", "tcp"])
def test_storm_toml_passes(oracle, transport):
    """the reference's own storm composition (50 x 10 dials x 1024 KiB in 4 KiB
    writes, concurrent_dials 2, unshaped) passes - 50/50 with no tail drops - once dials and writes
    are paced as storm.go paces them (dial / write semaphores, writes blocking on the send buffer;
    TCP: the Reno window). Round 2's all-at-once descriptor gave 0/50 with 78,000 tail drops."""
    r = storm_toml_run(oracle, transport)
    assert r["ok"].all(), r["failures"][:3]
    assert r["stats"]["overlimit"] == 0 and r["dials"] == 500 and r["bytes"] == 500 * 1024 * 1024
    assert r["chunks"] == 500 * 256
    if transport == "tcp":
        assert r["tcp"]["retransmissions"] == 0 and r["tcp"]["failed"] == 0 and r["tcp"]["delivered"] == 500 * 257


def test_storm_completes(oracle):
    env = env_for(oracle, 20, params={"conn_outgoing": 3, "conn_delay_ms": 1000, "data_size_kb": 10})
    ok = P.storm(env)
    assert ok.all(), env.failures
    assert env.delivered_chunks == 20 * 3 * 3          # 10 KiB in 4 KiB writes = 3 chunks per dial
    env.close()


# ---- api.Runner -----------------------------------------------------------------------------------

def test_runner_contract(oracle):
    r = LocalMI355XRunner(binding=oracle)
    assert r.id() == "local:mi355x"
    assert "exec:go" in r.compatible_builders()
    assert r.config_type()().window_ns == 1 * MS
    job = RunInput(run_id="r1", test_plan="splitbrain", test_case="drop", total_instances=12,
                   groups=[RunGroup("left", 5), RunGroup("right", 7)])
    out = r.run(job, io.StringIO())
    assert out.result.outcome == "success"
    assert {k: (v.total, v.ok) for k, v in out.result.outcomes.items()} == {"left": (5, 5), "right": (7, 7)}
    buf = io.BytesIO()
    r.collect_outputs("r1", buf)
    buf.seek(0)
    with tarfile.open(fileobj=buf, mode="r:gz") as tar:
        assert tar.getnames() == ["r1/result.json"]


def test_runner_reports_failures(oracle, monkeypatch):
    r = LocalMI355XRunner(binding=oracle)
    monkeypatch.setitem(P.PLANS, ("x", "y"), lambda env: np.arange(env.n) % 2 == 0)
    ow = io.StringIO()
    out = r.run(RunInput("r2", "x", "y", 4, [RunGroup("g", 4)]), ow)
    assert out.result.outcome == "failure" and out.result.outcomes["g"].ok == 2
    lines = ow.getvalue().splitlines()
    # pretty.go: START and an outcome per instance, then the printer's "N nodes failed"
    assert sum(" START " in x for x in lines) == 4 and sum("     OK << g[" in x for x in lines) == 2
    assert [x.split("<< ")[1].split(" >>")[0] for x in lines if "  FAIL << " in x] == ["g[1]", "g[3]"]
    assert "2 nodes failed" in lines and lines[-1] == "local:mi355x run r2: failure"


def test_runner_event_stream_and_printer():
    """collectOutcomes counts SuccessEvents per group and stops after every instance reported
    (local_docker.go:216-255); an instance with no outcome event is INCOMPLETE (pretty.go:127-135)."""
    from testground_amd.runner import (GroupOutcome, PrettyPrinter, Result, collect_outcomes, failure_event,
                                       start_event, success_event)
    res = Result(outcomes={"a": GroupOutcome(total=2), "b": GroupOutcome(total=1)})
    evs = [{"ts": 0, "event": start_event("a", {})}, {"ts": 5, "event": success_event("a")},
           {"ts": 6, "event": failure_event("b", "boom")}, {"ts": 7, "event": success_event("a")},
           {"ts": 8, "event": success_event("b")}]   # after every instance reported: not counted
    collect_outcomes(evs, res)
    assert (res.outcomes["a"].ok, res.outcomes["b"].ok, res.outcome) == (2, 0, "failure")
    ow = io.StringIO()
    pp = PrettyPrinter(ow)
    pp.manage("x[0]", [{"ts": 1_500_000_000, "event": start_event("x", {"TestPlan": "p"})}])
    pp.manage("x[1]", [{"ts": 2_000_000_000, "event": success_event("x")}])
    out = ow.getvalue().splitlines()
    assert out[0] == '1.5000s      START << x[0] >> {"TestGroupID": "x", "TestPlan": "p"}'
    assert out[1] == "0.0000s INCOMPLETE << x[0] >> " and out[2] == "2.0000s         OK << x[1] >> "
    assert pp.wait() == "1 nodes failed"


def test_runner_rejects_unknown_plan(oracle):
    r = LocalMI355XRunner(binding=oracle)
    with pytest.raises(ValueError, match="no workload descriptor"):
        r.run(RunInput("r3", "network", "nope", 2, [RunGroup("g", 2)]))
    with pytest.raises(ValueError, match="TotalInstances"):
        r.run(RunInput("r4", "network", "ping-pong", 3, [RunGroup("g", 2)]))


@pytest.mark.gpu
@pytest.mark.parametrize("plan,case,params", [("benchmarks", "netlinkshape", {"seed": "3"}),
                                              ("benchmarks", "subtree", {"subtree_iterations": "50"}),
                                              ("verify", "uses-data-network", {})])
def test_small_plan_cases_hip(hip, oracle, plan, case, params):
    out = []
    for b in (hip, oracle):
        env = P.PlanEnv(6, seed=1, test_case=case, params=params, binding=b)
        ok = P.PLANS[(plan, case)](env)
        out.append((ok.tolist(), env.sim.now, env.sync.count("end") if case == "subtree" else 0,
                    getattr(env, "time_to_shape_network", np.zeros(0)).tolist(),
                    {k: v.tolist() for k, v in getattr(env, "packet_loss", {}).items()}))
        env.close()
    assert out[0] == out[1] and all(out[0][0])


def test_placebo_outcomes(oracle):
    """plans/placebo through the runner: ok succeeds, panic crashes every instance (CrashEvent,
    counted not-ok as collectOutcomes does), stall ends 24 simulated hours later"""
    r = LocalMI355XRunner(binding=oracle)
    outs = {}
    for case in ("ok", "panic", "stall"):
        job = RunInput(run_id=f"placebo-{case}", test_plan="placebo", test_case=case, total_instances=3,
                       groups=[RunGroup(id="single", instances=3)])
        w = io.StringIO()
        outs[case] = (r.run(job, w).result, w.getvalue())
    assert outs["ok"][0].outcome == "success" and outs["stall"][0].outcome == "success"
    res, text = outs["panic"]
    assert res.outcome == "failure" and res.outcomes["single"].ok == 0
    assert text.count("CRASH") == 3 and "this is an intentional panic" in text


def test_example_sync_leader_releases_followers(oracle):
    """plans/example/sync.go: the leader (sequence 1 of "enrolled") releases every follower 6 s
    after the last one is ready"""
    env = env_for(oracle, 7, "sync", params={"seed": "4"})
    ok = P.example_sync(env)
    assert ok.all()
    rng = np.random.default_rng(4)
    t_ready = rng.integers(0, 5, 6) * 1_000_000_000
    assert np.all(env.released == t_ready.max() + 6_000_000_000)
    env.close()


def test_example_failure_through_the_runner(oracle):
    job = RunInput(run_id="ex-fail", test_plan="example", test_case="failure", total_instances=2,
                   groups=[RunGroup(id="g", instances=2)])
    w = io.StringIO()
    res = LocalMI355XRunner(binding=oracle).run(job, w).result
    assert res.outcome == "failure" and w.getvalue().count("FAIL") >= 2 and "intentional oops" in w.getvalue()


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["message", "tcp"])
def test_storm_toml_hip_matches_oracle(hip, oracle, transport):
    a, b = storm_toml_run(hip, transport), storm_toml_run(oracle, transport)
    assert a["ok"].all() and np.array_equal(a["ok"], b["ok"])
    for k in ("stats", "now", "chunks", "dials", "bytes") + (("tcp",) if transport == "tcp" else ()):
        assert a[k] == b[k], k
