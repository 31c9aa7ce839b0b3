"""sync.Client Publish / Subscribe as device-resident topic logs (tgsim_sync_publish /
tgsim_sync_subscribe). Semantics [EXT sdk-go]: ordered topics with full
history replay; positions are 1-based and, like SignalEntry sequence numbers, follow (t, instance)
order inside a batch (call sites: plans/network/pingpong.go:219-245, plans/benchmarks/storm.go:
232-255, plans/splitbrain/main.go:91-103)."""
import numpy as np
import pytest

from testground_amd import _abi as A
from testground_amd.sim import SimConfig, Simulator
from testground_amd.sync import SyncService


def _known_answers(binding):
    sim = Simulator(SimConfig(n_instances=16), binding=binding)
    sy = SyncService(sim)
    assert list(sy.publish("peers", [3, 1, 2], [5, 5, 1], ["a", {"x": 1}, [1, "b"]])) == [3, 2, 1]
    assert list(sy.publish("peers", [0], [7], ["z"])) == [4]
    assert sy.subscribe("peers") == [[1, "b"], {"x": 1}, "a", "z"]
    assert sy.subscribe("peers", until_t=5) == [[1, "b"], {"x": 1}, "a"]
    assert sy.subscribe("peers", until_t=0) == []
    assert sy.subscribe("nobody") == []
    tid = sy.state_id("topic:peers")
    inst, t, blobs = sim.subscribe(tid, from_pos=3)
    assert list(inst) == [3, 0] and list(t) == [5, 7] and blobs == [b'"a"', b'"z"']
    with pytest.raises(A.TgsimError) as e:                    # a batch may not go back in time
        sy.publish("peers", [4], [6], ["late"])
    assert e.value.code == A.ECAUSALITY
    # a topic counts like a state: SignalEntry on the same id continues the positions
    assert list(sim.publish([tid, tid], [9, 8], [9, 9], [b"", b"\x00\x01"])) == [6, 5]
    inst, t, blobs = sim.subscribe(tid, from_pos=5)
    assert list(inst) == [8, 9] and blobs == [b"\x00\x01", b""]
    sim.close()


def test_topics_known_answers_oracle(oracle):
    _known_answers(oracle)


@pytest.mark.gpu
def test_topics_known_answers_hip(hip):
    _known_answers(hip)


def _random_topics(binding, seed, n_inst=500, batches=40, restart=()):
    """Mixed batches over several topics (and a signal state), payloads of 0..300 bytes; every
    position returned and every subscription (several from / until cuts) is recorded. restart:
    batches after which the run is snapshotted and restored into a fresh context."""
    rng = np.random.default_rng(seed)
    cfg = SimConfig(n_instances=n_inst, max_states=64)
    sim = Simulator(cfg, binding=binding)
    out, t = [], 0
    for b in range(batches):
        n = int(rng.integers(1, 400))
        topics = rng.integers(0, 6, n).astype(np.uint32)
        inst = rng.integers(0, n_inst, n).astype(np.uint32)
        tt = t + rng.integers(0, 1000, n)
        payloads = [rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes() for _ in range(n)]
        out.append(sim.publish(topics, inst, tt, payloads))
        t = int(tt.max())
        if b % 7 == 3:
            out.append(sim.signal(np.full(5, 7), rng.integers(0, n_inst, 5), np.full(5, t)))
        if b in restart:
            image = sim.snapshot()
            sim.close()
            sim = Simulator(cfg, binding=binding)
            sim.restore(image)
    for topic in range(7):
        for frm in (1, 2, 50, 10_000):
            for until in (t // 3, t, (1 << 63) - 1):
                inst, ts, blobs = sim.subscribe(topic, frm, until)
                out.append((topic, frm, until, inst, ts, b"|".join(blobs), [len(x) for x in blobs]))
    sim.close()
    return out


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if isinstance(x, tuple):
            for u, v in zip(x, y):
                assert np.array_equal(np.asarray(u), np.asarray(v)) if isinstance(u, np.ndarray) else u == v
        else:
            assert np.array_equal(x, y)


def test_random_topics_properties_oracle(oracle):
    out = _random_topics(oracle, 1)
    for x in out:
        if isinstance(x, tuple):
            _, frm, until, inst, ts, _, _ = x
            assert np.all(np.diff(ts) >= 0) and (len(ts) == 0 or ts.max() <= until)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_random_topics_hip_matches_oracle(hip, oracle, seed):
    _same(_random_topics(hip, seed), _random_topics(oracle, seed))


@pytest.mark.gpu
def test_random_topics_resumed_matches_oracle(hip, oracle):
    """topic arenas and runs through tgsim_snapshot / tgsim_restore (a fresh context's arenas grow
    to the image's)"""
    _same(_random_topics(hip, 3, restart={0, 11, 25}), _random_topics(oracle, 3))


def _publish_random(sim, rng, n_inst, batches):
    t = 0
    for b in range(batches):
        n = int(rng.integers(1, 400))
        topics = rng.integers(0, 6, n).astype(np.uint32)
        inst = rng.integers(0, n_inst, n).astype(np.uint32)
        tt = t + rng.integers(0, 1000, n)
        payloads = [rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes() for _ in range(n)]
        sim.publish(topics, inst, tt, payloads)
        t = int(tt.max())
        if b % 7 == 3:
            sim.signal(np.full(5, 7), rng.integers(0, n_inst, 5), np.full(5, t))
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 4])
def test_subscribe_device_matches_oracle(hip, oracle, seed):
    """A batch of subscribers on the device (tgsim_sync_subscribe_device) reads, per subscriber,
    exactly the entries the oracle's Subscribe returns for (topic, from, until), cut at cap_each;
    topics past max_states and from = 0 read nothing; ids past entries_cap are not written."""
    import torch
    n_inst, batches = 500, 30
    sims = [Simulator(SimConfig(n_instances=n_inst, max_states=64), binding=b) for b in (hip, oracle)]
    t_last = [_publish_random(s, np.random.default_rng(seed), n_inst, batches) for s in sims][0]
    rng = np.random.default_rng(100 + seed)
    m = 3000
    topics = rng.integers(0, 9, m)
    topics[::97] = 64 + rng.integers(0, 5, len(topics[::97]))   # beyond max_states: empty
    frm = rng.integers(0, 1500, m)
    frm[::5] = 1
    until = rng.integers(0, t_last + 2, m)
    until[::3] = (1 << 63) - 1
    cap_each = 700
    dev = torch.device("cuda:0")
    tt = lambda a, d: torch.tensor(a, dtype=d, device=dev)
    offs, ids = sims[0].subscribe_device(tt(topics, torch.int32), tt(frm, torch.int32), tt(until, torch.int64), cap_each)
    offs, ids = offs.cpu().numpy(), ids.cpu().numpy()
    ar = sims[0].topic_arena()
    total = 0
    for i in range(m):
        if topics[i] >= 64 or frm[i] == 0:
            want_inst, want_t, want_b = [], [], []
        else:
            want_inst, want_t, want_b = sims[1].subscribe(int(topics[i]), int(frm[i]), int(until[i]))
            want_inst, want_t, want_b = want_inst[:cap_each], want_t[:cap_each], want_b[:cap_each]
        e = ids[offs[i]:offs[i + 1]]
        assert len(e) == len(want_inst), i
        assert np.array_equal(ar["instance"][e], want_inst) and np.array_equal(ar["t"][e], want_t)
        got_b = [ar["payload"][int(ar["payload_off"][k]):int(ar["payload_off"][k]) + int(ar["payload_len"][k])].tobytes()
                 for k in e]
        assert got_b == list(want_b)
        total += len(e)
    assert offs[m] == total and total > 0
    # counts only, then a short inbox buffer: the prefix that fits is written, the rest is not
    o2, none = sims[0].subscribe_device(tt(topics, torch.int32), tt(frm, torch.int32), tt(until, torch.int64), cap_each,
                                        entries=False)
    assert none is None and np.array_equal(o2.cpu().numpy(), offs)
    cut = total // 2
    _, short = sims[0].subscribe_device(tt(topics, torch.int32), tt(frm, torch.int32), tt(until, torch.int64), cap_each,
                                        entries_cap=cut)
    assert np.array_equal(short.cpu().numpy()[:cut], ids[:cut])
    for s in sims:
        s.close()


@pytest.mark.gpu
def test_address_exchange_fanout_on_device(hip):
    """storm.go:232-255 at 20k instances: every instance publishes its address, then every instance
    replays the whole topic — 4e8 deliveries written into per-subscriber inboxes on the device."""
    import torch
    n = 20_000
    sim = Simulator(SimConfig(n_instances=n, max_states=16), binding=hip)
    rng = np.random.default_rng(9)
    t_pub = np.sort(rng.integers(0, 10**6, n))
    order = rng.permutation(n).astype(np.uint32)
    payloads = [b"/ip4/16.0.%d.%d/tcp/2000" % (g >> 8, g & 255) for g in order]
    half = n // 2   # two publish batches (two runs), the second later in time
    sim.publish(0, order[:half], t_pub[:half], payloads[:half])
    sim.publish(0, order[half:], t_pub[half:], payloads[half:])
    dev = torch.device("cuda:0")
    subs = torch.zeros(n, dtype=torch.int32, device=dev)
    offs, ids = sim.subscribe_device(subs, subs + 1, torch.full((n,), 1 << 62, dtype=torch.int64, device=dev))
    assert int(offs[-1]) == n * n
    assert torch.equal(offs[:-1], torch.arange(n, device=dev, dtype=torch.int64) * n)
    # every inbox is the whole log in position order: entry ids 0..n-1 (one batch appends its
    # entries in position order)
    ref = torch.arange(n, device=dev, dtype=torch.int32)
    assert bool((ids.view(n, n) == ref).all())
    # a subscriber that stops at the first batch's last time sees exactly that batch
    cut = torch.full((1,), int(t_pub[half - 1]), dtype=torch.int64, device=dev)
    o1, _ = sim.subscribe_device(subs[:1], subs[:1] + 1, cut, entries=False)
    assert int(o1[-1]) == int(np.sum(t_pub <= t_pub[half - 1]))
    ar = sim.topic_arena()
    assert sorted(ar["instance"].tolist()) == list(range(n))
    sim.close()
