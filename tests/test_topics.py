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


def _random_topics(binding, seed, n_inst=500, batches=40):
    """Mixed batches over several topics (and a signal state), payloads of 0..300 bytes; every
    position returned and every subscription (several from / until cuts) is recorded."""
    rng = np.random.default_rng(seed)
    sim = Simulator(SimConfig(n_instances=n_inst, max_states=64), binding=binding)
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
