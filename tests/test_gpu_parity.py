"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the committed golden
fixtures, on identical seeded inputs. Bit-exact on every observable: statuses, delivery records
(all fields), inbox offsets, counters, sync sequence numbers and barrier release times."""
import numpy as np
import pytest

from testground_amd import _abi as A
from tests import golden_check as GC
from tests import scenarios as S
from tests import semantics_cases as SC
from tests.golden import make_golden as G

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_random_windows(hip, oracle, seed):
    S.assert_same(S.run_random(hip, seed), S.run_random(oracle, seed))


def test_random_windows_small_wheel(hip, oracle):
    kw = dict(wheel_slot_ns=3_000_000, wheel_slots=8)
    S.assert_same(S.run_random(hip, 11, cfg_kw=kw), S.run_random(oracle, 11, cfg_kw=kw))


@pytest.mark.parametrize("seed", [1, 2])
def test_bandwidth_limits_switched_mid_run(hip, oracle, seed):
    """The token-bucket stage is skipped until a sender is first limited, and kept after its limit
    is lifted while its copies are in flight (tests/scenarios.py run_limit_switch)."""
    S.assert_same(S.run_limit_switch(hip, seed), S.run_limit_switch(oracle, seed))


@pytest.mark.parametrize("n_inst", [64, 200, 1000])
def test_large_segments(hip, oracle, n_inst):
    S.assert_same(S.run_heavy(hip, 7, n_inst), S.run_heavy(oracle, 7, n_inst))


def test_many_large_segments(hip, oracle):
    """k_rest's task-parallel sort of several large segments at once."""
    a = S.run_many_large(hip, 11)
    S.assert_same(a, S.run_many_large(oracle, 11))
    assert max(np.diff(x["inbox"]).max() for x in a[:3]) > 8192


@pytest.mark.parametrize("seed", [1, 2])
def test_whole_inbox_sort(hip, oracle, seed):
    """Several long inboxes in one window - arrival ties with clone ties, arrivals over 1 us, a
    clustered one, arrivals over 20 ms, one of 15k - through k_rest's tasks. In the experiment build
    (-DTGSIM_WHOLE_SORT, loaded with TGSIM_LIB) the narrow ones are sorted by one workgroup in LDS
    instead (whole_sort) and the others handed back to the tasks: same outputs."""
    kc = []
    a = S.run_whole_inbox(hip, seed, counters=kc)
    S.assert_same(a, S.run_whole_inbox(oracle, seed))
    whole = np.diff([0] + [k["long_whole"] for k in kc])
    emit = np.diff([0] + [k["long_emit"] for k in kc])
    assert emit[0] > 25000 and emit[1] > 7000 and emit[2] > 3000 and emit[3] > 3000
    if whole.any():  # the experiment build
        assert whole[0] > 7000 and emit[0] > whole[0] + 12000   # two ~5k inboxes whole, the 15k one by tasks
        assert whole[1] == emit[1]                              # spread over 1 us: whole
        assert whole[2] == 0 and whole[3] == 0                  # clustered / wide keys: handed back


@pytest.mark.parametrize("seed", [1, 2])
def test_bucket_overflow_spans(hip, oracle, seed):
    """Fused buckets over their item capacity on the token bucket and the deliveries: their keys go
    to k_rest in spans of several keys (kMediumSpans), HIP = oracle."""
    kc = []
    a = S.run_bucket_overflow(hip, seed, counters=kc)
    S.assert_same(a, S.run_bucket_overflow(oracle, seed))
    assert kc[-1]["long_emit"] > 100_000 and kc[-1]["long_tb"] > 10_000  # the global form ran on both


@pytest.mark.parametrize("seed", [1, 2])
def test_token_bucket_rest_forms(hip, oracle, seed):
    """Busy and quiet token-bucket windows in runs: k_rest<TB> inside the window end's first launch
    and in a launch of its own (the host hint after a busy window), HIP = oracle."""
    kc = []
    a = S.run_rest_hint(hip, seed, counters=kc)
    S.assert_same(a, S.run_rest_hint(oracle, seed))
    longs = [kc[0]["long_tb"]] + [y["long_tb"] - x["long_tb"] for x, y in zip(kc, kc[1:])]
    assert all(v > 0 for v, b in zip(longs, (1, 1, 0, 1, 0, 0, 1, 1)) if b)  # every busy window went to k_rest


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_queue_limit_bursts(hip, oracle, seed):
    """netem's 1000-packet queue under every shape kind, across windows."""
    a, b = S.run_burst(hip, seed), S.run_burst(oracle, seed)
    S.assert_same(a, b)
    assert a[-1]["stats"]["overlimit"] > 1000


@pytest.mark.parametrize("seed", [1, 2])
def test_queue_limit_whole_sender(hip, oracle, seed):
    """k_shape_seq_wide and its fallbacks (repeated (t_send, seq), wide send spread, > 1024 messages,
    token bucket, no closed form) against the oracle's walk."""
    kc = {}
    a, b = S.run_wide(hip, seed, counters=kc), S.run_wide(oracle, seed)
    S.assert_same(a, b)
    assert a[-1]["stats"]["overlimit"] > 1000
    assert 0 < kc["wide"] < kc["deferred"]  # both lanes took senders


def test_sync_service(hip, oracle):
    S.assert_same(S.run_sync(hip, 3), S.run_sync(oracle, 3))


def test_storm_rounds(hip, oracle):
    S.assert_same(S.run_storm(hip), S.run_storm(oracle))


@pytest.mark.parametrize("n_inst,fanout", [(12, 10), (300, 5), (64, 1), (100, 32), (33, 3)])
def test_storm_fanouts(hip, oracle, n_inst, fanout):
    """Lane groups of the next power of two >= fanout; small populations force repeated draws
    (the lane-by-lane redraw of k_gen_storm) in most groups."""
    S.assert_same(S.run_storm(hip, n_inst=n_inst, rounds=3, fanout=fanout),
                  S.run_storm(oracle, n_inst=n_inst, rounds=3, fanout=fanout))


@pytest.mark.parametrize("case", SC.CASES, ids=lambda f: f.__name__[5:])
def test_semantics_hip(hip, case):
    case(hip)


@pytest.mark.parametrize("name", [s[0] for s in G.SCENARIOS])
def test_hip_matches_golden_scenario(hip, name):
    assert GC.check_scenario(hip, name) > 0


def test_hip_matches_golden_plans(hip):
    GC.check_plans(hip)


@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2)])
def test_sharded_on_one_device(hip, oracle, world, seed):
    """world shards of one run as separate contexts on cuda:0; the all-to-all is a set of
    device-to-device copies between their exchange buffers (the RCCL exchange of bench.py moves the
    same blocks between GPUs)."""
    import ctypes as C
    from testground_amd.sim import Simulator
    hiprt = C.CDLL("libamdhip64.so")
    hiprt.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    D2D = 3  # hipMemcpyDeviceToDevice

    def make(c):
        return Simulator(c)

    def exchange(sims):
        n = len(sims)
        bufs = [s.exchange_buffers() for s in sims]
        blk = bufs[0][2] // n
        for s in sims:
            s.sync()
        for q in range(n):
            for p in range(n):
                assert hiprt.hipMemcpy(bufs[p][1] + q * blk, bufs[q][0] + p * blk, blk, D2D) == 0
        # hipMemcpy D2D may return before the copy completes, and the contexts' streams are
        # non-blocking: finish the copies before any context reads its receive blocks
        assert hiprt.hipDeviceSynchronize() == 0

    outs, srcs = S.run_random_sharded(make, exchange, world, seed)
    S.assert_sharded_matches(outs, srcs, S.run_random(oracle, seed), world)


def _hip_with_transport(tr):
    from testground_amd.sim import Simulator

    def make(c):
        sim = Simulator(c)
        sim.set_transport(tr)
        return sim
    return make


@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2)])
def test_transport_on_one_device(hip, oracle, world, seed):
    """HIP shards on one GPU, one thread each, driven with the single-shard calls: the window's
    exchange runs inside tgsim_advance through a transport (device-to-device block copies here; the
    library's RCCL communicator between GPUs), equal to the single-shard oracle run."""
    outs = S.sharded_threads(world, lambda k, tr: S.run_random_sharded(
        _hip_with_transport(tr), None, world, seed, local=[k])[0][0], device=True)
    _, srcs = S.run_random_sharded(lambda c: S.Simulator(c, binding=oracle), S.memmove_exchange, world, seed)
    S.assert_sharded_matches(outs, srcs, S.run_random(oracle, seed), world)


@pytest.mark.parametrize("world,seed", [(2, 1), (3, 2)])
def test_transport_tight_exchange_on_one_device(hip, oracle, world, seed):
    """As above with the smallest sliced exchange block (exchange_cap 513: eight slices of 64
    records, include/tgsim.h): a few busy workgroups overrun their slices, and the token bucket's
    run spills into the next slice and the per-wave pushes rotate slices, so the capacity the block
    has is usable - no ECAPACITY, equal to the oracle."""
    outs = S.sharded_threads(world, lambda k, tr: S.run_random_sharded(
        _hip_with_transport(tr), None, world, seed, local=[k], exchange_cap=513)[0][0], device=True)
    _, srcs = S.run_random_sharded(lambda c: S.Simulator(c, binding=oracle), S.memmove_exchange, world, seed)
    S.assert_sharded_matches(outs, srcs, S.run_random(oracle, seed), world)


@pytest.mark.parametrize("n_msgs,ok", [(448, True), (512, True), (513, False)])
def test_skewed_exchange_on_one_device(hip, oracle, n_msgs, ok):
    """one or two netem workgroups send every record of a window to one peer, 7-8x a
    slice's 64 records (exchange_cap 513). Each overflowing wave goes on through the peer's other
    slices, so the device takes the whole block's 512 like the oracle (bit-exact) and refuses 513."""
    a, b = S.run_skewed_exchange(hip, n_msgs, device=True), S.run_skewed_exchange(oracle, n_msgs)
    if ok:
        assert [x[0] for x in a] == ["ok", "ok"], a
        S.assert_same(a, b)
    else:
        assert a[0] == ("err", A.ECAPACITY) and b[0] == ("err", A.ECAPACITY)


@pytest.mark.parametrize("world", [2, 4])
def test_storm_transport_on_one_device(hip, oracle, world):
    """bench.py's storm step on HIP shards: the storm batch's MAX all-reduce and the exchange go
    through the transport, rounds at the device clock (speculative generation); equal to the
    single-shard oracle run."""
    n, rounds = 2000, 6
    outs = S.sharded_threads(world, lambda k, tr: S.run_storm(
        hip, n_inst=n, rounds=rounds, cfg_kw=S.shard_cfg(world, k, exchange_cap=1 << 15),
        setup=lambda sim: sim.set_transport(tr), t_now=True), device=True)
    S.assert_storm_sharded(outs, S.run_storm(oracle, n_inst=n, rounds=rounds), world, n)


@pytest.mark.gpu
def test_rccl_communicator_one_rank(hip, oracle):
    """The native communicator comes up on the box (unique id, bootstrap, ncclCommInitRank - what
    bench.py --gpus N does on every rank) and a one-shard storm with it attached equals the oracle.
    RCCL refuses two ranks on one GPU, so the collectives themselves run only between GPUs."""
    from testground_amd.sim import Simulator
    uid = Simulator.comm_unique_id()
    kw = dict(n_inst=1500, rounds=4, t_now=True)
    S.assert_same(S.run_storm(hip, setup=lambda sim: sim.comm_init(uid, 1, 0), **kw), S.run_storm(oracle, **kw))


@pytest.mark.gpu
def test_storm_device_clock_speculation(hip, oracle):
    """bench.py's loop (rounds at TGSIM_T_NOW): each window's last launch generates the next round,
    which the next tgsim_gen_storm_round adopts. Calls that touch the staged arrays or the signal
    partials in between (an enqueue, a signal batch), a round of another size and a round staged
    at a host time each make the library generate the round itself; equal to the oracle throughout."""
    from testground_amd import _abi as A

    def between(r, sim):
        if r == 3:
            sim.enqueue([1, 2], [5, 6], [900000, 900000], [64, 64], [sim.now, sim.now])
        if r == 5:
            sim.signal([40, 40], [0, 1], [sim.now, sim.now])

    def size_of(r):
        return 512 if r == 7 else 1024

    kw = dict(n_inst=3000, rounds=11, t_now=True, size_of=size_of, between=between)
    S.assert_same(S.run_storm(hip, **kw), S.run_storm(oracle, **kw))


@pytest.mark.gpu
def test_shared_torch_stream_ordering(hip, oracle):
    """bench.py runs the library on torch's stream (tgsim_set_stream): torch kernels that produce the
    messages, the library's window and torch kernels that consume the deliveries are then ordered by
    the stream alone. Here the messages are computed by torch on a side stream, staged with
    tgsim_enqueue_device and advanced with tgsim_advance_async, and the deliveries are read back
    by torch from the device arrays (tgsim_deliveries_device) - with no synchronisation in between.
    Equal to the oracle fed the same messages."""
    import ctypes as C
    import torch
    from testground_amd import _abi as A
    from testground_amd.sim import SimConfig, Simulator, make_shape
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    n_inst, n = 64, 4096
    sims = [Simulator(SimConfig(n_instances=n_inst, seed=9, max_msgs_per_window=1 << 14, max_records=1 << 16),
                      binding=b) for b in (hip, oracle)]
    for sm in sims:
        for g in range(n_inst):
            sm.set_shape(g, make_shape(latency_ns=(g % 5) * 100_000, jitter_ns=50_000, loss=1.0))
    hs = sims[0]
    hs.set_stream(s.cuda_stream)
    with torch.cuda.stream(s):
        i = torch.arange(n, device=dev, dtype=torch.int64)
        src = (i * 7 % n_inst).to(torch.int32)
        dst = ((i * 13 + 5) % n_inst).to(torch.int32)
        seq = i.to(torch.int32)
        size = (64 + i % 512).to(torch.int32)
        t = (i * 97) % 1_000_000
        big = torch.empty(1 << 24, device=dev).normal_()   # a long torch kernel ahead of the staging
        soa = A.MsgSoA(src.data_ptr(), dst.data_ptr(), seq.data_ptr(), size.data_ptr(), t.data_ptr())
        assert hip.enqueue_device(hs._ctx, C.byref(soa), n) == 0
        assert hip.advance_async(hs._ctx, 3_000_000) == 0
        out = A.DeliverySoA()
        assert hip.deliveries_device(hs._ctx, C.byref(out)) == 0
        del big
    s.synchronize()
    src_h, dst_h, seq_h, size_h, t_h = (x.cpu().numpy() for x in (src, dst, seq, size, t))
    k = hs.delivery_count()
    # torch reads the device delivery arrays (stream-ordered after the window)
    with torch.cuda.stream(s):
        dt = torch.empty(k, dtype=torch.int64, device=dev)
        hip_memcpy = C.CDLL("libamdhip64.so").hipMemcpyAsync
        hip_memcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        assert hip_memcpy(dt.data_ptr(), out.t_deliver, 8 * k, 3, C.c_void_p(s.cuda_stream)) == 0
        dt2 = dt + 0                                       # a torch kernel on the copied data
    s.synchronize()
    got_t = dt2.cpu().numpy()
    sims[1].enqueue(src_h, dst_h, seq_h, size_h, t_h)
    sims[1].advance(3_000_000)
    want = sims[1].deliveries()
    assert np.array_equal(got_t, want["t_deliver"])
    assert np.array_equal(hs.deliveries()["seq"], want["seq"])
    for sm in sims:
        sm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mix", ["device", "device+device", "device+host", "host+device"])
def test_enqueue_device_in_place(hip, oracle, mix):
    """a tgsim_enqueue_device batch that is the window's only staging is read in
    place (no copy); one followed by more staging is copied in front of it at the window start; one
    after a host batch is copied during the call. Every mix equals the oracle fed the same messages,
    window by window, with the queue limit on (the sequential lane reads the batch too)."""
    import torch
    from testground_amd.sim import SimConfig, Simulator, make_shape
    dev = torch.device("cuda:0")
    n_inst, n = 4, 2500     # ~600 per sender per window, queued for 1-4 ms: the queue limit decides
    sims = [Simulator(SimConfig(n_instances=n_inst, seed=5, max_msgs_per_window=1 << 14, max_records=1 << 16),
                      binding=b) for b in (hip, oracle)]
    for sm in sims:
        for g in range(n_inst):
            sm.set_shape(g, make_shape(latency_ns=(1 + g % 4) * 1_000_000, jitter_ns=300_000, loss=2.0))
    rng = np.random.default_rng(11)
    outs = [[], []]
    seqc = np.zeros(n_inst, np.int64)
    for w in range(4):
        parts = []
        for kind in mix.split("+"):
            src = rng.integers(0, n_inst, n)
            dst = rng.integers(0, n_inst, n)
            seq = np.zeros(n, np.int64)
            for i in range(n):
                seq[i] = seqc[src[i]]
                seqc[src[i]] += 1
            t = w * 2_000_000 + np.sort(rng.integers(0, 2_000_000, n))
            parts.append((kind, src, dst, seq, np.full(n, 1500), t))
        keep = []
        for kind, src, dst, seq, size, t in parts:
            if kind == "device":
                cols = [torch.from_numpy(x.astype(np.int32)).to(dev) for x in (src, dst, seq, size)]
                cols.append(torch.from_numpy(t.astype(np.int64)).to(dev))
                torch.cuda.synchronize()
                keep.append(cols)   # read in place by the window: alive until it has run
                sims[0].enqueue_device(*(c.data_ptr() for c in cols), n)
            else:
                sims[0].enqueue(src, dst, seq, size, t)
            sims[1].enqueue(src, dst, seq, size, t)
        for k, sm in enumerate(sims):
            sm.advance((w + 1) * 2_000_000)
            outs[k].append(dict(status=sm.status(), deliv=sm.deliveries(), stats=S.parity_stats(sm)))
        del keep
    S.assert_same(outs[0], outs[1])
    for sm in sims:
        sm.close()
