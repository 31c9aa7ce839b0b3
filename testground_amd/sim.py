"""Python handle on one simulator context (one shard of one run).

``Simulator`` drives libtgsim.so (the HIP path). It takes an optional ``binding`` so that test
infrastructure can drive the CPU oracle through the identical interface; product code never
passes one.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi as A

DELIVERY_FIELDS = ("t_deliver", "src", "dst", "seq", "size", "flags", "corrupt_off")


@dataclass
class SimConfig:
    n_instances: int
    seed: int = 1
    shard_id: int = 0
    n_shards: int = 1
    device: int = 0
    data_subnet: str = "16.0.0.0"
    data_prefix_len: int = 16
    wheel_slot_ns: int = 1_000_000
    wheel_slots: int = 1024
    max_msgs_per_window: int = 1 << 20
    max_records: int = 1 << 22
    exchange_cap: int = 1 << 16
    max_states: int = 4096
    max_waiters: int = 65536
    max_signals: int = 1 << 24

    def to_c(self) -> A.Config:
        c = A.Config()
        c.n_instances = self.n_instances
        c.shard_id = self.shard_id
        c.n_shards = self.n_shards
        c.device = self.device
        c.seed = self.seed
        c.data_subnet = ip_to_int(self.data_subnet)
        c.data_prefix_len = self.data_prefix_len
        c.wheel_slot_ns = self.wheel_slot_ns
        c.wheel_slots = self.wheel_slots
        c.max_msgs_per_window = self.max_msgs_per_window
        c.max_records = self.max_records
        c.exchange_cap = self.exchange_cap
        c.max_states = self.max_states
        c.max_waiters = self.max_waiters
        c.max_signals = self.max_signals
        return c


def ip_to_int(ip: str) -> int:
    a, b, c, d = (int(x) for x in ip.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def int_to_ip(v: int) -> str:
    return f"{(v >> 24) & 255}.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}"


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class Simulator:
    def __init__(self, cfg: SimConfig, binding: A.Binding | None = None):
        self.lib = binding or A.hip_library()
        self.cfg = cfg
        self._ctx = C.c_void_p()
        c = cfg.to_c()
        rc = self.lib.create(C.byref(c), C.byref(self._ctx))
        if rc != A.OK:
            raise A.TgsimError(rc, f"{self.lib.name}: create failed")
        n, s, k = cfg.n_instances, cfg.n_shards, cfg.shard_id
        self.lo, self.hi = (k * n) // s, ((k + 1) * n) // s

    # ---- plumbing ---------------------------------------------------------------------------
    def _check(self, rc: int) -> None:
        if rc != A.OK:
            msg = self.lib.last_error(self._ctx)
            raise A.TgsimError(rc, msg.decode() if msg else "")

    def close(self) -> None:
        if self._ctx:
            self.lib.destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def now(self) -> int:
        return int(self.lib.now(self._ctx))

    @property
    def horizon(self) -> int:
        """Earliest admissible t_send: the start of the last completed window."""
        return int(self.lib.horizon(self._ctx))

    # ---- network configuration (sidecar.Network) ---------------------------------------------
    def configure_network(self, instance: int, cfg: A.NetworkConfig) -> None:
        self._check(self.lib.configure_network(self._ctx, instance, C.byref(cfg)))

    def configure(self, instance: int, cfg, order: str = "docker") -> None:
        """ConfigureNetwork for one instance from a testground_amd.network.Config, in the apply order
        of DockerNetwork (docker_network.go:51-148) or K8sNetwork (k8s_network.go:43-176)."""
        c, keep = cfg.to_c()
        code = {"docker": A.APPLY_DOCKER, "k8s": A.APPLY_K8S}[order]
        self._check(self.lib.configure_network_order(self._ctx, int(instance), C.byref(c), code))
        del keep

    def set_shape(self, instance: int, shape: A.LinkShape) -> None:
        self._check(self.lib.set_shape(self._ctx, instance, C.byref(shape)))

    def set_shapes(self, instances, shapes: list[A.LinkShape]) -> None:
        inst = np.ascontiguousarray(instances, dtype=np.uint32)
        arr = (A.LinkShape * max(1, len(shapes)))(*shapes)
        self._check(self.lib.set_shapes(self._ctx, _ptr(inst), arr, len(shapes)))

    def add_rules(self, instance: int, rules: list[A.LinkRule]) -> None:
        arr = (A.LinkRule * max(1, len(rules)))(*rules)
        self._check(self.lib.add_rules(self._ctx, instance, arr, len(rules)))

    def set_policy(self, instance: int, policy: int) -> None:
        self._check(self.lib.set_policy(self._ctx, instance, policy))

    def set_enabled(self, instance: int, enabled: bool, ip: int | None = None) -> None:
        self._check(self.lib.set_enabled(self._ctx, instance, int(enabled), int(ip is not None), ip or 0))

    def get_ip(self, instance: int) -> int:
        v = C.c_uint32()
        self._check(self.lib.get_ip(self._ctx, instance, C.byref(v)))
        return v.value

    # ---- data path --------------------------------------------------------------------------
    def enqueue(self, src, dst, seq, size, t_send) -> None:
        arrs = [np.ascontiguousarray(x, dtype=np.uint32) for x in (src, dst, seq, size)]
        t = np.ascontiguousarray(t_send, dtype=np.int64)
        n = len(t)
        assert all(len(a) == n for a in arrs)
        m = A.MsgSoA(_ptr(arrs[0]), _ptr(arrs[1]), _ptr(arrs[2]), _ptr(arrs[3]), _ptr(t))
        self._check(self.lib.enqueue(self._ctx, C.byref(m), n))

    def enqueue_device(self, src_ptr: int, dst_ptr: int, seq_ptr: int, size_ptr: int, t_ptr: int, n: int) -> None:
        """tgsim_enqueue_device: n messages already in device memory (SoA at the given addresses)."""
        m = A.MsgSoA(src_ptr, dst_ptr, seq_ptr, size_ptr, t_ptr)
        self._check(self.lib.enqueue_device(self._ctx, C.byref(m), n))

    # ---- TCP mode (tgsim_tcp_*) ------------------------------------------------
    def tcp_enable(self, mss: int = 0, header_bytes: int = 0, rto_ns: int = 0, max_attempts: int = 0,
                   max_writes: int = 0, max_segments: int = 0, acks: bool = False) -> None:
        """acks=True: ACK packets on the reverse path and retransmission timers (tgsim.h)."""
        cfg = A.TcpConfig(mss, header_bytes, rto_ns, max_attempts, int(acks), max_writes, max_segments)
        self._check(self.lib.tcp_enable(self._ctx, C.byref(cfg)))

    def tcp_send(self, src, dst, seq, size, t_send) -> None:
        arrs = [np.ascontiguousarray(np.broadcast_to(x, np.shape(t_send)), dtype=np.uint32) for x in (src, dst, seq, size)]
        t = np.ascontiguousarray(t_send, dtype=np.int64)
        m = A.MsgSoA(_ptr(arrs[0]), _ptr(arrs[1]), _ptr(arrs[2]), _ptr(arrs[3]), _ptr(t))
        self._check(self.lib.tcp_send(self._ctx, C.byref(m), len(t)))

    def tcp_react(self, wait: bool = True) -> int:
        """The window's TCP reaction. wait=False: asynchronous (no count returned, no read-back; the
        counters arrive with a later synchronising call)."""
        if not wait:
            self._check(self.lib.tcp_react(self._ctx, None))
            return -1
        n = C.c_size_t()
        self._check(self.lib.tcp_react(self._ctx, C.byref(n)))
        return n.value

    def tcp_writes(self) -> tuple[np.ndarray, np.ndarray]:
        """(state TCP_*, time) per write id: last segment's arrival, or the failure time."""
        n = C.c_size_t()
        self.lib.tcp_writes(self._ctx, None, None, 0, C.byref(n))  # size query (ECAPACITY when n > 0)
        st = np.zeros(n.value, np.uint8)
        t = np.zeros(n.value, np.int64)
        self._check(self.lib.tcp_writes(self._ctx, _ptr(st), _ptr(t), n.value, C.byref(n)))
        return st, t

    def tcp_writes_range(self, first: int, n: int) -> tuple[np.ndarray, np.ndarray]:
        """(state, time) of writes [first, first + n)."""
        st = np.zeros(n, np.uint8)
        t = np.zeros(n, np.int64)
        if n:
            self._check(self.lib.tcp_writes_range(self._ctx, int(first), n, _ptr(st), _ptr(t)))
        return st, t

    def tcp_connect(self, src, dst) -> np.ndarray:
        """Connections src[i] -> dst[i]; returns their ids."""
        s = np.ascontiguousarray(np.atleast_1d(src), dtype=np.uint32)
        d = np.ascontiguousarray(np.broadcast_to(dst, s.shape), dtype=np.uint32)
        out = np.zeros(len(s), np.uint32)
        self._check(self.lib.tcp_connect(self._ctx, _ptr(s), _ptr(d), len(s), _ptr(out)))
        return out

    def tcp_write(self, conn, size, t_send) -> None:
        c = np.ascontiguousarray(np.atleast_1d(conn), dtype=np.uint32)
        z = np.ascontiguousarray(np.broadcast_to(size, c.shape), dtype=np.uint32)
        t = np.ascontiguousarray(np.broadcast_to(t_send, c.shape), dtype=np.int64)
        self._check(self.lib.tcp_write(self._ctx, _ptr(c), _ptr(z), _ptr(t), len(c)))

    def tcp_conns(self, first: int = 0, n: int | None = None) -> dict:
        """Per connection: segments ACKed so far, cwnd, flight, queued (unsent)."""
        if n is None:
            n = self._n_conn() - first
        out = dict(acked=np.zeros(n, np.uint64), cwnd=np.zeros(n, np.uint32), flight=np.zeros(n, np.uint32),
                   queued=np.zeros(n, np.uint32))
        if n:
            self._check(self.lib.tcp_conns(self._ctx, first, n, *(_ptr(out[k]) for k in ("acked", "cwnd", "flight",
                                                                                        "queued"))))
        return out

    def _n_conn(self) -> int:
        lo, hi = 0, 1
        while self.lib.tcp_conns(self._ctx, 0, hi, None, None, None, None) == A.OK:
            lo, hi = hi, hi * 2
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if self.lib.tcp_conns(self._ctx, 0, mid, None, None, None, None) == A.OK:
                lo = mid
            else:
                hi = mid
        return lo

    def tcp_gen_storm_round(self, round_: int, t0: int, fanout: int, size: int, spread_ns: int, state: int) -> None:
        self._check(self.lib.tcp_gen_storm_round(self._ctx, round_, t0, fanout, size, spread_ns, state))

    def tcp_stats(self) -> dict:
        s = A.TcpStats()
        self._check(self.lib.tcp_get_stats(self._ctx, C.byref(s)))
        return {k: getattr(s, k) for k, _ in A.TcpStats._fields_}

    def advance(self, t_end: int, wait: bool = True) -> None:
        """One window [now, t_end). wait=False: tgsim_advance_async (no closing sync; device-side
        errors surface at the next synchronising call)."""
        fn = self.lib.advance if wait else self.lib.advance_async
        self._check(fn(self._ctx, int(t_end)))

    def advance_begin(self, t_end: int) -> None:
        self._check(self.lib.advance_begin(self._ctx, int(t_end)))

    def advance_end(self) -> None:
        self._check(self.lib.advance_end(self._ctx))

    def exchange_buffers(self) -> tuple[int, int, int]:
        s, r, b = C.c_void_p(), C.c_void_p(), C.c_size_t()
        self._check(self.lib.exchange_buffers(self._ctx, C.byref(s), C.byref(r), C.byref(b)))
        return s.value, r.value, b.value

    def set_exchange_buffers(self, send_dev: int, recv_dev: int, nbytes: int) -> None:
        self._check(self.lib.set_exchange_buffers(self._ctx, send_dev, recv_dev, nbytes))

    def advance_begin_device(self, t_end_dev: int, offset_ns: int = 0) -> None:
        self._check(self.lib.advance_begin_device(self._ctx, t_end_dev, int(offset_ns)))

    def storm_release_device(self, out_dev: int) -> None:
        self._check(self.lib.storm_release_device(self._ctx, out_dev))

    # ---- cross-shard transport ---------------------------------------------
    def comm_abort(self) -> None:
        """tgsim_comm_abort: this shard stops; no peer waits for it in a collective."""
        self._check(self.lib.comm_abort(self._ctx))

    def set_transport(self, transport) -> None:
        """A testground_amd.exchange transport (or None): tgsim_advance* then exchange inside the
        call, storm batches and signal batches reduce / gather across the shards."""
        self._transport = transport  # the callbacks must outlive the context's use of them
        self._check(self.lib.set_transport(self._ctx, C.byref(transport.c) if transport is not None else None))

    @staticmethod
    def comm_unique_id() -> bytes:
        """An RCCL unique id (one rank creates it, the caller distributes it)."""
        lib = A.hip_library()
        buf = (C.c_uint8 * A.COMM_ID_BYTES)()
        rc = lib.comm_unique_id(buf)
        if rc != A.OK:
            raise A.TgsimError(rc, "comm_unique_id failed")
        return bytes(buf)

    def comm_init(self, unique_id: bytes, nranks: int, rank: int) -> None:
        """The native RCCL communicator (collective over the shards)."""
        buf = (C.c_uint8 * A.COMM_ID_BYTES).from_buffer_copy(unique_id)
        self._check(self.lib.comm_init(self._ctx, buf, nranks, rank))

    def set_stream(self, stream: int | None) -> None:
        self._check(self.lib.set_stream(self._ctx, stream))

    def sync(self) -> None:
        self._check(self.lib.sync(self._ctx))

    def advance_to_barrier(self, waiter: int, offset_ns: int = 0) -> None:
        self._check(self.lib.advance_to_barrier(self._ctx, waiter, int(offset_ns)))

    def delivery_count(self) -> int:
        n = C.c_size_t()
        self._check(self.lib.delivery_count(self._ctx, C.byref(n)))
        return n.value

    def deliveries(self) -> dict[str, np.ndarray]:
        n = self.delivery_count()
        out = {"t_deliver": np.zeros(n, np.int64)}
        for f in DELIVERY_FIELDS[1:]:
            out[f] = np.zeros(n, np.uint32)
        soa = A.DeliverySoA(*[_ptr(out[f]) if n else None for f in DELIVERY_FIELDS])
        got = C.c_size_t()
        self._check(self.lib.copy_deliveries(self._ctx, C.byref(soa), n, C.byref(got)))
        assert got.value == n
        return out

    def inbox_offsets(self) -> np.ndarray:
        out = np.zeros(self.hi - self.lo + 1, np.uint32)
        self._check(self.lib.copy_inbox_offsets(self._ctx, _ptr(out), len(out)))
        return out

    def status(self) -> np.ndarray:
        n = C.c_size_t()
        buf = np.zeros(1 << 16, np.uint8)
        rc = self.lib.copy_status(self._ctx, _ptr(buf), len(buf), C.byref(n))
        if rc == A.ECAPACITY and n.value > len(buf):
            buf = np.zeros(n.value, np.uint8)
            rc = self.lib.copy_status(self._ctx, _ptr(buf), len(buf), C.byref(n))
        self._check(rc)
        return buf[: n.value].copy()

    def stats(self) -> dict[str, int]:
        s = A.Stats()
        self._check(self.lib.get_stats(self._ctx, C.byref(s)))
        return {name: getattr(s, name) for name, _ in A.Stats._fields_}

    # ---- checkpoint / resume (HIP library only; tgsim.h tgsim_snapshot) ----------------------
    def snapshot(self) -> bytes:
        """The context's state at this window boundary as an opaque image (tgsim_restore)."""
        n = C.c_size_t()
        self._check(self.lib.snapshot(self._ctx, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        self._check(self.lib.snapshot(self._ctx, buf, n.value, C.byref(n)))
        return buf.raw[:n.value]

    def restore(self, image: bytes) -> None:
        self._check(self.lib.restore(self._ctx, image, len(image)))

    # ---- profiling (HIP library only) --------------------------------------------------------
    def profile(self, kernels=None) -> None:
        """Enable HIP-event timing for the named kernel classes (None = all, [] = off)."""
        names = self.kernel_names()
        mask = (1 << len(names)) - 1 if kernels is None else sum(1 << names.index(k) for k in kernels)
        self._check(self.lib.profile_set(self._ctx, mask))

    def kernel_names(self) -> list[str]:
        return [self.lib.kernel_name(k).decode() for k in range(self.lib.kernel_classes())]

    def profile_read(self) -> dict[str, tuple[float, int]]:
        k = self.lib.kernel_classes()
        ms = np.zeros(k, np.float64)
        cnt = np.zeros(k, np.uint64)
        n = C.c_size_t()
        self._check(self.lib.profile_read(self._ctx, _ptr(ms), _ptr(cnt), k, C.byref(n)))
        return {name: (float(ms[i]), int(cnt[i])) for i, name in enumerate(self.kernel_names())}

    KERNEL_COUNTERS = ("deferred", "long_tb", "long_emit", "wide", "long_whole")

    def kernel_counters(self) -> dict[str, int]:
        """Cumulative implementation counters (tgsim_kernel_counters; HIP library only)."""
        out = np.zeros(len(self.KERNEL_COUNTERS), np.uint64)
        n = C.c_size_t()
        self._check(self.lib.kernel_counters(self._ctx, _ptr(out), len(out), C.byref(n)))
        return {k: int(out[i]) for i, k in enumerate(self.KERNEL_COUNTERS)}

    # ---- sync service -----------------------------------------------------------------------
    def signal(self, states, instances, t, want_seq: bool = True) -> np.ndarray | None:
        st = np.ascontiguousarray(states, dtype=np.uint32)
        ins = np.ascontiguousarray(instances, dtype=np.uint32)
        tt = np.ascontiguousarray(t, dtype=np.int64)
        n = len(st)
        seq = np.zeros(max(n, 1), np.uint32) if want_seq else None
        self._check(self.lib.sync_signal(self._ctx, _ptr(st), _ptr(ins), _ptr(tt), n,
                                         _ptr(seq) if want_seq else None))
        return seq[:n] if want_seq else None

    def barrier(self, state: int, target: int, t_wait: int) -> int:
        w = C.c_uint32()
        self._check(self.lib.sync_barrier(self._ctx, state, target, int(t_wait), C.byref(w)))
        return w.value

    def poll(self, waiter: int) -> int:
        r = C.c_int64()
        self._check(self.lib.sync_poll(self._ctx, waiter, C.byref(r)))
        return r.value

    def count(self, state: int) -> int:
        v = C.c_uint32()
        self._check(self.lib.sync_count(self._ctx, state, C.byref(v)))
        return v.value

    # ---- workloads --------------------------------------------------------------------------
    def gen_storm_round(self, round_: int, t0: int, fanout: int, size: int, spread_ns: int, state: int) -> None:
        self._check(self.lib.gen_storm_round(self._ctx, round_, int(t0), fanout, size, int(spread_ns), state))


    # ---- topics (sync.Client Publish / Subscribe, device-resident logs) ----------------------
    def publish(self, topics, instances, t, payloads: list[bytes]) -> np.ndarray:
        inst = np.ascontiguousarray(np.atleast_1d(instances), dtype=np.uint32)
        tp = np.ascontiguousarray(np.broadcast_to(np.asarray(topics, dtype=np.uint32), inst.shape))
        tt = np.ascontiguousarray(np.broadcast_to(np.asarray(t, dtype=np.int64), inst.shape))
        assert len(payloads) == len(inst)
        off = np.zeros(len(inst) + 1, np.uint64)
        off[1:] = np.cumsum([len(p) for p in payloads])
        blob = np.frombuffer(b"".join(payloads) or b"\0", dtype=np.uint8)
        pos = np.zeros(len(inst), np.uint32)
        self._check(self.lib.sync_publish(self._ctx, _ptr(tp), _ptr(inst), _ptr(tt), _ptr(off), _ptr(blob),
                                          len(inst), _ptr(pos)))
        return pos

    def subscribe(self, topic: int, from_pos: int = 1, until_t: int = (1 << 63) - 1,
                  cap: int = 1 << 20) -> tuple[np.ndarray, np.ndarray, list[bytes]]:
        """(instances, times, payloads) of the topic's entries from position from_pos on whose
        time is <= until_t, in position order."""
        n, nb = C.c_size_t(), C.c_size_t()
        inst = np.zeros(cap, np.uint32)
        tt = np.zeros(cap, np.int64)
        off = np.zeros(cap + 1, np.uint64)
        blob = np.zeros(1 << 12, np.uint8)
        while True:  # ECAPACITY reports the bytes needed
            rc = self.lib.sync_subscribe(self._ctx, topic, from_pos, until_t, cap, _ptr(inst), _ptr(tt), _ptr(off),
                                         _ptr(blob), len(blob), C.byref(n), C.byref(nb))
            if rc == A.ECAPACITY and nb.value > len(blob):
                blob = np.zeros(nb.value, np.uint8)
                continue
            self._check(rc)
            break
        k = n.value
        raw = blob.tobytes()
        return inst[:k].copy(), tt[:k].copy(), [raw[int(off[j]):int(off[j + 1])] for j in range(k)]

    def subscribe_device(self, topics, from_pos, until_t, cap_each: int = 0xFFFFFFFF, entries: bool = True,
                         entries_cap: int | None = None, wait: bool = True):
        """Subscribe for a batch of subscribers on the device (tgsim_sync_subscribe_device). Inputs
        are torch tensors on the context's device (uint32 topics / from_pos as int32 or int64
        tensors, int64 until_t). Returns (offsets [n+1] int64 tensor, entry ids int32 tensor or
        None); subscriber i's inbox is ids[offsets[i]:offsets[i+1]] (arena entries, topic_arena).
        The work runs on the context's stream: wait=False returns before it is done (the caller
        orders its own stream after it, e.g. by sharing the stream through set_stream)."""
        import torch
        dev = topics.device
        tp = topics.to(torch.int32).contiguous()
        fr = from_pos.to(torch.int32).contiguous()
        ut = until_t.to(torch.int64).contiguous()
        n = tp.numel()
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        torch.cuda.current_stream(dev).synchronize()  # the inputs were made on torch's stream
        ids = None
        if entries:
            if entries_cap is None:  # counts first (one host read) to size the inbox arrays exactly
                self._check(self.lib.sync_subscribe_device(self._ctx, n, tp.data_ptr(), fr.data_ptr(), ut.data_ptr(),
                                                           cap_each, offs.data_ptr(), None, 0))
                torch.cuda.synchronize(dev)
                entries_cap = int(offs[-1].item())
            ids = torch.empty(max(1, entries_cap), dtype=torch.int32, device=dev)
        self._check(self.lib.sync_subscribe_device(self._ctx, n, tp.data_ptr(), fr.data_ptr(), ut.data_ptr(), cap_each,
                                                   offs.data_ptr(), ids.data_ptr() if ids is not None else None,
                                                   entries_cap or 0))
        if wait:
            self.sync()
        return offs, ids

    def topic_arena(self) -> dict:
        """The topic arena copied to the host: per entry id instance, t, payload offset / length, and
        the payload bytes (tgsim_topic_arena_device)."""
        from .exchange import _D2H, _hip
        ptrs = [C.c_void_p() for _ in range(5)]
        n = C.c_size_t()
        self._check(self.lib.topic_arena_device(self._ctx, *[C.byref(p) for p in ptrs], C.byref(n)))
        self.sync()
        hip = _hip()
        k = n.value
        out = {"instance": np.zeros(k, np.uint32), "t": np.zeros(k, np.int64), "payload_off": np.zeros(k, np.uint64),
               "payload_len": np.zeros(k, np.uint32)}
        for p, key in zip(ptrs[:4], ("instance", "t", "payload_off", "payload_len")):
            if k:
                assert hip.hipMemcpy(out[key].ctypes.data, p.value, out[key].nbytes, _D2H) == 0
        nb = int((out["payload_off"][-1] + out["payload_len"][-1])) if k else 0
        out["payload"] = np.zeros(nb, np.uint8)
        if nb:
            assert hip.hipMemcpy(out["payload"].ctypes.data, ptrs[4].value, nb, _D2H) == 0
        return out

    # ---- sequential probes (tgsim_probe_*) ------------------------------------
    def probe_setup(self, order, request_bytes: int, reply_bytes: int, timeout_ns: int, window_ns: int) -> None:
        o = np.ascontiguousarray(order, dtype=np.uint32)
        self._probe_n = len(o)
        cfg = A.ProbeConfig(request_bytes, reply_bytes, timeout_ns, window_ns)
        self._check(self.lib.probe_setup(self._ctx, _ptr(o), len(o), C.byref(cfg)))

    def probe_start(self, t0: int) -> None:
        self._check(self.lib.probe_start(self._ctx, int(t0)))

    def probe_react(self, wait: bool = True):
        """After a window. wait: (proposed next window end, instances still probing); else None."""
        if not wait:
            self._check(self.lib.probe_react(self._ctx, None, None))
            return None
        ne, act = C.c_int64(), C.c_uint32()
        self._check(self.lib.probe_react(self._ctx, C.byref(ne), C.byref(act)))
        return ne.value, act.value

    def probe_state_device(self) -> tuple[int, int]:
        """Device addresses of the proposed next window end (int64) and the probers still active."""
        a, b = C.c_void_p(), C.c_void_p()
        self._check(self.lib.probe_state_device(self._ctx, C.byref(a), C.byref(b)))
        return a.value, b.value

    def probe_results(self) -> tuple[np.ndarray, np.ndarray]:
        """(outcome[local, position in order] of TGSIM_PROBE_*, t_done[local])."""
        nloc = self.hi - self.lo
        out = np.zeros((nloc, self._probe_n), np.uint8)
        t = np.zeros(nloc, np.int64)
        self._check(self.lib.probe_results(self._ctx, _ptr(out), _ptr(t), out.size))
        return out, t

    # ---- storm plan reactor (tgsim_storm_*) ----------------------------------
    def storm_setup(self, dst, t_ready, *, outgoing: int, concurrent: int, data_bytes: int, chunk_bytes: int = 4096,
                    header_bytes: int = 66, syn_bytes: int = 66, msg_window: int = 10,
                    dial_timeout_ns: int = 30 * 10**9, window_ns: int = 10**6) -> None:
        d = np.ascontiguousarray(dst, dtype=np.uint32)
        t = np.ascontiguousarray(t_ready, dtype=np.int64)
        assert len(d) == len(t) == self.cfg.n_instances * outgoing
        self._storm_n = (self.hi - self.lo) * outgoing  # the local instances' connections (sharded)
        cfg = A.StormConfig(outgoing, concurrent, chunk_bytes, header_bytes, data_bytes, syn_bytes, msg_window,
                            dial_timeout_ns, window_ns)
        self._check(self.lib.storm_setup(self._ctx, _ptr(d), _ptr(t), C.byref(cfg)))

    def storm_start(self) -> None:
        self._check(self.lib.storm_start(self._ctx))

    def storm_react(self, wait: bool = True):
        """After a window. wait: (proposed next window end, connections still active); else None."""
        if not wait:
            self._check(self.lib.storm_react(self._ctx, None, None))
            return None
        ne, act = C.c_int64(), C.c_uint32()
        self._check(self.lib.storm_react(self._ctx, C.byref(ne), C.byref(act)))
        return ne.value, act.value

    def storm_state_device(self) -> tuple[int, int]:
        a, b = C.c_void_p(), C.c_void_p()
        self._check(self.lib.storm_state_device(self._ctx, C.byref(a), C.byref(b)))
        return a.value, b.value

    def storm_dials(self) -> tuple[np.ndarray, np.ndarray]:
        """(outcome TGSIM_PROBE_* per connection, its end time): the local instances' connections,
        lo * outgoing .. hi * outgoing."""
        out = np.zeros(self._storm_n, np.uint8)
        t = np.zeros(self._storm_n, np.int64)
        self._check(self.lib.storm_dials(self._ctx, _ptr(out), _ptr(t), self._storm_n))
        return out, t

    def storm_write_start(self, t0: int) -> None:
        self._check(self.lib.storm_write_start(self._ctx, int(t0)))

    def storm_results(self) -> tuple[np.ndarray, np.ndarray, dict]:
        """(failed[local], t_last[local], totals)."""
        nloc = self.hi - self.lo
        f = np.zeros(nloc, np.uint8)
        t = np.zeros(nloc, np.int64)
        tot = A.StormTotals()
        self._check(self.lib.storm_results(self._ctx, _ptr(f), _ptr(t), nloc, C.byref(tot)))
        return f.astype(bool), t, {k: getattr(tot, k) for k, _ in A.StormTotals._fields_}

    def storm_end(self) -> None:
        self._check(self.lib.storm_end(self._ctx))

    # ---- flood workload (config 5) -----------------------------------------------------------
    def flood_set_graph(self, offsets, neighbors, max_pubs: int) -> None:
        off = np.ascontiguousarray(offsets, dtype=np.uint32)
        nbr = np.ascontiguousarray(neighbors, dtype=np.uint32)
        assert len(off) == self.cfg.n_instances + 1
        self._check(self.lib.flood_set_graph(self._ctx, _ptr(off), _ptr(nbr) if len(nbr) else None, max_pubs))

    def flood_publish(self, instances, pubs, t, size: int) -> None:
        inst = np.ascontiguousarray(instances, dtype=np.uint32)
        p = np.ascontiguousarray(pubs, dtype=np.uint32)
        tt = np.ascontiguousarray(np.broadcast_to(np.asarray(t, dtype=np.int64), inst.shape))
        self._check(self.lib.flood_publish(self._ctx, _ptr(inst), _ptr(p), _ptr(tt), len(inst), size))

    def flood_react(self, size: int, count: bool = True) -> int | None:
        """Stage the forwards of the last window's first receipts. count=False keeps it
        asynchronous (no host read; returns None)."""
        if not count:
            self._check(self.lib.flood_react(self._ctx, size, None))
            return None
        n = C.c_size_t()
        self._check(self.lib.flood_react(self._ctx, size, C.byref(n)))
        return n.value


def make_shape(latency_ns=0, jitter_ns=0, bandwidth_bps=0, loss=0.0, corrupt=0.0, reorder=0.0, duplicate=0.0,
               corrupt_corr=0.0, reorder_corr=0.0, duplicate_corr=0.0, filter=0) -> A.LinkShape:
    return A.LinkShape(int(latency_ns), int(jitter_ns), int(bandwidth_bps), loss, corrupt, corrupt_corr, reorder,
                       reorder_corr, duplicate, duplicate_corr, filter)


def make_rule(subnet: str, filter: int) -> A.LinkRule:
    ip, plen = subnet.split("/")
    return A.LinkRule(ip_to_int(ip), int(plen), make_shape(filter=filter))
