"""ctypes mirror of include/tgsim.h and the loader of the HIP library (testground_amd/libtgsim.so).

The product path binds ONLY libtgsim.so. If it is missing or cannot find a HIP device, every call
fails loudly (TgsimError); there is no CPU fallback. The CPU oracle (oracle/liboracle.so) exposes
the same entry points with a ``tgo_`` prefix and is bound by test infrastructure only
(oracle/pyoracle.py), through :func:`bind`.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libtgsim.so")

# ---- constants (tgsim.h) -------------------------------------------------------------------
OK = 0
EINVAL, ENOMEM, EHIP, ECAPACITY, ECAUSALITY, ENOTSUP, EUNSUPPORTED_NETWORK, ESTATE, ENODEV = (
    -1, -2, -3, -4, -5, -6, -7, -8, -9)
ERROR_NAMES = {EINVAL: "EINVAL", ENOMEM: "ENOMEM", EHIP: "EHIP", ECAPACITY: "ECAPACITY",
               ECAUSALITY: "ECAUSALITY", ENOTSUP: "ENOTSUP",
               EUNSUPPORTED_NETWORK: "EUNSUPPORTED_NETWORK", ESTATE: "ESTATE", ENODEV: "ENODEV"}

FILTER_ACCEPT, FILTER_REJECT, FILTER_DROP = 0, 1, 2
POLICY_DENY_ALL, POLICY_ALLOW_ALL = 0, 1
APPLY_DOCKER, APPLY_K8S = 0, 1
DST_EXTERNAL = 0xFFFFFFFF
T_NOW = -(1 << 63)  # TGSIM_T_NOW: "the current window start as the device knows it"

(ST_QUEUED, ST_LOST, ST_DROPPED, ST_REJECTED, ST_UNREACHABLE, ST_EXTERNAL, ST_DEST_DOWN, ST_LOCAL,
 ST_OVERLIMIT) = range(9)
ST_FLAG_DUP, ST_FLAG_CLONE_LOST, ST_FLAG_DUP_CANCEL, ST_FLAG_OVERLIMIT = 0x10, 0x20, 0x40, 0x80
F_CLONE, F_CORRUPT, F_REORDERED, F_STAGE_D, F_LOCAL, F_WHEEL = 1, 2, 4, 8, 128, 256
NETEM_LIMIT = 1000  # TGSIM_NETEM_LIMIT: netlink's default netem limit (link.go:169-179 sets none)


class TgsimError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code
        self.msg = msg


class LinkShape(C.Structure):
    _fields_ = [("latency_ns", C.c_int64), ("jitter_ns", C.c_int64), ("bandwidth_bps", C.c_uint64),
                ("loss", C.c_float), ("corrupt", C.c_float), ("corrupt_corr", C.c_float),
                ("reorder", C.c_float), ("reorder_corr", C.c_float), ("duplicate", C.c_float),
                ("duplicate_corr", C.c_float), ("filter", C.c_int32)]


class LinkRule(C.Structure):
    _fields_ = [("subnet_ip", C.c_uint32), ("prefix_len", C.c_uint32), ("shape", LinkShape)]


class NetworkConfig(C.Structure):
    _fields_ = [("network", C.c_char_p), ("enable", C.c_int32), ("routing_policy", C.c_int32),
                ("default_shape", LinkShape), ("rules", C.POINTER(LinkRule)), ("n_rules", C.c_size_t),
                ("has_ipv4", C.c_int32), ("ipv4", C.c_uint32)]


class Config(C.Structure):
    _fields_ = [("n_instances", C.c_uint32), ("shard_id", C.c_uint32), ("n_shards", C.c_uint32),
                ("device", C.c_uint32), ("seed", C.c_uint64), ("data_subnet", C.c_uint32),
                ("data_prefix_len", C.c_uint32), ("wheel_slot_ns", C.c_int64), ("wheel_slots", C.c_uint32),
                ("reserved0", C.c_uint32), ("max_msgs_per_window", C.c_uint64),
                ("max_records", C.c_uint64), ("exchange_cap", C.c_uint64), ("max_states", C.c_uint32),
                ("max_waiters", C.c_uint32), ("max_signals", C.c_uint64)]


class MsgSoA(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("seq", C.c_void_p), ("size", C.c_void_p),
                ("t_send", C.c_void_p)]


class DeliverySoA(C.Structure):
    _fields_ = [("t_deliver", C.c_void_p), ("src", C.c_void_p), ("dst", C.c_void_p), ("seq", C.c_void_p),
                ("size", C.c_void_p), ("flags", C.c_void_p), ("corrupt_off", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("msgs_in", "copies", "lost", "dropped", "rejected", "unreachable",
                                          "external", "dest_down", "local", "delivered", "windows",
                                          "inflight", "tb_items", "extracted", "inserted", "overlimit")]


class TcpConfig(C.Structure):
    _fields_ = [("mss", C.c_uint32), ("header_bytes", C.c_uint32), ("rto_ns", C.c_int64),
                ("max_attempts", C.c_uint32), ("acks", C.c_uint32), ("max_writes", C.c_uint64),
                ("max_segments", C.c_uint64)]


class TcpStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("writes", "segments", "packets", "retransmissions", "delivered",
                                          "failed", "pending_retx")]


TCP_PENDING, TCP_DELIVERED, TCP_TIMEOUT, TCP_REFUSED = 0, 1, 2, 3


class ProbeConfig(C.Structure):
    _fields_ = [("request_bytes", C.c_uint32), ("reply_bytes", C.c_uint32), ("timeout_ns", C.c_int64),
                ("window_ns", C.c_int64)]


class StormConfig(C.Structure):
    _fields_ = [("outgoing", C.c_uint32), ("concurrent", C.c_uint32), ("chunk_bytes", C.c_uint32),
                ("header_bytes", C.c_uint32), ("data_bytes", C.c_uint64), ("syn_bytes", C.c_uint32),
                ("msg_window", C.c_uint32), ("dial_timeout_ns", C.c_int64), ("window_ns", C.c_int64)]


class StormTotals(C.Structure):
    _fields_ = [("chunks_written", C.c_uint64), ("chunks_delivered", C.c_uint64), ("chunks_failed", C.c_uint64),
                ("bytes_written", C.c_uint64), ("dials_ok", C.c_uint32), ("dials_failed", C.c_uint32),
                ("dials_pending", C.c_uint32), ("conns_writing", C.c_uint32)]


STORM_SYN, STORM_DATA, STORM_SYNACK = 0x40000000, 0x80000000, 0xC0000000
PROBE_NONE, PROBE_OK, PROBE_REFUSED, PROBE_TIMEOUT = 0, 1, 2, 3
PROBE_REQ, PROBE_REP = 0x40000000, 0xC0000000
TCP_ACK_BIT = 0x80000000


# tgsim_transport (include/tgsim.h): caller-supplied cross-shard operations
ALLTOALL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
ABORT_FN = C.CFUNCTYPE(None, C.c_void_p)


class Transport(C.Structure):
    _fields_ = [("user", C.c_void_p), ("alltoall", ALLTOALL_FN), ("allreduce_max_i64", ALLREDUCE_FN),
                ("allgather", ALLGATHER_FN), ("abort", ABORT_FN)]


COMM_ID_BYTES = 128

RECORD_DTYPE_FIELDS = [("t", "<i8"), ("src", "<u4"), ("dst", "<u4"), ("seq", "<u4"), ("size", "<u4"),
                       ("meta", "<u4"), ("corrupt_off", "<u4")]

P = C.c_void_p
_SIGS = {
    "create": (C.c_int, [C.POINTER(Config), C.POINTER(P)]),
    "destroy": (None, [P]),
    "last_error": (C.c_char_p, [P]),
    "now": (C.c_int64, [P]),
    "horizon": (C.c_int64, [P]),
    "configure_network": (C.c_int, [P, C.c_uint32, C.POINTER(NetworkConfig)]),
    "configure_network_order": (C.c_int, [P, C.c_uint32, C.POINTER(NetworkConfig), C.c_int32]),
    "set_shape": (C.c_int, [P, C.c_uint32, C.POINTER(LinkShape)]),
    "set_shapes": (C.c_int, [P, C.c_void_p, C.POINTER(LinkShape), C.c_size_t]),
    "add_rules": (C.c_int, [P, C.c_uint32, C.POINTER(LinkRule), C.c_size_t]),
    "set_policy": (C.c_int, [P, C.c_uint32, C.c_int32]),
    "set_enabled": (C.c_int, [P, C.c_uint32, C.c_int32, C.c_int32, C.c_uint32]),
    "get_ip": (C.c_int, [P, C.c_uint32, C.POINTER(C.c_uint32)]),
    "enqueue": (C.c_int, [P, C.POINTER(MsgSoA), C.c_size_t]),
    "advance": (C.c_int, [P, C.c_int64]),
    "advance_async": (C.c_int, [P, C.c_int64]),
    "advance_begin": (C.c_int, [P, C.c_int64]),
    "exchange_buffers": (C.c_int, [P, C.POINTER(P), C.POINTER(P), C.POINTER(C.c_size_t)]),
    "advance_end": (C.c_int, [P]),
    "advance_to_barrier": (C.c_int, [P, C.c_uint32, C.c_int64]),
    "delivery_count": (C.c_int, [P, C.POINTER(C.c_size_t)]),
    "copy_deliveries": (C.c_int, [P, C.POINTER(DeliverySoA), C.c_size_t, C.POINTER(C.c_size_t)]),
    "copy_inbox_offsets": (C.c_int, [P, C.c_void_p, C.c_size_t]),
    "copy_status": (C.c_int, [P, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "get_stats": (C.c_int, [P, C.POINTER(Stats)]),
    "sync_signal": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "sync_barrier": (C.c_int, [P, C.c_uint32, C.c_uint32, C.c_int64, C.POINTER(C.c_uint32)]),
    "sync_poll": (C.c_int, [P, C.c_uint32, C.POINTER(C.c_int64)]),
    "sync_count": (C.c_int, [P, C.c_uint32, C.POINTER(C.c_uint32)]),
    "gen_storm_round": (C.c_int, [P, C.c_uint32, C.c_int64, C.c_uint32, C.c_uint32, C.c_int64, C.c_uint32]),
    "sync_publish": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                C.c_void_p]),
    "sync_subscribe": (C.c_int, [P, C.c_uint32, C.c_uint32, C.c_int64, C.c_size_t, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                  C.POINTER(C.c_size_t)]),
    "flood_set_graph": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_uint32]),
    "flood_publish": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32]),
    "flood_react": (C.c_int, [P, C.c_uint32, C.POINTER(C.c_size_t)]),
    "set_transport": (C.c_int, [P, C.POINTER(Transport)]),
    "comm_abort": (C.c_int, [P]),
    "tcp_enable": (C.c_int, [P, C.POINTER(TcpConfig)]),
    "tcp_send": (C.c_int, [P, C.POINTER(MsgSoA), C.c_size_t]),
    "tcp_react": (C.c_int, [P, C.POINTER(C.c_size_t)]),
    "tcp_writes": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "tcp_get_stats": (C.c_int, [P, C.POINTER(TcpStats)]),
    "tcp_gen_storm_round": (C.c_int, [P, C.c_uint32, C.c_int64, C.c_uint32, C.c_uint32, C.c_int64, C.c_uint32]),
    "tcp_writes_range": (C.c_int, [P, C.c_uint64, C.c_size_t, C.c_void_p, C.c_void_p]),
    "tcp_connect": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "tcp_write": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "tcp_conns": (C.c_int, [P, C.c_uint32, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "probe_setup": (C.c_int, [P, C.c_void_p, C.c_uint32, C.POINTER(ProbeConfig)]),
    "probe_start": (C.c_int, [P, C.c_int64]),
    "probe_react": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_uint32)]),
    "probe_results": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_size_t]),
    "storm_setup": (C.c_int, [P, C.c_void_p, C.c_void_p, C.POINTER(StormConfig)]),
    "storm_start": (C.c_int, [P]),
    "storm_react": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_uint32)]),
    "storm_dials": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_size_t]),
    "storm_write_start": (C.c_int, [P, C.c_int64]),
    "storm_results": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(StormTotals)]),
    "storm_end": (C.c_int, [P]),
}
# entry points only the HIP library has
_SIGS_HIP = {
    "version": (C.c_char_p, []),
    "abi_version": (C.c_int, []),
    "set_stream": (C.c_int, [P, P]),
    "shard_range": (C.c_int, [P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "sync": (C.c_int, [P]),
    "enqueue_device": (C.c_int, [P, C.POINTER(MsgSoA), C.c_size_t]),
    "deliveries_device": (C.c_int, [P, C.POINTER(DeliverySoA)]),
    "profile_set": (C.c_int, [P, C.c_uint32]),
    "profile_read": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "kernel_classes": (C.c_int, []),
    "kernel_name": (C.c_char_p, [C.c_int]),
    "set_exchange_buffers": (C.c_int, [P, P, P, C.c_size_t]),
    "advance_begin_device": (C.c_int, [P, P, C.c_int64]),
    "storm_release_device": (C.c_int, [P, P]),
    "comm_unique_id": (C.c_int, [C.c_void_p]),
    "comm_init": (C.c_int, [P, C.c_void_p, C.c_uint32, C.c_uint32]),
    "sync_subscribe_device": (C.c_int, [P, C.c_size_t, P, P, P, C.c_uint32, P, P, C.c_size_t]),
    "topic_arena_device": (C.c_int, [P, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                     C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "snapshot": (C.c_int, [P, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "restore": (C.c_int, [P, C.c_void_p, C.c_size_t]),
    "debug_fail_alloc": (C.c_int, [P, C.c_uint32]),
    "probe_state_device": (C.c_int, [P, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "storm_state_device": (C.c_int, [P, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "kernel_counters": (C.c_int, [P, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
}


class Binding:
    """A loaded library + its symbol prefix; attribute access returns the typed C function."""

    def __init__(self, cdll: C.CDLL, prefix: str, name: str):
        self.cdll = cdll
        self.prefix = prefix
        self.name = name
        sigs = dict(_SIGS)
        if prefix == "tgsim_":
            sigs.update(_SIGS_HIP)
        for short, (res, args) in sigs.items():
            fn = getattr(cdll, prefix + short)
            fn.restype = res
            fn.argtypes = args
            setattr(self, short, fn)


def bind(path: str, prefix: str, name: str) -> Binding:
    return Binding(C.CDLL(path), prefix, name)


_HIP: Binding | None = None


def hip_library() -> Binding:
    """The product library. Raises if it was not built (run __graft_entry__.build()). TGSIM_LIB
    names an experiment build of the same sources to load instead (tools/ timing probes)."""
    global _HIP
    if _HIP is None:
        path = os.environ.get("TGSIM_LIB") or LIB_PATH
        if not os.path.exists(path):
            raise TgsimError(ENODEV, f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        # torch bundles its own libamdhip64 (soname libamdhip64.so.7). Loaded first, it also serves
        # libtgsim.so, so the process has one HIP runtime; loaded after /opt/rocm's copy, torch would
        # bring up a second runtime that finds no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _HIP = bind(path, "tgsim_", "hip")
    return _HIP


def header_symbols(header: str | None = None) -> list[str]:
    """Every function the public header declares (for the ABI export test)."""
    import re
    header = header or os.path.join(os.path.dirname(HERE), "include", "tgsim.h")
    text = open(header).read()
    return sorted(set(re.findall(r"\b(tgsim_[a-z_0-9]+)\s*\(", text)))
