"""sdk-go ``network`` package types, restated for the simulator (host side).

The reference consumes these types but does not vendor them: ``github.com/testground/sdk-go``
(``go.mod:33``, v0.3.1-0.20211012114808-49c90fa75405) defines ``network.Config``, ``LinkShape``,
``LinkRule``, ``FilterAction`` and ``RoutingPolicyType``; the sidecar reads them at
``pkg/sidecar/link.go:155-217``, ``pkg/sidecar/route.go:102-117`` and
``pkg/sidecar/docker_network.go:51-148``. Field names follow the Go names (snake_case) so a plan
restated here reads like the Go plan (compare ``plans/network/pingpong.go:29-41``).

``Config.to_c()`` lowers a config to the C ABI struct ``tgsim_network_config`` (include/tgsim.h).
The callback fields (``callback_state``, ``callback_target``) never reach the C ABI: the sidecar
handler consumes them (``pkg/sidecar/sidecar_handler.go:75-79``), which lives in
:mod:`testground_amd.sidecar`.
"""
from __future__ import annotations

import ctypes as C
import enum
from dataclasses import dataclass, field
from typing import Optional

from . import _abi as A

MS = 1_000_000
SECOND = 1_000_000_000


class FilterAction(enum.IntEnum):
    """network.FilterAction: iota order Accept, Reject, Drop [EXT sdk-go network/types.go]."""
    Accept = A.FILTER_ACCEPT
    Reject = A.FILTER_REJECT
    Drop = A.FILTER_DROP


Accept, Reject, Drop = FilterAction.Accept, FilterAction.Reject, FilterAction.Drop


class RoutingPolicyType(str, enum.Enum):
    """network.RoutingPolicyType. Only "allow_all" enables external routes; "deny_all" and any other
    value, including the zero value "", disable them (route.go:105-113)."""
    AllowAll = "allow_all"
    DenyAll = "deny_all"


AllowAll, DenyAll = RoutingPolicyType.AllowAll, RoutingPolicyType.DenyAll


def policy_code(p) -> int:
    return A.POLICY_ALLOW_ALL if p == RoutingPolicyType.AllowAll or p == "allow_all" else A.POLICY_DENY_ALL


def ip_to_int(ip: str) -> int:
    a, b, c, d = (int(x) for x in ip.split("."))
    for x in (a, b, c, d):
        if not 0 <= x <= 255:
            raise ValueError(f"bad IPv4 address {ip!r}")
    return (a << 24) | (b << 16) | (c << 8) | d


def int_to_ip(v: int) -> str:
    return f"{(v >> 24) & 255}.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}"


@dataclass(frozen=True)
class IPNet:
    """net.IPNet (IPv4 only): address + prefix length. ``IPNet.parse("16.0.0.5/32")``."""
    ip: int
    prefix_len: int

    @staticmethod
    def parse(s: str) -> "IPNet":
        ip, _, plen = s.partition("/")
        p = int(plen) if plen else 32
        if not 0 <= p <= 32:
            raise ValueError(f"bad prefix length in {s!r}")
        return IPNet(ip_to_int(ip), p)

    @property
    def mask(self) -> int:
        return (0xFFFFFFFF << (32 - self.prefix_len)) & 0xFFFFFFFF if self.prefix_len else 0

    def contains(self, ip: int) -> bool:
        return (ip & self.mask) == (self.ip & self.mask)

    def __str__(self) -> str:
        return f"{int_to_ip(self.ip)}/{self.prefix_len}"


@dataclass
class LinkShape:
    """network.LinkShape. Durations in integer nanoseconds (time.Duration), rates in bits/s,
    probabilities in percent (float32 on the wire)."""
    latency: int = 0
    jitter: int = 0
    bandwidth: int = 0
    filter: FilterAction = FilterAction.Accept
    loss: float = 0.0
    corrupt: float = 0.0
    corrupt_corr: float = 0.0
    reorder: float = 0.0
    reorder_corr: float = 0.0
    duplicate: float = 0.0
    duplicate_corr: float = 0.0

    def to_c(self) -> A.LinkShape:
        return A.LinkShape(int(self.latency), int(self.jitter), int(self.bandwidth), self.loss, self.corrupt,
                           self.corrupt_corr, self.reorder, self.reorder_corr, self.duplicate,
                           self.duplicate_corr, int(self.filter))


@dataclass
class LinkRule:
    """network.LinkRule = LinkShape + Subnet. Only ``shape.filter`` is applied (link.go:185-186)."""
    subnet: IPNet
    shape: LinkShape = field(default_factory=LinkShape)

    def to_c(self) -> A.LinkRule:
        return A.LinkRule(self.subnet.ip, self.subnet.prefix_len, self.shape.to_c())


@dataclass
class Config:
    """network.Config. ``callback_target == 0`` means "all instances" (network.Client [EXT])."""
    network: str = ""
    enable: bool = False
    default: LinkShape = field(default_factory=LinkShape)
    rules: list = field(default_factory=list)
    callback_state: str = ""
    callback_target: int = 0
    routing_policy: str = ""
    ipv4: Optional[IPNet] = None
    ipv6: Optional[str] = None

    def to_c(self):
        """Returns (tgsim_network_config, keepalive) - keep the second alive during the call."""
        if self.ipv6:
            raise A.TgsimError(A.ENOTSUP, "IPv6 data networks are not simulated")
        rules = (A.LinkRule * max(1, len(self.rules)))(*[r.to_c() for r in self.rules])
        name = self.network.encode()
        cfg = A.NetworkConfig(name, int(bool(self.enable)), policy_code(self.routing_policy), self.default.to_c(),
                              C.cast(rules, C.POINTER(A.LinkRule)), len(self.rules),
                              int(self.ipv4 is not None), self.ipv4.ip if self.ipv4 is not None else 0)
        return cfg, (rules, name)
