"""sdk-go ``network`` package types, restated for the simulator (host side).

The reference consumes these types but does not vendor them: ``github.com/testground/sdk-go``
(``go.mod:33``, v0.3.1-0.20211012114808-49c90fa75405) defines ``network.Config``, ``LinkShape``,
``LinkRule``, ``FilterAction`` and ``RoutingPolicyType``; the sidecar reads them at
``pkg/sidecar/link.go:155-217``, ``pkg/sidecar/route.go:102-117`` and
``pkg/sidecar/docker_network.go:51-148``. Field names follow the Go names (snake_case) so a plan
restated here reads like the Go plan (compare ``plans/network/pingpong.go:29-41``).

``Config.to_c()`` lowers a config to the C ABI struct ``tgsim_network_config`` (include/tgsim.h).
``Config.to_wire()`` / ``Config.from_wire()`` are the JSON form a config travels in on the sync
topic ``network:<hostname>`` that the sidecar subscribes to (``pkg/sidecar/sidecar_handler.go:49-
80``): Go ``encoding/json`` of sdk-go's types [EXT]: ``network``, ``enable``, ``default``, ``rules``,
``callback_state``, ``routing_policy`` tags, ``IPv4`` / ``IPv6`` as ``net.IPNet`` objects
(``{"IP": "a.b.c.d", "Mask": <base64 bytes>}``), untagged ``LinkShape`` fields by Go name, durations
in integer nanoseconds, ``LinkRule`` = the embedded ``LinkShape`` fields + ``Subnet``.
``CallbackTarget`` is ``json:"-"``: it never travels. Decoding matches keys case-insensitively, as
Go does, and also takes the JS SDK's spellings (``callbackState``, ``routingPolicy``, ``IPv4`` as
``"a.b.c.d/n"``: ``plans/example-js/pingpong.js:25-33``).
The callback fields (``callback_state``, ``callback_target``) never reach the C ABI: the sidecar
handler consumes them (``pkg/sidecar/sidecar_handler.go:75-79``), which lives in
:mod:`testground_amd.sidecar`.
"""
from __future__ import annotations

import base64
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

    def to_wire(self) -> dict:
        return {go: (int(getattr(self, py)) if py in _INT_FIELDS else float(getattr(self, py)))
                for go, py in _SHAPE_FIELDS}

    @staticmethod
    def from_wire(d: dict) -> "LinkShape":
        sh = LinkShape()
        for go, py in _SHAPE_FIELDS:
            v = _get(d, go)
            if v is not None:
                setattr(sh, py, FilterAction(int(v)) if py == "filter" else (int(v) if py in _INT_FIELDS else float(v)))
        return sh


# Go field name -> Python attribute of network.LinkShape (untagged fields: encoding/json uses the names)
_SHAPE_FIELDS = (("Latency", "latency"), ("Jitter", "jitter"), ("Bandwidth", "bandwidth"), ("Filter", "filter"),
                 ("Loss", "loss"), ("Corrupt", "corrupt"), ("CorruptCorr", "corrupt_corr"), ("Reorder", "reorder"),
                 ("ReorderCorr", "reorder_corr"), ("Duplicate", "duplicate"), ("DuplicateCorr", "duplicate_corr"))
_INT_FIELDS = {"latency", "jitter", "bandwidth", "filter"}


def _get(d: dict, *names):
    """encoding/json's key match: exact first, then case-insensitive."""
    for n in names:
        if n in d:
            return d[n]
    low = {k.lower(): v for k, v in d.items()}
    for n in names:
        if n.lower() in low:
            return low[n.lower()]
    return None


def ipnet_to_wire(n: IPNet) -> dict:
    """net.IPNet's JSON: IP as text, Mask ([]byte) as base64."""
    return {"IP": int_to_ip(n.ip), "Mask": base64.b64encode(n.mask.to_bytes(4, "big")).decode()}


def ipnet_from_wire(v) -> IPNet:
    if isinstance(v, str):
        return IPNet.parse(v)
    mask = int.from_bytes(base64.b64decode(_get(v, "Mask")), "big")
    plen = bin(mask).count("1")
    if mask != ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF if plen else 0):
        raise ValueError(f"non-canonical netmask {mask:#010x}")
    return IPNet(ip_to_int(_get(v, "IP")), plen)


@dataclass
class LinkRule:
    """network.LinkRule = LinkShape + Subnet. Only ``shape.filter`` is applied (link.go:185-186)."""
    subnet: IPNet
    shape: LinkShape = field(default_factory=LinkShape)

    def to_c(self) -> A.LinkRule:
        return A.LinkRule(self.subnet.ip, self.subnet.prefix_len, self.shape.to_c())

    def to_wire(self) -> dict:
        return {**self.shape.to_wire(), "Subnet": ipnet_to_wire(self.subnet)}

    @staticmethod
    def from_wire(d: dict) -> "LinkRule":
        return LinkRule(ipnet_from_wire(_get(d, "Subnet")), LinkShape.from_wire(d))


class RuleList(tuple):
    """A rule list that many Configs share (splitbrain: every region-A node installs the same
    /32 block). It is immutable and snapshots its rules' C form when it is built, so every Config
    that carries it passes the same array without rebuilding it (a mutable list whose
    cache was keyed on its length could hand out a stale array after an in-place edit)."""

    def __new__(cls, rules=()):
        self = super().__new__(cls, rules)
        self.c_array = (A.LinkRule * max(1, len(self)))(*[r.to_c() for r in self])
        return self


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

    def to_wire(self) -> dict:
        """The JSON object published on network:<hostname> (callback_target does not travel)."""
        return {"network": self.network, "IPv4": ipnet_to_wire(self.ipv4) if self.ipv4 is not None else None,
                "IPv6": self.ipv6, "enable": bool(self.enable), "default": self.default.to_wire(),
                "rules": [r.to_wire() for r in self.rules], "callback_state": self.callback_state,
                "routing_policy": str(getattr(self.routing_policy, "value", self.routing_policy))}

    @staticmethod
    def from_wire(d: dict) -> "Config":
        ip4 = _get(d, "IPv4")
        return Config(network=_get(d, "network") or "", enable=bool(_get(d, "enable")),
                      default=LinkShape.from_wire(_get(d, "default") or {}),
                      rules=[LinkRule.from_wire(r) for r in (_get(d, "rules") or [])],
                      callback_state=_get(d, "callback_state", "callbackState") or "",
                      routing_policy=_get(d, "routing_policy", "routingPolicy") or "",
                      ipv4=ipnet_from_wire(ip4) if ip4 else None, ipv6=_get(d, "IPv6") or None)

    def to_c(self):
        """Returns (tgsim_network_config, keepalive) - keep the second alive during the call."""
        if self.ipv6:
            raise A.TgsimError(A.ENOTSUP, "IPv6 data networks are not simulated")
        if isinstance(self.rules, RuleList):
            rules = self.rules.c_array
        else:
            rules = (A.LinkRule * max(1, len(self.rules)))(*[r.to_c() for r in self.rules])
        name = self.network.encode()
        cfg = A.NetworkConfig(name, int(bool(self.enable)), policy_code(self.routing_policy), self.default.to_c(),
                              C.cast(rules, C.POINTER(A.LinkRule)), len(self.rules),
                              int(self.ipv4 is not None), self.ipv4.ip if self.ipv4 is not None else 0)
        return cfg, (rules, name)
