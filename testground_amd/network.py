"""Mirror of the sdk-go ``network`` package types the reference sidecar consumes.

Field names follow sdk-go exactly (``network.Config``, ``network.LinkShape``, ``network.LinkRule``,
``network.FilterAction``, ``network.RoutingPolicyType``) as used by the reference:
pkg/sidecar/link.go:155-217, pkg/sidecar/route.go:102-117, pkg/sidecar/docker_network.go:51-148,
plans/network/pingpong.go:29-42, plans/splitbrain/main.go:111-131.  Durations are Go
``time.Duration`` values, i.e. integer nanoseconds (constants below).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import enum
import ipaddress
from typing import List, Optional, Union

import numpy as np

from . import abi

Nanosecond = 1
Microsecond = 1_000
Millisecond = 1_000_000
Second = 1_000_000_000
Hour = 3600 * Second


class FilterAction(enum.IntEnum):
    Accept = 0
    Reject = 1
    Drop = 2


class RoutingPolicyType(str, enum.Enum):
    AllowAll = "allow_all"
    DenyAll = "deny_all"


@dataclasses.dataclass
class LinkShape:
    Latency: int = 0          # time.Duration (ns)
    Jitter: int = 0           # time.Duration (ns)
    Bandwidth: int = 0        # bits/s, 0 = unlimited
    Filter: FilterAction = FilterAction.Accept
    Loss: float = 0.0         # percent
    Corrupt: float = 0.0
    CorruptCorr: float = 0.0
    Reorder: float = 0.0
    ReorderCorr: float = 0.0
    Duplicate: float = 0.0
    DuplicateCorr: float = 0.0


IPNetLike = Union[str, ipaddress.IPv4Interface, ipaddress.IPv4Network, tuple]


def _ipnet(x: IPNetLike) -> tuple:
    """Returns (address as int, prefix length) without masking host bits (the kernel rejects
    routes whose prefix carries host bits; the engine reproduces that error).  IPv4 only: the
    engine's rules are IPv4 prefixes, and an IPv6 subnet is refused here rather than truncated."""
    if isinstance(x, tuple):
        ip, plen = x
        a = ipaddress.ip_address(ip)
        if a.version != 4:
            raise ValueError(f"IPv6 subnet {ip}/{plen}: link rules are IPv4 only")
        return int(a), int(plen)
    if isinstance(x, (ipaddress.IPv4Network, ipaddress.IPv6Network)):
        if x.version != 4:
            raise ValueError(f"IPv6 subnet {x}: link rules are IPv4 only")
        return int(x.network_address), x.prefixlen
    iface = ipaddress.ip_interface(x)
    if iface.version != 4:
        raise ValueError(f"IPv6 subnet {x}: link rules are IPv4 only")
    return int(iface.ip), iface.network.prefixlen


def _ipv6(x) -> bytes:
    """cfg.IPv6 (an address or interface string, or an IPv6Address/Interface) -> 16 bytes."""
    if isinstance(x, (ipaddress.IPv6Address, ipaddress.IPv6Interface)):
        return (x.ip if isinstance(x, ipaddress.IPv6Interface) else x).packed
    return ipaddress.IPv6Interface(x).ip.packed


@dataclasses.dataclass
class LinkRule:
    Subnet: IPNetLike = "0.0.0.0/0"
    LinkShape: LinkShape = dataclasses.field(default_factory=LinkShape)


@dataclasses.dataclass
class Config:
    Network: str = ""
    IPv4: Optional[IPNetLike] = None
    IPv6: Optional[Union[str, ipaddress.IPv6Interface, ipaddress.IPv6Address]] = None
    Enable: bool = False
    Default: LinkShape = dataclasses.field(default_factory=LinkShape)
    Rules: List[LinkRule] = dataclasses.field(default_factory=list)
    CallbackState: str = ""
    CallbackTarget: int = 0
    RoutingPolicy: Union[RoutingPolicyType, str] = ""


_POLICY = {RoutingPolicyType.AllowAll: 1, RoutingPolicyType.DenyAll: 2, "allow_all": 1, "deny_all": 2}


def to_c(cfg: Config):
    """Flattens a Config into the C struct; returns (struct, keep-alive objects)."""
    c = abi.Config()
    net = (cfg.Network or "").encode()
    c.network = net
    c.enable = 1 if cfg.Enable else 0
    c.routing_policy = _POLICY.get(cfg.RoutingPolicy, 0)
    if cfg.IPv4 is not None:
        ip, _ = _ipnet(cfg.IPv4)
        c.has_ipv4 = 1
        c.ipv4 = ip
    if cfg.IPv6 is not None:
        c.has_ipv6 = 1
        c.ipv6[:] = list(_ipv6(cfg.IPv6))
    s = cfg.Default
    c.shape.latency_ns = int(s.Latency)
    c.shape.jitter_ns = int(s.Jitter)
    c.shape.bandwidth_bps = int(s.Bandwidth)
    c.shape.loss = s.Loss
    c.shape.corrupt = s.Corrupt
    c.shape.corrupt_corr = s.CorruptCorr
    c.shape.reorder = s.Reorder
    c.shape.reorder_corr = s.ReorderCorr
    c.shape.duplicate = s.Duplicate
    c.shape.duplicate_corr = s.DuplicateCorr
    rules = (abi.Rule * max(1, len(cfg.Rules)))()
    for i, r in enumerate(cfg.Rules):
        ip, plen = _ipnet(r.Subnet)
        rules[i].prefix = ip
        rules[i].len = plen
        rules[i].action = int(r.LinkShape.Filter)
    c.rules = rules
    c.n_rules = len(cfg.Rules)
    return c, (net, rules)


def shape_to_c(s: LinkShape) -> abi.Shape:
    return to_c(Config(Network="default", Enable=True, Default=s))[0].shape


_DEFAULT_NET = b"default"
_DEFAULT_NET_BUF = C.create_string_buffer(_DEFAULT_NET)


def configs_array(latency_ns, jitter_ns=0, bandwidth_bps=0, loss=0.0, corrupt=0.0, reorder=0.0, duplicate=0.0,
                  routing_policy: int = 0) -> np.ndarray:
    """Vectorised Config{Network: "default", Enable: true, Default: LinkShape{...}} records (no
    rules, no re-addressing) for tgsim_configure_batch; correlations 0."""
    lat = np.asarray(latency_ns, dtype=np.int64)
    n = lat.shape[0]
    a = np.zeros(n, dtype=abi.CONFIG_DTYPE)
    a["network"] = C.addressof(_DEFAULT_NET_BUF)
    a["enable"] = 1
    a["routing_policy"] = routing_policy
    sh = a["shape"]
    sh["latency_ns"] = lat
    sh["jitter_ns"] = jitter_ns
    sh["bandwidth_bps"] = bandwidth_bps
    sh["loss"] = loss
    sh["corrupt"] = corrupt
    sh["reorder"] = reorder
    sh["duplicate"] = duplicate
    a["shape"] = sh
    return a
