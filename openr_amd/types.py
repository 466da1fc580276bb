"""Python mirror of the thrift structs on the Decision route-computation path.

Field names, defaults and enum values follow the reference IDL:
  - Adjacency / AdjacencyDatabase          openr/if/Types.thrift:74-175
  - PrefixMetrics / PrefixEntry            openr/if/Types.thrift:297-430
  - BinaryAddress / IpPrefix / MplsAction /
    NextHopThrift / PrefixType             openr/if/Network.thrift:48-131
  - PrefixForwardingType / Algorithm       openr/if/OpenrConfig.thrift:162-182

Between Python and the C++ modules (the HIP-backed host library and the test
oracle) these objects travel as plain tuples (``to_wire`` / ``*_from_wire``),
so neither C++ module depends on the other's type definitions.
"""
from __future__ import annotations

import ipaddress
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

# Testing area name of the reference fixtures (openr/common/Util.h:62).
K_TESTING_AREA = "test_area_name"


class MplsActionCode:  # Network.thrift:24-31
    PUSH = 0
    SWAP = 1
    PHP = 2
    POP_AND_LOOKUP = 3
    NOOP = 4


class PrefixType:  # Network.thrift:105-120
    LOOPBACK = 1
    DEFAULT = 2
    BGP = 3
    PREFIX_ALLOCATOR = 4
    BREEZE = 5
    RIB = 6


class PrefixForwardingType:  # OpenrConfig.thrift:162-167
    IP = 0
    SR_MPLS = 1


class PrefixForwardingAlgorithm:  # OpenrConfig.thrift:169-182
    SP_ECMP = 0
    KSP2_ED_ECMP = 1


def addr_bytes(text: str) -> bytes:
    """toBinaryAddress(IPAddress(text)): 4 bytes for v4, 16 for v6."""
    return ipaddress.ip_address(text).packed


@dataclass(frozen=True)
class BinaryAddress:
    addr: bytes = b""
    ifName: Optional[str] = None

    @staticmethod
    def of(text: str, ifName: Optional[str] = None) -> "BinaryAddress":
        return BinaryAddress(addr_bytes(text), ifName)

    def __str__(self) -> str:
        if not self.addr:
            return ""
        ip = ipaddress.ip_address(self.addr)
        return f"{ip}%{self.ifName}" if self.ifName else str(ip)


@dataclass(frozen=True)
class IpPrefix:
    prefixAddress: BinaryAddress
    prefixLength: int

    @staticmethod
    def of(text: str) -> "IpPrefix":
        """toIpPrefix("a.b.c.d/len"); the network is masked like
        folly::IPAddress::createNetwork (openr/common/NetworkUtil.h:100-130)."""
        net = ipaddress.ip_network(text, strict=False)
        return IpPrefix(BinaryAddress(net.network_address.packed), net.prefixlen)

    def is_v4(self) -> bool:
        return len(self.prefixAddress.addr) == 4

    def __str__(self) -> str:
        return f"{ipaddress.ip_address(self.prefixAddress.addr)}/{self.prefixLength}"


@dataclass(frozen=True)
class MplsAction:
    action: int
    swapLabel: Optional[int] = None
    pushLabels: Optional[Tuple[int, ...]] = None


@dataclass(frozen=True)
class NextHopThrift:
    address: BinaryAddress
    weight: int = 0
    mplsAction: Optional[MplsAction] = None
    metric: int = 0
    area: Optional[str] = None
    neighborNodeName: Optional[str] = None

    def sort_key(self):
        a = self.mplsAction
        return (
            self.address.addr,
            self.address.ifName or "",
            self.weight,
            (-1,) if a is None else (a.action, a.swapLabel or -1, a.pushLabels or ()),
            self.metric,
            self.area or "",
            self.neighborNodeName or "",
        )


@dataclass
class Adjacency:
    otherNodeName: str
    ifName: str
    nextHopV6: BinaryAddress
    nextHopV4: BinaryAddress
    metric: int
    adjLabel: int = 0
    isOverloaded: bool = False
    rtt: int = 0
    timestamp: int = 0
    weight: int = 1
    otherIfName: str = ""

    def to_wire(self):
        return (self.otherNodeName, self.ifName, self.nextHopV6.addr,
                self.nextHopV4.addr, int(self.metric), int(self.adjLabel),
                bool(self.isOverloaded), int(self.rtt), int(self.timestamp),
                int(self.weight), self.otherIfName)


@dataclass
class AdjacencyDatabase:
    thisNodeName: str
    isOverloaded: bool = False
    adjacencies: List[Adjacency] = field(default_factory=list)
    nodeLabel: int = 0
    area: str = K_TESTING_AREA

    def to_wire(self):
        return (self.thisNodeName, bool(self.isOverloaded),
                [a.to_wire() for a in self.adjacencies], int(self.nodeLabel),
                self.area)


@dataclass(frozen=True)
class PrefixMetrics:
    version: int = 1
    path_preference: int = 0
    source_preference: int = 0
    distance: int = 0


@dataclass
class PrefixEntry:
    prefix: IpPrefix
    type: int = PrefixType.LOOPBACK
    data: Optional[bytes] = None
    forwardingType: int = PrefixForwardingType.IP
    forwardingAlgorithm: int = PrefixForwardingAlgorithm.SP_ECMP
    # legacy BGP MetricVector (Types.thrift:237-290) as
    # (version, ((type, priority, op, isBestPathTieBreaker, (metric, ...)), ...))
    mv: Optional[tuple] = None
    minNexthop: Optional[int] = None
    prependLabel: Optional[int] = None
    metrics: PrefixMetrics = field(default_factory=PrefixMetrics)
    tags: tuple = ()  # Types.thrift PrefixEntry.tags (RibPolicy tag matcher)

    def to_wire(self):
        m = self.metrics
        return (self.prefix.prefixAddress.addr, int(self.prefix.prefixLength),
                int(self.type), int(self.forwardingType),
                int(self.forwardingAlgorithm), self.minNexthop,
                self.prependLabel,
                (int(m.path_preference), int(m.source_preference), int(m.distance)),
                self.mv, self.data, tuple(sorted(self.tags)))


def prefix_entry_from_wire(w) -> PrefixEntry:
    addr, plen, typ, ft, fa, mn, pl, (pp, sp, d), mv, data = w[:10]
    tags = tuple(w[10]) if len(w) > 10 and w[10] is not None else ()
    if mv is not None:
        mv = (mv[0], tuple((t, p, o, tb, tuple(m)) for t, p, o, tb, m in mv[1]))
    return PrefixEntry(IpPrefix(BinaryAddress(addr), plen), typ, data, ft, fa,
                       mv, mn, pl, PrefixMetrics(1, pp, sp, d), tags)


def nexthop_from_wire(w) -> NextHopThrift:
    addr, ifname, weight, act, metric, area, nbr = w
    action = None
    if act is not None:
        code, swap, push = act
        action = MplsAction(code, swap, tuple(push) if push is not None else None)
    return NextHopThrift(BinaryAddress(addr, ifname), weight, action, metric,
                         area, nbr)


@dataclass
class UnicastRoute:
    """RibUnicastEntry (openr/decision/RibEntry.h:38-99) in canonical form."""
    dest: IpPrefix
    nextHops: List[NextHopThrift]
    doNotInstall: bool = False
    bestArea: str = ""
    bestPrefixEntry: Optional[PrefixEntry] = None

    def nexthop_set(self):
        return frozenset(self.nextHops)


@dataclass
class MplsRoute:
    """RibMplsEntry (openr/decision/RibEntry.h:101-144) in canonical form."""
    topLabel: int
    nextHops: List[NextHopThrift]

    def nexthop_set(self):
        return frozenset(self.nextHops)


@dataclass
class RouteDb:
    """DecisionRouteDb (openr/decision/Decision.h:78-119); routes keyed by
    prefix / label, nexthops sorted (canonical order)."""
    unicastRoutes: dict
    mplsRoutes: dict

    @staticmethod
    def from_wire(w) -> "RouteDb":
        ucast_w, mpls_w = w
        uc = {}
        for addr, plen, nhs, dni, best_area, best_entry in ucast_w:
            dest = IpPrefix(BinaryAddress(addr), plen)
            hops = sorted((nexthop_from_wire(n) for n in nhs),
                          key=NextHopThrift.sort_key)
            uc[dest] = UnicastRoute(
                dest, hops, dni, best_area,
                prefix_entry_from_wire(best_entry) if best_entry else None)
        mp = {}
        for label, nhs in mpls_w:
            hops = sorted((nexthop_from_wire(n) for n in nhs),
                          key=NextHopThrift.sort_key)
            mp[label] = MplsRoute(label, hops)
        db = RouteDb(uc, mp)
        db.wire = w  # the backend's own form, for calculate_update / apply_update
        return db

    def canonical(self):
        """Comparable form: nexthops as sets (the reference compares
        unordered_set<NextHopThrift>, DecisionTest.cpp:245-246)."""
        return (
            {str(k): (v.nexthop_set(), v.doNotInstall) for k, v in self.unicastRoutes.items()},
            {k: v.nexthop_set() for k, v in self.mplsRoutes.items()},
        )

    def canonical_full(self):
        """canonical() plus each route's bestArea and bestPrefixEntry (part of
        RibUnicastEntry equality, RibEntry.h:65-69), tags included."""
        def entry(e):
            if e is None:
                return None
            return (e.prefix, e.type, e.data, e.forwardingType, e.forwardingAlgorithm, e.mv,
                    e.minNexthop, e.prependLabel, e.metrics, tuple(sorted(e.tags)))
        return (
            {str(k): (v.nexthop_set(), v.doNotInstall, v.bestArea, entry(v.bestPrefixEntry))
             for k, v in self.unicastRoutes.items()},
            {k: v.nexthop_set() for k, v in self.mplsRoutes.items()},
        )


@dataclass
class RouteDbDelta:
    """DecisionRouteUpdate (openr/decision/RouteUpdate.h:23-41) as produced by
    DecisionRouteDb::calculateUpdate (Decision.cpp:108-143); list order is
    the backend's container order, so compare through canonical()."""
    unicastRoutesToUpdate: dict
    unicastRoutesToDelete: list
    mplsRoutesToUpdate: dict
    mplsRoutesToDelete: list

    @staticmethod
    def from_wire(w) -> "RouteDbDelta":
        uu, ud, mu, md = w
        upd = RouteDb.from_wire((uu, mu))
        return RouteDbDelta(upd.unicastRoutes,
                            [IpPrefix(BinaryAddress(a), l) for a, l in ud],
                            upd.mplsRoutes, list(md))

    def canonical(self):
        return (
            {str(k): (v.nexthop_set(), v.doNotInstall) for k, v in self.unicastRoutesToUpdate.items()},
            sorted(str(p) for p in self.unicastRoutesToDelete),
            {k: v.nexthop_set() for k, v in self.mplsRoutesToUpdate.items()},
            sorted(self.mplsRoutesToDelete),
        )


# ---------------------------------------------------------------------------
# Builders restating openr/common/Util.cpp helpers used by the fixtures
# ---------------------------------------------------------------------------

def create_adjacency(other: str, if_name: str, remote_if: str, nh_v6: str,
                     nh_v4: str, metric: int, adj_label: int,
                     weight: int = 1) -> Adjacency:
    """createAdjacency (openr/common/Util.cpp:582-604): rtt = metric*100."""
    return Adjacency(other, if_name, BinaryAddress.of(nh_v6),
                     BinaryAddress.of(nh_v4), metric, adj_label, False,
                     metric * 100, 0, weight, remote_if)


def create_adj_db(node: str, adjs: List[Adjacency], node_label: int,
                  overloaded: bool = False,
                  area: str = K_TESTING_AREA) -> AdjacencyDatabase:
    """createAdjDb (openr/common/Util.cpp:606-620)."""
    return AdjacencyDatabase(node, overloaded, list(adjs), node_label, area)


def create_prefix_entry(prefix: IpPrefix, typ: int = PrefixType.LOOPBACK,
                        forwarding_type: int = PrefixForwardingType.IP,
                        forwarding_algo: int = PrefixForwardingAlgorithm.SP_ECMP,
                        mv=None, min_nexthop: Optional[int] = None) -> PrefixEntry:
    """createPrefixEntry (openr/common/Util.cpp:638-656)."""
    return PrefixEntry(prefix, typ, None, forwarding_type, forwarding_algo,
                       mv, min_nexthop)


def create_mpls_action(code: int, swap: Optional[int] = None,
                       push: Optional[List[int]] = None) -> MplsAction:
    """createMplsAction (openr/common/Util.cpp:793-803)."""
    return MplsAction(code, swap, tuple(push) if push is not None else None)


def create_next_hop(addr: BinaryAddress, if_name: Optional[str] = None,
                    metric: int = 0, action: Optional[MplsAction] = None,
                    area: Optional[str] = None,
                    nbr: Optional[str] = None) -> NextHopThrift:
    """createNextHop (openr/common/Util.cpp:775-789); metric is int32."""
    return NextHopThrift(BinaryAddress(addr.addr, if_name), 0, action,
                         _i32(metric), area, nbr)


def _i32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v
