"""RibPolicy facade (openr/decision/RibPolicy.{h,cpp}; thrift types from
OpenrCtrl.thrift RibPolicy / RibPolicyStatement / RibRouteActionWeight).

The policy logic runs in the native host library (csrc/host/rib_policy.cpp);
these classes carry the thrift-shaped arguments and convert routes to and
from the wire tuples the library takes.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Sequence

from . import host_module
from .types import IpPrefix, NextHopThrift, PrefixEntry, UnicastRoute, nexthop_from_wire, \
    prefix_entry_from_wire, BinaryAddress


@dataclass
class RibRouteActionWeight:
    default_weight: int = 0
    area_to_weight: Dict[str, int] = field(default_factory=dict)
    neighbor_to_weight: Dict[str, int] = field(default_factory=dict)


@dataclass
class RibPolicyStatement:
    name: str = ""
    prefixes: Optional[List[IpPrefix]] = None  # matcher.prefixes
    tags: Optional[List[str]] = None           # matcher.tags
    set_weight: Optional[RibRouteActionWeight] = None  # action.set_weight

    def to_wire(self):
        w = self.set_weight
        return (self.name,
                None if self.prefixes is None else
                [(p.prefixAddress.addr, int(p.prefixLength)) for p in self.prefixes],
                None if self.tags is None else list(self.tags),
                None if w is None else (int(w.default_weight), dict(w.area_to_weight),
                                        dict(w.neighbor_to_weight)))


def create_policy_statement(prefixes: Optional[Sequence[IpPrefix]], tags: Optional[Sequence[str]],
                            default_weight: int, area_to_weight: Dict[str, int],
                            neighbor_to_weight: Optional[Dict[str, int]] = None,
                            name: str = "TestStatement") -> RibPolicyStatement:
    """createPolicyStatement of the reference tests (RibPolicyTest.cpp:22-41)."""
    return RibPolicyStatement(name, None if prefixes is None else list(prefixes),
                              None if tags is None else list(tags),
                              RibRouteActionWeight(default_weight, dict(area_to_weight),
                                                   dict(neighbor_to_weight or {})))


def route_to_wire(r: UnicastRoute):
    return (r.dest.prefixAddress.addr, int(r.dest.prefixLength),
            [_nh_to_wire(n) for n in r.nextHops], bool(r.doNotInstall), r.bestArea,
            r.bestPrefixEntry.to_wire() if r.bestPrefixEntry is not None else None)


def route_from_wire(w) -> UnicastRoute:
    addr, plen, nhs, dni, best_area, best_entry = w
    hops = sorted((nexthop_from_wire(n) for n in nhs), key=NextHopThrift.sort_key)
    return UnicastRoute(IpPrefix(BinaryAddress(addr), plen), hops, dni, best_area,
                        prefix_entry_from_wire(best_entry) if best_entry else None)


def _nh_to_wire(n: NextHopThrift):
    a = n.mplsAction
    act = None if a is None else (a.action, a.swapLabel,
                                  None if a.pushLabels is None else tuple(a.pushLabels))
    return (n.address.addr, n.address.ifName, int(n.weight), act, int(n.metric), n.area,
            n.neighborNodeName)


def unicast_entry(prefix: str, nexthops: Sequence[NextHopThrift] = (),
                  tags: Sequence[str] = ()) -> UnicastRoute:
    """RibUnicastEntry(prefix, nexthops) with an optional best prefix entry
    carrying `tags` (the tests' bestPrefixEntry.tags_ref()->insert)."""
    p = IpPrefix.of(prefix)
    best = PrefixEntry(p, tags=tuple(tags)) if tags else None
    return UnicastRoute(p, sorted(nexthops, key=NextHopThrift.sort_key), False, "", best)


class RibPolicyStatementCheck:
    """A lone RibPolicyStatement (match / applyAction). `module`: the native
    module that implements it (default: the product host library; the tests
    also pass the CPU oracle's, which has the same surface)."""

    def __init__(self, stmt: RibPolicyStatement, module=None):
        self._impl = (module or host_module()).RibPolicyStatement(stmt.to_wire())

    def match(self, route: UnicastRoute) -> bool:
        return self._impl.match(route_to_wire(route))

    def apply_action(self, route: UnicastRoute):
        changed, w = self._impl.apply_action(route_to_wire(route))
        return changed, route_from_wire(w)


class RibPolicy:
    """RibPolicy(thrift::RibPolicy): statements + ttl_secs."""

    def __init__(self, statements: Sequence[RibPolicyStatement], ttl_secs: int, module=None):
        self._impl = (module or host_module()).RibPolicy([s.to_wire() for s in statements],
                                                         int(ttl_secs))

    def is_active(self) -> bool:
        return self._impl.is_active()

    def get_ttl_duration_ms(self) -> int:
        return self._impl.ttl_ms()

    def match(self, route: UnicastRoute) -> bool:
        return self._impl.match(route_to_wire(route))

    def apply_action(self, route: UnicastRoute):
        changed, w = self._impl.apply_action(route_to_wire(route))
        return changed, route_from_wire(w)

    def apply_policy(self, routes: Dict[IpPrefix, UnicastRoute]):
        """Applies to every route; returns (updated prefixes, deleted
        prefixes, transformed routes keyed by prefix)."""
        up, dele, out = self._impl.apply_policy([route_to_wire(r) for r in routes.values()])
        res = {}
        for w in out:
            r = route_from_wire(w)
            res[r.dest] = r
        conv = [IpPrefix(BinaryAddress(a), l) for a, l in up]
        return conv, [IpPrefix(BinaryAddress(a), l) for a, l in dele], res

    @property
    def invalidated_routes(self) -> int:
        return self._impl.invalidated_routes
