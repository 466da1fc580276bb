"""Pythonic facade over a wire-level Decision backend module.

Mirrors the reference's public interface for the route-computation path:
  LinkState          openr/decision/LinkState.h:177-469
  PrefixState        openr/decision/PrefixState.h:22-70
  SpfSolver          openr/decision/Decision.h:200-251
with snake_case method names and Python value types (openr_amd.types).

``Backend(module)`` wraps any extension module that implements the wire-level
API (tuples in, tuples out).  The product module is ``openr_amd._openr_host``
(C++ host library over libopenr_hip); the test suite also wraps the CPU
oracle with the same facade, so a parity test is the same code run twice.
"""
from __future__ import annotations

from collections import namedtuple
from typing import Iterable, List, Optional

from .types import (AdjacencyDatabase, BinaryAddress, IpPrefix, NextHopThrift,
                    PrefixEntry, RouteDb, RouteDbDelta, UnicastRoute, nexthop_from_wire,
                    prefix_entry_from_wire)

LinkStateChange = namedtuple(
    "LinkStateChange", "topologyChanged linkAttributesChanged nodeLabelChanged")

# (firstNodeName, ifName on first, secondNodeName, ifName on second)
LinkDesc = namedtuple("LinkDesc", "n1 if1 n2 if2")


class NodeSpfResult:
    __slots__ = ("metric", "nextHops", "pathLinks")

    def __init__(self, metric, next_hops, path_links=()):
        self.metric = metric
        self.nextHops = frozenset(next_hops)
        self.pathLinks = [(LinkDesc(*l), prev) for l, prev in path_links]

    def __repr__(self):
        return f"NodeSpfResult(metric={self.metric}, nextHops={sorted(self.nextHops)})"


class LinkState:
    def __init__(self, impl):
        self._impl = impl

    def update_adjacency_database(self, db: AdjacencyDatabase, hold_up_ttl: int = 0,
                                  hold_down_ttl: int = 0) -> LinkStateChange:
        return LinkStateChange(*self._impl.update_adjacency_database(
            db.to_wire(), hold_up_ttl, hold_down_ttl))

    def delete_adjacency_database(self, node: str) -> LinkStateChange:
        return LinkStateChange(*self._impl.delete_adjacency_database(node))

    def decrement_holds(self) -> LinkStateChange:
        return LinkStateChange(*self._impl.decrement_holds())

    def has_holds(self) -> bool:
        return self._impl.has_holds()

    def has_node(self, node: str) -> bool:
        return self._impl.has_node(node)

    def is_node_overloaded(self, node: str) -> bool:
        return self._impl.is_node_overloaded(node)

    def num_links(self) -> int:
        return self._impl.num_links()

    def num_nodes(self) -> int:
        return self._impl.num_nodes()

    @property
    def spf_runs(self) -> int:
        return self._impl.spf_runs

    def links_from_node(self, node: str) -> List[LinkDesc]:
        return [LinkDesc(*l) for l in self._impl.links_from_node(node)]

    def get_spf_result(self, node: str, use_link_metric: bool = True):
        raw = self._impl.get_spf_result(node, use_link_metric)
        return {k: NodeSpfResult(*v) for k, v in raw.items()}

    def get_kth_paths(self, src: str, dst: str, k: int) -> List[List[LinkDesc]]:
        return [[LinkDesc(*l) for l in p] for p in self._impl.get_kth_paths(src, dst, k)]

    def get_metric_from_a_to_b(self, a: str, b: str, use_link_metric: bool = True):
        return self._impl.get_metric_from_a_to_b(a, b, use_link_metric)

    def get_hops_from_a_to_b(self, a: str, b: str):
        return self._impl.get_hops_from_a_to_b(a, b)

    def get_max_hops_to_node(self, node: str) -> int:
        return self._impl.get_max_hops_to_node(node)

    def metric_from_node(self, link: LinkDesc, node: str) -> int:
        return self._impl.metric_from_node(link.n1, link.if1, node)


class AreaLinkStates:
    """std::unordered_map<std::string /* area */, LinkState>."""

    def __init__(self, backend_mod, lane: int = 0):
        self._impl = backend_mod.AreaLinkStates(lane) if lane else backend_mod.AreaLinkStates()
        self._areas = {}

    def add_area(self, area: str) -> LinkState:
        self._impl.add_area(area)
        self._areas[area] = LinkState(self._impl.area(area))
        return self._areas[area]

    def area(self, area: str) -> LinkState:
        return self._areas[area]

    def __getitem__(self, area: str) -> LinkState:
        return self._areas[area]

    def areas(self):
        return list(self._areas)


class PrefixState:
    def __init__(self, backend_mod):
        self._impl = backend_mod.PrefixState()

    def update_prefix(self, node: str, area: str, entry: PrefixEntry):
        return {IpPrefix(BinaryAddress(a), l)
                for a, l in self._impl.update_prefix(node, area, entry.to_wire())}

    def delete_prefix(self, node: str, area: str, prefix: IpPrefix):
        return {IpPrefix(BinaryAddress(a), l) for a, l in self._impl.delete_prefix(
            node, area, prefix.prefixAddress.addr, prefix.prefixLength)}

    def num_prefixes(self) -> int:
        return self._impl.num_prefixes()


def _route_from_wire(w) -> UnicastRoute:
    addr, plen, nhs, dni, best_area, best = w
    hops = sorted((nexthop_from_wire(n) for n in nhs), key=NextHopThrift.sort_key)
    return UnicastRoute(IpPrefix(BinaryAddress(addr), plen), hops, dni, best_area,
                        prefix_entry_from_wire(best) if best else None)


def _nh_to_wire(nh: NextHopThrift):
    a = nh.mplsAction
    act = None if a is None else (a.action, a.swapLabel,
                                  list(a.pushLabels) if a.pushLabels is not None else None)
    return (nh.address.addr, nh.address.ifName, nh.weight, act, nh.metric, nh.area,
            nh.neighborNodeName)


class SpfSolver:
    def __init__(self, backend_mod, my_node: str, enable_v4: bool,
                 enable_ordered_fib: bool = False, bgp_dry_run: bool = False,
                 enable_best_route_selection: bool = False):
        self._impl = backend_mod.SpfSolver(my_node, enable_v4, enable_ordered_fib,
                                           bgp_dry_run, enable_best_route_selection)

    def build_route_db(self, my_node: str, als: AreaLinkStates,
                       ps: PrefixState) -> Optional[RouteDb]:
        w = self._impl.build_route_db(my_node, als._impl, ps._impl)
        return None if w is None else RouteDb.from_wire(w)

    def build_route_db_with_policy(self, my_node: str, als: AreaLinkStates, ps: PrefixState,
                                   policy) -> Optional[RouteDb]:
        """buildRouteDb, then RibPolicy::applyPolicy over its unicast routes
        (Decision::rebuildRoutes, Decision.cpp:1888-1900); `policy` is an
        openr_amd.rib_policy.RibPolicy of the same backend."""
        w = self._impl.build_route_db_with_policy(my_node, als._impl, ps._impl, policy._impl)
        return None if w is None else RouteDb.from_wire(w)

    def create_route_for_prefix_or_get_static_route(self, my_node, als, ps,
                                                    prefix: IpPrefix):
        w = self._impl.create_route_for_prefix_or_get_static_route(
            my_node, als._impl, ps._impl, prefix.prefixAddress.addr, prefix.prefixLength)
        return None if w is None else _route_from_wire(w)

    def update_static_unicast_routes(self, upd, dele: Iterable[IpPrefix] = ()):
        self._impl.update_static_unicast_routes(
            [(p.prefixAddress.addr, p.prefixLength, [_nh_to_wire(n) for n in nhs])
             for p, nhs in upd],
            [(p.prefixAddress.addr, p.prefixLength) for p in dele])

    def update_static_mpls_routes(self, upd, dele: Iterable[int] = ()):
        self._impl.update_static_mpls_routes(
            [(label, [_nh_to_wire(n) for n in nhs]) for label, nhs in upd], list(dele))

    @property
    def route_build_runs(self) -> int:
        return self._impl.route_build_runs

    @property
    def device_selected(self) -> int:
        """Prefixes of the last build selected by the device kernel (product only)."""
        return getattr(self._impl, "device_selected", 0)

    @property
    def host_selected(self) -> int:
        return getattr(self._impl, "host_selected", 0)


class Backend:
    """Bundle of the facade classes bound to one wire-level module."""

    def __init__(self, module, name: str):
        self.module = module
        self.name = name

    def area_link_states(self, *areas, lane: int = 0) -> AreaLinkStates:
        """lane > 0: the areas' device work goes to stream lane `lane` (its own
        context and HIP stream), so independent topologies overlap on the GPU."""
        als = AreaLinkStates(self.module, lane) if lane else AreaLinkStates(self.module)
        for a in areas:
            als.add_area(a)
        return als

    def prefix_state(self) -> PrefixState:
        return PrefixState(self.module)

    def spf_solver(self, my_node: str, enable_v4: bool, enable_ordered_fib=False,
                   bgp_dry_run=False, enable_best_route_selection=False) -> SpfSolver:
        return SpfSolver(self.module, my_node, enable_v4, enable_ordered_fib,
                         bgp_dry_run, enable_best_route_selection)

    def rib_policy(self, statements, ttl_secs: int):
        """RibPolicy(thrift::RibPolicy) of this backend (RibPolicy.cpp:164-178)."""
        from .rib_policy import RibPolicy
        return RibPolicy(statements, ttl_secs, module=self.module)

    def calculate_update(self, old_db: RouteDb, new_db: RouteDb) -> RouteDbDelta:
        """DecisionRouteDb::calculateUpdate (Decision.cpp:108-143)."""
        return RouteDbDelta.from_wire(self.module.calculate_update(old_db.wire, new_db.wire))

    def apply_update(self, db: RouteDb, delta_wire) -> RouteDb:
        """DecisionRouteDb::update (Decision.cpp:146-160)."""
        return RouteDb.from_wire(self.module.apply_update(db.wire, delta_wire))

    def __repr__(self):
        return f"Backend({self.name})"


def load_topology(backend: Backend, adj_dbs, prefixes, als=None, ps=None, lane: int = 0):
    """Feed generator output (openr_amd.topology) into a backend."""
    if als is None:
        areas = sorted({db.area for db in adj_dbs} | {a for _, a, _ in prefixes})
        als = backend.area_link_states(*areas, lane=lane) if lane else backend.area_link_states(*areas)
    if ps is None:
        ps = backend.prefix_state()
    for db in adj_dbs:
        als[db.area].update_adjacency_database(db)
    # PrefixState::updatePrefix for every advertisement, in order, a chunk per
    # call (no changed-prefix set is built for the caller)
    chunk = 1 << 16
    for i in range(0, len(prefixes), chunk):
        ps._impl.update_prefixes([(node, area, entry.to_wire()) for node, area, entry in prefixes[i:i + chunk]])
    return als, ps
