"""The wire output of device-built route databases (SURVEY.md §8f f3;
Types.thrift:1003-1060 RouteDatabase / RouteDatabaseDelta, Decision.h:92-104
DecisionRouteDb::toThrift).

The product builds the route database on the device path and serialises it in
C++ (SpfSolver build_route_db_thrift, DecisionRib rebuild_routes_thrift);
those bytes must equal the same Compact serialiser run over the oracle's
databases (and deltas: calculateUpdate of the oracle's builds), and decode
with the independent schema-less decoder (tests/compact_decode.py). The
serialiser writes routes in prefix / label order and nexthops in
NextHopThrift order (the reference lists unordered_* iteration order, see
DESIGN.md §9), so equal databases give equal bytes.

  C1 grid (node / adjacency labels)               RouteDatabase
  C3 Clos at 3,000 prefixes, both selection modes RouteDatabase
  random topologies with SR_MPLS / KSP2 prefixes   RouteDatabase
  C5 at 3,000 prefixes with the UCMP policy        RouteDatabase + two
                                                   RouteDatabaseDeltas (whole
                                                   and delta rebuilds)
"""
import random

import pytest

from compact_decode import decode
from openr_amd import host_module
from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid
from openr_amd.types import (IpPrefix, K_TESTING_AREA, PrefixEntry, PrefixForwardingAlgorithm,
                             PrefixForwardingType, PrefixMetrics, create_prefix_entry)
from openr_amd.workloads import C5_AREAS, c3_fabric, c5_multi_area

from test_gpu_parity import random_topology
from test_gpu_policy import _ucmp

pytestmark = pytest.mark.gpu


def _same_bytes(hip, oracle, adj, pfx, me, best_route=False):
    mod = host_module()
    als_h, ps_h = load_topology(hip, adj, pfx)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    sh = hip.spf_solver(me, True, enable_best_route_selection=best_route)
    got = sh._impl.build_route_db_thrift(me, als_h._impl, ps_h._impl)
    wire = oracle.spf_solver(me, True, enable_best_route_selection=best_route)._impl.build_route_db(
        me, als_o._impl, ps_o._impl)
    want = mod.route_db_thrift(wire, me)
    assert got == want
    d = decode(got)
    assert d[1] == me.encode()
    assert len(d[4]) == len(wire[0]) and len(d.get(5, [])) == len(wire[1])
    return d, sh


def test_route_db_bytes_c1(hip, oracle):
    adj, pfx = bench_grid(10, 1)
    d, sh = _same_bytes(hip, oracle, adj, pfx, "1")
    assert len(d[4]) == 99 and len(d[5]) == 99 + 3


@pytest.mark.parametrize("best_route", [False, True])
def test_route_db_bytes_c3(hip, oracle, best_route):
    adj, pfx = c3_fabric(num_prefixes=3000)
    d, sh = _same_bytes(hip, oracle, adj, pfx, "2-0-0", best_route)
    assert len(d[4]) > 2900
    assert sh.device_selected > 2900  # the device selection built them


@pytest.mark.parametrize("seed", range(2))
def test_route_db_bytes_ksp2_random(hip, oracle, seed):
    """SR_MPLS / KSP2 prefixes (PUSH / SWAP / PHP label stacks, KSP2 second
    paths traced on the device) on random graphs with parallel links."""
    dbs = random_topology(6100 + seed, n=20, extra=30, parallel=0.3)
    rng = random.Random(seed)
    pfx = []
    for i in range(60):
        for db in rng.sample(dbs, rng.randint(1, 3)):
            e = create_prefix_entry(IpPrefix.of(f"fc00:{seed}::{i:x}/128"))
            if rng.random() < 0.5:
                e.forwardingType = PrefixForwardingType.SR_MPLS
                if rng.random() < 0.6:
                    e.forwardingAlgorithm = PrefixForwardingAlgorithm.KSP2_ED_ECMP
            pfx.append((db.thisNodeName, K_TESTING_AREA, e))
    me = sorted(db.thisNodeName for db in dbs)[seed]
    d, _ = _same_bytes(hip, oracle, dbs, pfx, me)
    assert any(3 in nh for r in d[4] for nh in r[4])  # MPLS actions on the wire


def test_route_delta_bytes_c5_policy(hip, oracle):
    """Decision::rebuildRoutes with the C5 UCMP policy on the product
    (DecisionRib: a whole rebuild, then full rebuilds after prefix and metric
    changes, which run as deltas) against the oracle's buildRouteDb +
    applyPolicy and calculateUpdate, as RouteDatabase / RouteDatabaseDelta
    bytes."""
    mod = host_module()
    areas, pfx = c5_multi_area(num_prefixes=3000)
    adj = [db for a in C5_AREAS for db in areas[a]]
    als_h, ps_h = load_topology(hip, adj, pfx)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    sh = hip.spf_solver("me", True, enable_best_route_selection=True)
    so = oracle.spf_solver("me", True, enable_best_route_selection=True)
    ph = hip.rib_policy(_ucmp(), 3600)
    rib = hip.module.DecisionRib()
    prev_wire = ([], [])
    rng = random.Random(12)
    for rnd in range(3):
        delta = rib.rebuild_routes_thrift(sh._impl, "me", als_h._impl, ps_h._impl, True, [], ph._impl)
        cur = so._impl.build_route_db_with_policy("me", als_o._impl, ps_o._impl,
                                                  oracle.rib_policy(_ucmp(), 3600)._impl)
        assert delta == mod.route_delta_thrift(prev_wire, cur), rnd
        assert rib.route_db_thrift("me") == mod.route_db_thrift(cur, "me"), rnd
        dd = decode(delta)
        assert rnd > 0 or len(dd[2]) == len(cur[0])
        prev_wire = cur
        for _ in range(150):
            node, area, e = pfx[rng.randrange(len(pfx))]
            e2 = PrefixEntry(e.prefix, metrics=PrefixMetrics(1, rng.randint(0, 3), rng.randint(0, 3),
                                                             rng.randint(0, 3)), tags=e.tags)
            ps_h.update_prefix(node, area, e2)
            ps_o.update_prefix(node, area, e2)
        a = C5_AREAS[rnd % 4]
        db = areas[a][rng.randrange(len(areas[a]) - 1)]
        db.adjacencies[0].metric = rng.randint(1, 4)
        als_h[a].update_adjacency_database(db)
        als_o[a].update_adjacency_database(db)
    assert rib.delta_rebuilds >= 1


def _lists(wire):
    """prefix / label -> the nexthop list in the backend's unordered_set
    iteration order (what DecisionRouteDb::toThrift would list)."""
    uc = {(r[0], r[1]): [tuple(n) for n in r[2]] for r in wire[0]}
    mp = {m[0]: [tuple(n) for n in m[1]] for m in wire[1]}
    return uc, mp


def _ksp2_random(seed):
    dbs = random_topology(6200 + seed, n=20, extra=30, parallel=0.4)
    rng = random.Random(seed)
    pfx = []
    for i in range(60):
        for db in rng.sample(dbs, rng.randint(1, 3)):
            e = create_prefix_entry(IpPrefix.of(f"fc00:{seed}::{i:x}/128"))
            if rng.random() < 0.5:
                e.forwardingType = PrefixForwardingType.SR_MPLS
                if rng.random() < 0.6:
                    e.forwardingAlgorithm = PrefixForwardingAlgorithm.KSP2_ED_ECMP
            pfx.append((db.thisNodeName, K_TESTING_AREA, e))
    return dbs, pfx, sorted(db.thisNodeName for db in dbs)[seed]


@pytest.mark.parametrize("case", ["c1", "c3", "ksp2_0", "ksp2_1", "c5_policy", "c3_policy"])
def test_nexthop_list_order(hip, oracle, case):
    """every route's nexthops iterate - and toThrift would
    list them - in the oracle's order, i.e. std::unordered_set<NextHopThrift>
    with std::hash<NextHopThrift> (NetworkUtil.cpp:24-66) filled in the
    reference's insertion sequence: getNextHopsThrift's area / LinkSet loops
    (Decision.cpp:1245-1246, parallel links included), KSP2 paths, node-label
    SWAP / PHP routes, and RibPolicy's rebuild of a transformed route
    (RibPolicy.cpp:116-141). Routes built on the device (selection + template
    materialisation) and on the host path alike."""
    me, policy = "1", None
    if case == "c1":
        adj, pfx = bench_grid(10, 1)
    elif case == "c3":
        adj, pfx = c3_fabric(num_prefixes=3000)
        me = "2-0-0"
    elif case.startswith("ksp2"):
        adj, pfx, me = _ksp2_random(int(case[-1]))
    elif case == "c5_policy":
        areas, pfx = c5_multi_area(num_prefixes=3000)
        adj = [db for a in C5_AREAS for db in areas[a]]
        me, policy = "me", _ucmp()
    else:  # ~36-way ECMP routes rebuilt by a policy: some neighbours dropped, others reweighted
        from openr_amd.rib_policy import RibPolicyStatement, RibRouteActionWeight
        adj, pfx = c3_fabric(num_prefixes=3000)
        me = "2-0-0"
        nbrs = sorted({a.otherNodeName for db in adj if db.thisNodeName == me for a in db.adjacencies})
        rng = random.Random(77)
        weights = {n: rng.choice([0, 1, 3, 5]) for n in rng.sample(nbrs, len(nbrs) // 2)}
        some = rng.sample(sorted({e.prefix for _, _, e in pfx}, key=str), 1500)
        policy = [RibPolicyStatement("nbr", some, None, RibRouteActionWeight(2, {}, weights))]
    als_h, ps_h = load_topology(hip, adj, pfx)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    best = case.endswith("policy")
    sh = hip.spf_solver(me, True, enable_best_route_selection=best)._impl
    so = oracle.spf_solver(me, True, enable_best_route_selection=best)._impl
    if policy:
        wh = sh.build_route_db_with_policy(me, als_h._impl, ps_h._impl, hip.rib_policy(policy, 3600)._impl)
        wo = so.build_route_db_with_policy(me, als_o._impl, ps_o._impl, oracle.rib_policy(policy, 3600)._impl)
    else:
        wh = sh.build_route_db(me, als_h._impl, ps_h._impl)
        wo = so.build_route_db(me, als_o._impl, ps_o._impl)
    (uh, mh), (uo, mo) = _lists(wh), _lists(wo)
    assert uh.keys() == uo.keys() and mh.keys() == mo.keys()
    bad = [k for k in uo if uh[k] != uo[k]] + [k for k in mo if mh[k] != mo[k]]
    assert not bad, f"{len(bad)} of {len(uo) + len(mo)} routes list their nexthops in another order, e.g. {bad[0]}"
    if case != "c5_policy":  # (C5's `me` has one link per area: single-nexthop routes)
        assert sum(len(v) > 1 for v in list(uo.values()) + list(mo.values())) >= 5  # orders that can differ


def test_nexthop_list_order_after_linkset_rehash(hip, oracle):
    """the shared nexthop sets are cached across builds while the
    templates stay; a non-tight parallel link added to `me` leaves the tight
    templates as they were but can rehash my LinkSet and so reorder the
    links getNextHopsThrift inserts (Decision.cpp:1245-1246). After each of
    several such additions (both ends, so the link is up), every route's
    nexthop list must still be in the oracle's order."""
    import copy
    adj, pfx = c3_fabric(num_prefixes=2000)
    me = "2-0-0"
    by_name = {db.thisNodeName: db for db in adj}
    als_h, ps_h = load_topology(hip, adj, pfx)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    sh = hip.spf_solver(me, True)._impl
    so = oracle.spf_solver(me, True)._impl
    mine = list(by_name[me].adjacencies)
    rng = random.Random(808)
    multi = 0
    for step in range(5):
        (uh, mh), (uo, mo) = _lists(sh.build_route_db(me, als_h._impl, ps_h._impl)), \
            _lists(so.build_route_db(me, als_o._impl, ps_o._impl))
        assert uh.keys() == uo.keys() and mh.keys() == mo.keys()
        bad = [k for k in uo if uh[k] != uo[k]] + [k for k in mo if mh[k] != mo[k]]
        assert not bad, f"step {step}: {len(bad)} routes list their nexthops in another order, e.g. {bad[0]}"
        multi += sum(len(v) > 1 for v in uo.values())
        for i in range(12):  # non-tight parallel links me <-> a neighbour
            a = rng.choice(mine)
            peer = by_name[a.otherNodeName]
            back = next(b for b in peer.adjacencies if b.otherNodeName == me)
            tag = f"-p{step}.{i}"
            fwd, rev = copy.copy(a), copy.copy(back)
            fwd.ifName, fwd.otherIfName = a.ifName + tag, a.otherIfName + tag
            rev.ifName, rev.otherIfName = back.ifName + tag, back.otherIfName + tag
            fwd.metric = rev.metric = 5 + i
            # no adjacency label: a repeated one is a duplicate MPLS route,
            # which the reference CHECK-fails on (Decision.h:115-118)
            fwd.adjLabel = rev.adjLabel = 0
            by_name[me].adjacencies.append(fwd)
            peer.adjacencies.append(rev)
            for als in (als_h, als_o):
                als[K_TESTING_AREA].update_adjacency_database(peer)
        for als in (als_h, als_o):
            als[K_TESTING_AREA].update_adjacency_database(by_name[me])
    assert multi >= 5
