"""More known-answer tests transcribed from openr/decision/tests/DecisionTest.cpp
(best-route selection, connectivity, overload, KSP2 on the ring and ring-mesh
fixtures, BGP metric-vector redistribution, multi-area). Every expected value
is the reference's own assertion, cited by line. Each test runs on the CPU
oracle (``-m "not gpu"``) and on the HIP product (``-m gpu``), so these pins
are independent of both implementations' reading of Decision.cpp.
"""
import pytest

from helpers import PHP, adj_label_nexthops, nh_from_adj, pop_route, push, route_map, swap
from openr_amd.topology import adj
from openr_amd.types import (K_TESTING_AREA, IpPrefix, PrefixEntry, PrefixForwardingAlgorithm,
                             PrefixForwardingType, PrefixMetrics, PrefixType, create_adj_db,
                             create_adjacency, create_prefix_entry)

A = K_TESTING_AREA
ADDR = {i: IpPrefix.of(f"::ffff:10.{i}.{i}.{i}/128") for i in range(1, 5)}  # :87-90
ADDR_V4 = {i: IpPrefix.of(f"10.{i}.{i}.{i}/32") for i in range(1, 5)}     # :93-96

# :46-85 adjacencies not in openr_amd.topology.RING_ADJ
ADJ12_OLD_1 = lambda: create_adjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 1000021)
ADJ12_OLD_2 = lambda: create_adjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 20, 1000022)
ADJ13_OLD = lambda: create_adjacency("3", "1/3", "3/1", "fe80::3", "192.168.0.3", 10, 1000031)
ADJ21_OLD_1 = lambda: create_adjacency("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 1000011)
ADJ31_OLD = lambda: create_adjacency("1", "3/1", "1/3", "fe80::1", "192.168.0.1", 10, 1000011)


def _pfx(addr):
    return create_prefix_entry(addr)


def _validate_pop_and_adj(rm, node, db):
    """validatePopLabelRoute + validateAdjLabelRoutes (:336-368)."""
    assert rm[(node, str(db.nodeLabel))] == {pop_route()}
    for label, nhs in adj_label_nexthops(db.adjacencies).items():
        assert rm[(node, str(label))] == nhs


# ---------------------------------------------------------------------------
# Decision.BestRouteSelection (:1139-1272)
# ---------------------------------------------------------------------------

def test_best_route_selection(backend):
    als = backend.area_link_states(A)
    ls = als[A]
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False, enable_best_route_selection=True)
    assert not ls.update_adjacency_database(create_adj_db("1", [adj("adj12"), adj("adj13")], 1)).topologyChanged
    assert ls.update_adjacency_database(create_adj_db("2", [adj("adj21")], 2)).topologyChanged
    assert ls.update_adjacency_database(create_adj_db("3", [adj("adj31")], 3)).topologyChanged

    def entry(pp, sp, d, ft=PrefixForwardingType.IP):
        return PrefixEntry(ADDR[1], PrefixType.DEFAULT, None, ft,
                           PrefixForwardingAlgorithm.SP_ECMP, None, None, None,
                           PrefixMetrics(1, pp, sp, d))

    assert ps.update_prefix("2", A, entry(200, 0, 0))
    assert ps.update_prefix("3", A, entry(200, 0, 0))
    # Case-1: ECMP towards {2, 3}; best node area "2" (:1185-1213)
    db = solver.build_route_db("1", als, ps)
    assert len(db.unicastRoutes) == 1
    r = db.unicastRoutes[ADDR[1]]
    assert r.nexthop_set() == {nh_from_adj(adj("adj12"), False, 10),
                               nh_from_adj(adj("adj13"), False, 10)}
    assert r.bestArea == A and r.bestPrefixEntry.metrics == PrefixMetrics(1, 200, 0, 0)
    # Case-2: node 2 preferred by source preference (:1216-1246)
    assert ps.update_prefix("2", A, entry(200, 100, 0))
    db = solver.build_route_db("1", als, ps)
    assert len(db.unicastRoutes) == 1
    r = db.unicastRoutes[ADDR[1]]
    assert r.nexthop_set() == {nh_from_adj(adj("adj12"), False, 10)}
    assert r.bestPrefixEntry.metrics == PrefixMetrics(1, 200, 100, 0)
    # forwarding type taken from the best entry: node 2's SR_MPLS (:1248-1271)
    assert ps.update_prefix("2", A, entry(200, 100, 0, PrefixForwardingType.SR_MPLS))
    db = solver.build_route_db("3", als, ps)
    assert len(db.unicastRoutes) == 1
    assert db.unicastRoutes[ADDR[1]].nexthop_set() == {
        nh_from_adj(adj("adj31"), False, 20, push(2))}


# ---------------------------------------------------------------------------
# ConnectivityTest (:1281-1558)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("partitioned", [False, True])
def test_graph_connected_or_partitioned(backend, partitioned):
    db1 = create_adj_db("1", [] if partitioned else [adj("adj12")], 1)
    db2 = create_adj_db("2", [adj("adj21"), adj("adj23")], 2)
    db3 = create_adj_db("3", [] if partitioned else [adj("adj32")], 3)
    als = backend.area_link_states(A)
    ls = als[A]
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    assert tuple(ls.update_adjacency_database(db1)) == (False, False, True)
    assert tuple(ls.update_adjacency_database(db2)) == (not partitioned, False, True)
    assert tuple(ls.update_adjacency_database(db3)) == (not partitioned, False, True)
    for i in (1, 2, 3):
        assert ps.update_prefix(str(i), A, _pfx(ADDR[i]))
    db = solver.build_route_db("1", als, ps)
    found_v6 = db is not None and ADDR[3] in db.unicastRoutes
    found_label = db is not None and 3 in db.mplsRoutes
    assert partitioned == (not found_v6)
    assert partitioned == (not found_label)


def test_connectivity_overload_node(backend):
    """1 - 2 - 3 with node 2 overloaded (:1348-1435)."""
    als = backend.area_link_states(A)
    ls = als[A]
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    db1 = create_adj_db("1", [adj("adj12")], 1)
    db2 = create_adj_db("2", [adj("adj21"), adj("adj23")], 2, True)
    db3 = create_adj_db("3", [adj("adj32")], 3)
    for i in (1, 2, 3):
        assert ps.update_prefix(str(i), A, _pfx(ADDR[i]))
    assert not ls.update_adjacency_database(db1).topologyChanged
    assert ls.update_adjacency_database(db2).topologyChanged
    assert ls.update_adjacency_database(db3).topologyChanged
    rm = route_map(solver, ["1", "2", "3"], als, ps)
    assert len(rm) == 15
    assert rm[("1", str(ADDR[2]))] == {nh_from_adj(adj("adj12"), False, 10)}
    assert rm[("1", "2")] == {nh_from_adj(adj("adj12"), False, 10, PHP)}
    _validate_pop_and_adj(rm, "1", db1)
    assert rm[("2", str(ADDR[3]))] == {nh_from_adj(adj("adj23"), False, 10)}
    assert rm[("2", str(ADDR[1]))] == {nh_from_adj(adj("adj21"), False, 10)}
    assert rm[("2", "1")] == {nh_from_adj(adj("adj21"), False, 10, PHP)}
    assert rm[("2", "3")] == {nh_from_adj(adj("adj23"), False, 10, PHP)}
    _validate_pop_and_adj(rm, "2", db2)
    assert rm[("3", str(ADDR[2]))] == {nh_from_adj(adj("adj32"), False, 10)}
    assert rm[("3", "2")] == {nh_from_adj(adj("adj32"), False, 10, PHP)}
    _validate_pop_and_adj(rm, "3", db3)


def test_connectivity_compatibility_node(backend):
    """Adjacencies re-advertised with old labels / metrics (:1446-1558)."""
    als = backend.area_link_states(A)
    ls = als[A]
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    db1 = create_adj_db("1", [ADJ12_OLD_1()], 1)
    db2 = create_adj_db("2", [ADJ21_OLD_1(), adj("adj23")], 2)
    db3 = create_adj_db("3", [adj("adj32"), ADJ31_OLD()], 3)
    for i in (1, 2, 3):
        assert ps.update_prefix(str(i), A, _pfx(ADDR[i]))
    assert not ls.update_adjacency_database(db2).topologyChanged
    assert ls.update_adjacency_database(db3).topologyChanged
    assert ls.update_adjacency_database(db1).topologyChanged
    db1 = create_adj_db("1", [ADJ12_OLD_1(), ADJ13_OLD()], 1)
    assert ls.update_adjacency_database(db1).topologyChanged
    db1 = create_adj_db("1", [ADJ12_OLD_2(), ADJ13_OLD()], 1)
    assert ls.update_adjacency_database(db1).topologyChanged
    rm = route_map(solver, ["1", "2", "3"], als, ps)
    assert len(rm) == 21
    assert rm[("1", str(ADDR[2]))] == {nh_from_adj(ADJ12_OLD_2(), False, 20),
                                       nh_from_adj(ADJ13_OLD(), False, 20)}
    assert rm[("1", str(ADDR[3]))] == {nh_from_adj(adj("adj13"), False, 10)}
    assert rm[("1", "2")] == {nh_from_adj(ADJ12_OLD_2(), False, 20, PHP),
                              nh_from_adj(ADJ13_OLD(), False, 20, swap(2))}
    assert rm[("1", "3")] == {nh_from_adj(ADJ13_OLD(), False, 10, PHP)}
    _validate_pop_and_adj(rm, "1", db1)
    assert rm[("2", str(ADDR[3]))] == {nh_from_adj(adj("adj23"), False, 10)}
    assert rm[("2", str(ADDR[1]))] == {nh_from_adj(adj("adj21"), False, 10)}
    assert rm[("2", "1")] == {nh_from_adj(adj("adj21"), False, 10, PHP)}
    assert rm[("2", "3")] == {nh_from_adj(adj("adj23"), False, 10, PHP)}
    assert rm[("3", str(ADDR[2]))] == {nh_from_adj(adj("adj32"), False, 10)}
    assert rm[("3", str(ADDR[1]))] == {nh_from_adj(adj("adj31"), False, 10)}
    assert rm[("3", "1")] == {nh_from_adj(adj("adj31"), False, 10, PHP)}
    assert rm[("3", "2")] == {nh_from_adj(adj("adj32"), False, 10, PHP)}
    _validate_pop_and_adj(rm, "3", db3)
    # removals (:1550-1557)
    assert ls.update_adjacency_database(create_adj_db("1", [ADJ12_OLD_2()], 0)).topologyChanged
    assert not ls.update_adjacency_database(create_adj_db("3", [adj("adj32")], 0)).topologyChanged
    assert not ls.update_adjacency_database(
        create_adj_db("1", [ADJ12_OLD_2(), ADJ13_OLD()], 0)).topologyChanged


# ---------------------------------------------------------------------------
# MplsRoutes.BasicTest (:737-780)
# ---------------------------------------------------------------------------

def test_mpls_routes_basic(backend):
    als = backend.area_link_states(A)
    ls = als[A]
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    db1 = create_adj_db("1", [adj("adj12")], 1)
    db2 = create_adj_db("2", [adj("adj23")], 0)
    db3 = create_adj_db("3", [adj("adj32")], 3)
    assert tuple(ls.update_adjacency_database(db1)) == (False, False, True)
    assert tuple(ls.update_adjacency_database(db1)) == (False, False, False)
    assert tuple(ls.update_adjacency_database(db2)) == (False, False, False)
    assert tuple(ls.update_adjacency_database(db3)) == (True, False, True)
    rm = route_map(solver, ["1", "2", "3"], als, ps)
    assert len(rm) == 5
    assert rm[("1", "1")] == {pop_route()}
    for label, nhs in adj_label_nexthops([adj("adj23")]).items():
        assert rm[("2", str(label))] == nhs
    _validate_pop_and_adj(rm, "3", db3)


# ---------------------------------------------------------------------------
# Simple ring (:1766-1892) and ring-mesh (:1571-1680) fixtures
# ---------------------------------------------------------------------------

def _ring_setup(backend, v4, ksp2, bgp, mesh=False):
    if mesh:
        names = {1: ("adj12", "adj13", "adj14"), 2: ("adj21", "adj23", "adj24"),
                 3: ("adj31", "adj32", "adj34"), 4: ("adj41", "adj42", "adj43")}
    else:
        names = {1: ("adj12", "adj13"), 2: ("adj21", "adj24"), 3: ("adj31", "adj34"),
                 4: ("adj42", "adj43")}
    dbs = {i: create_adj_db(str(i), [adj(n) for n in names[i]], i) for i in range(1, 5)}
    als = backend.area_link_states(A)
    ls = als[A]
    assert tuple(ls.update_adjacency_database(dbs[1])) == (False, False, True)
    for i in (2, 3, 4):
        assert tuple(ls.update_adjacency_database(dbs[i])) == (True, False, True)
    ps = backend.prefix_state()
    for i in range(1, 5):
        e = _pfx((ADDR_V4 if v4 else ADDR)[i])
        entries = [e]
        if ksp2:  # createPrefixDbWithKspfAlgo (:167-206)
            e.forwardingType = PrefixForwardingType.SR_MPLS
            e.forwardingAlgorithm = PrefixForwardingAlgorithm.KSP2_ED_ECMP
            if bgp:
                e.type = PrefixType.BGP
                e.mv = (0, ())
                lo = IpPrefix.of(f"172.0.0.{i}/32" if v4 else f"fd00::{i}/128")  # :156-165
                entries.append(_pfx(lo))
        for x in entries:
            ps.update_prefix(str(i), A, x)
    solver = backend.spf_solver("1", v4)
    return dbs, als, ps, solver


@pytest.mark.parametrize("v4", [False, True])
@pytest.mark.parametrize("bgp", [False, True])
def test_ring_mesh_ksp2(backend, v4, bgp):
    """SimpleRingMeshTopologyFixture.Ksp2EdEcmp (:1682-1754)."""
    dbs, als, ps, solver = _ring_setup(backend, v4, True, bgp, mesh=True)
    rm = route_map(solver, ["1"], als, ps)
    addr = ADDR_V4 if v4 else ADDR
    a = adj
    assert rm[("1", str(addr[4]))] == {nh_from_adj(a("adj14"), v4, 10),
                                       nh_from_adj(a("adj12"), v4, 20, push(4)),
                                       nh_from_adj(a("adj13"), v4, 20, push(4))}
    assert rm[("1", "4")] == {nh_from_adj(a("adj14"), False, 10, PHP)}
    assert rm[("1", str(addr[3]))] == {nh_from_adj(a("adj13"), v4, 10),
                                       nh_from_adj(a("adj12"), v4, 20, push(3)),
                                       nh_from_adj(a("adj14"), v4, 20, push(3))}
    assert rm[("1", str(addr[2]))] == {nh_from_adj(a("adj12"), v4, 10),
                                       nh_from_adj(a("adj13"), v4, 20, push(2)),
                                       nh_from_adj(a("adj14"), v4, 20, push(2))}
    _validate_pop_and_adj(rm, "1", dbs[1])
    dbs[3].isOverloaded = True
    assert als[A].update_adjacency_database(dbs[3]).topologyChanged
    rm = route_map(solver, ["1"], als, ps)
    assert rm[("1", str(addr[4]))] == {nh_from_adj(a("adj14"), v4, 10),
                                       nh_from_adj(a("adj12"), v4, 20, push(4))}


@pytest.mark.parametrize("v4", [False, True])
@pytest.mark.parametrize("bgp", [False, True])
def test_ring_ksp2(backend, v4, bgp):
    """SimpleRingTopologyFixture.Ksp2EdEcmp (:2398-2600), including the
    decision.spf_runs count of 16 (4 memoized + 12 k=2 re-runs)."""
    dbs, als, ps, solver = _ring_setup(backend, v4, True, bgp)
    ls = als[A]
    runs0 = ls.spf_runs
    rm = route_map(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == (48 if bgp else 36)
    assert ls.spf_runs - runs0 == 16
    addr = ADDR_V4 if v4 else ADDR
    a = adj
    u = lambda n, d: rm[(n, str(addr[d]))]
    assert u("1", 4) == {nh_from_adj(a("adj12"), v4, 20, push(4)),
                         nh_from_adj(a("adj13"), v4, 20, push(4))}
    assert rm[("1", "4")] == {nh_from_adj(a("adj12"), False, 20, swap(4)),
                              nh_from_adj(a("adj13"), False, 20, swap(4))}
    assert u("1", 3) == {nh_from_adj(a("adj13"), v4, 10), nh_from_adj(a("adj12"), v4, 30, push(3, 4))}
    assert rm[("1", "3")] == {nh_from_adj(a("adj13"), False, 10, PHP)}
    assert u("1", 2) == {nh_from_adj(a("adj12"), v4, 10), nh_from_adj(a("adj13"), v4, 30, push(2, 4))}
    assert rm[("1", "2")] == {nh_from_adj(a("adj12"), False, 10, PHP)}
    _validate_pop_and_adj(rm, "1", dbs[1])
    assert u("2", 4) == {nh_from_adj(a("adj24"), v4, 10), nh_from_adj(a("adj21"), v4, 30, push(4, 3))}
    assert rm[("2", "4")] == {nh_from_adj(a("adj24"), False, 10, PHP)}
    assert u("2", 3) == {nh_from_adj(a("adj21"), v4, 20, push(3)),
                         nh_from_adj(a("adj24"), v4, 20, push(3))}
    assert rm[("2", "3")] == {nh_from_adj(a("adj21"), False, 20, swap(3)),
                              nh_from_adj(a("adj24"), False, 20, swap(3))}
    assert u("2", 1) == {nh_from_adj(a("adj21"), v4, 10), nh_from_adj(a("adj24"), v4, 30, push(1, 3))}
    assert rm[("2", "1")] == {nh_from_adj(a("adj21"), False, 10, PHP)}
    _validate_pop_and_adj(rm, "2", dbs[2])
    assert u("3", 4) == {nh_from_adj(a("adj34"), v4, 10), nh_from_adj(a("adj31"), v4, 30, push(4, 2))}
    assert u("3", 2) == {nh_from_adj(a("adj31"), v4, 20, push(2)),
                         nh_from_adj(a("adj34"), v4, 20, push(2))}
    assert rm[("3", "2")] == {nh_from_adj(a("adj31"), False, 20, swap(2)),
                              nh_from_adj(a("adj34"), False, 20, swap(2))}
    assert u("3", 1) == {nh_from_adj(a("adj31"), v4, 10), nh_from_adj(a("adj34"), v4, 30, push(1, 2))}
    _validate_pop_and_adj(rm, "3", dbs[3])
    assert u("4", 3) == {nh_from_adj(a("adj43"), v4, 10), nh_from_adj(a("adj42"), v4, 30, push(3, 1))}
    assert u("4", 2) == {nh_from_adj(a("adj42"), v4, 10), nh_from_adj(a("adj43"), v4, 30, push(2, 1))}
    assert u("4", 1) == {nh_from_adj(a("adj42"), v4, 20, push(1)),
                         nh_from_adj(a("adj43"), v4, 20, push(1))}
    assert rm[("4", "1")] == {nh_from_adj(a("adj42"), False, 20, swap(1)),
                              nh_from_adj(a("adj43"), False, 20, swap(1))}
    _validate_pop_and_adj(rm, "4", dbs[4])
    # node 3 overloaded and link 1-2 drained: no route from 1 to 2 or 4 (:2579-2599)
    dbs[1].adjacencies[0].isOverloaded = True
    dbs[3].isOverloaded = True
    assert ls.update_adjacency_database(dbs[1]).topologyChanged
    assert ls.update_adjacency_database(dbs[3]).topologyChanged
    rm = route_map(solver, ["1"], als, ps)
    assert ("1", str(addr[4])) not in rm
    assert rm[("1", str(addr[3]))] == {nh_from_adj(a("adj13"), v4, 10)}
    assert ("1", str(addr[2])) not in rm


@pytest.mark.parametrize("v4", [False, True])
def test_ring_overload_node(backend, v4):
    """SimpleRingTopologyFixture.OverloadNodeTest (:2974-3087)."""
    dbs, als, ps, solver = _ring_setup(backend, v4, False, False)
    ls = als[A]
    dbs[2].isOverloaded = True
    dbs[3].isOverloaded = True
    assert ls.update_adjacency_database(dbs[2]).topologyChanged
    assert ls.update_adjacency_database(dbs[3]).topologyChanged
    rm = route_map(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == 32
    addr = ADDR_V4 if v4 else ADDR
    a = adj
    u = lambda n, d: rm[(n, str(addr[d]))]
    assert u("1", 3) == {nh_from_adj(a("adj13"), v4, 10)}
    assert rm[("1", "3")] == {nh_from_adj(a("adj13"), False, 10, PHP)}
    assert u("1", 2) == {nh_from_adj(a("adj12"), v4, 10)}
    assert rm[("1", "2")] == {nh_from_adj(a("adj12"), False, 10, PHP)}
    _validate_pop_and_adj(rm, "1", dbs[1])
    assert u("2", 4) == {nh_from_adj(a("adj24"), v4, 10)}
    assert u("2", 3) == {nh_from_adj(a("adj21"), v4, 20), nh_from_adj(a("adj24"), v4, 20)}
    assert rm[("2", "3")] == {nh_from_adj(a("adj21"), False, 20, swap(3)),
                              nh_from_adj(a("adj24"), False, 20, swap(3))}
    assert u("2", 1) == {nh_from_adj(a("adj21"), v4, 10)}
    _validate_pop_and_adj(rm, "2", dbs[2])
    assert u("3", 4) == {nh_from_adj(a("adj34"), v4, 10)}
    assert u("3", 2) == {nh_from_adj(a("adj31"), v4, 20), nh_from_adj(a("adj34"), v4, 20)}
    assert rm[("3", "2")] == {nh_from_adj(a("adj31"), False, 20, swap(2)),
                              nh_from_adj(a("adj34"), False, 20, swap(2))}
    assert u("3", 1) == {nh_from_adj(a("adj31"), v4, 10)}
    _validate_pop_and_adj(rm, "3", dbs[3])
    assert u("4", 3) == {nh_from_adj(a("adj43"), v4, 10)}
    assert u("4", 2) == {nh_from_adj(a("adj42"), v4, 10)}
    assert rm[("4", "2")] == {nh_from_adj(a("adj42"), False, 10, PHP)}
    _validate_pop_and_adj(rm, "4", dbs[4])


@pytest.mark.parametrize("v4", [False, True])
def test_ring_overload_link(backend, v4):
    """SimpleRingTopologyFixture.OverloadLinkTest (:3093-3274)."""
    dbs, als, ps, solver = _ring_setup(backend, v4, False, False)
    ls = als[A]
    dbs[3].adjacencies[0].isOverloaded = True  # adj31
    assert ls.update_adjacency_database(dbs[3]).topologyChanged
    rm = route_map(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == 36
    addr = ADDR_V4 if v4 else ADDR
    a = adj
    u = lambda n, d: rm[(n, str(addr[d]))]
    assert u("1", 4) == {nh_from_adj(a("adj12"), v4, 20)}
    assert rm[("1", "4")] == {nh_from_adj(a("adj12"), False, 20, swap(4))}
    assert u("1", 3) == {nh_from_adj(a("adj12"), v4, 30)}
    assert rm[("1", "3")] == {nh_from_adj(a("adj12"), False, 30, swap(3))}
    assert u("1", 2) == {nh_from_adj(a("adj12"), v4, 10)}
    _validate_pop_and_adj(rm, "1", dbs[1])
    assert u("2", 4) == {nh_from_adj(a("adj24"), v4, 10)}
    assert u("2", 3) == {nh_from_adj(a("adj24"), v4, 20)}
    assert rm[("2", "3")] == {nh_from_adj(a("adj24"), False, 20, swap(3))}
    assert u("2", 1) == {nh_from_adj(a("adj21"), v4, 10)}
    assert u("3", 4) == {nh_from_adj(a("adj34"), v4, 10)}
    assert u("3", 2) == {nh_from_adj(a("adj34"), v4, 20)}
    assert rm[("3", "2")] == {nh_from_adj(a("adj34"), False, 20, swap(2))}
    assert u("3", 1) == {nh_from_adj(a("adj34"), v4, 30)}
    assert rm[("3", "1")] == {nh_from_adj(a("adj34"), False, 30, swap(1))}
    _validate_pop_and_adj(rm, "3", dbs[3])
    assert u("4", 3) == {nh_from_adj(a("adj43"), v4, 10)}
    assert u("4", 2) == {nh_from_adj(a("adj42"), v4, 10)}
    assert u("4", 1) == {nh_from_adj(a("adj42"), v4, 20)}
    assert rm[("4", "1")] == {nh_from_adj(a("adj42"), False, 20, swap(1))}
    # adj34 too: node 3 disconnected (:3205-3273)
    dbs[3].adjacencies[1].isOverloaded = True
    assert ls.update_adjacency_database(dbs[3]).topologyChanged
    rm = route_map(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == 24
    assert u("1", 4) == {nh_from_adj(a("adj12"), v4, 20)}
    assert u("1", 2) == {nh_from_adj(a("adj12"), v4, 10)}
    assert u("2", 4) == {nh_from_adj(a("adj24"), v4, 10)}
    assert u("2", 1) == {nh_from_adj(a("adj21"), v4, 10)}
    assert u("4", 2) == {nh_from_adj(a("adj42"), v4, 10)}
    assert u("4", 1) == {nh_from_adj(a("adj42"), v4, 20)}
    assert rm[("4", "1")] == {nh_from_adj(a("adj42"), False, 20, swap(1))}
    _validate_pop_and_adj(rm, "3", dbs[3])


# ---------------------------------------------------------------------------
# BGPRedistribution (:782-1137)
# ---------------------------------------------------------------------------

def _mv(last_metric=4, tie_breaker=False, tie_last=None):
    """MetricVector of 5 WIN_IF_PRESENT entities, type = priority = i,
    metric = {i} (:805-820)."""
    ents = []
    for i in range(5):
        m = last_metric if i == 4 else i
        tb = tie_breaker if i == 4 else False
        ents.append((i, i, 1, tb, (m,)))
    return (0, tuple(ents))


def _bgp_entry(prefix, data, mv):
    return PrefixEntry(prefix, PrefixType.BGP, data, PrefixForwardingType.IP,
                       PrefixForwardingAlgorithm.SP_ECMP, mv)


def test_bgp_redistribution_basic(backend):
    als = backend.area_link_states(A)
    ls = als[A]
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    assert not ls.update_adjacency_database(create_adj_db("1", [adj("adj12"), adj("adj13")], 0)).topologyChanged
    assert ls.update_adjacency_database(create_adj_db("2", [adj("adj21")], 0)).topologyChanged
    assert ls.update_adjacency_database(create_adj_db("3", [adj("adj31")], 0)).topologyChanged
    bgp = ADDR[3]
    ps.update_prefix("1", A, _pfx(ADDR[1]))
    ps.update_prefix("1", A, _bgp_entry(bgp, b"data1", _mv()))
    ps.update_prefix("2", A, _pfx(ADDR[2]))

    def bgp_route(node):
        return solver.build_route_db(node, als, ps).unicastRoutes.get(bgp)

    db = solver.build_route_db("2", als, ps)
    assert len(db.unicastRoutes) == 2
    r = db.unicastRoutes[bgp]  # route1 (:838-845)
    assert r.nexthop_set() == {nh_from_adj(adj("adj21"), False, 10)}
    assert r.bestPrefixEntry.type == PrefixType.BGP and r.bestPrefixEntry.data == b"data1"
    assert not r.doNotInstall
    # same metric vector at node 2: no best path (:847-861)
    ps.update_prefix("2", A, _bgp_entry(bgp, b"data2", _mv()))
    assert len(solver.build_route_db("1", als, ps).unicastRoutes) == 1
    # node 2's last metric decreased: route towards node 1 (:863-877)
    ps.update_prefix("2", A, _bgp_entry(bgp, b"data2", _mv(3)))
    r = bgp_route("2")
    assert r.nexthop_set() == {nh_from_adj(adj("adj21"), False, 10)}
    assert r.bestPrefixEntry.data == b"data1"
    # node 2 better (:879-899)
    ps.update_prefix("2", A, _bgp_entry(bgp, b"data2", _mv(5)))
    db = solver.build_route_db("1", als, ps)
    assert len(db.unicastRoutes) == 2
    r = db.unicastRoutes[bgp]
    assert r.nexthop_set() == {nh_from_adj(adj("adj12"), False, 10)}
    assert r.bestPrefixEntry.data == b"data2"
    # tie breaker on the last metric: multipath at node 3 (:901-939)
    ps.update_prefix("1", A, _bgp_entry(bgp, b"data1", _mv(4, True)))
    ps.update_prefix("2", A, _bgp_entry(bgp, b"data2", _mv(5, True)))
    assert len(solver.build_route_db("1", als, ps).unicastRoutes) == 1
    db = solver.build_route_db("3", als, ps)
    assert len(db.unicastRoutes) == 3
    r = db.unicastRoutes[bgp]
    assert r.bestPrefixEntry.data == b"data2"
    assert r.nexthop_set() == {nh_from_adj(adj("adj31"), False, 10)}
    # disconnect node 1: nodes 1 and 2 program no BGP route (:941-959)
    assert ls.update_adjacency_database(create_adj_db("1", [], 0)).topologyChanged
    assert bgp_route("1") is None
    assert bgp_route("2") is None


def test_bgp_redistribution_igp_metric(backend):
    """BGPRedistribution.IgpMetric (:973-1137)."""
    als = backend.area_link_states(A)
    ls = als[A]
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    mv2 = (0, tuple((i, i, 1, i == 4, (i,)) for i in range(5)))
    mv3 = (0, tuple((i, i, 1, i == 4, (100 if i == 4 else i,)) for i in range(5)))
    db1 = create_adj_db("1", [adj("adj12"), adj("adj13")], 0)
    assert not ls.update_adjacency_database(db1).topologyChanged
    assert ls.update_adjacency_database(create_adj_db("2", [adj("adj21")], 0)).topologyChanged
    assert ls.update_adjacency_database(create_adj_db("3", [adj("adj31")], 0)).topologyChanged
    ps.update_prefix("2", A, _pfx(ADDR[2]))
    ps.update_prefix("2", A, _bgp_entry(ADDR[1], b"data1", mv2))
    ps.update_prefix("3", A, _pfx(ADDR[3]))
    ps.update_prefix("3", A, _bgp_entry(ADDR[1], b"data1", mv3))

    def check(n_routes, hops):
        db = solver.build_route_db("1", als, ps)
        assert len(db.unicastRoutes) == n_routes
        r = db.unicastRoutes[ADDR[1]]
        assert r.bestPrefixEntry.data == b"data1"
        assert r.nexthop_set() == hops

    a12, a13 = adj("adj12"), adj("adj13")
    check(3, {nh_from_adj(a12, False, 10), nh_from_adj(a13, False, 10)})
    db1.adjacencies[1].metric = 20
    assert ls.update_adjacency_database(db1).topologyChanged
    check(3, {nh_from_adj(a12, False, 10)})
    db1.adjacencies[0].isOverloaded = True
    assert ls.update_adjacency_database(db1).topologyChanged
    a13_20 = adj("adj13")
    a13_20.metric = 20
    check(2, {nh_from_adj(a13_20, False, 20)})
    db1.adjacencies[0].metric = 20
    assert ls.update_adjacency_database(db1).topologyChanged
    check(2, {nh_from_adj(a13_20, False, 20)})
    db1.adjacencies[0].isOverloaded = False
    assert ls.update_adjacency_database(db1).topologyChanged
    a12_20 = adj("adj12")
    a12_20.metric = 20
    check(3, {nh_from_adj(a12_20, False, 20), nh_from_adj(a13_20, False, 20)})


# ---------------------------------------------------------------------------
# DecisionTestFixture.MultiAreaBestPathCalculation (:5411-5552), driven
# through LinkState / PrefixState directly (the fixture feeds the same
# adjacency and prefix databases through KvStore publications)
# ---------------------------------------------------------------------------

def test_multi_area_best_path(backend):
    als = backend.area_link_states("A", "B")
    ps = backend.prefix_state()
    a = adj
    for db in (create_adj_db("1", [a("adj12")], 1, False, "A"),
               create_adj_db("2", [a("adj21"), a("adj24")], 2, False, "A"),
               create_adj_db("4", [a("adj42")], 4, False, "A")):
        als["A"].update_adjacency_database(db)
    ps.update_prefix("1", "A", _pfx(ADDR[1]))
    ps.update_prefix("2", "A", _pfx(ADDR[2]))
    for db in (create_adj_db("1", [a("adj13")], 1, False, "B"),
               create_adj_db("3", [a("adj31"), a("adj34")], 3, False, "B"),
               create_adj_db("4", [a("adj43")], 4, False, "B")):
        als["B"].update_adjacency_database(db)
    ps.update_prefix("3", "B", _pfx(ADDR[3]))
    ps.update_prefix("4", "B", _pfx(ADDR[4]))

    def routes(node):
        db = backend.spf_solver(node, False).build_route_db(node, als, ps)
        return {p: r.nexthop_set() for p, r in db.unicastRoutes.items()}

    nh = lambda x, m, area: nh_from_adj(a(x), False, m, None, area)
    assert routes("1") == {ADDR[2]: {nh("adj12", 10, "A")}, ADDR[3]: {nh("adj13", 10, "B")},
                           # addr4 only in B, reached through A as well (area ignored)
                           ADDR[4]: {nh("adj12", 20, "A"), nh("adj13", 20, "B")}}
    assert routes("2") == {ADDR[1]: {nh("adj21", 10, "A")}}
    assert routes("3") == {ADDR[4]: {nh("adj34", 10, "B")}}
    assert routes("4") == {ADDR[2]: {nh("adj42", 10, "A")}, ADDR[3]: {nh("adj43", 10, "B")},
                           ADDR[1]: {nh("adj42", 20, "A"), nh("adj43", 20, "B")}}
    ps.update_prefix("1", "B", _pfx(ADDR[1]))  # (:5521-5551)
    assert routes("3")[ADDR[1]] == {nh("adj31", 10, "B")}
    assert routes("4")[ADDR[1]] == {nh("adj43", 20, "B"), nh("adj42", 20, "A")}
