"""Known-answer tests transcribed from openr/decision/tests/DecisionTest.cpp.

Each runs against the CPU oracle (``-m "not gpu"``) and the HIP product
(``-m gpu``).  Expected values are the reference's own assertions; line
numbers cite them.
"""
import pytest

from helpers import (PHP, adj_label_nexthops, nh_from_adj, pop_route, push,
                     route_map, swap)
from openr_amd.facade import load_topology
from openr_amd.topology import (RING_ADDR_V4, RING_ADDR_V6, adj, ring,
                                unittest_grid, unittest_grid_prefix)
from openr_amd.types import (K_TESTING_AREA, IpPrefix, PrefixForwardingAlgorithm,
                             PrefixForwardingType, PrefixType, create_adj_db,
                             create_adjacency, create_prefix_entry)

A = K_TESTING_AREA
ADDR = {i: IpPrefix.of(f"::ffff:10.{i}.{i}.{i}/128") for i in range(1, 5)}


def _prefix(node: int):
    return create_prefix_entry(ADDR[node])


# ---------------------------------------------------------------------------
# ShortestPathTest.* (DecisionTest.cpp:471-593)
# ---------------------------------------------------------------------------

def test_unreachable_nodes(backend):
    als = backend.area_link_states(A)
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    assert not als[A].update_adjacency_database(create_adj_db("1", [], 0)).topologyChanged
    assert not als[A].update_adjacency_database(create_adj_db("2", [], 0)).topologyChanged
    assert ps.update_prefix("1", A, _prefix(1))
    assert ps.update_prefix("2", A, _prefix(2))
    for node in ("1", "2"):
        db = solver.build_route_db(node, als, ps)
        assert db is not None
        assert len(db.unicastRoutes) == 0 and len(db.mplsRoutes) == 0


def test_missing_neighbor_adjacency_db(backend):
    als = backend.area_link_states(A)
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    assert not als[A].update_adjacency_database(create_adj_db("1", [adj("adj12")], 0)).topologyChanged
    ps.update_prefix("1", A, _prefix(1))
    ps.update_prefix("2", A, _prefix(2))
    db = solver.build_route_db("1", als, ps)
    assert db is not None and len(db.unicastRoutes) == 0 and len(db.mplsRoutes) == 0


def test_empty_neighbor_adjacency_db(backend):
    als = backend.area_link_states(A)
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    assert not als[A].update_adjacency_database(create_adj_db("1", [adj("adj12")], 0)).topologyChanged
    assert not als[A].update_adjacency_database(create_adj_db("2", [], 0)).topologyChanged
    ps.update_prefix("1", A, _prefix(1))
    ps.update_prefix("2", A, _prefix(2))
    assert len(solver.build_route_db("1", als, ps).unicastRoutes) == 0
    assert len(solver.build_route_db("2", als, ps).unicastRoutes) == 0


def test_unknown_node(backend):
    als = backend.area_link_states(A)
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    assert solver.build_route_db("1", als, ps) is None
    assert solver.build_route_db("2", als, ps) is None


# ---------------------------------------------------------------------------
# SpfSolver.AdjacencyUpdate (DecisionTest.cpp:598-731)
# ---------------------------------------------------------------------------

def test_adjacency_update(backend):
    from openr_amd.types import BinaryAddress
    db1 = create_adj_db("1", [adj("adj12")], 1)
    db2 = create_adj_db("2", [adj("adj21")], 2)
    als = backend.area_link_states(A)
    ps = backend.prefix_state()
    solver = backend.spf_solver("1", False)
    ls = als[A]
    r = ls.update_adjacency_database(db1)
    assert not r.topologyChanged and r.nodeLabelChanged
    r = ls.update_adjacency_database(db2)
    assert r.topologyChanged and r.nodeLabelChanged
    ps.update_prefix("1", A, _prefix(1))
    ps.update_prefix("2", A, _prefix(2))

    def check():
        for node in ("1", "2"):
            db = solver.build_route_db(node, als, ps)
            assert len(db.unicastRoutes) == 1
            assert len(db.mplsRoutes) == 3  # two node labels + one adj label

    check()
    db1.adjacencies[0].nextHopV6 = BinaryAddress.of("fe80::1234:b00c")
    r = ls.update_adjacency_database(db1)
    assert not r.topologyChanged and r.linkAttributesChanged
    check()
    db2.adjacencies[0].nextHopV6 = BinaryAddress.of("fe80::5678:b00c")
    r = ls.update_adjacency_database(db2)
    assert not r.topologyChanged and r.linkAttributesChanged
    check()
    db1.adjacencies[0].adjLabel = 111
    r = ls.update_adjacency_database(db1)
    assert not r.topologyChanged and r.linkAttributesChanged
    db2.adjacencies[0].adjLabel = 222
    r = ls.update_adjacency_database(db2)
    assert not r.topologyChanged and r.linkAttributesChanged
    db1.nodeLabel = 11
    r = ls.update_adjacency_database(db1)
    assert (r.topologyChanged, r.linkAttributesChanged, r.nodeLabelChanged) == (False, False, True)
    db2.nodeLabel = 22
    r = ls.update_adjacency_database(db2)
    assert (r.topologyChanged, r.linkAttributesChanged, r.nodeLabelChanged) == (False, False, True)


# ---------------------------------------------------------------------------
# SimpleRingTopologyFixture.ShortestPathTest (DecisionTest.cpp:1897-2028)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("v4", [False, True])
def test_ring_shortest_path(backend, v4):
    adj_dbs, prefixes = ring(v4)
    als = backend.area_link_states(A)
    ls = als[A]
    expect_change = [(False, False, True), (True, False, True), (True, False, True),
                     (True, False, True)]
    for db, exp in zip(adj_dbs, expect_change):
        assert tuple(ls.update_adjacency_database(db)) == exp
    _, ps = load_topology(backend, [], prefixes, als=als)
    solver = backend.spf_solver("1", v4)
    spf_before = ls.spf_runs
    rm = route_map(solver, ["1", "2", "3", "4"], als, ps)
    # unicast 4*3 + node label 4*4 + adj label 4*2
    assert len(rm) == 36
    assert ls.spf_runs - spf_before == 4  # decision.spf_runs.count
    addr = RING_ADDR_V4 if v4 else RING_ADDR_V6

    def u(node, dst):
        return rm[(node, str(addr[dst]))]

    def lbl(node, label):
        return rm[(node, str(label))]

    a = adj
    assert u("1", 4) == {nh_from_adj(a("adj12"), v4, 20), nh_from_adj(a("adj13"), v4, 20)}
    assert lbl("1", 4) == {nh_from_adj(a("adj12"), False, 20, swap(4)),
                           nh_from_adj(a("adj13"), False, 20, swap(4))}
    assert u("1", 3) == {nh_from_adj(a("adj13"), v4, 10)}
    assert lbl("1", 3) == {nh_from_adj(a("adj13"), False, 10, PHP)}
    assert u("1", 2) == {nh_from_adj(a("adj12"), v4, 10)}
    assert lbl("1", 2) == {nh_from_adj(a("adj12"), False, 10, PHP)}
    assert lbl("1", 1) == {pop_route()}

    assert u("2", 4) == {nh_from_adj(a("adj24"), v4, 10)}
    assert lbl("2", 4) == {nh_from_adj(a("adj24"), False, 10, PHP)}
    assert u("2", 3) == {nh_from_adj(a("adj21"), v4, 20), nh_from_adj(a("adj24"), v4, 20)}
    assert lbl("2", 3) == {nh_from_adj(a("adj21"), False, 20, swap(3)),
                           nh_from_adj(a("adj24"), False, 20, swap(3))}
    assert u("2", 1) == {nh_from_adj(a("adj21"), v4, 10)}
    assert lbl("2", 1) == {nh_from_adj(a("adj21"), False, 10, PHP)}

    assert u("3", 4) == {nh_from_adj(a("adj34"), v4, 10)}
    assert u("3", 2) == {nh_from_adj(a("adj31"), v4, 20), nh_from_adj(a("adj34"), v4, 20)}
    assert lbl("3", 2) == {nh_from_adj(a("adj31"), False, 20, swap(2)),
                           nh_from_adj(a("adj34"), False, 20, swap(2))}
    assert u("3", 1) == {nh_from_adj(a("adj31"), v4, 10)}

    assert u("4", 3) == {nh_from_adj(a("adj43"), v4, 10)}
    assert u("4", 2) == {nh_from_adj(a("adj42"), v4, 10)}
    assert u("4", 1) == {nh_from_adj(a("adj42"), v4, 20), nh_from_adj(a("adj43"), v4, 20)}
    assert lbl("4", 1) == {nh_from_adj(a("adj42"), False, 20, swap(1)),
                           nh_from_adj(a("adj43"), False, 20, swap(1))}
    for node, db in zip("1234", adj_dbs):
        assert lbl(node, db.nodeLabel) == {pop_route()}
        for label, nhs in adj_label_nexthops(db.adjacencies).items():
            assert rm[(node, str(label))] == nhs


# ---------------------------------------------------------------------------
# GridTopologyFixture.ShortestPathTest (DecisionTest.cpp:4479-4533)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("n", [2, 4, 6, 8, 10, 12, 14, 16])
def test_grid_all_sources(backend, n):
    adj_dbs, prefixes = unittest_grid(n)
    als, ps = load_topology(backend, adj_dbs, prefixes)
    solver = backend.spf_solver("1", False)
    nodes = [str(i) for i in range(n * n)]
    rm = route_map(solver, nodes, als, ps)
    assert len(rm) == 2 * n ** 4 + 3 * n * n - 4 * n
    # every unicast route's nexthops carry the Manhattan distance
    for src in range(0, n * n, max(1, n * n // 8)):
        for dst in range(n * n):
            if dst == src:
                continue
            hops = rm[(str(src), str(unittest_grid_prefix(dst)))]
            d = abs(src % n - dst % n) + abs(src // n - dst // n)
            assert {h.metric for h in hops} == {d}


# ---------------------------------------------------------------------------
# ParallelAdjRingTopologyFixture (DecisionTest.cpp:3293-3878)
# ---------------------------------------------------------------------------

def _par_adjs():
    c = create_adjacency
    return {
        "adj12_1": c("2", "2/1", "1/1", "fe80::2:1", "192.168.2.1", 11, 201),
        "adj12_2": c("2", "2/2", "1/2", "fe80::2:2", "192.168.2.2", 11, 202),
        "adj12_3": c("2", "2/3", "1/3", "fe80::2:3", "192.168.2.3", 20, 203),
        "adj13_1": c("3", "3/1", "1/1", "fe80::3:1", "192.168.3.1", 11, 301),
        "adj21_1": c("1", "1/1", "2/1", "fe80::1:1", "192.168.1.1", 11, 101),
        "adj21_2": c("1", "1/2", "2/2", "fe80::1:2", "192.168.1.2", 11, 102),
        "adj21_3": c("1", "1/3", "2/3", "fe80::1:3", "192.168.1.3", 20, 103),
        "adj24_1": c("4", "4/1", "2/1", "fe80::4:1", "192.168.4.1", 11, 401),
        "adj31_1": c("1", "1/1", "3/1", "fe80::1:1", "192.168.1.1", 11, 101),
        "adj34_1": c("4", "4/1", "3/1", "fe80::4:1", "192.168.4.1", 11, 401),
        "adj34_2": c("4", "4/2", "3/2", "fe80::4:2", "192.168.4.2", 20, 402),
        "adj34_3": c("4", "4/3", "3/3", "fe80::4:3", "192.168.4.3", 20, 403),
        "adj42_1": c("2", "2/1", "4/1", "fe80::2:1", "192.168.2.1", 11, 201),
        "adj43_1": c("3", "3/1", "4/1", "fe80::3:1", "192.168.3.1", 11, 301),
        "adj43_2": c("3", "3/2", "4/2", "fe80::3:2", "192.168.3.2", 20, 302),
        "adj43_3": c("3", "3/3", "4/3", "fe80::3:3", "192.168.3.3", 20, 303),
    }


def _par_setup(backend, ksp2=False, bgp=False):
    a = _par_adjs()
    dbs = [
        create_adj_db("1", [a["adj12_1"], a["adj12_2"], a["adj12_3"], a["adj13_1"]], 1),
        create_adj_db("2", [a["adj21_1"], a["adj21_2"], a["adj21_3"], a["adj24_1"]], 2),
        create_adj_db("3", [a["adj31_1"], a["adj34_1"], a["adj34_2"], a["adj34_3"]], 3),
        create_adj_db("4", [a["adj42_1"], a["adj43_1"], a["adj43_2"], a["adj43_3"]], 4),
    ]
    als = backend.area_link_states(A)
    ls = als[A]
    assert not ls.update_adjacency_database(dbs[0]).topologyChanged
    for db in dbs[1:]:
        assert ls.update_adjacency_database(db).topologyChanged
    ps = backend.prefix_state()
    entries = {}
    for i in range(1, 5):
        e = _prefix(i)
        node_entries = [e]
        if ksp2:
            # createPrefixDbWithKspfAlgo (DecisionTest.cpp:167-206)
            e.forwardingType = PrefixForwardingType.SR_MPLS
            e.forwardingAlgorithm = PrefixForwardingAlgorithm.KSP2_ED_ECMP
            if bgp:
                e.type = PrefixType.BGP
                e.mv = (0, ())
                node_entries.append(create_prefix_entry(IpPrefix.of(f"fd00::{i}/128")))
        for ne in node_entries:
            ps.update_prefix(str(i), A, ne)
        entries[i] = node_entries
    return a, dbs, als, ps, entries


def test_parallel_adj_ring_shortest_path(backend):
    a, dbs, als, ps, _ = _par_setup(backend)
    solver = backend.spf_solver("1", False)
    rm = route_map(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == 44
    u = lambda n, d: rm[(n, str(ADDR[d]))]
    lbl = lambda n, l: rm[(n, str(l))]
    assert u("1", 4) == {nh_from_adj(a["adj12_2"], False, 22), nh_from_adj(a["adj13_1"], False, 22),
                         nh_from_adj(a["adj12_1"], False, 22)}
    assert lbl("1", 4) == {nh_from_adj(a["adj12_2"], False, 22, swap(4)),
                           nh_from_adj(a["adj13_1"], False, 22, swap(4)),
                           nh_from_adj(a["adj12_1"], False, 22, swap(4))}
    assert u("1", 3) == {nh_from_adj(a["adj13_1"], False, 11)}
    assert u("1", 2) == {nh_from_adj(a["adj12_2"], False, 11), nh_from_adj(a["adj12_1"], False, 11)}
    assert lbl("1", 2) == {nh_from_adj(a["adj12_2"], False, 11, PHP),
                           nh_from_adj(a["adj12_1"], False, 11, PHP)}
    assert u("2", 4) == {nh_from_adj(a["adj24_1"], False, 11)}
    assert u("2", 3) == {nh_from_adj(a["adj21_2"], False, 22), nh_from_adj(a["adj21_1"], False, 22),
                         nh_from_adj(a["adj24_1"], False, 22)}
    assert lbl("2", 3) == {nh_from_adj(a["adj21_2"], False, 22, swap(3)),
                           nh_from_adj(a["adj21_1"], False, 22, swap(3)),
                           nh_from_adj(a["adj24_1"], False, 22, swap(3))}
    assert u("2", 1) == {nh_from_adj(a["adj21_2"], False, 11), nh_from_adj(a["adj21_1"], False, 11)}
    assert u("3", 4) == {nh_from_adj(a["adj34_1"], False, 11)}
    assert u("3", 2) == {nh_from_adj(a["adj31_1"], False, 22), nh_from_adj(a["adj34_1"], False, 22)}
    assert u("3", 1) == {nh_from_adj(a["adj31_1"], False, 11)}
    assert u("4", 3) == {nh_from_adj(a["adj43_1"], False, 11)}
    assert u("4", 2) == {nh_from_adj(a["adj42_1"], False, 11)}
    assert u("4", 1) == {nh_from_adj(a["adj42_1"], False, 22), nh_from_adj(a["adj43_1"], False, 22)}
    assert lbl("4", 1) == {nh_from_adj(a["adj42_1"], False, 22, swap(1)),
                           nh_from_adj(a["adj43_1"], False, 22, swap(1))}
    for node, db in zip("1234", dbs):
        assert lbl(node, db.nodeLabel) == {pop_route()}
        for label, nhs in adj_label_nexthops(db.adjacencies).items():
            assert rm[(node, str(label))] == nhs


@pytest.mark.parametrize("bgp", [False, True])
def test_parallel_adj_ring_ksp2(backend, bgp):
    """Ksp2EdEcmp (DecisionTest.cpp:3694-3878), including the parallel-link
    tie pinned at :3743-3761 (KSP2 picks adj12_2, not adj12_1)."""
    a, dbs, als, ps, entries = _par_setup(backend, ksp2=True, bgp=bgp)
    solver = backend.spf_solver("1", False)
    rm = route_map(solver, ["1"], als, ps)
    assert rm[("1", str(ADDR[2]))] == {nh_from_adj(a["adj12_1"], False, 11),
                                       nh_from_adj(a["adj12_2"], False, 11),
                                       nh_from_adj(a["adj12_3"], False, 20)}

    bgp1 = IpPrefix.of("2401:1::10.1.1.1/32")
    new = create_prefix_entry(bgp1, PrefixType.LOOPBACK, PrefixForwardingType.SR_MPLS,
                              PrefixForwardingAlgorithm.KSP2_ED_ECMP, None, 4)
    ps.update_prefix("4", A, new)
    rm = route_map(solver, ["1"], als, ps)
    assert ("1", str(bgp1)) not in rm  # minNexthop 4 not met

    new.minNexthop = 2
    ps.update_prefix("4", A, new)
    rm = route_map(solver, ["1"], als, ps)
    assert rm[("1", str(bgp1))] == {nh_from_adj(a["adj12_2"], False, 22, push(4)),
                                    nh_from_adj(a["adj13_1"], False, 22, push(4))}

    new3 = create_prefix_entry(bgp1, PrefixType.LOOPBACK, PrefixForwardingType.SR_MPLS,
                               PrefixForwardingAlgorithm.KSP2_ED_ECMP, None, 4)
    ps.update_prefix("3", A, new3)
    rm = route_map(solver, ["1"], als, ps)
    assert ("1", str(bgp1)) not in rm

    ps.delete_prefix("4", A, bgp1)
    ps.delete_prefix("3", A, bgp1)

    ls = als[A]
    dbs[0].adjacencies[1].isOverloaded = True
    dbs[2].adjacencies[2].isOverloaded = True
    assert ls.update_adjacency_database(dbs[0]).topologyChanged
    assert ls.update_adjacency_database(dbs[2]).topologyChanged
    rm = route_map(solver, ["1", "2", "3", "4"], als, ps)
    assert len(rm) == (56 if bgp else 44)
    u = lambda n, d: rm[(n, str(ADDR[d]))]
    assert u("1", 4) == {nh_from_adj(a["adj12_1"], False, 22, push(4)),
                         nh_from_adj(a["adj13_1"], False, 22, push(4))}
    assert u("1", 3) == {nh_from_adj(a["adj13_1"], False, 11),
                         nh_from_adj(a["adj12_1"], False, 33, push(3, 4))}
    assert u("1", 2) == {nh_from_adj(a["adj12_1"], False, 11),
                         nh_from_adj(a["adj12_3"], False, 20)}
    assert u("2", 4) == {nh_from_adj(a["adj24_1"], False, 11),
                         nh_from_adj(a["adj21_1"], False, 33, push(4, 3))}
    assert u("2", 3) == {nh_from_adj(a["adj21_1"], False, 22, push(3)),
                         nh_from_adj(a["adj24_1"], False, 22, push(3))}
    assert u("2", 1) == {nh_from_adj(a["adj21_1"], False, 11),
                         nh_from_adj(a["adj21_3"], False, 20)}
    assert u("3", 4) == {nh_from_adj(a["adj34_1"], False, 11),
                         nh_from_adj(a["adj34_3"], False, 20)}
    assert u("3", 2) == {nh_from_adj(a["adj31_1"], False, 22, push(2)),
                         nh_from_adj(a["adj34_1"], False, 22, push(2))}
    assert u("3", 1) == {nh_from_adj(a["adj31_1"], False, 11),
                         nh_from_adj(a["adj34_1"], False, 33, push(1, 2))}
    assert u("4", 3) == {nh_from_adj(a["adj43_1"], False, 11),
                         nh_from_adj(a["adj43_3"], False, 20)}
    assert u("4", 2) == {nh_from_adj(a["adj42_1"], False, 11),
                         nh_from_adj(a["adj43_1"], False, 33, push(2, 1))}
    assert u("4", 1) == {nh_from_adj(a["adj42_1"], False, 22, push(1)),
                         nh_from_adj(a["adj43_1"], False, 22, push(1))}
