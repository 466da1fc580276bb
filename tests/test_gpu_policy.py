"""RibPolicy decided on the device (orh_route_policy; SURVEY.md §8a a31,
§8f f2) against the oracle's restatement of RibPolicy.cpp:19-247.

The product's buildRouteDbWithPolicy selects routes on the device, decides
per route which statement applies (tag / prefix matchers, keep-if-all-dropped
with the invalidated count) in route_policy_kernel, and sets the statement's
weights while it materialises the routes; host-path routes (SR_MPLS, KSP2,
...) and static routes take RibPolicy::applyAction. The oracle builds the
route DB with its restatement of buildRouteDb and then runs its restatement
of RibPolicy::applyPolicy over it, as Decision::rebuildRoutes does
(Decision.cpp:1888-1900). Whole databases are compared, nexthop weights
included, plus the invalidated-routes counters.

  C5 (4 areas, `me` in all four) at 3,000 prefixes, the BASELINE UCMP
  statement {A:1, B:2, C:3, D:4} on the C5 tag       full canonical DBs
  the same topology with mixed tag sets, prefix matchers, neighbour weights,
  zero weights (dropped nexthops, invalidated routes), an inert statement,
  SR_MPLS prefixes (host path) and a static route    full canonical DBs
  tag sets past the device's ids (ORH_POL_HOST), and 33 statements (host
  applyPolicy)                                       full canonical DBs
  C5 at 1M prefixes with the UCMP statement         whole-DB digests
  DecisionRib full rebuilds (whole and delta) with the policy vs the oracle
"""
import random

import pytest

from openr_amd.facade import load_topology
from openr_amd.rib_policy import RibPolicyStatement, RibRouteActionWeight
from openr_amd.types import BinaryAddress, IpPrefix, NextHopThrift, PrefixEntry, PrefixForwardingType
from openr_amd.workloads import C5_AREAS, C5_TAG, c5_multi_area

pytestmark = pytest.mark.gpu


def _c5(n, retag=None):
    areas, prefixes = c5_multi_area(num_prefixes=n)
    adj = [db for a in C5_AREAS for db in areas[a]]
    if retag is not None:
        prefixes = [retag(i, node, area, e) for i, (node, area, e) in enumerate(prefixes)]
    return adj, prefixes


def _ucmp():
    """BASELINE.json C5: set_weight{area_to_weight: {A:1, B:2, C:3, D:4}}."""
    return [RibPolicyStatement("ucmp", None, [C5_TAG],
                               RibRouteActionWeight(0, {"A": 1, "B": 2, "C": 3, "D": 4}, {}))]


def _build_both(hip, oracle, adj, pfx, stmts, me="me", best_route=True, static=None, tag_id_limit=None):
    ps_h = hip.prefix_state()
    if tag_id_limit is not None:
        ps_h._impl.set_tag_set_id_limit(tag_id_limit)
    als_h, ps_h = load_topology(hip, adj, pfx, ps=ps_h)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    sh = hip.spf_solver(me, True, enable_best_route_selection=best_route)
    so = oracle.spf_solver(me, True, enable_best_route_selection=best_route)
    if static:
        sh.update_static_unicast_routes(static)
        so.update_static_unicast_routes(static)
    ph = hip.rib_policy(stmts, 3600)
    po = oracle.rib_policy(stmts, 3600)
    h = sh.build_route_db_with_policy(me, als_h, ps_h, ph)
    o = so.build_route_db_with_policy(me, als_o, ps_o, po)
    # the same build once more, for the policy statistics (routes decided on
    # the device; the counters of a separate policy object)
    stats = sh._impl.time_build_route_db_with_policy(me, als_h._impl, ps_h._impl,
                                                     hip.rib_policy(stmts, 3600)._impl)
    return h, o, ph, po, stats


@pytest.mark.parametrize("best_route", [False, True])
def test_c5_ucmp_policy_small(hip, oracle, best_route):
    h, o, ph, po, _ = _build_both(hip, oracle, *_c5(3000), _ucmp(), best_route=best_route)
    assert h is not None and o is not None
    assert h.canonical_full() == o.canonical_full()
    assert ph.invalidated_routes == po.invalidated_routes
    weights = {nh.weight for r in h.unicastRoutes.values() for nh in r.nextHops}
    assert weights == {1, 2, 3, 4}  # every route's nexthops took their area's weight


def _mixed_retag(seed):
    rng = random.Random(seed)
    tagsets = [(), (C5_TAG,), ("T1",), ("T2", "X"), ("X",), (C5_TAG, "T1")]

    def retag(i, node, area, e):
        tags = rng.choice(tagsets)
        fwd = PrefixForwardingType.SR_MPLS if rng.random() < 0.03 else e.forwardingType
        return node, area, PrefixEntry(e.prefix, e.type, e.data, fwd, e.forwardingAlgorithm, e.mv,
                                       e.minNexthop, e.prependLabel, e.metrics, tags)
    return retag


def _mixed_statements(prefixes, seed):
    rng = random.Random(seed)
    uniq = sorted({e.prefix for _, _, e in prefixes}, key=str)
    some = rng.sample(uniq, len(uniq) // 20)
    more = rng.sample(uniq, len(uniq) // 10)
    return [
        # prefix matcher; area B dropped by its neighbour weight, A by area weight
        RibPolicyStatement("p", some, None, RibRouteActionWeight(1, {"A": 0, "C": 5}, {"B0": 0})),
        # tag matcher whose weights drop every nexthop of C / D routes
        # (invalidated; the next statement is tried)
        RibPolicyStatement("t12", None, ["T1", "T2"], RibRouteActionWeight(0, {"A": 3, "B": 4}, {})),
        # both matchers
        RibPolicyStatement("pt", more, [C5_TAG, "X"], RibRouteActionWeight(2, {}, {"D0": 9})),
        # present but empty matchers: never matches (RibPolicy.cpp:74-76)
        RibPolicyStatement("inert", [], [], RibRouteActionWeight(7, {}, {})),
        # catch-all on the C5 tag
        RibPolicyStatement("ucmp", None, [C5_TAG], RibRouteActionWeight(0, {"A": 1, "B": 2, "C": 3, "D": 4}, {})),
    ]


@pytest.mark.parametrize("seed", [1, 2])
def _static(i):
    """A static route for a prefix no node advertises, via B0."""
    sp = IpPrefix(BinaryAddress(bytes([0xfc, 0x99, 0, i] + [0] * 12)), 64)
    snh = NextHopThrift(BinaryAddress(bytes([0xfe, 0x80] + [0] * 13 + [7]), "static0"), 0, None, 0, "B",
                        "B0")
    return sp, snh


def _fillers(k):
    """k statements whose prefix matchers name prefixes nobody advertises."""
    return [RibPolicyStatement(f"f{i}", [IpPrefix(BinaryAddress(bytes([0xfd, 0x77, i] + [0] * 13)), 48)],
                               None, RibRouteActionWeight(1, {}, {})) for i in range(k)]


@pytest.mark.parametrize("seed", [1, 2])
def test_c5_mixed_policy_small(hip, oracle, seed):
    adj, pfx = _c5(3000, _mixed_retag(seed))
    stmts = _mixed_statements(pfx, seed)
    # a static route (host policy path)
    sp, snh = _static(0)
    h, o, ph, po, stats = _build_both(hip, oracle, adj, pfx, stmts + [RibPolicyStatement(
        "static", [sp], None, RibRouteActionWeight(6, {}, {}))], static=[(sp, [snh])])
    assert h.canonical_full() == o.canonical_full()
    assert ph.invalidated_routes == po.invalidated_routes > 0
    assert h.unicastRoutes[sp].nextHops[0].weight == 6
    weights = {nh.weight for r in h.unicastRoutes.values() for nh in r.nextHops}
    assert {0, 1, 2, 3, 4, 5, 9}.issubset(weights)
    assert stats[4] > 0.8 * stats[1]  # most routes decided on the device


def test_c5_policy_tag_ids_saturated(hip, oracle):
    """Tag sets beyond the device's id space (ORH_ADV_TAGSET_OVF; the limit is
    lowered so 2 of the 5 sets get ids): their routes come back ORH_POL_HOST
    from route_policy_kernel and take RibPolicy::applyAction on the host as
    they materialise - the result and the counters are the reference's."""
    adj, pfx = _c5(3000, _mixed_retag(3))
    stmts = _mixed_statements(pfx, 3)
    h, o, ph, po, stats = _build_both(hip, oracle, adj, pfx, stmts, tag_id_limit=3)
    assert h.canonical_full() == o.canonical_full()
    assert ph.invalidated_routes == po.invalidated_routes > 0
    _, routes, updated, invalidated, on_device, _ = stats
    assert invalidated == po.invalidated_routes
    assert 0 < on_device < 0.7 * routes  # tagged routes of 3 sets went to the host


def test_c5_policy_33_statements(hip, oracle):
    """More statements than the device's masks hold (ORH_POL_MAX_STMTS = 32):
    RibPolicy::applyPolicy over the built database on the host."""
    adj, pfx = _c5(3000, _mixed_retag(4))
    stmts = _fillers(28) + _mixed_statements(pfx, 4)
    assert len(stmts) == 33
    h, o, ph, po, stats = _build_both(hip, oracle, adj, pfx, stmts)
    assert h.canonical_full() == o.canonical_full()
    assert ph.invalidated_routes == po.invalidated_routes > 0
    assert stats[4] == 0 and stats[3] == po.invalidated_routes


def test_c5_ucmp_policy_1m_digest(hip, oracle):
    """C5 at BASELINE size: 1M prefixes, best-route selection, the UCMP
    statement; whole-DB digests (nexthop weights included)."""
    adj, pfx = _c5(1_000_000)
    als_h, ps_h = load_topology(hip, adj, pfx)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    sh = hip.spf_solver("me", True, enable_best_route_selection=True)
    so = oracle.spf_solver("me", True, enable_best_route_selection=True)
    ph = hip.rib_policy(_ucmp(), 3600)
    po = oracle.rib_policy(_ucmp(), 3600)
    dh = sh._impl.build_route_db_with_policy_digest("me", als_h._impl, ps_h._impl, ph._impl)
    do = so._impl.build_route_db_with_policy_digest("me", als_o._impl, ps_o._impl, po._impl)
    assert dh[:2] == do[:2] and dh[0] > 900_000
    if dh[2] != do[2]:
        import numpy as np
        bad = np.nonzero(np.frombuffer(dh[2], np.uint64) != np.frombuffer(do[2], np.uint64))[0]
        raise AssertionError(f"{len(bad)} routes differ, first at canonical index {bad[0]}")
    # the same policy applied by the host pass over buildRouteDb's map (A/B)
    secs, updated = sh._impl.time_host_apply_policy("me", als_h._impl, ps_h._impl,
                                                     hip.rib_policy(_ucmp(), 3600)._impl)
    assert updated == dh[0]


@pytest.mark.parametrize("variant", ["device", "tag_ids_saturated", "33_statements"])
def test_decision_rib_rebuild_with_policy(hip, oracle, variant):
    """DecisionRib full rebuilds with the policy (the first whole, the later
    ones as deltas against routeDb_) equal the oracle's buildRouteDb +
    applyPolicy after the same prefix and metric changes, and the policy's
    invalidated-routes counter accumulates what the reference's full rebuilds
    count (RibPolicy.cpp:149-150): the device's count of the selected routes,
    host-path routes, and static routes the delta did not rebuild - one
    invalidated (every nexthop weighted 0), one shadowed by an advertisement.
    With tag sets past the device's ids (ORH_POL_HOST) the delta materialises
    those routes to count them; with 33 statements every rebuild is whole."""
    from openr_amd.types import RouteDb
    adj, pfx = _c5(3000, _mixed_retag(5))
    sp, snh = _static(1)
    shadow = pfx[7][2].prefix
    stmts = [RibPolicyStatement("static0", [sp, shadow], None, RibRouteActionWeight(0, {}, {}))]
    stmts += _mixed_statements(pfx, 5) + (_fillers(27) if variant == "33_statements" else [])
    ps_h = hip.prefix_state()
    if variant == "tag_ids_saturated":
        ps_h._impl.set_tag_set_id_limit(3)
    als_h, ps_h = load_topology(hip, adj, pfx, ps=ps_h)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    sh = hip.spf_solver("me", True, enable_best_route_selection=True)
    so = oracle.spf_solver("me", True, enable_best_route_selection=True)
    statics = [(sp, [snh]), (shadow, [snh])]
    sh.update_static_unicast_routes(statics)
    so.update_static_unicast_routes(statics)
    ph = hip.rib_policy(stmts, 3600)
    rib = hip.module.DecisionRib()
    rng = random.Random(9)
    want_inv = 0
    for rnd in range(3):
        rib.rebuild_routes(sh._impl, "me", als_h._impl, ps_h._impl, True, [], ph._impl, wire=False)
        po = oracle.rib_policy(stmts, 3600)
        want = so.build_route_db_with_policy("me", als_o, ps_o, po)
        want_inv += po.invalidated_routes
        got = RouteDb.from_wire(rib.route_db())
        assert got.canonical_full() == want.canonical_full(), rnd
        assert sp in got.unicastRoutes
        assert ph.invalidated_routes == want_inv, rnd
        # prefix re-advertisements with new metrics and one adjacency metric change
        for _ in range(200):
            node, area, e = pfx[rng.randrange(len(pfx))]
            e2 = PrefixEntry(e.prefix, e.type, e.data, e.forwardingType, e.forwardingAlgorithm, e.mv,
                             e.minNexthop, e.prependLabel,
                             type(e.metrics)(1, rng.randint(0, 3), rng.randint(0, 3), rng.randint(0, 3)),
                             e.tags)
            ps_h.update_prefix(node, area, e2)
            ps_o.update_prefix(node, area, e2)
        db = adj[rng.randrange(len(adj))]
        if db.adjacencies:
            db.adjacencies[0].metric = rng.randint(1, 3)
            als_h[db.area].update_adjacency_database(db)
            als_o[db.area].update_adjacency_database(db)
    assert want_inv >= 3
    if variant == "33_statements":
        assert rib.delta_rebuilds == 0
    else:
        assert rib.delta_rebuilds >= 1
