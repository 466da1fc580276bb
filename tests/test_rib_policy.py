"""RibPolicy known-answer tests transcribed from
openr/decision/tests/RibPolicyTest.cpp, run against both
the CPU oracle's restatement (oracle/src/oracle_rib_policy.cpp, pinning it to
the reference's assertions) and the product's RibPolicy class (host C++; the
device form of applyPolicy, orh_route_policy, is checked against the oracle
in tests/test_gpu_policy.py)."""
import time

import pytest

from openr_amd.rib_policy import (RibPolicy, RibPolicyStatement, RibPolicyStatementCheck,
                                  RibRouteActionWeight, create_policy_statement, unicast_entry)
from openr_amd.types import BinaryAddress, IpPrefix, create_next_hop
from dataclasses import replace


@pytest.fixture(params=["oracle", "product"])
def pmod(request):
    if request.param == "oracle":
        return request.getfixturevalue("oracle_mod")
    from openr_amd import host_module
    return host_module()


def P(s):
    return IpPrefix.of(s)


def nh(ifname, area=None, nbr=None):
    return create_next_hop(BinaryAddress.of("fe80::1"), ifname, 0, None, area, nbr)


def weighted(n, w):
    return replace(n, weight=w)


def test_statement_errors(pmod):
    # RibPolicyTest.cpp:38-65: no action / no matcher -> OpenrError
    with pytest.raises(ValueError):
        RibPolicyStatementCheck(RibPolicyStatement("s", [P("fc00::/64")], None, None), pmod)
    with pytest.raises(ValueError):
        RibPolicyStatementCheck(RibPolicyStatement("s", None, None, RibRouteActionWeight()), pmod)


def test_policy_error_no_statements(pmod):
    # RibPolicyTest.cpp:67-73
    with pytest.raises(ValueError):
        RibPolicy([], 3, pmod)


def test_statement_apply_action(pmod):
    # RibPolicyTest.cpp:75-117
    st = RibPolicyStatementCheck(create_policy_statement(
        [P("fc00::/64")], None, 1, {"area1": 0, "area2": 2}), pmod)
    nh_default = nh("iface-default")
    nh1 = nh("iface1", "area1")
    nh2 = nh("iface2", "area2")
    entry = unicast_entry("fd00::/64", [nh_default, nh1, nh2])
    changed, out = st.apply_action(entry)
    assert not changed and out == entry
    changed, out = st.apply_action(unicast_entry("fc00::/64", [nh_default, nh1, nh2]))
    assert changed
    assert set(out.nextHops) == {weighted(nh_default, 1), weighted(nh2, 2)}


def test_statement_match(pmod):
    # RibPolicyTest.cpp:119-196
    st = RibPolicyStatementCheck(create_policy_statement([P("10.0.0.0/8")], None, 1, {"test-area": 2}), pmod)
    assert st.match(unicast_entry("10.0.0.0/8", tags=["COMMODITY:EGRESS"]))
    assert not st.match(unicast_entry("11.0.0.0/8", tags=["COMMODITY:EGRESS"]))

    st = RibPolicyStatementCheck(create_policy_statement(None, ["COMMODITY:EGRESS"], 1, {"test-area": 2}), pmod)
    assert st.match(unicast_entry("11.0.0.0/8", tags=["COMMODITY:EGRESS"]))
    assert not st.match(unicast_entry("11.0.0.0/8", tags=["COMMODITY:INGRESS:pod1"]))

    st = RibPolicyStatementCheck(create_policy_statement(
        [P("10.0.0.0/8")], ["COMMODITY:EGRESS"], 1, {"test-area": 2}), pmod)
    assert st.match(unicast_entry("10.0.0.0/8", tags=["COMMODITY:EGRESS"]))
    assert not st.match(unicast_entry("11.0.0.0/8", tags=["COMMODITY:EGRESS"]))
    assert not st.match(unicast_entry("10.0.0.0/8", tags=["COMMODITY:INGRESS:pod1"]))
    assert not st.match(unicast_entry("11.0.0.0/8", tags=["COMMODITY:INGRES:pod1"]))

    st = RibPolicyStatementCheck(create_policy_statement([], [], 1, {"test-area": 2}), pmod)
    assert not st.match(unicast_entry("10.0.0.0/8", tags=["COMMODITY:EGRESS"]))


def test_policy_api(pmod):
    # RibPolicyTest.cpp:198-238 (toThrift round trip is not restated)
    policy = RibPolicy([create_policy_statement([P("10.0.0.0/8")], ["TAG1"], 1, {"test-area": 2})], 3, pmod)
    assert 0 < policy.get_ttl_duration_ms() <= 3000
    assert policy.is_active()
    assert policy.match(unicast_entry("10.0.0.0/8", tags=["TAG1"]))
    assert not policy.match(unicast_entry("99.0.0.0/8", tags=["TAG1"]))


def test_policy_is_active(pmod):
    # RibPolicyTest.cpp:240-255
    policy = RibPolicy([create_policy_statement([P("10.0.0.0/8")], None, 1, {})], 1, pmod)
    assert policy.is_active()
    time.sleep(1.0)
    assert not policy.is_active()


def test_policy_apply_action_first_statement_wins(pmod):
    # RibPolicyTest.cpp:257-320
    s1 = create_policy_statement([P("fc01::/64")], None, 1, {"area1": 99})
    s2 = create_policy_statement([P("fc00::/64"), P("fc02::/64")], None, 1, {"area2": 99})
    policy = RibPolicy([s1, s2], 1, pmod)
    nh1 = nh("iface1", "area1")
    nh2 = nh("iface2", "area2")
    changed, out = policy.apply_action(unicast_entry("fc01::/64", [nh1, nh2]))
    assert changed and set(out.nextHops) == {weighted(nh1, 99), weighted(nh2, 1)}
    changed, out = policy.apply_action(unicast_entry("fc02::/64", [nh1, nh2]))
    assert changed and set(out.nextHops) == {weighted(nh1, 1), weighted(nh2, 99)}
    entry = unicast_entry("fc03::/64", [nh1, nh2])
    changed, out = policy.apply_action(entry)
    assert not changed and out == entry


def test_policy_apply_policy(pmod):
    # RibPolicyTest.cpp:322-396: neighbour weight beats area weight; a route
    # whose nexthops would all be dropped is kept unchanged and counted
    s1 = create_policy_statement([P("fc01::/64")], None, 1, {"area1": 99}, {"nbr3": 98})
    s2 = create_policy_statement([P("fc00::/64"), P("fc02::/64")], None, 1, {"area2": 0})
    policy = RibPolicy([s1, s2], 1, pmod)
    nh1 = nh("iface1", "area1", "nbr1")
    nh2 = nh("iface2", "area2", "nbr2")
    nh3 = nh("iface3", "area1", "nbr3")
    e1 = unicast_entry("fc01::/64", [nh1, nh2, nh3])
    e2 = unicast_entry("fc02::/64", [nh2])
    updated, deleted, routes = policy.apply_policy({e1.dest: e1, e2.dest: e2})
    assert updated == [e1.dest] and deleted == []
    assert policy.invalidated_routes == 1
    assert len(routes) == 2
    assert set(routes[e1.dest].nextHops) == {weighted(nh1, 99), weighted(nh2, 1), weighted(nh3, 98)}
    assert routes[e2.dest].nextHops == e2.nextHops
    time.sleep(1.0)
    assert not policy.is_active()
    updated, deleted, _ = policy.apply_policy({e1.dest: e1, e2.dest: e2})
    assert updated == [] and deleted == []


def test_apply_policy_c5_cross_check(oracle):
    """At scale on CPU: the oracle's restatement and the product's host
    RibPolicy applied to the same oracle-built C5 route DB (3,000 prefixes,
    mixed tag sets, prefix / tag / both matchers, neighbour and zero
    weights) give the same routes, updated lists and invalidated counts."""
    import random
    from openr_amd import host_module
    from openr_amd.facade import load_topology
    from openr_amd.types import PrefixEntry, RouteDb
    from openr_amd.workloads import C5_AREAS, C5_TAG, c5_multi_area
    areas, pfx = c5_multi_area(num_prefixes=3000)
    rng = random.Random(3)
    tagsets = [(), (C5_TAG,), ("T1",), ("T2", "X"), ("X",)]
    pfx = [(n, a, PrefixEntry(e.prefix, e.type, e.data, e.forwardingType, e.forwardingAlgorithm, e.mv,
                              e.minNexthop, e.prependLabel, e.metrics, rng.choice(tagsets)))
           for n, a, e in pfx]
    als, ps = load_topology(oracle, [db for a in C5_AREAS for db in areas[a]], pfx)
    db = oracle.spf_solver("me", True, enable_best_route_selection=True).build_route_db("me", als, ps)
    uniq = sorted(db.unicastRoutes, key=str)
    stmts = [
        RibPolicyStatement("p", rng.sample(uniq, 150), None, RibRouteActionWeight(1, {"A": 0, "C": 5}, {"B0": 0})),
        RibPolicyStatement("t", None, ["T1", "T2"], RibRouteActionWeight(0, {"A": 3, "B": 4}, {})),
        RibPolicyStatement("u", None, [C5_TAG, "X"], RibRouteActionWeight(0, {"A": 1, "B": 2, "C": 3, "D": 4}, {})),
    ]
    routes = {p: r for p, r in db.unicastRoutes.items()}
    outs = []
    for mod in (oracle.module, host_module()):
        pol = RibPolicy(stmts, 3600, mod)
        up, dele, res = pol.apply_policy(routes)
        outs.append((sorted(map(str, up)), dele,
                     RouteDb(res, {}).canonical_full(), pol.invalidated_routes))
    assert outs[0] == outs[1]
    assert outs[0][3] > 0 and len(outs[0][0]) > 1000
