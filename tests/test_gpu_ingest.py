"""KvStore publication ingest against the oracle (``-m gpu``).

Decision::processPublication (Decision.cpp:1682-1824): "adj:" keys carry
Compact-encoded AdjacencyDatabases, "prefix:" keys PrefixDatabases with one
entry, expired keys delete, values without a payload are TTL refreshes. The
product decodes the publication bytes in C++ and applies them to its
LinkState / PrefixState (device mirrors follow at the next build); the
oracle gets the same databases through its direct update calls. Route
databases built afterwards must be equal, and DecisionPendingUpdates must
report what the reference's would (Decision.cpp:40-100).
"""
import random

import pytest

from openr_amd.facade import load_topology
from openr_amd.types import K_TESTING_AREA as A_DEF, IpPrefix, PrefixMetrics, RouteDb, create_prefix_entry

from test_gpu_parity import random_topology

pytestmark = pytest.mark.gpu
AREA = "area0"


def _prefix_key(node, entry):
    import ipaddress
    p = entry.prefix
    addr = ipaddress.ip_address(p.prefixAddress.addr)
    return f"prefix:{node}:{AREA}:[{addr}/{p.prefixLength}]"


def _routes(be, als_impl, ps_impl, me):
    w = be.spf_solver(me, True)._impl.build_route_db(me, als_impl, ps_impl)
    return None if w is None else RouteDb.from_wire(w).canonical()


def test_publication_ingest(hip, oracle):
    mod = hip.module
    dbs = random_topology(6000, n=24, extra=36, max_metric=9)
    for db in dbs:
        db.area = AREA
    rng = random.Random(6)
    pfx = []
    for i in range(40):
        for db in rng.sample(dbs, rng.randint(1, 2)):
            pfx.append((db.thisNodeName, AREA, create_prefix_entry(IpPrefix.of(f"fd00:{i:x}::/64"))))

    def adj_val(db):
        return (1, db.thisNodeName, mod.adj_db_to_compact(db.to_wire()), 3600000, 1)

    def pfx_val(node, e, delete=False):
        return (1, node, mod.prefix_db_to_compact(node, AREA, [e.to_wire()], delete), 3600000, 1)

    als_h = hip.area_link_states()
    ps_h = hip.prefix_state()
    ingest = mod.DecisionIngest(dbs[0].thisNodeName, False)
    # adjacency databases in three publications, prefixes in one
    for chunk in (dbs[:8], dbs[8:16], dbs[16:]):
        pub = mod.publication_to_compact(AREA, {f"adj:{db.thisNodeName}": adj_val(db) for db in chunk}, [])
        ingest.process_publication(pub, als_h._impl, ps_h._impl)
    pend = ingest.pending()
    assert pend["needs_full_rebuild"] and pend["count"] == len(dbs)
    ingest.reset()
    kv = {_prefix_key(n, e): pfx_val(n, e) for n, _, e in pfx}
    kv["fibtime:" + dbs[1].thisNodeName] = (1, "x", b"1234", 1000, 1)
    kv["adj:" + dbs[2].thisNodeName + "-ttl"] = (2, "x", None, 1000, 2)  # TTL refresh: no value
    ingest.process_publication(mod.publication_to_compact(AREA, kv, []), als_h._impl, ps_h._impl)
    pend = ingest.pending()
    assert not pend["needs_full_rebuild"] and len(pend["updated_prefixes"]) == 40
    assert ingest.fib_times() == {dbs[1].thisNodeName: 1234}
    st = ingest.stats()
    assert st["adj_db_update"] == len(dbs) and st["prefix_db_update"] == len(pfx) and st["ttl_refresh"] == 1

    als_o, ps_o = load_topology(oracle, dbs, pfx)
    names = sorted(db.thisNodeName for db in dbs)
    for me in names[:6]:
        assert _routes(hip, als_h._impl, ps_h._impl, me) == _routes(oracle, als_o._impl, ps_o._impl, me), me

    # expiry: two adjacency databases and three prefix keys
    ingest.reset()
    gone_adj = [dbs[3].thisNodeName, dbs[5].thisNodeName]
    gone_pfx = pfx[:3]
    expired = [f"adj:{n}" for n in gone_adj] + [_prefix_key(n, e) for n, _, e in gone_pfx]
    ingest.process_publication(mod.publication_to_compact(AREA, {}, expired), als_h._impl, ps_h._impl)
    for n in gone_adj:
        als_o[AREA].delete_adjacency_database(n)
    for n, _, e in gone_pfx:
        ps_o.delete_prefix(n, AREA, e.prefix)
    pend = ingest.pending()
    assert pend["needs_full_rebuild"]
    assert len(pend["updated_prefixes"]) == len({e.prefix for _, _, e in gone_pfx})
    for me in names[6:12]:
        assert _routes(hip, als_h._impl, ps_h._impl, me) == _routes(oracle, als_o._impl, ps_o._impl, me), me

    # a delete-flagged PrefixDatabase and a malformed value
    ingest.reset()
    n, _, e = pfx[10]
    bad = (1, "x", b"\x19\x05", 1000, 1)
    ingest.process_publication(mod.publication_to_compact(
        AREA, {_prefix_key(n, e): pfx_val(n, e, delete=True), "adj:broken": bad}, []), als_h._impl, ps_h._impl)
    ps_o.delete_prefix(n, AREA, e.prefix)
    assert ingest.stats()["error"] == 1
    assert _routes(hip, als_h._impl, ps_h._impl, names[0]) == _routes(oracle, als_o._impl, ps_o._impl, names[0])


def test_publication_metric_change_is_local_attribute(hip, oracle):
    """A metric change on a remote node is a topology change (full rebuild);
    link attribute changes only count when they are local (Decision.cpp:46-52)."""
    mod = hip.module
    dbs = random_topology(6100, n=12, extra=10, max_metric=5, overload=0.0, link_overload=0.0)
    for db in dbs:
        db.area = AREA
    als_h = hip.area_link_states()
    ps_h = hip.prefix_state()
    me = dbs[0].thisNodeName
    ingest = mod.DecisionIngest(me, False)
    pub = mod.publication_to_compact(
        AREA, {f"adj:{db.thisNodeName}": (1, db.thisNodeName, mod.adj_db_to_compact(db.to_wire()), 1, 1)
               for db in dbs}, [])
    ingest.process_publication(pub, als_h._impl, ps_h._impl)
    als_o, _ = load_topology(oracle, dbs, [])
    ingest.reset()
    other = dbs[4]
    other.adjacencies[0].metric += 7
    change = als_o[AREA].update_adjacency_database(other)
    ingest.process_publication(mod.publication_to_compact(
        AREA, {f"adj:{other.thisNodeName}": (2, other.thisNodeName, mod.adj_db_to_compact(other.to_wire()), 1, 1)},
        []), als_h._impl, ps_h._impl)
    assert ingest.pending()["needs_full_rebuild"] == bool(change.topologyChanged or change.nodeLabelChanged)


def test_multi_area_best_path_via_publications(hip):
    """DecisionTestFixture.MultiAreaBestPathCalculation (DecisionTest.cpp:5411-5552)
    as the reference runs it: KvStore publications per area into Decision,
    then route DBs of every node (expected values: the test's own)."""
    from helpers import nh_from_adj
    from openr_amd.topology import adj
    from openr_amd.types import create_adj_db
    from test_ka_decision_more import ADDR, _pfx
    mod = hip.module
    als = hip.area_link_states()
    ps = hip.prefix_state()

    def adj_kv(db):
        return f"adj:{db.thisNodeName}", (1, db.thisNodeName, mod.adj_db_to_compact(db.to_wire()), 1, 1)

    def pfx_kv(node, addr, area):  # createPrefixKeyValue (DecisionTestUtils)
        e = _pfx(addr)
        return _prefix_key_in(node, e, area), (1, node, mod.prefix_db_to_compact(node, area, [e.to_wire()]), 1, 1)

    a = adj
    pub_a = dict([adj_kv(create_adj_db("1", [a("adj12")], 1, False, "A")),
                  adj_kv(create_adj_db("2", [a("adj21"), a("adj24")], 2, False, "A")),
                  adj_kv(create_adj_db("4", [a("adj42")], 4, False, "A")),
                  pfx_kv("1", ADDR[1], "A"), pfx_kv("2", ADDR[2], "A")])
    pub_b = dict([adj_kv(create_adj_db("1", [a("adj13")], 1, False, "B")),
                  adj_kv(create_adj_db("3", [a("adj31"), a("adj34")], 3, False, "B")),
                  adj_kv(create_adj_db("4", [a("adj43")], 4, False, "B")),
                  pfx_kv("3", ADDR[3], "B"), pfx_kv("4", ADDR[4], "B")])
    g = mod.DecisionIngest("1", False)
    g.process_publication(mod.publication_to_compact("A", pub_a, []), als._impl, ps._impl)
    g.process_publication(mod.publication_to_compact("B", pub_b, []), als._impl, ps._impl)
    assert sorted(als._impl.areas()) == ["A", "B"]

    def routes(node):
        w = hip.spf_solver(node, False)._impl.build_route_db(node, als._impl, ps._impl)
        db = RouteDb.from_wire(w)
        return {p: r.nexthop_set() for p, r in db.unicastRoutes.items()}

    nh = lambda x, m, area: nh_from_adj(a(x), False, m, None, area)
    assert routes("1") == {ADDR[2]: {nh("adj12", 10, "A")}, ADDR[3]: {nh("adj13", 10, "B")},
                           ADDR[4]: {nh("adj12", 20, "A"), nh("adj13", 20, "B")}}   # :5471-5483
    assert routes("2") == {ADDR[1]: {nh("adj21", 10, "A")}}                        # :5486-5489
    assert routes("3") == {ADDR[4]: {nh("adj34", 10, "B")}}                        # :5492-5495
    assert routes("4") == {ADDR[2]: {nh("adj42", 10, "A")}, ADDR[3]: {nh("adj43", 10, "B")},
                           ADDR[1]: {nh("adj42", 20, "A"), nh("adj43", 20, "B")}}   # :5498-5512
    # "1" also originates addr1 into B (:5521-5551)
    g.process_publication(mod.publication_to_compact("B", dict([pfx_kv("1", ADDR[1], "B")]), []),
                          als._impl, ps._impl)
    assert routes("3")[ADDR[1]] == {nh("adj31", 10, "B")}
    assert routes("4")[ADDR[1]] == {nh("adj43", 20, "B"), nh("adj42", 20, "A")}


def _prefix_key_in(node, entry, area):
    import ipaddress
    p = entry.prefix
    return f"prefix:{node}:{area}:[{ipaddress.ip_address(p.prefixAddress.addr)}/{p.prefixLength}]"


def test_ordered_fib_publication_holds(hip, oracle):
    """Ordered FIB (Decision.cpp:1715-1723): each adjacency
    update gets hold TTLs from hop counts (me -> node, max hops from node),
    whose SPFs the product fetches for the whole publication in one batch.
    The oracle applies the same databases one by one with TTLs from its own
    hop queries; holds, their expiry and the route DBs must agree."""
    from openr_amd.topology import bench_grid
    mod = hip.module
    dbs, pfx = bench_grid(6, 1)
    for db in dbs:
        db.area = AREA
    pfx = [(n, AREA, e) for n, _, e in pfx]
    me = "0"
    als_h = hip.area_link_states()
    ps_h = hip.prefix_state()
    als_o = oracle.area_link_states(AREA)
    ps_o = oracle.prefix_state()
    ingest = mod.DecisionIngest(me, True)

    def oracle_update(db):
        ls = als_o[AREA]
        up = down = 0
        hops = ls.get_hops_from_a_to_b(me, db.thisNodeName)
        if hops is not None:
            up = hops
            down = ls.get_max_hops_to_node(db.thisNodeName) - up
        ls.update_adjacency_database(db, up, down)

    def adj_val(db, ver):
        return (ver, db.thisNodeName, mod.adj_db_to_compact(db.to_wire()), 1, 1)

    for db in dbs:  # one publication per database: a defined order
        ingest.process_publication(mod.publication_to_compact(AREA, {f"adj:{db.thisNodeName}": adj_val(db, 1)}, []),
                                   als_h._impl, ps_h._impl)
        oracle_update(db)
    kv = {f"prefix:{n}:{AREA}:[{__import__('ipaddress').ip_address(e.prefix.prefixAddress.addr)}/"
          f"{e.prefix.prefixLength}]": (1, n, mod.prefix_db_to_compact(n, AREA, [e.to_wire()]), 1, 1)
          for n, _, e in pfx}
    ingest.process_publication(mod.publication_to_compact(AREA, kv, []), als_h._impl, ps_h._impl)
    for n, a, e in pfx:
        ps_o.update_prefix(n, a, e)
    # one publication of metric changes on many nodes: hop counts do not depend
    # on metrics, so the per-update TTLs are the same in any order
    changed = [db for db in dbs if int(db.thisNodeName) % 5 == 2]
    for db in changed:
        for adj in db.adjacencies:
            adj.metric += 3
    ingest.process_publication(mod.publication_to_compact(
        AREA, {f"adj:{db.thisNodeName}": adj_val(db, 2) for db in changed}, []), als_h._impl, ps_h._impl)
    for db in changed:
        oracle_update(db)
    ls_h = als_h._impl.area(AREA)
    assert ls_h.has_holds() and als_o[AREA].has_holds()  # the metric increases are held
    for tick in range(12):
        assert _routes(hip, als_h._impl, ps_h._impl, me) == _routes(oracle, als_o._impl, ps_o._impl, me), tick
        ls_h.decrement_holds()
        als_o[AREA].decrement_holds()
        assert ls_h.has_holds() == als_o[AREA].has_holds(), tick


def test_rebuild_routes_incremental(hip, oracle):
    """Decision::rebuildRoutes (Decision.cpp:1865-1930): a full rebuild, then
    prefix-only updates rebuilt incrementally (only the updated prefixes; the
    device-selection batch from 64 prefixes on, the per-prefix host path
    below). After each rebuild the route database equals a full build of the
    same state on the oracle; with a RibPolicy, the incremental result equals
    a full rebuild with that policy."""
    from openr_amd.rib_policy import RibPolicy, RibPolicyStatement, RibRouteActionWeight
    mod = hip.module
    dbs = random_topology(6200, n=24, extra=36, max_metric=9)
    rng = random.Random(62)
    pfx = []
    for i in range(80):
        for db in rng.sample(dbs, rng.randint(1, 3)):
            pfx.append((db.thisNodeName, A_DEF, create_prefix_entry(IpPrefix.of(f"fd00:{i:x}::/64"))))
    als_h, ps_h = load_topology(hip, dbs, pfx)
    als_o, ps_o = load_topology(oracle, dbs, pfx)
    me = sorted(db.thisNodeName for db in dbs)[3]
    solver = hip.spf_solver(me, True)._impl
    rib = mod.DecisionRib()
    rib.rebuild_routes(solver, me, als_h._impl, ps_h._impl, True, [])
    assert RouteDb.from_wire(rib.route_db()).canonical() == _routes(oracle, als_o._impl, ps_o._impl, me)

    def prefix_round(n_changes, policy=None):
        changed = set()
        for _ in range(n_changes):
            r = rng.random()
            if r < 0.4:  # withdraw an advertisement
                node, area, e = pfx[rng.randrange(len(pfx))]
                for be_ps in (ps_h, ps_o):
                    changed |= {(p.prefixAddress.addr, p.prefixLength) for p in be_ps.delete_prefix(node, area, e.prefix)}
            elif r < 0.7:  # a new prefix
                node = rng.choice(dbs).thisNodeName
                e = create_prefix_entry(IpPrefix.of(f"fd01:{rng.randrange(1 << 16):x}::/64"))
                pfx.append((node, A_DEF, e))
                for be_ps in (ps_h, ps_o):
                    changed |= {(p.prefixAddress.addr, p.prefixLength) for p in be_ps.update_prefix(node, A_DEF, e)}
            else:  # re-advertise with other metrics
                node, area, e = pfx[rng.randrange(len(pfx))]
                e2 = create_prefix_entry(e.prefix)
                e2.metrics = PrefixMetrics(1, rng.randint(0, 2), rng.randint(0, 2), rng.randint(0, 2))
                for be_ps in (ps_h, ps_o):
                    changed |= {(p.prefixAddress.addr, p.prefixLength) for p in be_ps.update_prefix(node, area, e2)}
        rib.rebuild_routes(solver, me, als_h._impl, ps_h._impl, False, sorted(changed),
                           policy._impl if policy else None)
        return changed

    for n in (120, 10):  # device-batched, then per-prefix host path
        prefix_round(n)
        assert RouteDb.from_wire(rib.route_db()).canonical() == _routes(oracle, als_o._impl, ps_o._impl, me), n

    policy = RibPolicy([RibPolicyStatement("w", None, ["t"], RibRouteActionWeight(3, {A_DEF: 2}, {}))], 3600)
    # tag every prefix advertisement so the statement matches, then rebuild
    tagged = []
    for node, area, e in pfx:
        e2 = create_prefix_entry(e.prefix)
        e2.tags = ("t",)
        tagged.append((node, area, e2))
        ps_h.update_prefix(node, area, e2)
    rib.rebuild_routes(solver, me, als_h._impl, ps_h._impl, False,
                       sorted({(e.prefix.prefixAddress.addr, e.prefix.prefixLength) for _, _, e in tagged}),
                       policy._impl)
    fresh = mod.DecisionRib()
    fresh.rebuild_routes(solver, me, als_h._impl, ps_h._impl, True, [], policy._impl)
    got = RouteDb.from_wire(rib.route_db())
    assert got.canonical_full() == RouteDb.from_wire(fresh.route_db()).canonical_full()
    assert any(nh.weight == 2 for r in got.unicastRoutes.values() for nh in r.nextHops)


def test_hostile_publication_values_counted_as_errors(hip, oracle):
    """Peer-supplied values the decoders reject (list count beyond the input,
    201 nested structs in an unknown field, a prefix of 129 bits) are counted
    as errors ("Failed to deserialize", Decision.cpp:1785-1788) and change
    nothing; the valid keys of the same publication still apply."""
    mod = hip.module
    dbs = random_topology(6100, n=12, extra=16, max_metric=5)
    for db in dbs:
        db.area = AREA
    als_h = hip.area_link_states()
    ps_h = hip.prefix_state()
    ingest = mod.DecisionIngest(dbs[0].thisNodeName, False)
    kv = {f"adj:{db.thisNodeName}": (1, db.thisNodeName, mod.adj_db_to_compact(db.to_wire()), 3600000, 1)
          for db in dbs}
    huge = b"\xff\xff\xff\xff\x0f"
    good = create_prefix_entry(IpPrefix.of("fd00:1::/64"))
    bad = create_prefix_entry(IpPrefix.of("fd00:2::/64"))
    bad.prefix = IpPrefix(bad.prefix.prefixAddress, 129)
    node = dbs[3].thisNodeName
    adj = mod.adj_db_to_compact(dbs[4].to_wire())
    kv.update({
        _prefix_key(node, good): (1, node, mod.prefix_db_to_compact(node, AREA, [good.to_wire()]), 3600000, 1),
        f"prefix:{node}:{AREA}:[fd00:3::/64]": (1, node, b"\x18\x01a\x29\xfc" + huge, 3600000, 1),
        f"prefix:{node}:{AREA}:[fd00:2::/64]": (1, node, mod.prefix_db_to_compact(node, AREA, [bad.to_wire()]),
                                                3600000, 1),
        "adj:deep": (1, "x", adj[:-1] + b"\xec" + b"\x1c" * 200 + b"\x00" * 202, 3600000, 1),
    })
    ingest.process_publication(mod.publication_to_compact(AREA, kv, []), als_h._impl, ps_h._impl)
    st = ingest.stats()
    assert st["error"] == 3 and st["adj_db_update"] == len(dbs) and st["prefix_db_update"] == 1
    als_o, ps_o = load_topology(oracle, dbs, [(node, AREA, good)])
    for me in sorted(db.thisNodeName for db in dbs)[:4]:
        assert _routes(hip, als_h._impl, ps_h._impl, me) == _routes(oracle, als_o._impl, ps_o._impl, me), me


@pytest.mark.parametrize("with_policy", [False, True])
def test_full_rebuild_delta(hip, oracle, with_policy):
    """Full rebuilds after topology changes (adjacency metric changes, a link
    drained, a node's database deleted and restored) together with prefix
    changes, run as deltas against the DecisionRib's database
    (SpfSolver::buildRouteDelta: device selection compared on the device
    with the previous snapshot, orh_route_diff). After every rebuild the
    database equals a whole build of the same state on the oracle (with the
    policy: a whole rebuild of the product with that policy), and the
    returned update equals calculateUpdate(previous, rebuilt)
    (Decision.cpp:108-143)."""
    from openr_amd.rib_policy import RibPolicy, RibPolicyStatement, RibRouteActionWeight
    from openr_amd.types import RouteDbDelta
    mod = hip.module
    dbs = random_topology(6300, n=30, extra=50, max_metric=7)
    rng = random.Random(63)
    pfx = []
    for i in range(400):
        for db in rng.sample(dbs, rng.randint(1, 3)):
            e = create_prefix_entry(IpPrefix.of(f"fd02:{i:x}::/64"))
            e.tags = ("t",) if i % 3 else ()
            pfx.append((db.thisNodeName, A_DEF, e))
    als_h, ps_h = load_topology(hip, dbs, pfx)
    als_o, ps_o = load_topology(oracle, dbs, pfx)
    me = sorted(db.thisNodeName for db in dbs)[5]
    solver = hip.spf_solver(me, True)._impl
    policy = (RibPolicy([RibPolicyStatement("w", None, ["t"], RibRouteActionWeight(1, {A_DEF: 3}, {}))],
                        3600) if with_policy else None)
    pol = policy._impl if policy else None
    rib = mod.DecisionRib()
    rib.rebuild_routes(solver, me, als_h._impl, ps_h._impl, True, [], pol)
    assert rib.whole_rebuilds == 1
    by_name = {db.thisNodeName: db for db in dbs}
    # topology changes away from me: my nexthop templates (my tight links)
    # stay, so the rebuilds can run as deltas (a template change is a whole
    # rebuild by design)
    near = {me} | {a.otherNodeName for a in by_name[me].adjacencies}
    far = sorted(n for n in by_name if n not in near)
    for rnd in range(6):
        before = rib.route_db()
        changed = set()
        for _ in range(rng.randint(1, 4)):  # topology
            db = by_name[rng.choice(far)]
            r = rng.random()
            if r < 0.6 and db.adjacencies:
                db.adjacencies[rng.randrange(len(db.adjacencies))].metric = rng.randint(1, 7)
                for als in (als_h, als_o):
                    als[A_DEF].update_adjacency_database(db)
            elif r < 0.8 and db.adjacencies:
                a = db.adjacencies[rng.randrange(len(db.adjacencies))]
                a.isOverloaded = not a.isOverloaded
                for als in (als_h, als_o):
                    als[A_DEF].update_adjacency_database(db)
            else:
                for als in (als_h, als_o):
                    als[A_DEF].delete_adjacency_database(db.thisNodeName)
                    als[A_DEF].update_adjacency_database(db)
        for _ in range(rng.randint(0, 20)):  # prefixes
            node, area, e = pfx[rng.randrange(len(pfx))]
            if rng.random() < 0.3:
                for ps in (ps_h, ps_o):
                    changed |= {(p.prefixAddress.addr, p.prefixLength) for p in ps.delete_prefix(node, area, e.prefix)}
            else:
                e2 = create_prefix_entry(e.prefix)
                e2.metrics = PrefixMetrics(1, rng.randint(0, 2), rng.randint(0, 2), rng.randint(0, 2))
                e2.tags = e.tags
                for ps in (ps_h, ps_o):
                    changed |= {(p.prefixAddress.addr, p.prefixLength) for p in ps.update_prefix(node, area, e2)}
        delta, _ = rib.rebuild_routes(solver, me, als_h._impl, ps_h._impl, True, sorted(changed), pol)
        after = rib.route_db()
        if policy is None:
            assert RouteDb.from_wire(after).canonical() == _routes(oracle, als_o._impl, ps_o._impl, me), rnd
        fresh = mod.DecisionRib()
        fresh.rebuild_routes(hip.spf_solver(me, True)._impl, me, als_h._impl, ps_h._impl, True, [], pol)
        assert RouteDb.from_wire(after).canonical_full() == RouteDb.from_wire(fresh.route_db()).canonical_full()
        want = RouteDbDelta.from_wire(mod.calculate_update(before, after)).canonical()
        assert RouteDbDelta.from_wire(delta).canonical() == want, rnd
    assert rib.delta_rebuilds >= 4 and rib.delta_rebuilds + rib.whole_rebuilds == 7
