"""Test helpers restating the reference test utilities.

  route_map              getRouteMap + fillRouteMap (DecisionTest.cpp:256-320)
  nh_from_adj            createNextHopFromAdj (DecisionTest.cpp:208-222)
  update_prefix_database updatePrefixDatabase (DecisionTest.cpp:436-463)
"""
from openr_amd.types import (K_TESTING_AREA, MplsActionCode, NextHopThrift,
                             create_mpls_action, create_next_hop)


def route_map(solver, nodes, als, ps):
    """(node, prefix-string | label-string) -> frozenset(nexthops); a route
    with no nexthops adds no key, exactly as fillRouteMap's per-nexthop
    emplace does."""
    out = {}
    for node in nodes:
        db = solver.build_route_db(node, als, ps)
        if db is None:
            continue
        for pfx, r in db.unicastRoutes.items():
            for nh in r.nextHops:
                out.setdefault((node, str(pfx)), set()).add(nh)
        for label, r in db.mplsRoutes.items():
            for nh in r.nextHops:
                out.setdefault((node, str(label)), set()).add(nh)
    return {k: frozenset(v) for k, v in out.items()}


def nh_from_adj(adj, v4, metric, action=None, area=K_TESTING_AREA) -> NextHopThrift:
    return create_next_hop(adj.nextHopV4 if v4 else adj.nextHopV6, adj.ifName, metric,
                           action, area, adj.otherNodeName)


PHP = create_mpls_action(MplsActionCode.PHP)
POP = create_mpls_action(MplsActionCode.POP_AND_LOOKUP)


def swap(label):
    return create_mpls_action(MplsActionCode.SWAP, label)


def push(*labels):
    return create_mpls_action(MplsActionCode.PUSH, None, list(labels))


def update_prefix_database(ps, node, entries, area=K_TESTING_AREA, old=()):
    """Replace node's advertisements: update every entry, delete keys that
    were in ``old`` but not in ``entries``."""
    changed = set()
    new_keys = set()
    for e in entries:
        changed |= ps.update_prefix(node, area, e)
        new_keys.add(e.prefix)
    for e in old:
        if e.prefix not in new_keys:
            changed |= ps.delete_prefix(node, area, e.prefix)
    return changed


def pop_route(area=K_TESTING_AREA):
    from openr_amd.types import BinaryAddress
    return NextHopThrift(BinaryAddress(bytes(16)), 0, POP, 0, area, None)


def adj_label_nexthops(adjs, area=K_TESTING_AREA):
    """validateAdjLabelRoutes (DecisionTest.cpp:354-368)."""
    return {a.adjLabel: frozenset({nh_from_adj(a, False, a.metric, PHP, area)}) for a in adjs}


def assert_digests_equal(solver_h, solver_o, me, als_h, ps_h, als_o, ps_o):
    """Whole-route-DB parity at full size through the per-route canonical
    digests both backends compute natively (build_route_db_digest); on a
    mismatch, report the first differing route index."""
    h = solver_h._impl.build_route_db_digest(me, als_h._impl, ps_h._impl)
    o = solver_o._impl.build_route_db_digest(me, als_o._impl, ps_o._impl)
    assert (h is None) == (o is None), me
    if h is None:
        return 0
    assert h[:2] == o[:2], f"route counts differ: hip {h[:2]} oracle {o[:2]}"
    if h[2] != o[2]:
        import numpy as np
        a = np.frombuffer(h[2], dtype=np.uint64)
        b = np.frombuffer(o[2], dtype=np.uint64)
        bad = np.nonzero(a != b)[0]
        raise AssertionError(f"{len(bad)} routes differ (first canonical index {bad[0]} "
                             f"of {h[0]} unicast + {h[1]} mpls)")
    return h[0] + h[1]


_M1, _M2 = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB
_G, _K = 0x9E3779B97F4A7C15, 0xC2B2AE3D27D4EB4F


def _fmix64(z):
    import numpy as np
    z = z ^ (z >> np.uint64(30))
    z = z * np.uint64(_M1)
    z = z ^ (z >> np.uint64(27))
    z = z * np.uint64(_M2)
    return z ^ (z >> np.uint64(31))


def row_digest(dist, nh):
    """orh_row_digest (include/openr_hip.h) of one row, restated in numpy:
    sum over v of mix(v, dist[v], nh[v][0..words)) mod 2^64. dist: [N] u32,
    nh: [N] or [N, words] u32."""
    import numpy as np
    dist = np.asarray(dist, dtype=np.uint64)
    nh = np.asarray(nh, dtype=np.uint64).reshape(len(dist), -1)
    v = np.arange(len(dist), dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _fmix64(v * np.uint64(_G) + dist)
        for k in range(nh.shape[1]):
            h = _fmix64(h ^ (nh[:, k] + np.uint64(k) * np.uint64(_K)))
        return int(np.sum(h, dtype=np.uint64))


def assert_tiers_match(info, info1, search_large):
    """Per-request what-if info (ORH_WHATIF_TIER | affected << 3) of a split
    job against the single job's: equal, except that with
    ORH_WHATIF_SEARCH_LARGE (a 4-way or wider split) some tier 2 / 3
    requests are searched in full (tier 4, no affected count). The rows
    themselves are compared by digest by the caller."""
    import numpy as np
    info = np.asarray(info, dtype=np.uint64)
    info1 = np.asarray(info1, dtype=np.uint64)
    full = (info & 7) == 4
    if not search_large:
        assert np.array_equal(info, info1)
        return
    # the searches take tier 1's overflow (no tier 2 in such a job): what the
    # single job repaired in tier 2 or 3 is searched, or repaired in a slot
    # (tier 3) once the searches' cap is reached, with the same affected count
    assert np.all(np.isin(info1[full] & 7, [2, 3])), "a request searched in full was not a tier 2 / 3 repair"
    slot = ((info & 7) == 3) & ((info1 & 7) == 2)
    assert np.array_equal(info[slot] >> 3, info1[slot] >> 3)
    rest = ~full & ~slot
    assert np.array_equal(info[rest], info1[rest])
