"""Parity of the HIP product against the CPU oracle (``-m gpu``).

Bit-exact bar: distances, first-hop sets, pathLinks order, KSP2 paths and
whole route databases must equal the oracle's on the same inputs.
"""
import random

import numpy as np
import pytest

from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid, fabric, int_topology, ring, unittest_grid, wan
from openr_amd.types import (K_TESTING_AREA, AdjacencyDatabase, PrefixForwardingAlgorithm,
                             PrefixForwardingType, create_adj_db, create_adjacency,
                             create_prefix_entry, IpPrefix)

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA


def random_topology(seed, n=24, extra=30, max_metric=20, parallel=0.15, overload=0.1,
                    link_overload=0.05, min_metric=1):
    """Seeded graph with parallel links, directional metrics, drained nodes
    and drained adjacencies (both link-down and node-overload semantics)."""
    rng = random.Random(seed)
    links = []
    for i in range(1, n):
        links.append((rng.randrange(i), i))
    for _ in range(extra):
        a, b = rng.randrange(n), rng.randrange(n)
        if a != b:
            links.append((a, b))
    adjs = {i: [] for i in range(n)}
    count = {}
    for a, b in links:
        reps = 2 if rng.random() < parallel else 1
        for _ in range(reps):
            k = count.get((a, b), 0) + count.get((b, a), 0)
            count[(a, b)] = count.get((a, b), 0) + 1
            m_ab, m_ba = rng.randint(min_metric, max_metric), rng.randint(min_metric, max_metric)
            # adjacency labels unique per node (the reference CHECKs duplicates)
            ab = create_adjacency(f"n{b}", f"{a}-{b}-{k}", f"{b}-{a}-{k}", f"fe80::{a}:{b}:{k}",
                                  f"10.{a}.{b}.{k}", m_ab, 10000 + a * 256 + len(adjs[a]))
            ba = create_adjacency(f"n{a}", f"{b}-{a}-{k}", f"{a}-{b}-{k}", f"fe80::{b}:{a}:{k}",
                                  f"10.{b}.{a}.{k}", m_ba, 10000 + b * 256 + len(adjs[b]))
            ab.isOverloaded = rng.random() < link_overload
            adjs[a].append(ab)
            adjs[b].append(ba)
    dbs = [create_adj_db(f"n{i}", adjs[i], 100 + i, rng.random() < overload) for i in range(n)]
    order = list(range(n))
    rng.shuffle(order)
    return [dbs[i] for i in order]


def spf_view(ls, node, use_link_metric=True):
    return {k: (v.metric, v.nextHops, tuple(v.pathLinks))
            for k, v in ls.get_spf_result(node, use_link_metric).items()}


@pytest.mark.parametrize("seed", range(8))
def test_spf_random_graphs(hip, oracle, seed):
    dbs = random_topology(seed)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    for db in dbs:
        for metric in (True, False):
            assert spf_view(als_h[A], db.thisNodeName, metric) == \
                spf_view(als_o[A], db.thisNodeName, metric), (seed, db.thisNodeName, metric)


@pytest.mark.parametrize("seed", range(4))
def test_spf_ignoring_links(hip, oracle, seed):
    dbs = random_topology(100 + seed)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    rng = random.Random(seed)
    for db in dbs[:8]:
        src = db.thisNodeName
        links = als_o[A].links_from_node(src)
        ignore = [tuple(l) for l in rng.sample(links, min(2, len(links)))]
        h = als_h[A]._impl.run_spf_ignoring(src, ignore)
        o = als_o[A]._impl.run_spf_ignoring(src, ignore)
        assert h == o


@pytest.mark.parametrize("seed", range(6))
def test_kth_paths_random(hip, oracle, seed):
    dbs = random_topology(200 + seed, n=16, extra=24, max_metric=3, parallel=0.4, overload=0.0,
                          link_overload=0.0)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    for src in names[:5]:
        for dst in names:
            for k in (1, 2):
                assert als_h[A].get_kth_paths(src, dst, k) == als_o[A].get_kth_paths(src, dst, k), \
                    (seed, src, dst, k)


def _route_dbs_equal(hip, oracle, adj_dbs, prefixes, nodes, **solver_kw):
    als_h, ps_h = load_topology(hip, adj_dbs, prefixes)
    als_o, ps_o = load_topology(oracle, adj_dbs, prefixes)
    for node in nodes:
        sh = hip.spf_solver(node, solver_kw.get("enable_v4", True))
        so = oracle.spf_solver(node, solver_kw.get("enable_v4", True))
        h = sh.build_route_db(node, als_h, ps_h)
        o = so.build_route_db(node, als_o, ps_o)
        assert (h is None) == (o is None)
        if h is not None:
            assert h.canonical() == o.canonical(), node


def test_route_db_bench_grid_10x10(hip, oracle):
    """Config C1: createGrid(10, 1, SP_ECMP), every node as myNode."""
    adj_dbs, prefixes = bench_grid(10)
    _route_dbs_equal(hip, oracle, adj_dbs, prefixes, [str(i) for i in range(100)])


def test_route_db_grid_ksp2(hip, oracle):
    adj_dbs, prefixes = bench_grid(5, 1, PrefixForwardingAlgorithm.KSP2_ED_ECMP)
    _route_dbs_equal(hip, oracle, adj_dbs, prefixes, [str(i) for i in range(0, 25, 3)])


def test_route_db_fabric(hip, oracle):
    adj_dbs, _ = fabric(344, bug_compatible=False)
    prefixes = [(db.thisNodeName, A, create_prefix_entry(IpPrefix.of(f"fd00::{i:x}/128")))
                for i, db in enumerate(adj_dbs) if db.thisNodeName.startswith("3-")]
    _route_dbs_equal(hip, oracle, adj_dbs, prefixes, ["2-0-0", "3-0-1", "1-0-0"])


@pytest.mark.parametrize("seed", range(3))
def test_route_db_random_with_anycast(hip, oracle, seed):
    dbs = random_topology(300 + seed)
    rng = random.Random(seed)
    prefixes = []
    for i in range(30):
        advertisers = rng.sample(dbs, rng.randint(1, 3))
        for db in advertisers:
            e = create_prefix_entry(IpPrefix.of(f"fc00:{seed}::{i:x}/128"))
            if rng.random() < 0.3:
                e.forwardingType = PrefixForwardingType.SR_MPLS
            prefixes.append((db.thisNodeName, A, e))
    _route_dbs_equal(hip, oracle, dbs, prefixes, [db.thisNodeName for db in dbs[:6]])


def test_all_sources_sweep_100x100(hip, oracle):
    """Config C2 at full size: the device sweep over all 10,000 sources.
    Exact comparison with the oracle on sampled sources; size-independent
    properties (Manhattan distances, first-hop masks) on all of them."""
    n = 100
    adj_dbs, _ = bench_grid(n)
    als_h, _ = load_topology(hip, adj_dbs, [])
    ls = als_h[A]
    names = [str(i) for i in range(n * n)]
    sweep = ls._impl.sweep(names, True)
    sweep.run()
    sweep.sync()
    node_ids = {name: i for i, name in enumerate(ls._impl.node_names())}
    ids = np.array([node_ids[str(v)] for v in range(n * n)])  # grid id -> device id
    row_of = np.empty(n * n, dtype=np.int64)
    row_of[ids] = np.arange(n * n)
    rr, cc = np.divmod(np.arange(n * n), n)
    for s in range(0, n * n, 97):
        dist, nh = sweep.fetch(s)
        d = dist[ids]
        manhattan = np.abs(rr - rr[s]) + np.abs(cc - cc[s])
        assert np.array_equal(d, manhattan)
        m = nh[ids]
        assert m[s] == 0 and np.all(m[np.arange(n * n) != s] != 0)
    als_o, _ = load_topology(oracle, adj_dbs, [])
    for s in (0, 1, 4950, 9999):
        dist, nh = sweep.fetch(s)
        ref = als_o[A].get_spf_result(str(s))
        for v in range(n * n):
            assert dist[node_ids[str(v)]] == ref[str(v)].metric
        hres = ls.get_spf_result(str(s))
        assert {k: (v.metric, v.nextHops) for k, v in hres.items()} == \
            {k: (v.metric, v.nextHops) for k, v in ref.items()}


def test_incremental_mirror_updates(hip, oracle):
    """Metric / overload / link add-remove deltas applied to both; SPF and
    route results must track the oracle after every delta."""
    adj_dbs, prefixes = bench_grid(6)
    als_h, ps_h = load_topology(hip, adj_dbs, prefixes)
    als_o, ps_o = load_topology(oracle, adj_dbs, prefixes)
    rng = random.Random(7)
    for step in range(12):
        db = adj_dbs[rng.randrange(len(adj_dbs))]
        kind = step % 4
        if kind == 0 and db.adjacencies:
            db.adjacencies[rng.randrange(len(db.adjacencies))].metric = rng.randint(1, 9)
        elif kind == 1:
            db.isOverloaded = not db.isOverloaded
        elif kind == 2 and db.adjacencies:
            db.adjacencies[rng.randrange(len(db.adjacencies))].isOverloaded ^= True
        elif kind == 3 and len(db.adjacencies) > 1:
            db.adjacencies.pop(rng.randrange(len(db.adjacencies)))
        ch = als_h[A].update_adjacency_database(db)
        co = als_o[A].update_adjacency_database(db)
        assert ch == co, step
        for node in ("0", "1", "35", db.thisNodeName):
            assert spf_view(als_h[A], node) == spf_view(als_o[A], node), (step, node)
        h = hip.spf_solver("1", True).build_route_db("1", als_h, ps_h)
        o = oracle.spf_solver("1", True).build_route_db("1", als_o, ps_o)
        assert h.canonical() == o.canonical(), step


def test_ordered_fib_holds(hip, oracle):
    """Hold TTLs (ordered FIB, LinkState.cpp:500-514) keep the old value in
    the SPF until they expire."""
    adj_dbs, _ = bench_grid(4)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    db = adj_dbs[5]
    db.adjacencies[0].metric = 5
    assert als_h[A].update_adjacency_database(db, 2, 3) == als_o[A].update_adjacency_database(db, 2, 3)
    for _ in range(4):
        assert spf_view(als_h[A], "5") == spf_view(als_o[A], "5")
        assert als_h[A].has_holds() == als_o[A].has_holds()
        assert als_h[A].decrement_holds() == als_o[A].decrement_holds()
    assert spf_view(als_h[A], "5") == spf_view(als_o[A], "5")


def _star_dbs(center_links, extra_ring=True):
    """hub "h" with `leaves` leaves, plus a stub node "s" attached to the hub;
    leaves are chained into a ring so they also have lateral paths."""
    adjs = {}

    def link(a, b, m=1, k=0):
        adjs.setdefault(a, []).append(create_adjacency(b, f"{a}>{b}:{k}", f"{b}>{a}:{k}",
                                                       "fe80::1", "10.0.0.1", m, 0))
        adjs.setdefault(b, []).append(create_adjacency(a, f"{b}>{a}:{k}", f"{a}>{b}:{k}",
                                                       "fe80::2", "10.0.0.2", m, 0))

    link("s", "h", 3)
    for i in range(center_links):
        link("h", f"l{i}", 1 + i % 3)
    if extra_ring:
        for i in range(center_links):
            link(f"l{i}", f"l{(i + 1) % center_links}", 2)
    return [create_adj_db(n, a, 0) for n, a in adjs.items()]


def test_frontier_overflow_path(hip, oracle):
    """1,500 nodes settle in one level from "s": more than the frontier buffer
    holds, exercising the inline-settle path of phase A."""
    dbs = _star_dbs(1500)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    for node in ("s", "l7"):
        assert spf_view(als_h[A], node) == spf_view(als_o[A], node)


def test_wide_mask_variant(hip, oracle):
    """A source with 40 distinct neighbours needs two mask words (Wide)."""
    dbs = _star_dbs(40)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    for node in ("h", "s", "l3"):
        assert spf_view(als_h[A], node) == spf_view(als_o[A], node)


def test_k32_variant_large_metrics(hip, oracle):
    """Path metrics beyond 16 bits select the 64-bit packed state."""
    dbs = random_topology(55, n=40, extra=40, max_metric=60000)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    for db in dbs[:10]:
        assert spf_view(als_h[A], db.thisNodeName) == spf_view(als_o[A], db.thisNodeName)
