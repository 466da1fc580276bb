"""Structural mirror deltas (orh_graph_apply_delta) against the oracle
(``-m gpu``).

Adjacency databases lose and regain adjacencies (links removed and added,
LinkState.cpp:564-719) and nodes lose their databases (:721-738). The
product rewrites only the changed CSR rows on the device; after every step
its SPF results (metric, nexthops, ordered pathLinks), KSP2 paths and
route database equal the oracle's, and the mirror stats show row deltas, not
full reloads.
"""
import copy
import random

import pytest

from helpers import assert_digests_equal
from openr_amd.facade import load_topology
from openr_amd.types import K_TESTING_AREA, IpPrefix, create_prefix_entry

from test_gpu_parity import random_topology, spf_view

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA


def _views_equal(als_h, als_o, names, tag):
    for nm in names:
        for metric in (True, False):
            assert spf_view(als_h[A], nm, metric) == spf_view(als_o[A], nm, metric), (tag, nm, metric)


@pytest.mark.parametrize("seed", range(3))
def test_link_remove_add_sequence(hip, oracle, seed):
    rng = random.Random(seed)
    dbs = random_topology(2000 + seed, n=30, extra=50, max_metric=6, parallel=0.2)
    prefixes = [(db.thisNodeName, A, create_prefix_entry(IpPrefix.of(f"fd00:{i:x}::/64")))
                for i, db in enumerate(dbs)]
    als_h, ps_h = load_topology(hip, dbs, prefixes)
    als_o, ps_o = load_topology(oracle, dbs, prefixes)
    names = sorted(db.thisNodeName for db in dbs)
    _views_equal(als_h, als_o, names, "initial")
    loads0, _ = als_h[A]._impl.mirror_stats()
    current = {db.thisNodeName: copy.deepcopy(db) for db in dbs}
    removed = {}
    for step in range(12):
        node = rng.choice(names)
        db = current[node]
        if removed.get(node) and rng.random() < 0.5:  # restore an adjacency
            db.adjacencies.append(removed[node].pop())
        elif db.adjacencies:  # drop one
            removed.setdefault(node, []).append(db.adjacencies.pop(rng.randrange(len(db.adjacencies))))
        for ls in (als_h[A], als_o[A]):
            ls.update_adjacency_database(copy.deepcopy(db))
        _views_equal(als_h, als_o, names, step)
        src = rng.choice(names)
        for dst in names[:8]:
            for k in (1, 2):
                assert als_h[A].get_kth_paths(src, dst, k) == als_o[A].get_kth_paths(src, dst, k)
        me = rng.choice(names)
        assert_digests_equal(hip.spf_solver(me, True), oracle.spf_solver(me, True), me,
                             als_h, ps_h, als_o, ps_o)
    loads, deltas = als_h[A]._impl.mirror_stats()
    assert deltas >= 6 and loads == loads0, (loads0, loads, deltas)


def test_delete_adjacency_database(hip, oracle):
    dbs = random_topology(2100, n=24, extra=30, max_metric=4)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    for victim in names[:3]:
        for ls in (als_h[A], als_o[A]):
            ls.delete_adjacency_database(victim)
        _views_equal(als_h, als_o, names, victim)
    loads, deltas = als_h[A]._impl.mirror_stats()
    # one row delta per deletion that still removed links (a victim whose
    # links all went with earlier victims changes no row), never a reload
    assert 1 <= deltas <= 3 and loads == 1, (loads, deltas)
