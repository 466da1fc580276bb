"""The independent fast checker (oracle/src/oracle_fast.h; test
infrastructure) against the faithful oracle (-m "not gpu").

FastChecker restates runSpf (LinkState.cpp:808-882) in the closed form of
SURVEY.md Appendix A.1 with flat arrays and a binary heap, pathLinks in
(distance, name) then LinkSet order (A.2) and getKthPaths / traceOnePath
(:762-791, :398-419). It is what pins the product at the configs' full sizes
(tests/test_gpu_at_scale.py), so here it must agree with the faithful oracle -
itself pinned by the transcribed reference known answers - on every row and
path of random graphs with parallel links, drained nodes and drained
adjacencies, on ignore sets, and on a 3,000-node slice of the C4 WAN generator.
"""
import random

import numpy as np
import pytest

from helpers import row_digest
from openr_amd.facade import LinkDesc, load_topology
from openr_amd.topology import wan
from openr_amd.types import K_TESTING_AREA
from test_gpu_parity import random_topology

A = K_TESTING_AREA


def _checker(oracle, dbs):
    als, _ = load_topology(oracle, dbs, [])
    ls = als[A]._impl
    order = sorted(db.thisNodeName for db in dbs)
    return ls, order, oracle.module.FastChecker(ls, order)


def _oracle_rows(ls, fc, order, srcs, ignores=None):
    nbrs = [[order[v] for v in fc.neighbours(s)] for s in srcs]
    descs = []
    if ignores is not None:
        for ign in ignores:
            descs.append([fc.link_desc(l)[:3] for l in ign])
    return ls.spf_tables([order[s] for s in srcs], order, nbrs, 4, descs)


@pytest.mark.parametrize("seed", range(6))
def test_fast_rows_match_oracle_random(oracle, seed):
    dbs = random_topology(2100 + seed, n=40, extra=60, max_metric=6, parallel=0.3, overload=0.15,
                          link_overload=0.08)
    ls, order, fc = _checker(oracle, dbs)
    srcs = list(range(len(order)))
    dist, nh = fc.spf_rows(srcs, [], 4)
    od, on = _oracle_rows(ls, fc, order, srcs)
    assert np.array_equal(dist, od)
    assert np.array_equal(nh[:, :, :1], on[:, :, :1])
    # one digest per row, as orh_row_digest computes it on the device
    dig = fc.row_digests(srcs, [], 4)
    for i in range(0, len(srcs), 7):
        assert int(dig[i]) == row_digest(dist[i], nh[i][:, 0])


@pytest.mark.parametrize("seed", range(4))
def test_fast_rows_with_ignore_sets(oracle, seed):
    dbs = random_topology(2200 + seed, n=36, extra=50, max_metric=5, parallel=0.3, overload=0.1,
                          link_overload=0.05)
    ls, order, fc = _checker(oracle, dbs)
    rng = random.Random(seed)
    srcs = [rng.randrange(len(order)) for _ in range(40)]
    ignores = [rng.sample(range(fc.links), rng.randint(1, 4)) for _ in srcs]
    dist, nh = fc.spf_rows(srcs, ignores, 4)
    od, on = _oracle_rows(ls, fc, order, srcs, ignores)
    assert np.array_equal(dist, od)
    assert np.array_equal(nh[:, :, :1], on[:, :, :1])


@pytest.mark.parametrize("seed", range(6))
def test_fast_kth_paths_match_oracle_random(oracle, seed):
    """getKthPaths k = 1, 2 for every (src, dst) pair: link by link, in order
    (parallel-link ties follow LinkSet order)."""
    dbs = random_topology(2300 + seed, n=18, extra=30, max_metric=3, parallel=0.4, overload=0.1,
                          link_overload=0.05)
    ls, order, fc = _checker(oracle, dbs)
    pairs = [(s, d) for s in range(len(order)) for d in range(len(order))]
    got = fc.kth_paths(pairs, 4)
    for (s, d), (k1, k2) in zip(pairs, got):
        for k, paths in ((1, k1), (2, k2)):
            want = [[LinkDesc(*l) for l in p] for p in ls.get_kth_paths(order[s], order[d], k)]
            assert [[LinkDesc(*l) for l in p] for p in paths] == want, (order[s], order[d], k)


def test_fast_checker_wan_slice(oracle):
    """The C4 WAN generator (log-normal metrics) at 3,000 nodes: rows of 12
    sources with and without a single ignored link, and KSP2 paths of 12
    pairs, against the faithful oracle."""
    dbs, _ = wan(3000, seed=4)
    ls, order, fc = _checker(oracle, dbs)
    rng = random.Random(9)
    srcs = [rng.randrange(len(order)) for _ in range(12)]
    ign = [[rng.randrange(fc.links)] for _ in srcs]
    for ignores in (None, ign):
        dist, nh = fc.spf_rows(srcs, ignores or [], 8)
        od, on = _oracle_rows(ls, fc, order, srcs, ignores)
        assert np.array_equal(dist, od)
        assert np.array_equal(nh[:, :, :1], on[:, :, :1])
    pairs = [(rng.randrange(len(order)), rng.randrange(len(order))) for _ in range(12)]
    got = fc.kth_paths(pairs, 8)
    for (s, d), (k1, k2) in zip(pairs, got):
        for k, paths in ((1, k1), (2, k2)):
            want = [[LinkDesc(*l) for l in p] for p in ls.get_kth_paths(order[s], order[d], k)]
            assert [[LinkDesc(*l) for l in p] for p in paths] == want, (order[s], order[d], k)


def test_fast_checker_rejects_zero_metrics(oracle):
    dbs = random_topology(2400, n=10, extra=10, max_metric=2, min_metric=0, parallel=0.0, overload=0.0,
                          link_overload=0.0)
    _, _, fc = _checker(oracle, dbs)
    with pytest.raises(ValueError, match="zero-metric"):
        fc.spf_rows(list(range(10)), [], 2)
