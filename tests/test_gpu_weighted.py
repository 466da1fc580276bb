"""Weighted sweeps (general integer metrics), LinkState::runSpf semantics
(LinkState.cpp:808-882, first hops :857-873), on the two LDS plans:
  spf_wms_kernel (ORH_VARIANT_WMS, >= 256 sources): 4-source Bellman-Ford
      batches with u16 labels in LDS, then the first-hop phase over u32 rows
  spf_lds_nh_kernel (ORH_VARIANT_LDS_NH, fewer sources or ignore sets):
      {dist, first-hop mask} labels in LDS, first hops fused, one workgroup per
      source

  C2w 100x100 grid, metrics 1..64      all 10,000 rows (WMS) vs the fast
                                       checker, 200 of them vs the oracle
  packed labels past 16 bits           a ladder at metric 30,000: every row
                                       overflows the u32 label and is redone
                                       with u64 labels
  17..32 distinct neighbours           u64 labels directly
  ignore sets                          per-source ignore sets (KSP2-style
                                       host path) on a random weighted graph
"""
import gc
import random

import numpy as np
import pytest

from openr_amd import host_module
from openr_amd.facade import load_topology
from openr_amd.topology import ladder
from openr_amd.types import K_TESTING_AREA

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA
LDS_NH, WMS = 12, 13  # ORH_VARIANT_LDS_NH, ORH_VARIANT_WMS


def _compare_rows(sweep, names, rows, dist_w, nh_w, label):
    W = sweep.words
    Wc = nh_w.shape[2]
    w = min(W, Wc)
    for k, i in enumerate(rows):
        d, m = sweep.fetch(i)
        m = m.reshape(-1, W)
        assert np.array_equal(d, dist_w[k]), (label, "dist", names[i])
        if not np.array_equal(m[:, :w], nh_w[k][:, :w]):
            bad = np.nonzero(np.any(m[:, :w] != nh_w[k][:, :w], axis=1))[0]
            raise AssertionError(f"{label}: first hops of {names[i]} differ at {len(bad)} nodes")
        assert not m[:, w:].any() and not nh_w[k][:, w:].any(), names[i]


def test_c2w_sweep_all_rows_vs_checker(hip, oracle):
    """The benched weighted sweep (bench_legs.leg_c2w): every one of the
    10,000 rows, dist and first-hop masks in full, against the independent
    fast checker (binary-heap Dijkstra + the closed-form first hops); 200
    seeded rows against the faithful oracle's runSpf tables too."""
    from openr_amd.workloads import c2_weighted_grid
    adj, _ = c2_weighted_grid()
    als_h, _ = load_topology(hip, adj, [])
    ls = als_h[A]._impl
    order = ls.node_names()
    names = [db.thisNodeName for db in adj]
    sw = ls.sweep(names, True)
    sw.run()
    sw.sync()
    info = sw.info()
    assert info["variant"] == WMS and info["rows"] == len(names) and info["hop_nodes"] == 1, info
    als_o, _ = load_topology(oracle, adj, [])
    fc = oracle.module.FastChecker(als_o[A]._impl, order)
    ids = {n: i for i, n in enumerate(order)}
    for lo in range(0, len(names), 1000):
        rows = list(range(lo, min(len(names), lo + 1000)))
        dist, nh = fc.spf_rows([ids[names[i]] for i in rows], [], 16)
        _compare_rows(sw, names, rows, dist, nh, "checker")
        del dist, nh
        gc.collect()
    rng = random.Random(2024)
    rows = rng.sample(range(len(names)), 200)
    srcs = [names[i] for i in rows]
    dist_o, nh_o = als_o[A]._impl.spf_tables(srcs, order, [ls.neighbors(s) for s in srcs], 16)
    _compare_rows(sw, names, rows, dist_o, nh_o, "oracle")
    # not a degenerate workload: ECMP somewhere, distances well past the BFS depth
    d, m = sw.fetch(0)
    assert int(d.max()) > 2000
    assert any(bin(int(x)).count("1") > 1 for x in sw.fetch(len(names) // 2)[1])


def _random_weighted(seed, n, extra, max_metric):
    from test_gpu_parity import random_topology
    return random_topology(seed, n=n, extra=extra, max_metric=max_metric, parallel=0.1,
                           overload=0.05, link_overload=0.02)


def _all_rows_vs_oracle(hip, oracle, dbs, expect_variant=LDS_NH, repeat=1):
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    ls = als_h[A]._impl
    order = ls.node_names()
    names = sorted(db.thisNodeName for db in dbs) * repeat  # repeat: >= 256 rows take the WMS plan
    sw = ls.sweep(names, True)
    sw.run()
    sw.sync()
    info = sw.info()
    assert info["variant"] == expect_variant, info
    uniq = sorted(set(names))
    dist_o, nh_o = als_o[A]._impl.spf_tables(uniq, order, [ls.neighbors(s) for s in uniq], 16)
    at = {s: k for k, s in enumerate(uniq)}
    _compare_rows(sw, names, list(range(len(names))), dist_o[[at[s] for s in names]],
                  nh_o[[at[s] for s in names]], "oracle")
    return info


def test_packed_overflow_redone_with_u64_labels(hip, oracle):
    """Ladder at metric 30,000: distances reach ~0xFFFF within a few rungs,
    so every packed search overflows and its row comes from the u64 form."""
    dbs, _ = ladder(120, metric=30_000)
    for db in dbs[::7]:  # not uniform: the weighted plan
        db.adjacencies[0].metric = 29_999
    _all_rows_vs_oracle(hip, oracle, dbs)


@pytest.mark.parametrize("seed", [81, 82])
def test_random_weighted_all_rows(hip, oracle, seed):
    """Random graphs with parallel links, overloaded nodes and links: all
    rows, packed labels (degree <= 16)."""
    dbs = _random_weighted(seed, n=250, extra=600, max_metric=20)
    _all_rows_vs_oracle(hip, oracle, dbs)


@pytest.mark.parametrize("env", [{}, {"ORH_WMS_SKIP": "1"}, {"ORH_WMS_BAND": "0"},
                                 {"ORH_WMS_BAND": "0", "ORH_WMS_SKIP": "1"}, {"ORH_WMS_SOURCES": "4"}])
@pytest.mark.parametrize("seed", [85, 86])
def test_random_weighted_wms(hip, oracle, monkeypatch, seed, env):
    """The same kind of graph (parallel links, overloaded nodes - sources
    among them - and drained links), every node twice as a source: the WMS
    batches (repeated sources inside a batch, overloaded sources reaching
    only their neighbours), all rows vs the oracle; the default schedule
    (8-source batches, bands swept both ways, no activity skip) and the
    opt-in variants."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    dbs = _random_weighted(seed, n=250, extra=250, max_metric=30)
    for db in dbs:  # WMS needs every in-link in the ELL row: cap the degree
        db.adjacencies = db.adjacencies[:8]
    info = _all_rows_vs_oracle(hip, oracle, dbs, expect_variant=WMS, repeat=2)
    assert info["rows"] >= 500


def test_wms_overflow_redone(hip, oracle):
    """Ladder at metric 20,000: distances pass 16 bits within a few rungs, so
    every WMS batch flags its rows and the u64 LDS search redoes them."""
    dbs, _ = ladder(130, metric=20_000)
    for db in dbs[::5]:
        db.adjacencies[0].metric = 19_999
    _all_rows_vs_oracle(hip, oracle, dbs, expect_variant=WMS, repeat=2)


def test_many_neighbours_u64_labels(hip, oracle):
    """A hub with 24 distinct neighbours: its row needs more than 16 mask
    bits, so the batch runs with u64 labels."""
    from openr_amd.types import Adjacency, BinaryAddress, create_adj_db
    rng = random.Random(91)
    n = 300
    adjs = {i: [] for i in range(n)}

    def link(a, b, w):
        k = {a: len(adjs[a]), b: len(adjs[b])}  # interface names: the two ends name each other
        for x, y in ((a, b), (b, a)):
            adjs[x].append(Adjacency(f"n{y}", f"n{x}-n{y}-{k[x]}", BinaryAddress.of("fe80::1"),
                                     BinaryAddress.of("10.0.0.1"), w, 0, False, 0, 0, 1,
                                     f"n{y}-n{x}-{k[y]}"))

    for i in range(1, n):
        link(i, rng.randrange(i), rng.randint(1, 9))
    for j in range(1, 25):
        link(0, j * 11, rng.randint(1, 9))
    for _ in range(200):
        a, b = rng.randrange(n), rng.randrange(n)
        if a != b:
            link(a, b, rng.randint(1, 9))
    dbs = [create_adj_db(f"n{i}", adjs[i], i + 1, False, A) for i in range(n)]
    als_h, _ = load_topology(hip, dbs, [])
    assert len(als_h[A]._impl.neighbors("n0")) > 16
    _all_rows_vs_oracle(hip, oracle, dbs)


def test_ignore_sets_lds_nh(hip, oracle):
    """Per-source ignore sets through the fused LDS search: runSpf(src, true,
    {links}) for a batch the what-if repair does not take (repair off)."""
    dbs = _random_weighted(83, n=250, extra=500, max_metric=15)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    mod = host_module()
    mod.set_repair_mode(0)
    try:
        ls = als_h[A]._impl
        desc = dict(ls.link_ids())
        links = sorted(desc)
        rng = random.Random(84)
        names = sorted(db.thisNodeName for db in dbs)
        srcs = rng.sample(names, 40)
        sets = [rng.sample(links, 3) for _ in srcs]
        sw = ls.what_if_sweep(srcs, sets)
        sw.run()
        sw.sync()
        assert sw.info()["variant"] == LDS_NH, sw.info()
        order = ls.node_names()
        dist_o, nh_o = als_o[A]._impl.spf_tables(
            srcs, order, [ls.neighbors(s) for s in srcs], 16,
            [[tuple(desc[l][:3]) for l in st] for st in sets])
        _compare_rows(sw, srcs, list(range(len(srcs))), dist_o, nh_o, "oracle")
    finally:
        mod.set_repair_mode(1)
