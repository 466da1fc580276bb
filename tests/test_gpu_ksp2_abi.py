"""orh_ksp2 (the C-ABI KSP2 entry point) against the oracle's getKthPaths
(``-m gpu``): k = 1 and k = 2 paths, link by link, in order.

Covers parallel links (tie order = CSR row order = LinkSet order), drained
nodes and adjacencies, zero and 64-bit metrics (exact kernel rows), and the
C4 WAN at full size (50,000 nodes) on sampled (src, dst) pairs - the batched
k = 2 SPFs of one call run in one launch.
"""
import random

import pytest

from openr_amd.facade import LinkDesc, load_topology
from openr_amd.topology import wan
from openr_amd.types import K_TESTING_AREA

from test_gpu_parity import random_topology

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA


def _check(als_h, als_o, src, dsts):
    got = als_h[A]._impl.ksp2_abi(src, dsts)
    for d, (k1, k2) in zip(dsts, got):
        for k, paths in ((1, k1), (2, k2)):
            mine = [[LinkDesc(*l) for l in p] for p in paths]
            assert mine == als_o[A].get_kth_paths(src, d, k), (src, d, k)


@pytest.mark.parametrize("seed", range(4))
def test_ksp2_abi_random(hip, oracle, seed):
    dbs = random_topology(1900 + seed, n=18, extra=30, max_metric=3, parallel=0.4, overload=0.1,
                          link_overload=0.05)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    for src in names[:5]:
        _check(als_h, als_o, src, names)


@pytest.mark.parametrize("lo,hi", [(0, 2), (1 << 30, (1 << 31) - 1)])
def test_ksp2_abi_exact_rows(hip, oracle, lo, hi):
    from test_gpu_exact import _topology
    dbs = _topology(1950, n=16, extra=24, min_metric=lo, max_metric=hi, parallel=0.4, overload=0.0,
                    link_overload=0.0)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    for src in names[:4]:
        _check(als_h, als_o, src, names)


def test_ksp2_abi_wan_50k(hip, oracle):
    """C4's WAN: one source, 3 sampled destinations in one call (the oracle's
    runSpf takes ~10 s per fresh SPF at this size)."""
    adj_dbs, _ = wan(50000, seed=4)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    rng = random.Random(4)
    dsts = [f"w{rng.randrange(50000)}" for _ in range(3)]
    _check(als_h, als_o, "w17", dsts)


def test_ksp2_prefetch_wan_50k(hip, oracle):
    """The LinkState path at C4 size: prefetchKthPaths over sampled pairs
    (all k = 2 re-runs in one launch), then the memoized getKthPaths."""
    adj_dbs, _ = wan(50000, seed=4)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    rng = random.Random(44)
    pairs = [("w17", f"w{rng.randrange(50000)}") for _ in range(2)]
    als_h[A]._impl.prefetch_kth_paths(pairs)
    for s, d in pairs:
        for k in (1, 2):
            assert als_h[A].get_kth_paths(s, d, k) == als_o[A].get_kth_paths(s, d, k), (s, d, k)


@pytest.mark.parametrize("seed", range(4))
def test_ksp2_device_batch_random(hip, oracle, seed):
    """prefetchKthPaths through orh_ksp2_batch (k = 1 traces, k = 2 searches
    and k = 2 traces on the device) over every (src, dst) pair of random
    graphs with parallel links (LinkSet tie order), drained nodes and
    adjacencies: every pair's k = 1 and k = 2 paths equal the oracle's
    getKthPaths (LinkState.cpp:762-791), link by link, and spf_runs counts
    the reference's runs (one per source, one per pair with k = 1 paths)."""
    dbs = random_topology(2100 + seed, n=20, extra=34, max_metric=4, parallel=0.4, overload=0.1,
                          link_overload=0.06)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    pairs = [(s, d) for s in names for d in names]
    ls = als_h[A]._impl
    runs0 = ls.spf_runs
    ls.prefetch_kth_paths(pairs)
    dev, host = ls.ksp_stats()
    assert dev == len(pairs) and host == 0
    runs_o0 = als_o[A]._impl.spf_runs
    for s, d in pairs:
        for k in (1, 2):
            assert als_h[A].get_kth_paths(s, d, k) == als_o[A].get_kth_paths(s, d, k), (s, d, k)
    assert ls.spf_runs - runs0 == als_o[A]._impl.spf_runs - runs_o0


def test_ksp2_device_batch_c4(hip, oracle, monkeypatch):
    """The C4 KSP2 batch as bench_legs.leg_c4 runs it: c4_wan() (seed 4004),
    1,024 seeded (src, dst) pairs through the device batch. All 1,024 pairs'
    paths equal the product's host traces over device rows (ORH_KSP_HOST=1,
    the traceOnePath restatement checked against the oracle above), and
    three sampled pairs equal the oracle's getKthPaths at full size."""
    from openr_amd.workloads import C4_KSP2_PAIRS, c4_ksp2_pairs, c4_wan
    adj, _ = c4_wan()
    als_h, _ = load_topology(hip, adj, [])
    ls = als_h[A]._impl
    pairs = c4_ksp2_pairs(ls.node_names(), C4_KSP2_PAIRS)
    ls.prefetch_kth_paths(pairs)
    dev, host = ls.ksp_stats()
    assert dev == len(set(pairs)) and host == 0
    got = {(s, d, k): als_h[A].get_kth_paths(s, d, k) for s, d in pairs for k in (1, 2)}
    assert sum(len(v) for v in got.values()) > len(pairs)
    monkeypatch.setenv("ORH_KSP_HOST", "1")
    als_r, _ = load_topology(hip, adj, [])
    als_r[A]._impl.prefetch_kth_paths(pairs)
    assert als_r[A]._impl.ksp_stats()[0] == 0
    for (s, d, k), v in got.items():
        assert v == als_r[A].get_kth_paths(s, d, k), (s, d, k)
    als_o, _ = load_topology(oracle, adj, [])
    for s, d in random.Random(7).sample(pairs, 3):
        for k in (1, 2):
            assert got[(s, d, k)] == als_o[A].get_kth_paths(s, d, k), (s, d, k)


def test_ksp2_device_batch_c4_vs_oracle(hip, oracle):
    """The benched C4 KSP2 batch (c4_wan(), 1,024 seeded pairs, one device
    batch) against the oracle's own getKthPaths (LinkState.cpp:762-791) on 40
    of its pairs: the 20 with the most k = 1 + k = 2 paths and 20 seeded
    others, k = 1 and k = 2, link by link. The oracle runs them on 16
    threads, each with a LinkState copy loaded in the same order as the
    product's (same LinkSet iteration order)."""
    from openr_amd.workloads import C4_KSP2_PAIRS, c4_ksp2_pairs, c4_wan
    adj, _ = c4_wan()
    als_h, _ = load_topology(hip, adj, [])
    ls = als_h[A]._impl
    pairs = c4_ksp2_pairs(ls.node_names(), C4_KSP2_PAIRS)
    ls.prefetch_kth_paths(pairs)
    assert ls.ksp_stats() == (len(set(pairs)), 0)
    got = {(s, d): (als_h[A].get_kth_paths(s, d, 1), als_h[A].get_kth_paths(s, d, 2)) for s, d in pairs}
    ranked = sorted(set(pairs), key=lambda p: (-(len(got[p][0]) + len(got[p][1])), p))
    pick = ranked[:20]
    rest = [p for p in sorted(set(pairs)) if p not in set(pick)]
    pick += random.Random(41).sample(rest, 20)
    assert sum(len(got[p][0]) + len(got[p][1]) for p in pick) > 60
    als_o, _ = load_topology(oracle, adj, [])
    want = als_o[A]._impl.kth_paths_threaded(pick, 16, [db.thisNodeName for db in adj])
    for p, (k1, k2) in zip(pick, want):
        assert got[p][0] == [[LinkDesc(*l) for l in path] for path in k1], (p, 1)
        assert got[p][1] == [[LinkDesc(*l) for l in path] for path in k2], (p, 2)


def test_kth_paths_link_handles(hip, oracle):
    """getKthPaths in the reference's type: paths of LinkRef handles walked as
    selectBestPathsKsp2 walks them (Decision.cpp:1035-1076:
    link->getMetricFromNode(cur), getOtherNodeName, getIfaceFromNode,
    getNhV6FromNode of the first link), equal to the oracle's links and
    directional metrics."""
    dbs = random_topology(2200, n=16, extra=26, max_metric=6, parallel=0.4, overload=0.0,
                          link_overload=0.0)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    adj = {(db.thisNodeName, a.ifName): a for db in dbs for a in db.adjacencies}
    walked = 0
    for src in names[:4]:
        for dst in names:
            for k in (1, 2):
                got = als_h[A]._impl.walk_kth_paths(src, dst, k)
                want = als_o[A].get_kth_paths(src, dst, k)
                assert len(got) == len(want), (src, dst, k)
                for (hops, nh6, if0), path in zip(got, want):
                    cur = src
                    for (metric, iface, other, area, up), l in zip(hops, path):
                        near_if, far = (l.if1, l.n2) if l.n1 == cur else (l.if2, l.n1)
                        assert (iface, other, area, up) == (near_if, far, A, True)
                        assert metric == als_o[A]._impl.metric_from_node(l.n1, l.if1, cur)
                        cur = far
                        walked += 1
                    assert cur == dst
                    assert nh6 == adj[(src, if0)].nextHopV6.addr
    assert walked > 50


@pytest.mark.parametrize("lds", ["1", "0"])
@pytest.mark.parametrize("seed,lo,hi", [(2300, 1, 5), (2301, 20000, 40000)])
def test_ksp2_device_batch_lds16(hip, oracle, monkeypatch, lds, seed, lo, hi):
    """The batch's k = 1 / k = 2 searches with u16 distances in LDS
    (spf_lds16_kernel, the default when a graph fits) and with the HBM kernel
    alone (ORH_KSP_LDS=0). At metrics 20,000-40,000 a path of two or three
    links needs 17 bits: those rows leave nodes unreached in the u16 search
    and are re-run by the HBM kernel from the fallback list. Every pair
    equals the oracle's getKthPaths."""
    monkeypatch.setenv("ORH_KSP_LDS", lds)
    dbs = random_topology(seed, n=22, extra=36, min_metric=lo, max_metric=hi, parallel=0.4,
                          overload=0.1, link_overload=0.06)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    pairs = [(s, d) for s in names for d in names]
    ls = als_h[A]._impl
    ls.prefetch_kth_paths(pairs)
    assert ls.ksp_stats() == (len(pairs), 0)
    for s, d in pairs:
        for k in (1, 2):
            assert als_h[A].get_kth_paths(s, d, k) == als_o[A].get_kth_paths(s, d, k), (s, d, k)


def test_ksp2_c4_lds16_vs_hbm(hip, monkeypatch):
    """The benched C4 batch (1,024 pairs on the 50k-node WAN) through the u16
    LDS searches and through the HBM kernel alone: the same paths for every
    pair, k = 1 and k = 2 (the HBM path is pinned to the oracle above)."""
    from openr_amd.workloads import C4_KSP2_PAIRS, c4_ksp2_pairs, c4_wan
    adj, _ = c4_wan()
    got = []
    for lds in ("1", "0"):
        monkeypatch.setenv("ORH_KSP_LDS", lds)
        als_h, _ = load_topology(hip, adj, [])
        ls = als_h[A]._impl
        pairs = c4_ksp2_pairs(ls.node_names(), C4_KSP2_PAIRS)
        ls.prefetch_kth_paths(pairs)
        assert ls.ksp_stats() == (len(set(pairs)), 0)
        got.append({(s, d, k): als_h[A].get_kth_paths(s, d, k) for s, d in pairs for k in (1, 2)})
    assert got[0] == got[1]
    assert sum(len(v) for v in got[0].values()) > C4_KSP2_PAIRS


def test_ksp2_lds16_spill_table_full(hip, oracle):
    """A 2,400-node ladder at metric 30,000: every node more than two links
    away needs the spill table, which holds 2,048 nodes, so every search
    overflows it and its row is re-run by the HBM kernel - sampled pairs
    equal the oracle's getKthPaths."""
    from openr_amd.topology import ladder
    L = 1200
    dbs, _ = ladder(L, 30000)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    # pairs on one rail: one shortest path each (a cross-rail pair has one
    # per rung, more than a device trace holds)
    pairs = [("a0", f"a{L - 1}"), ("b5", f"b{L - 100}"), (f"a{L // 2}", "a3"), (f"b{L - 1}", "b0")]
    ls = als_h[A]._impl
    ls.prefetch_kth_paths(pairs)
    assert sum(ls.ksp_stats()) == len(set(pairs))
    found = 0
    for s, d in pairs:
        for k in (1, 2):
            got = als_h[A].get_kth_paths(s, d, k)
            assert got == als_o[A].get_kth_paths(s, d, k), (s, d, k)
            found += len(got)
    assert found > len(pairs)
