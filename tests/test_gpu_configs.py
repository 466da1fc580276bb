"""Full-size BASELINE configs and every kernel variant, bit-exact against the
oracle (``-m gpu``).

Each sweep test asserts which kernel plan ran (orh_last_spf_info), so the
variant the bench times is the variant that is checked:

  C2 100x100 grid, all 10,000 sources   MS-BFS u32 masks + first_hop_lvl<16>;
                                        opt-in u64 masks and interval skip
  ladder 2 x 4,100 (BFS depth > 254)    MS-BFS levels >= 254 written directly
                                        (kLvlDirect) + first_hop_lvl<16>
  ladder 2 x 300, all sources           kLvlDirect + first_hop_lvl<4>
  150x150 grid (N = 22,500)             MS-BFS u16 masks (u32 exceeds LDS)
  C3 Clos (2,472 nodes)                 all 288 spines + sampled others
  C3 / C5 route databases               whole-DB canonical digests

Distances and first-hop sets are compared as whole tables: the oracle's
runSpf (LinkState.cpp:808-882) nextHops become bitmasks over the product's
own neighbour order (LinkState::neighbors), so every (source, node) pair is
checked, not a property of it.
"""
import gc
import random

import numpy as np
import pytest

from helpers import assert_digests_equal
from openr_amd import host_module
from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid, ladder
from openr_amd.types import K_TESTING_AREA
from openr_amd.workloads import C5_AREAS, c3_fabric, c5_multi_area

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA
MSBFS, BFS8, BFS16, BFS32, DIST16, DIST32 = 1, 2, 3, 4, 5, 6


def _sweep_tables(ls_h, ls_o, names, check, threads=16):
    """Run the all-sources sweep over `names` on the product, then compare the
    rows of `check` (indices into names) with the oracle's tables."""
    sweep = ls_h._impl.sweep(names, True)
    sweep.run()
    sweep.sync()
    info = sweep.info()
    order = ls_h._impl.node_names()
    srcs = [names[i] for i in check]
    nbrs = [ls_h._impl.neighbors(s) for s in srcs]
    dist_o, nh_o = ls_o._impl.spf_tables(srcs, order, nbrs, threads)
    W = sweep.words
    for k, i in enumerate(check):
        dist, nh = sweep.fetch(i)
        assert np.array_equal(dist, dist_o[k]), ("dist", names[i])
        got = nh.reshape(len(order), W)
        want = nh_o[k][:, :W]
        assert not np.any(nh_o[k][:, W:]), names[i]
        if not np.array_equal(got, want):
            bad = np.nonzero(np.any(got != want, axis=1))[0]
            raise AssertionError(f"first hops of {names[i]} differ at {len(bad)} nodes, "
                                 f"e.g. {order[bad[0]]}: {got[bad[0]]} vs {want[bad[0]]}")
    return info


@pytest.mark.parametrize("variant", [0, 1, 7])
def test_c2_sweep_first_hops_exact(hip, oracle, variant):
    """The bench's own sweeps (C2, all 10,000 sources in one launch): the
    grid itself (variant 0) and two of the timed what-if variants (the grid
    with one seeded link drained, bench.drain_what_if_link: SKIP records in
    the MS-BFS and in first_hop_lvl_kernel<8>). Dist rows and first-hop
    masks of 300 sources compared in full: the four corners, the edges'
    midpoints, the centre, both ends of the drained link and their
    neighbours, and seeded others."""
    from bench import drain_what_if_link
    n = 100
    adj_dbs, _ = bench_grid(n)
    special = [0, n - 1, n * (n - 1), n * n - 1, n // 2, n * (n // 2), n * (n // 2) + n - 1,
               n * (n - 1) + n // 2, n * (n // 2) + n // 2]
    if variant:
        drained = drain_what_if_link(adj_dbs, n, variant)
        assert drained and all(a.isOverloaded for a in drained)
        ends = {int(a.otherNodeName) for a in drained}
        for e in sorted(ends):
            special += [e] + [int(x.otherNodeName) for x in adj_dbs[e].adjacencies]
        special = list(dict.fromkeys(special))
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = [str(i) for i in range(n * n)]
    rng = random.Random(22 + variant)
    check = special + rng.sample([i for i in range(n * n) if i not in special], 300 - len(special))
    info = _sweep_tables(als_h[A], als_o[A], names, check)
    assert info["variant"] == MSBFS and info["mask_bits"] == 32, info
    assert info["batch_sources"] == 32, info
    assert info["hop_nodes"] == 8, info  # first_hop_lvl_kernel<8>, as benched


@pytest.mark.parametrize("variant", [0, 7])
def test_c2_sweep_all_sources_exact(hip, oracle, variant):
    """Every one of the 10,000 rows of a benched C2 sweep (the grid, and the
    what-if variant 7 with its seeded drained link) against the oracle's
    runSpf tables on 16 threads, dist rows and first-hop masks in full, in
    chunks of 1,000 sources (~11 s of oracle time per variant)."""
    from bench import drain_what_if_link
    n = 100
    adj_dbs, _ = bench_grid(n)
    if variant:
        assert drain_what_if_link(adj_dbs, n, variant)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = [str(i) for i in range(n * n)]
    ls_h, ls_o = als_h[A], als_o[A]
    sweep = ls_h._impl.sweep(names, True)
    sweep.run()
    sweep.sync()
    info = sweep.info()
    assert info["variant"] == MSBFS and info["hop_nodes"] == 8, info
    assert info["ms_direct"] == 0, info  # Cuthill-McKee layout: rows through ms_finalize_kernel, as benched
    order = ls_h._impl.node_names()
    W = sweep.words
    for lo in range(0, n * n, 1000):
        srcs = names[lo:lo + 1000]
        dist_o, nh_o = ls_o._impl.spf_tables(srcs, order, [ls_h._impl.neighbors(s) for s in srcs], 16)
        for k, s in enumerate(srcs):
            dist, nh = sweep.fetch(lo + k)
            assert np.array_equal(dist, dist_o[k]), ("dist", s)
            assert not np.any(nh_o[k][:, W:]), s
            assert np.array_equal(nh.reshape(len(order), W), nh_o[k][:, :W]), ("first hops", s)
        del dist_o, nh_o
        gc.collect()


@pytest.mark.parametrize("env", [{"ORH_MS_WIDE": "1"}, {"ORH_MS_SKIP": "1"}, {"ORH_MS_ORDER": "host"},
                                 {"ORH_MS_ORDER": "host", "ORH_MS_DIRECT": "0"},
                                 {"ORH_MS_SKIP": "1", "ORH_MS_ORDER": "host"}])
def test_c2_sweep_opt_in_variants(hip, oracle, monkeypatch, env):
    """The opt-in MS-BFS variants on the same sweep, 64 sources compared in
    full: u64 masks (250 batches of 40 sources), the interval skip, the host
    layout with its rows written by the search kernel and through
    ms_finalize_kernel (the default is the Cuthill-McKee layout: ms_lvl scratch
    + ms_finalize_kernel)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n = 100
    adj_dbs, _ = bench_grid(n)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = [str(i) for i in range(n * n)]
    rng = random.Random(32)
    check = [0, n * n - 1] + rng.sample(range(1, n * n - 1), 62)
    info = _sweep_tables(als_h[A], als_o[A], names, check)
    wide = "ORH_MS_WIDE" in env
    assert info["variant"] == MSBFS and info["mask_bits"] == (64 if wide else 32), info
    assert info["batch_sources"] == (40 if wide else 32), info
    direct = not wide and env.get("ORH_MS_ORDER") == "host" and "ORH_MS_DIRECT" not in env
    assert info["ms_direct"] == (1 if direct else 0), info


@pytest.mark.parametrize("order", ["host", "cm"])
@pytest.mark.parametrize("length,metric,hop_nodes", [(4100, 3, 8), (300, 1, 4)])
def test_ladder_deep_levels(hip, oracle, monkeypatch, length, metric, hop_nodes, order):
    """BFS depth beyond the u8 level encoding (levels >= 254 are written to
    the distance rows directly and read back through them), with the rows
    written by the search kernel (ORH_MS_ORDER=host) and through
    ms_finalize_kernel (Cuthill-McKee layout, the default)."""
    monkeypatch.setenv("ORH_MS_ORDER", order)
    adj_dbs, _ = ladder(length, metric)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = sorted(db.thisNodeName for db in adj_dbs)
    rng = random.Random(length)
    ends = [names.index(x) for x in ("a0", "b0", f"a{length - 1}", f"b{length - 1}")]
    check = ends + rng.sample(range(len(names)), 28)
    info = _sweep_tables(als_h[A], als_o[A], names, check)
    assert info["variant"] == MSBFS, info
    assert info["hop_nodes"] == hop_nodes, info
    assert info["ms_direct"] == (1 if order == "host" else 0), info


def test_u16_mask_msbfs_150x150(hip, oracle):
    """N = 22,500: two u32 frontier arrays exceed the 160 KB LDS, so the
    planner takes 16-source (u16) masks."""
    n = 150
    adj_dbs, _ = bench_grid(n)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = [str(i) for i in range(0, n * n, 37)] + [str(n * n - 1)]
    rng = random.Random(150)
    check = [0, len(names) - 1] + rng.sample(range(1, len(names) - 1), 30)
    info = _sweep_tables(als_h[A], als_o[A], names, check)
    assert info["variant"] == MSBFS and info["mask_bits"] == 16, info


def test_c3_clos_sweep(hip, oracle):
    """C3's 2,472-node Clos (full spine mesh), all sources in one sweep;
    every spine (36 x 8, the widest first-hop masks) and 64 seeded others
    compared in full."""
    adj_dbs, _ = c3_fabric(num_prefixes=0)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = [db.thisNodeName for db in adj_dbs]
    spines = [i for i, x in enumerate(names) if x.startswith("1-")]
    assert len(spines) == 288
    rng = random.Random(33)
    others = rng.sample([i for i in range(len(names)) if i not in set(spines)], 64)
    info = _sweep_tables(als_h[A], als_o[A], names, spines + others)
    assert info["variant"] == MSBFS, info


@pytest.mark.parametrize("best_route", [False, True])
def test_c3_route_db_full(hip, oracle, best_route):
    """C3 buildRouteDb("2-0-0") over 100k prefixes (5% anycast) in default and
    best-route mode: whole-DB digest parity, bestPrefixEntry included."""
    adj_dbs, prefixes = c3_fabric()
    als_h, ps_h = load_topology(hip, adj_dbs, prefixes)
    als_o, ps_o = load_topology(oracle, adj_dbs, prefixes)
    me = "2-0-0"
    sh = hip.spf_solver(me, True, enable_best_route_selection=best_route)
    so = oracle.spf_solver(me, True, enable_best_route_selection=best_route)
    n = assert_digests_equal(sh, so, me, als_h, ps_h, als_o, ps_o)
    assert n > 100_000


def _c5(num_prefixes):
    areas, prefixes = c5_multi_area(num_prefixes=num_prefixes)
    return [db for a in C5_AREAS for db in areas[a]], prefixes


@pytest.mark.parametrize("best_route", [False, True])
def test_c5_multi_area_small(hip, oracle, best_route):
    """C5 topology (4 areas, `me` in all four) at 3,000 prefixes: full
    canonical comparison including bestArea / bestPrefixEntry, for `me` and
    for nodes inside one area (multi-area getMinCostNodes ignores the area,
    Decision.cpp:1152-1175; per-area ECMP union, :1177-1228)."""
    adj, pfx = _c5(3000)
    als_h, ps_h = load_topology(hip, adj, pfx)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    for me in ("me", "A0", "B1249", "D2499"):
        h = hip.spf_solver(me, True, enable_best_route_selection=best_route).build_route_db(
            me, als_h, ps_h)
        o = oracle.spf_solver(me, True, enable_best_route_selection=best_route).build_route_db(
            me, als_o, ps_o)
        assert (h is None) == (o is None), me
        if h is not None:
            assert h.canonical_full() == o.canonical_full(), me


def test_c5_route_db_1m_digest(hip, oracle):
    """C5 at full size: 1M prefixes, best-route selection, whole-DB digest."""
    adj, pfx = _c5(1_000_000)
    als_h, ps_h = load_topology(hip, adj, pfx)
    als_o, ps_o = load_topology(oracle, adj, pfx)
    sh = hip.spf_solver("me", True, enable_best_route_selection=True)
    so = oracle.spf_solver("me", True, enable_best_route_selection=True)
    assert assert_digests_equal(sh, so, "me", als_h, ps_h, als_o, ps_o) > 900_000


def test_recreated_link_state_same_context(hip, oracle):
    """A LinkState destroyed and a new one built on the shared context must
    not reuse the first one's staged request (same source ids, new graph at
    a possibly recycled address)."""
    adj1, _ = bench_grid(6)
    als1, _ = load_topology(hip, adj1, [])
    names = [str(i) for i in range(36)]
    sw = als1[A]._impl.sweep(names, True)
    sw.run()
    sw.sync()
    als1[A].get_spf_result("0")
    del sw, als1
    gc.collect()
    adj2, _ = bench_grid(5)  # same names "0".."24", different topology
    als2, _ = load_topology(hip, adj2, [])
    als_o, _ = load_topology(oracle, adj2, [])
    got = {k: (v.metric, v.nextHops) for k, v in als2[A].get_spf_result("0").items()}
    want = {k: (v.metric, v.nextHops) for k, v in als_o[A].get_spf_result("0").items()}
    assert got == want
    names2 = [str(i) for i in range(25)]
    _sweep_tables(als2[A], als_o[A], names2, list(range(25)))


@pytest.mark.parametrize("mode", [1, 0])
def test_many_workgroups_per_cu(hip, oracle, mode):
    """Per-source LDS kernels with thousands of small workgroups (8+ per CU):
    the regime where a level-exit flag race would cut searches short. Uniform
    metrics (BFS kernel) and mixed metrics (level-synchronous Dijkstra)."""
    from test_gpu_parity import random_topology
    mod = host_module()
    mod.set_spf_mode(mode)
    try:
        for seed, max_metric in ((71, 1), (72, 9)):
            dbs = random_topology(seed, n=250, extra=450, max_metric=max_metric, parallel=0.1,
                                  overload=0.05, link_overload=0.02)
            als_h, _ = load_topology(hip, dbs, [])
            als_o, _ = load_topology(oracle, dbs, [])
            names = sorted(db.thisNodeName for db in dbs) * 10  # 2,500 rows
            info = _sweep_tables(als_h[A], als_o[A], names, list(range(0, 250, 3)))
            if mode == 1:
                assert info["variant"] in ((BFS8, BFS16) if max_metric == 1 else (DIST16,)), info
    finally:
        mod.set_spf_mode(0)


def test_device_selection_covers_bulk(hip, oracle):
    """The IP / SP_ECMP prefixes of C3 are selected by route_select_kernel
    (not the host path), and the result equals both the oracle's and the
    product's own host-path selection (ORH_HOST_SELECT)."""
    import os
    adj_dbs, prefixes = c3_fabric(num_prefixes=20_000)
    als_h, ps_h = load_topology(hip, adj_dbs, prefixes)
    als_o, ps_o = load_topology(oracle, adj_dbs, prefixes)
    me = "2-0-0"
    sh = hip.spf_solver(me, True, enable_best_route_selection=True)
    so = oracle.spf_solver(me, True, enable_best_route_selection=True)
    assert_digests_equal(sh, so, me, als_h, ps_h, als_o, ps_o)
    assert sh.device_selected >= 20_000 and sh.host_selected == 0
    os.environ["ORH_HOST_SELECT"] = "1"
    try:
        assert_digests_equal(sh, so, me, als_h, ps_h, als_o, ps_o)
        assert sh.device_selected == 0
    finally:
        del os.environ["ORH_HOST_SELECT"]


def test_prefix_mirror_incremental(hip, oracle):
    """Prefix deltas (add, withdraw, metric / forwarding changes, anycast
    growth) applied in rounds: the device mirror is patched incrementally
    (orh_prefix_apply_delta, id reuse, pool compaction) and every round's
    route DB equals the oracle's."""
    from openr_amd.types import (PrefixEntry, PrefixForwardingAlgorithm, PrefixForwardingType,
                                 PrefixMetrics, IpPrefix, BinaryAddress)
    adj_dbs, _ = bench_grid(12)
    als_h, ps_h = load_topology(hip, adj_dbs, [])
    als_o, ps_o = load_topology(oracle, adj_dbs, [])
    nodes = [db.thisNodeName for db in adj_dbs]
    rng = random.Random(77)
    live = {}

    def pfx(i):
        return IpPrefix(BinaryAddress(bytes([0xfd, 1, (i >> 8) & 255, i & 255]) + bytes(12)), 64)

    for rnd in range(30):
        for _ in range(400):
            i = rng.randrange(3000)
            node = rng.choice(nodes)
            op = rng.random()
            if op < 0.25 and (i, node) in live:
                ps_h.delete_prefix(node, A, pfx(i))
                ps_o.delete_prefix(node, A, pfx(i))
                del live[(i, node)]
                continue
            e = PrefixEntry(pfx(i), metrics=PrefixMetrics(1, rng.randint(0, 2), rng.randint(0, 2),
                                                            rng.randint(0, 2)))
            if op > 0.95:
                e.forwardingType = PrefixForwardingType.SR_MPLS
            if op > 0.98:
                e.forwardingAlgorithm = PrefixForwardingAlgorithm.KSP2_ED_ECMP
            ps_h.update_prefix(node, A, e)
            ps_o.update_prefix(node, A, e)
            live[(i, node)] = e
        me = str(rng.randrange(144))
        best = rnd % 2 == 1
        sh = hip.spf_solver(me, True, enable_best_route_selection=best)
        so = oracle.spf_solver(me, True, enable_best_route_selection=best)
        assert_digests_equal(sh, so, me, als_h, ps_h, als_o, ps_o)
        assert sh.device_selected > 0


@pytest.mark.parametrize("lat", ["1", "2", "0"])
@pytest.mark.parametrize("variant", [0, 7])
def test_c2_latency_plan(hip, oracle, monkeypatch, lat, variant):
    """A sweep over a shard of the grid's sources (20 batches, each with a CU
    to itself): the latency plan's 1,024-thread workgroups with the interval
    skip (ORH_MS_LATENCY=2), without it (default) and the 512-thread plan
    (ORH_MS_LATENCY=0); 64 rows in full against the oracle each time."""
    from bench import drain_what_if_link
    monkeypatch.setenv("ORH_MS_LATENCY", lat)
    n = 100
    adj_dbs, _ = bench_grid(n)
    if variant:
        assert drain_what_if_link(adj_dbs, n, variant)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = [str(i) for i in random.Random(640 + variant).sample(range(n * n), 640)]
    info = _sweep_tables(als_h[A], als_o[A], names, list(range(0, 640, 10)))
    assert info["variant"] == MSBFS and info["batch_sources"] == 32, info
    assert info["ms_threads"] == (512 if lat == "0" else 1024), info
    assert info["ms_skip"] == (1 if lat == "2" else 0), info
