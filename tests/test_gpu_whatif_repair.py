"""What-if repair (whatif_kernels.hip) against the oracle (``-m gpu``).

An ignore-set batch whose sources repeat - runSpf(src, true, {link}) for a few
sources x many links, the C4 what-if shape - is answered from the plain SPF
rows of its distinct sources: only the nodes below a tight ignored link are
re-derived (LinkState.cpp:808-882 semantics on the reduced graph). Every
request must equal the oracle's runSpf with that ignore set: metric and
nexthop set per reachable node, unreachable nodes absent. Cases: random
graphs with parallel links, directional metrics, drained nodes and links
(both metric-uniform and general metrics, one- and multi-link ignore sets),
links that are not on any shortest path (the row is the base row), an
affected set larger than the workgroup's LDS (the flagged full-search
fallback), the existing ignore-set tests re-run with the repair forced on,
and the 50k-node WAN (every row against the non-repair device path, sampled
rows against the oracle).
"""
import random

import numpy as np
import pytest

from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid
from openr_amd.types import K_TESTING_AREA

from test_gpu_parity import random_topology

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA
VARIANT_REPAIR = 11


@pytest.fixture
def repair_mode(hip):
    mod = hip.module

    def set_mode(m):
        mod.set_repair_mode(m)

    yield set_mode
    mod.set_repair_mode(1)


def _batch(ls_h, ls_o, srcs, sets, link_desc, expect_repair=True):
    got = ls_h._impl.run_spf_batch(srcs, sets)
    if expect_repair:
        assert ls_h._impl.last_spf_info()["variant"] == VARIANT_REPAIR
    for src, ids, g in zip(srcs, sets, got):
        ref = ls_o._impl.run_spf_ignoring(src, [link_desc[i][:3] for i in ids])
        assert g == ref, (src, [link_desc[i] for i in ids])


@pytest.mark.parametrize("seed", range(8))
def test_repair_random_graphs(hip, oracle, seed):
    """Few sources x every link (single-link sets) plus two- and three-link
    sets, on graphs with parallel links and drained nodes / adjacencies."""
    uniform = seed % 2 == 1
    dbs = random_topology(3000 + seed, n=28, extra=40, max_metric=1 if uniform else 12,
                          parallel=0.25, overload=0.1, link_overload=0.08)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    rng = random.Random(seed)
    links = als_h[A]._impl.link_ids()
    desc = dict(links)
    lids = [lid for lid, _ in links]
    names = sorted(db.thisNodeName for db in dbs)
    srcs_pool = rng.sample(names, 4)
    srcs, sets = [], []
    for lid in lids:
        for s in srcs_pool:
            srcs.append(s)
            sets.append([lid])
    for _ in range(len(srcs) // 4):
        srcs.append(rng.choice(srcs_pool))
        sets.append(rng.sample(lids, rng.choice((2, 3))))
    _batch(als_h[A], als_o[A], srcs, sets, desc)


def test_repair_sources_neighbours(hip, oracle):
    """Every link incident to the source (the affected set starts at a first
    hop) and links between its neighbours."""
    dbs = random_topology(3100, n=20, extra=30, max_metric=5, parallel=0.3, overload=0.0,
                          link_overload=0.0)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    links = als_h[A]._impl.link_ids()
    desc = dict(links)
    names = sorted(db.thisNodeName for db in dbs)
    srcs, sets = [], []
    for s in names[:3]:
        mine = [lid for lid, d in links if s in (d[0], d[2])]
        for lid in mine:
            srcs += [s, s]
            sets += [[lid], [lid, mine[0]]]
    _batch(als_h[A], als_o[A], srcs, sets, desc)


def test_repair_fallback_large_affected_set(hip, oracle):
    """A 60x60 grid: ignoring a link at the corner source puts ~3,500 nodes
    below it (more than the LDS node list holds). Such requests are repaired
    again in global slots (64 per batch); repeated 40 times each (80 big
    requests), the ones beyond the slots take the full-search fallback."""
    dbs, _ = bench_grid(60, 0)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    links = als_h[A]._impl.link_ids()
    desc = dict(links)
    corner = [lid for lid, d in links if "0" in (d[0], d[2])]
    far = [lid for lid, d in links if "1830" in (d[0], d[2])]
    srcs = ["0"] * (40 * len(corner)) + ["1830"] * len(far) + ["0"] * len(far)
    sets = [[x] for x in corner] * 40 + [[x] for x in far] * 2
    got = als_h[A]._impl.run_spf_batch(srcs, sets)
    assert als_h[A]._impl.last_spf_info()["variant"] == VARIANT_REPAIR
    ref = {}
    for src, ids, g in zip(srcs, sets, got):
        key = (src, ids[0])
        if key not in ref:
            ref[key] = als_o[A]._impl.run_spf_ignoring(src, [desc[ids[0]][:3]])
        assert g == ref[key], key


def test_repair_forced_single_requests(hip, oracle, repair_mode):
    """Single runSpf(src, true, ignore) calls with the repair forced on
    (ORH_REPAIR_ALWAYS): two-link sets on general graphs."""
    repair_mode(2)
    for seed in range(4):
        dbs = random_topology(3200 + seed)
        als_h, _ = load_topology(hip, dbs, [])
        als_o, _ = load_topology(oracle, dbs, [])
        rng = random.Random(seed)
        for db in dbs[:8]:
            src = db.thisNodeName
            links = als_o[A].links_from_node(src)
            ignore = [tuple(l) for l in rng.sample(links, min(2, len(links)))]
            assert als_h[A]._impl.run_spf_ignoring(src, ignore) == \
                als_o[A]._impl.run_spf_ignoring(src, ignore)


@pytest.mark.parametrize("seed", range(3))
def test_repair_forced_ksp2(hip, oracle, repair_mode, seed):
    """KSP2 second paths (k = 2 re-runs ignore the k = 1 path links) with the
    repair forced on, including the batched prefetch."""
    repair_mode(2)
    dbs = random_topology(3300 + seed, n=16, extra=24, max_metric=3, parallel=0.4, overload=0.0,
                          link_overload=0.0)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    als_h[A]._impl.prefetch_kth_paths([(s, d) for s in names[:4] for d in names if d != s])
    for src in names[:4]:
        for dst in names:
            for k in (1, 2):
                assert als_h[A].get_kth_paths(src, dst, k) == als_o[A].get_kth_paths(src, dst, k), \
                    (seed, src, dst, k)


def test_repair_wan_50k(hip, oracle, repair_mode):
    """C4 shape on the 50k-node WAN: 64 links x 4 sources. Every row (dist
    and first-hop mask) equals the non-repair device path's (itself checked
    against the oracle at this size in test_wan_50k_hbm_kernel), and the
    request that changes the most nodes equals the oracle's runSpf."""
    from openr_amd.workloads import c4_wan, c4_what_if_pairs
    adj, _ = c4_wan()
    als_h, _ = load_topology(hip, adj, [])
    ls = als_h[A]._impl
    names = ls.node_names()
    links = ls.link_ids()
    desc = dict(links)
    pairs = c4_what_if_pairs([lid for lid, _ in links], names, 64, 4)
    srcs = [s for s, _ in pairs]
    sets = [[l] for _, l in pairs]
    rows = {}
    for mode in (1, 0):
        repair_mode(mode)
        sw = ls.what_if_sweep(srcs, sets)
        sw.run()
        sw.sync()
        assert (sw.info()["variant"] == VARIANT_REPAIR) == (mode == 1)
        rows[mode] = [sw.fetch(i) for i in range(len(pairs))]
        del sw
    changed = []
    for i in range(len(pairs)):
        np.testing.assert_array_equal(rows[1][i][0], rows[0][i][0], err_msg=str(pairs[i]))
        np.testing.assert_array_equal(rows[1][i][1], rows[0][i][1], err_msg=str(pairs[i]))
    # the request whose row differs most from its source's plain row
    base = {}
    repair_mode(1)
    for s in set(srcs):
        sw = ls.sweep([s], True)
        sw.run()
        sw.sync()
        base[s] = sw.fetch(0)
    for i, (s, _) in enumerate(pairs):
        changed.append((int(np.sum(rows[1][i][0] != base[s][0]) + np.sum(rows[1][i][1] != base[s][1])), i))
    n_changed, i = max(changed)
    assert n_changed > 0
    als_o, _ = load_topology(oracle, adj, [])
    ref = als_o[A]._impl.run_spf_ignoring(srcs[i], [desc[sets[i][0]][:3]])
    nbrs = ls.neighbors(srcs[i])
    dist, nh = rows[1][i]
    got = {}
    for v in np.nonzero(dist != 0xFFFFFFFF)[0]:
        m = int(nh[v])
        got[names[v]] = (int(dist[v]), sorted(nbrs[b] for b in range(32) if m >> b & 1))
    assert got == ref


def _oracle_rows(ls_o, order, nbrs, srcs, ignores, threads=16):
    dist, nh = ls_o._impl.spf_tables(srcs, order, nbrs, threads, ignores)
    return dist, nh[:, :, 0]


def test_c4_bench_batch_vs_oracle(hip, oracle):
    """The C4 what-if batch exactly as bench_legs.leg_c4 runs it: c4_wan()
    (seed 4004), 4,096 links x 64 sources = 262,144 runSpf(src, true, {link})
    through one what-if job in chunks of C4_WHATIF_CHUNK. Every request's tier and
    affected-node count come back from the product; then, against the
    oracle's runSpf (LinkState.cpp:808-882) in full (dist + first hops of all
    50k nodes): all 64 base rows, the 24 requests with the largest affected
    sets, 24 seeded repaired ones and 8 seeded ones whose source row stands."""
    from openr_amd.workloads import C4_WHATIF_CHUNK, c4_wan, c4_what_if_job
    adj, _ = c4_wan()
    als_h, _ = load_topology(hip, adj, [])
    ls = als_h[A]._impl
    names = ls.node_names()
    links = ls.link_ids()
    desc = dict(links)
    srcs, idx, sets = c4_what_if_job([lid for lid, _ in links], names)
    assert len(srcs) == 64 and len(idx) == 4096 * 64
    big = ls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK)
    big.run()
    big.sync()
    info = big.info()
    tier, affected = info & 7, info >> 3
    # tiers 1-3 repair (affected > 0); tier 4 searches in full the slot
    # tier's queue (the subtrees too large for LDS) and reports no count
    assert int(tier.max()) <= 4
    assert np.array_equal((tier >= 1) & (tier <= 3), affected > 0)
    assert not np.any(affected[tier == 0])
    searched = [int(i) for i in np.nonzero(tier == 4)[0]]
    repaired = np.nonzero(affected)[0]
    assert 0 < len(repaired) < len(idx)
    rng = random.Random(44)
    top = [int(i) for i in repaired[np.argsort(-affected[repaired], kind="stable")[:24]]]
    rest = sorted(set(int(i) for i in repaired) - set(top))
    pick = (top + rng.sample(rest, 24) + rng.sample(searched, min(16, len(searched))) +
            rng.sample([int(i) for i in np.nonzero(tier == 0)[0]], 8))
    sub = ls.what_if_batch(srcs, [idx[i] for i in pick], [sets[i] for i in pick], len(pick))
    sub.run()
    sub.sync()
    assert np.array_equal(sub.info(), info[pick])
    got = [sub.fetch(k) for k in range(len(pick))]

    als_o, _ = load_topology(oracle, adj, [])
    nbrs = {s: ls.neighbors(s) for s in srcs}
    base = ls.sweep(srcs, True)
    base.run()
    base.sync()
    q_srcs = srcs + [srcs[idx[i]] for i in pick]
    q_ign = [[] for _ in srcs] + [[desc[sets[i][0]][:3]] for i in pick]
    dist_o, nh_o = _oracle_rows(als_o[A], names, [nbrs[s] for s in q_srcs], q_srcs, q_ign)
    for k, s in enumerate(srcs):
        d, m = base.fetch(k)
        np.testing.assert_array_equal(d, dist_o[k], err_msg=f"base dist {s}")
        np.testing.assert_array_equal(m, nh_o[k], err_msg=f"base nh {s}")
    for k, i in enumerate(pick):
        d, m = got[k]
        np.testing.assert_array_equal(d, dist_o[len(srcs) + k], err_msg=f"request {i} dist")
        np.testing.assert_array_equal(m, nh_o[len(srcs) + k], err_msg=f"request {i} nh")
        if 1 <= tier[i] <= 3:
            changed = int(np.sum((d != dist_o[idx[i]]) | (m != nh_o[idx[i]])))
            assert changed <= affected[i], (i, changed, affected[i])
    assert affected[top[0]] > 100  # the largest sets leave the small LDS tier


def test_c4_shared_base_rows(hip):
    """ORH_WHATIF_SHARE_BASE on the C4 job: the same tiers and affected
    counts, and every sampled request's row (repaired rows from the row
    buffer, source rows from the job's base rows) equals the dense job's."""
    from openr_amd.workloads import C4_WHATIF_CHUNK, c4_wan, c4_what_if_job
    adj, _ = c4_wan()
    als_h, _ = load_topology(hip, adj, [])
    ls = als_h[A]._impl
    names = ls.node_names()
    links = ls.link_ids()
    srcs, idx, sets = c4_what_if_job([lid for lid, _ in links], names)
    rows = {}
    infos = {}
    for share in (False, True):
        b = ls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK, share_base=share)
        b.run()
        b.sync()
        infos[share] = b.info()
        last = len(idx) - C4_WHATIF_CHUNK
        rng = random.Random(7)
        tier = infos[share] & 7
        pick = (rng.sample([i for i in range(last, len(idx)) if tier[i] == 0], 12) +
                rng.sample([i for i in range(last, len(idx)) if tier[i] != 0], 12))
        rows[share] = {i: b.fetch(i) for i in pick}
        del b
    assert np.array_equal(infos[False], infos[True])
    for i, (d, m) in rows[False].items():
        np.testing.assert_array_equal(rows[True][i][0], d, err_msg=f"request {i} dist")
        np.testing.assert_array_equal(rows[True][i][1], m, err_msg=f"request {i} nh")
