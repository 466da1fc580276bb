"""Multi-device SPF inside the library (openr_amd/csrc/host/multi_device.h;
SURVEY.md §8e): ReplicatedLinkState mirrors one topology on several device
contexts and MultiDeviceSweep splits the all-sources SPF over them in
contiguous equal-work blocks. On a one-GPU box the "devices" are contexts on
device 0 (own streams), which exercises the same code: replication of every
mutation, block cuts, per-block sweeps, fetch / gather.

Every row equals the single-context sweep's, which test_gpu_configs.py pins
to the oracle (and here a sample is compared with the oracle directly)."""
import numpy as np
import pytest

from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid
from openr_amd.types import K_TESTING_AREA
from openr_amd.workloads import c3_fabric

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA


def _replicated(hip, adj_dbs, devices):
    rls = hip.module.ReplicatedLinkState(A, devices)
    for db in adj_dbs:
        rls.update_adjacency_database(db.to_wire())
    return rls


@pytest.mark.parametrize("replicas", [2, 4])
def test_multi_device_sweep_grid(hip, oracle, replicas):
    n = 40
    adj, _ = bench_grid(n)
    rls = _replicated(hip, adj, [0] * replicas)
    assert rls.replicas == replicas
    names = [str(i) for i in range(n * n)]
    sw = rls.sweep(names, True)
    assert sw.blocks == replicas
    cuts = [sw.block(r) for r in range(replicas)]
    assert cuts[0][0] == 0 and cuts[-1][1] == n * n
    assert all(cuts[r][1] == cuts[r + 1][0] for r in range(replicas - 1))
    sizes = [hi - lo for lo, hi in cuts]
    assert max(sizes) - min(sizes) <= n  # equal work on a grid: near-equal blocks
    sw.run()
    sw.sync()
    dist, nh = sw.gather()
    # the single-context sweep over the same sources
    als, _ = load_topology(hip, adj, [])
    one = als[A]._impl.sweep(names, True, sw.words)
    one.run()
    one.sync()
    for i in range(0, n * n, 7):
        d1, h1 = one.fetch(i)
        assert np.array_equal(dist[i], d1) and np.array_equal(nh[i], h1), names[i]
        d2, h2 = sw.fetch(i)
        assert np.array_equal(d2, d1) and np.array_equal(h2, h1), names[i]
    # and a sample against the oracle's runSpf tables
    als_o, _ = load_topology(oracle, adj, [])
    order = rls.replica(0).node_names()
    srcs = [names[i] for i in (0, n - 1, n * n // 2, n * n - 1)]
    dist_o, nh_o = als_o[A]._impl.spf_tables(srcs, order, [rls.replica(0).neighbors(s) for s in srcs], 4)
    for k, s in enumerate(srcs):
        i = int(s)
        assert np.array_equal(dist[i], dist_o[k])
        assert np.array_equal(nh[i].reshape(len(order), sw.words), nh_o[k][:, :sw.words])
    assert all(sw.last_ms(r) > 0 for r in range(replicas))


def test_multi_device_replicas_follow_mutations(hip):
    """A metric change and a deleted node reach every replica's mirror."""
    adj, _ = bench_grid(12)
    rls = _replicated(hip, adj, [0, 0, 0])
    db = adj[13]
    db.adjacencies[0].metric = 5
    rls.update_adjacency_database(db.to_wire())
    rls.delete_adjacency_database("77")
    names = [str(i) for i in range(144) if i != 77]
    sw = rls.sweep(names, True)
    sw.run()
    sw.sync()
    dist, _ = sw.gather()
    order = rls.replica(0).node_names()
    for r in range(1, 3):
        assert rls.replica(r).node_names() == order
    # every block's rows agree with the primary's own single-source SPF
    ls0 = rls.replica(0)
    for i in (0, 40, 100, len(names) - 1):
        res = ls0.get_spf_result(names[i], True)
        want = np.array([res[v][0] if v in res else 0xFFFFFFFF for v in order], dtype=np.uint32)
        assert np.array_equal(dist[i], want), names[i]


def test_replicas_share_one_host_store(hip):
    """Replicas 1.. are device views of replica 0's host graph store: a
    mutation is applied once, through the primary (a replica refuses one),
    and reaches every replica - new nodes and links included."""
    adj, _ = bench_grid(6)
    rls = _replicated(hip, adj[:30], [0, 0, 0])
    with pytest.raises(RuntimeError):
        rls.replica(1).update_adjacency_database(adj[0].to_wire())
    for db in adj[30:]:
        rls.update_adjacency_database(db.to_wire())
    names = [str(i) for i in range(36)]
    for r in range(3):
        assert rls.replica(r).node_names() == rls.replica(0).node_names()
    sw = rls.sweep(names, True)
    sw.run()
    sw.sync()
    dist, _ = sw.gather()
    order = rls.replica(0).node_names()
    pos = {v: i for i, v in enumerate(order)}
    for i, s in enumerate(names):  # unit grid: Manhattan distances, every block
        r0, c0 = divmod(int(s), 6)
        want = [abs(r0 - int(v) // 6) + abs(c0 - int(v) % 6) for v in order]
        assert list(dist[i]) == want, s
    assert pos


def test_multi_device_sweep_clos_weighted(hip):
    """C3 Clos: blocks cut by work (1 + links / 16 per source), so the 288
    spines (84 links each) do not all land in one block."""
    adj, _ = c3_fabric(num_prefixes=0)
    rls = _replicated(hip, adj, [0, 0, 0, 0])
    names = [db.thisNodeName for db in adj]
    sw = rls.sweep(names, True)
    deg = {db.thisNodeName: len(db.adjacencies) for db in adj}
    work = [sum(1 + deg[names[i]] / 16 for i in range(*sw.block(r))) for r in range(4)]
    assert max(work) / min(work) < 1.1
    sw.run()
    sw.sync()
    dist, nh = sw.gather()
    als, _ = load_topology(hip, adj, [])
    one = als[A]._impl.sweep(names, True, sw.words)
    one.run()
    one.sync()
    for i in range(0, len(names), 97):
        d1, h1 = one.fetch(i)
        assert np.array_equal(dist[i], d1) and np.array_equal(nh[i], h1), names[i]


def test_multi_device_sweep_follows_topology_changes(hip):
    """A sweep made before a metric change sweeps the changed topology (the
    replicas' pending deltas are flushed at run); a topology that grew a node
    since the sweep was made is refused instead of overrunning its rows."""
    from openr_amd.types import Adjacency, BinaryAddress, create_adj_db
    adj, _ = bench_grid(12)
    rls = _replicated(hip, adj, [0, 0])
    names = [str(i) for i in range(144)]
    sw = rls.sweep(names, True)
    db = adj[20]
    db.adjacencies[0].metric = 7
    rls.update_adjacency_database(db.to_wire())
    sw.run()
    sw.sync()
    dist, nh = sw.gather()
    als, _ = load_topology(hip, adj, [])
    one = als[A]._impl.sweep(names, True, sw.words)
    one.run()
    one.sync()
    for i in range(0, 144, 11):
        d1, h1 = one.fetch(i)
        assert np.array_equal(dist[i], d1) and np.array_equal(nh[i], h1), names[i]
    # a new node (with a link to node 0) changes the row shape
    new = Adjacency("0", "if_new_0", BinaryAddress.of("fe80::99"), BinaryAddress.of("10.9.9.9"), 1, 0,
                    False, 100, 10000, 1, "if_0_new")
    back = Adjacency("new", "if_0_new", BinaryAddress.of("fe80::98"), BinaryAddress.of("10.9.9.8"), 1, 0,
                     False, 100, 10000, 1, "if_new_0")
    adj[0].adjacencies.append(back)
    rls.update_adjacency_database(adj[0].to_wire())
    rls.update_adjacency_database(create_adj_db("new", [new], 0, False, A).to_wire())
    with pytest.raises(RuntimeError, match="changed shape"):
        sw.run()


def _c4(hip):
    from openr_amd.workloads import c4_wan, c4_what_if_job
    adj, _ = c4_wan()
    als, _ = load_topology(hip, adj, [])
    ls = als[A]._impl
    names = ls.node_names()
    srcs, idx, sets = c4_what_if_job([lid for lid, _ in ls.link_ids()], names)
    return adj, als, ls, names, srcs, idx, sets


@pytest.mark.parametrize("replicas", [2, 4])
def test_multi_device_what_if_c4_union(hip, replicas):
    """The benched C4 what-if job (262,144 runSpf(src, true, {link})) split
    over `replicas` device contexts by source block: every request's tier,
    affected count (slot-tier requests of a 4-way split may be searched in
    full instead) and row digest (dist + first hops of all 50,000 nodes,
    orh_row_digest) equal the single-context job's. The split runs
    copy-on-write (the bench's mode) against the dense single job, so the
    shared base rows are pinned too. Blocks run one at a time and release
    their rows (one GPU stands in for the devices)."""
    from openr_amd.workloads import C4_WHATIF_CHUNK
    adj, als, ls, names, srcs, idx, sets = _c4(hip)
    one = ls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK)
    one.set_digests()
    one.run()
    one.sync()
    info1, dig1 = one.info(), one.digests()
    one.release()
    del one
    rls = _replicated(hip, adj, [0] * replicas)
    assert rls.replica(0).node_names() == names
    md = rls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK, share_base=True)
    assert md.blocks == replicas
    cuts = [md.source_block(r) for r in range(replicas)]
    assert cuts[0][0] == 0 and cuts[-1][1] == len(srcs)
    assert sum(md.block_requests(r) for r in range(replicas)) == len(idx)
    assert max(md.block_requests(r) for r in range(replicas)) <= len(idx) // replicas + 4096
    md.set_digests()
    for r in range(replicas):
        md.run_block(r)
        md.sync()
        md.release(r)
    # 4 blocks search their largest repairs in full (ORH_WHATIF_SEARCH_LARGE)
    from helpers import assert_tiers_match
    assert_tiers_match(md.info(), info1, replicas >= 4)
    if replicas >= 4:
        assert np.any((np.asarray(md.info()) & 7) == 4)
    dig = md.digests()
    bad = np.nonzero(dig != dig1)[0]
    assert len(bad) == 0, f"{len(bad)} requests differ, first {bad[:5]}"


def test_multi_device_what_if_concurrent_run(hip):
    """MultiDeviceWhatIf.run drives every block from its own host thread at
    once (as on separate GPUs); a reduced C4 job (512 links x 64 sources)
    gives the same tiers and row digests as the single-context job."""
    adj, als, ls, names, srcs, idx, sets = _c4(hip)
    n = 512 * 64
    idx, sets = idx[:n], sets[:n]
    one = ls.what_if_batch(srcs, idx, sets, 8192)
    one.set_digests()
    one.run()
    one.sync()
    info1, dig1 = one.info(), one.digests()
    del one
    rls = _replicated(hip, adj, [0, 0, 0])
    md = rls.what_if_batch(srcs, idx, sets, 8192)
    md.set_digests()
    md.run()
    md.sync()
    assert np.array_equal(md.info(), info1)
    assert np.array_equal(md.digests(), dig1)
    # a second run refreshes the jobs and gives the same rows
    md.run()
    md.sync()
    assert np.array_equal(md.digests(), dig1)


def test_what_if_digests_match_fetched_rows(hip):
    """orh_row_digest of a job's rows equals the numpy restatement
    (tests/helpers.row_digest) over the same rows copied out."""
    from helpers import row_digest
    adj, als, ls, names, srcs, idx, sets = _c4(hip)
    pick = list(range(0, 64 * 40, 5))
    for share in (False, True):
        b = ls.what_if_batch(srcs, [idx[i] for i in pick], [sets[i] for i in pick], len(pick), share_base=share)
        b.set_digests()
        b.run()
        b.sync()
        dig = b.digests()
        for k in range(0, len(pick), 37):
            d, m = b.fetch(k)
            assert row_digest(d, m) == int(dig[k]), (share, k)


@pytest.mark.parametrize("replicas", [2, 4])
def test_multi_device_ksp2_c4_union(hip, replicas):
    """The benched 1,024 C4 KSP2 pairs split over device contexts by source:
    every pair's k = 1 and k = 2 paths equal the single LinkState's
    getKthPaths (prefetchKthPaths, which test_gpu_ksp2_abi pins to the
    oracle)."""
    from openr_amd.workloads import C4_KSP2_PAIRS, c4_ksp2_pairs
    adj, als, ls, names, *_ = _c4(hip)
    kp = c4_ksp2_pairs(names, C4_KSP2_PAIRS)
    ls.prefetch_kth_paths(kp)
    rls = _replicated(hip, adj, [0] * replicas)
    mk = rls.kth_paths_batch(kp)
    assert mk.blocks == replicas and sum(mk.block_pairs(r) for r in range(replicas)) == len(kp)
    mk.run()
    assert mk.device_pairs > 0.9 * len(kp)
    for i, (s, d) in enumerate(kp):
        for k in (1, 2):
            assert mk.paths(i, k) == ls.get_kth_path_ids(s, d, k), (i, s, d, k)


@pytest.mark.parametrize("best_route", [False, True])
def test_sharded_route_builder_c3(hip, oracle, best_route):
    """C3's 100k-prefix buildRouteDb sharded over 8 device contexts
    (ShardedRouteBuilder: shard r selects, policies and materialises prefix-id
    block r on device r from its own thread; the unicast maps are spliced):
    the merged DecisionRouteDb's digest equals the oracle's
    (Decision.cpp:615-792), and again after 2,000 prefix updates / withdrawals
    (each device's prefix mirror takes its own delta)."""
    import random
    from openr_amd.types import PrefixEntry, PrefixMetrics
    adj, pfx = c3_fabric()
    me = "2-0-0"
    _, ps = load_topology(hip, adj, pfx)
    ras = hip.module.ReplicatedAreaLinkStates([0] * 8)
    for db in adj:
        ras.update_adjacency_database(db.to_wire())
    b = ras.route_builder(me, True, enable_best_route_selection=best_route)
    assert b.shards == 8
    als_o, ps_o = load_topology(oracle, adj, pfx)
    so = oracle.spf_solver(me, True, enable_best_route_selection=best_route)

    def check():
        h = b.build_route_db_digest(me, ps._impl)
        o = so._impl.build_route_db_digest(me, als_o._impl, ps_o._impl)
        assert h[:2] == o[:2]
        assert h[2] == o[2]
        return h[0]

    assert check() > 90_000
    rng = random.Random(77)
    for i in range(2000):
        node, area, e = pfx[rng.randrange(len(pfx))]
        if i % 3 == 0:
            ps.delete_prefix(node, area, e.prefix)
            ps_o.delete_prefix(node, area, e.prefix)
        else:
            ne = PrefixEntry(e.prefix, metrics=PrefixMetrics(1, rng.randint(0, 3), rng.randint(0, 3),
                                                             rng.randint(0, 3)))
            ps.update_prefix(node, area, ne)
            ps_o.update_prefix(node, area, ne)
    check()
    sec, routes, shard_ms, merge_ms = b.time_build_route_db(me, ps._impl)
    assert routes > 90_000 and len(shard_ms) == 8 and all(x > 0 for x in shard_ms)


def test_prefix_shard_solver_builds_only_its_block(hip):
    """A SpfSolver with setPrefixShard(r, 8) builds about an eighth of C3's
    unicast routes, and the 8 shards' route counts add up to the whole
    build's (MPLS routes only on shard 0)."""
    adj, pfx = c3_fabric()
    me = "2-0-0"
    als, ps = load_topology(hip, adj, pfx)
    whole = hip.spf_solver(me, True)._impl.build_route_db_digest(me, als._impl, ps._impl)
    counts = []
    for r in range(8):
        s = hip.spf_solver(me, True)
        s._impl.set_prefix_shard(r, 8)
        d = s._impl.build_route_db_digest(me, als._impl, ps._impl)
        counts.append(d[:2])
    assert sum(c[0] for c in counts) == whole[0]
    assert counts[0][1] == whole[1] and all(c[1] == 0 for c in counts[1:])
    assert max(c[0] for c in counts) < whole[0] / 8 * 1.2
