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
