"""Every distance kernel against the oracle (``-m gpu``).

libopenr_hip picks among three distance kernels (orh_set_spf_mode): the
multi-source BFS (uniform metrics, no ignore sets), the LDS-resident
per-source kernels, and the HBM frontier kernel (graphs beyond LDS, such as
the 50k-node WAN of config C4). Results must be identical in every mode, so
the parity cases run once per mode.
"""
import random

import numpy as np
import pytest

from openr_amd import host_module
from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid, fabric, wan
from openr_amd.types import K_TESTING_AREA

from test_gpu_parity import random_topology, spf_view

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA
MODES = {"auto": 0, "per_source": 1, "global": 2, "global_two_phase": 3, "exact": 4}


@pytest.fixture(params=list(MODES))
def spf_mode(request, hip):
    mod = host_module()
    mod.set_spf_mode(MODES[request.param])
    yield request.param
    mod.set_spf_mode(0)


@pytest.mark.parametrize("seed", range(4))
def test_modes_random_graphs(hip, oracle, spf_mode, seed):
    dbs = random_topology(500 + seed, n=40, extra=60)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    for db in dbs:
        for metric in (True, False):
            assert spf_view(als_h[A], db.thisNodeName, metric) == \
                spf_view(als_o[A], db.thisNodeName, metric), (spf_mode, seed, db.thisNodeName)


def test_modes_ignore_sets(hip, oracle, spf_mode):
    dbs = random_topology(600, n=30, extra=40)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    rng = random.Random(3)
    for db in dbs[:10]:
        links = als_o[A].links_from_node(db.thisNodeName)
        ignore = [tuple(l) for l in rng.sample(links, min(2, len(links)))]
        assert als_h[A]._impl.run_spf_ignoring(db.thisNodeName, ignore) == \
            als_o[A]._impl.run_spf_ignoring(db.thisNodeName, ignore)


def test_modes_sweep_fabric(hip, oracle, spf_mode):
    """Clos fabric (uniform metrics, high-degree spines with ELL overflow
    records): an all-sources sweep in each mode, compared with the oracle on
    every 7th source."""
    adj_dbs, _ = fabric(600, bug_compatible=False)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = [db.thisNodeName for db in adj_dbs]
    sweep = als_h[A]._impl.sweep(names, True)
    sweep.run()
    sweep.sync()
    node_names = als_h[A]._impl.node_names()
    for i in range(0, len(names), 7):
        dist, _ = sweep.fetch(i)
        ref = als_o[A].get_spf_result(names[i])
        got = {node_names[v]: int(d) for v, d in enumerate(dist) if d != 0xFFFFFFFF}
        assert got == {k: v.metric for k, v in ref.items()}, (spf_mode, names[i])
        hv = {k: (v.metric, v.nextHops) for k, v in als_h[A].get_spf_result(names[i]).items()}
        assert hv == {k: (v.metric, v.nextHops) for k, v in ref.items()}


def test_modes_grid_sweep_properties(hip, spf_mode):
    """40x40 grid, all sources: dist = Manhattan distance in every mode."""
    n = 40
    adj_dbs, _ = bench_grid(n)
    als_h, _ = load_topology(hip, adj_dbs, [])
    ls = als_h[A]
    sweep = ls._impl.sweep([str(i) for i in range(n * n)], True)
    sweep.run()
    sweep.sync()
    node_ids = {name: i for i, name in enumerate(ls._impl.node_names())}
    ids = np.array([node_ids[str(v)] for v in range(n * n)])
    rr, cc = np.divmod(np.arange(n * n), n)
    for s in range(0, n * n, 13):
        dist, nh = sweep.fetch(s)
        assert np.array_equal(dist[ids], np.abs(rr - rr[s]) + np.abs(cc - cc[s])), (spf_mode, s)


def test_modes_split_grid_sweep_unreached(hip, oracle, spf_mode):
    """40x40 grid cut in two between rows 19 and 20, all sources: half of
    every row is unreachable, so every (node, source) level byte the search
    never reaches must come out "unreached" (the multi-source search writes
    those at its end; no pre-filled scratch). Compared with the oracle."""
    n = 40
    adj_dbs, _ = bench_grid(n)
    for db in adj_dbs:
        row = int(db.thisNodeName) // n
        db.adjacencies = [a for a in db.adjacencies
                          if (int(a.otherNodeName) // n >= 20) == (row >= 20)]
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    names = [db.thisNodeName for db in adj_dbs]
    sweep = als_h[A]._impl.sweep(names, True)
    sweep.run()
    sweep.sync()
    node_names = als_h[A]._impl.node_names()
    for i in list(range(0, n * n, 11)) + [n * n - 1]:
        dist, _ = sweep.fetch(i)
        ref = als_o[A].get_spf_result(names[i])
        assert len(ref) == n * n // 2
        got = {node_names[v]: int(d) for v, d in enumerate(dist) if d != 0xFFFFFFFF}
        assert got == {k: v.metric for k, v in ref.items()}, (spf_mode, names[i])


def test_wan_50k_hbm_kernel(hip, oracle):
    """Config C4's 50k-node WAN (log-normal metrics): too large for the
    LDS-resident kernels, so AUTO selects the HBM frontier kernel. Exact
    comparison with the oracle on sampled sources, including first hops and
    an ignore-set (what-if) SPF."""
    adj_dbs, _ = wan(50000, seed=4)
    als_h, _ = load_topology(hip, adj_dbs, [])
    als_o, _ = load_topology(oracle, adj_dbs, [])
    for src in ("w0", "w49999"):
        h = als_h[A].get_spf_result(src)
        o = als_o[A].get_spf_result(src)
        assert {k: (v.metric, v.nextHops) for k, v in h.items()} == \
            {k: (v.metric, v.nextHops) for k, v in o.items()}, src
    links = als_o[A].links_from_node("w777")
    ignore = [tuple(links[0])]
    assert als_h[A]._impl.run_spf_ignoring("w777", ignore) == \
        als_o[A]._impl.run_spf_ignoring("w777", ignore)


@pytest.mark.parametrize("seed", range(3))
def test_what_if_batch(hip, oracle, seed):
    """Batched single-link what-if SPFs (runSpf(src, true, {link}) for many
    (src, link) pairs in one launch) against the oracle, pair by pair."""
    dbs = random_topology(700 + seed, n=30, extra=40)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    links = als_h[A]._impl.link_ids()
    rng = random.Random(seed)
    srcs, ign, descs = [], [], []
    for _ in range(40):
        lid, desc = links[rng.randrange(len(links))]
        srcs.append(dbs[rng.randrange(len(dbs))].thisNodeName)
        ign.append([lid])
        descs.append(desc)
    got = als_h[A]._impl.run_spf_batch(srcs, ign)
    for src, desc, g in zip(srcs, descs, got):
        assert g == als_o[A]._impl.run_spf_ignoring(src, [(desc[0], desc[1], desc[2])]), (src, desc)


def test_what_if_sweep_device_rows(hip, oracle):
    """Device-resident what-if sweep (the bench path) row by row."""
    dbs = random_topology(800, n=30, extra=40)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    links = als_h[A]._impl.link_ids()
    names = als_h[A]._impl.node_names()
    srcs = [dbs[i % len(dbs)].thisNodeName for i in range(24)]
    picks = [links[(7 * i) % len(links)] for i in range(24)]
    sweep = als_h[A]._impl.what_if_sweep(srcs, [[lid] for lid, _ in picks])
    sweep.run()
    sweep.sync()
    for i, (src, (lid, desc)) in enumerate(zip(srcs, picks)):
        dist, _ = sweep.fetch(i)
        ref = als_o[A]._impl.run_spf_ignoring(src, [(desc[0], desc[1], desc[2])])
        got = {names[v]: int(d) for v, d in enumerate(dist) if d != 0xFFFFFFFF}
        assert got == {k: v[0] for k, v in ref.items()}, (src, desc)


@pytest.mark.parametrize("seed", range(3))
def test_ksp2_batch_prefetch(hip, oracle, seed):
    """All k = 2 re-runs of many (src, dst) pairs in one launch: the memo then
    returns exactly the oracle's paths."""
    dbs = random_topology(900 + seed, n=16, extra=24, max_metric=3, parallel=0.4, overload=0.0,
                          link_overload=0.0)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    pairs = [(s, d) for s in names[:4] for d in names]
    als_h[A]._impl.prefetch_kth_paths(pairs)
    for s, d in pairs:
        for k in (1, 2):
            assert als_h[A].get_kth_paths(s, d, k) == als_o[A].get_kth_paths(s, d, k), (s, d, k)


def test_stream_lanes_concurrent_sweeps(hip, oracle):
    """Independent topologies on different stream lanes (own context and HIP
    stream each, bench.py --lanes): sweeps launched back to back overlap on
    the GPU and each equals the oracle on sampled sources."""
    from openr_amd.facade import load_topology as lt
    tops = [random_topology(7000 + i, n=40, extra=60, max_metric=1 if i % 2 else 9) for i in range(4)]
    sweeps = []
    for lane, dbs in enumerate(tops):
        als_h, _ = lt(hip, dbs, [], lane=lane)
        names = sorted(db.thisNodeName for db in dbs)
        sw = als_h[A]._impl.sweep(names, True)
        sweeps.append((dbs, als_h, names, sw))
    for _ in range(3):
        for *_, sw in sweeps:
            sw.run()
    for *_, sw in sweeps:
        sw.sync()
    for dbs, als_h, names, sw in sweeps:
        als_o, _ = lt(oracle, dbs, [])
        ids = als_h[A]._impl.node_names()
        for i in (0, len(names) // 2, len(names) - 1):
            dist, _ = sw.fetch(i)
            ref = als_o[A].get_spf_result(names[i], True)
            got = {ids[v]: int(d) for v, d in enumerate(dist) if d != 0xFFFFFFFF}
            assert got == {k: v.metric for k, v in ref.items()}, names[i]
