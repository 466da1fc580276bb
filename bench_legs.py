"""The other BASELINE.json configs, reported under bench.py's "legs" (N = 1).

Each leg times the HIP product with its inputs resident on the device, and
(unless --no-cpu-baseline) the CPU oracle, a restatement of the reference's
LinkState / SpfSolver with its containers, on a bounded sample of the same
work, stating the sample.

  c1  createGrid(10): buildRouteDb("1") ms (reference BM_DecisionGrid shape)
  c2w the 100x100 grid with integer metrics 1..64: all-sources SPF sweep
  c3  Clos (~2.5k nodes, full spine mesh): all-sources SPF sweep + 100k-prefix
      buildRouteDb, default and best-route selection
  c4  50k-node WAN: batched single-link what-if SPFs and KSP2 (src, dst) pairs
  c5  4 areas + 1M prefixes, best-route selection, RibPolicy area weights
"""
import importlib
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle", "build"))
    from openr_amd.facade import Backend
    return Backend(importlib.import_module("openr_oracle"), "oracle")


def _route_ms(solver, me, als, ps, reps):
    return statistics.median(solver._impl.time_build_route_db(me, als._impl, ps._impl)[0] * 1e3
                             for _ in range(reps))


def _route_runs(solver, me, als, ps, reps):
    """Every run's ms with their spread, the phase times / page faults of the
    builds (bench.profiled_build) and the cgroup's CFS throttling over them
    (bench.cgroup_cpu_stat)."""
    import bench
    st0 = bench.cgroup_cpu_stat()
    runs = [bench.profiled_build(solver._impl, me, als._impl, ps._impl) for _ in range(reps)]
    ms = [r["ms"] for r in runs]
    return ms, {"ms": bench.spread(ms), "phases": bench.phase_summary(runs),
                "cgroup_throttling": bench.throttle_delta(st0, bench.cgroup_cpu_stat())}


def _select_roofline(solver, me, als, ps):
    """Route-selection kernel of one build: device time and B_sel roofline."""
    solver._impl.time_build_route_db(me, als._impl, ps._impl)
    ms = solver._impl.last_select_ms
    b = solver._impl.last_select_bytes
    if ms <= 0:
        return {"select_kernel": None}
    gbs = b / (ms * 1e-3) / 1e9
    return {"select_kernel": {"ms": round(ms, 4), "bytes": b, "achieved_gbs": round(gbs, 1),
                              "frac": round(gbs / 8000.0, 4),
                              "prefixes_selected_on_device": solver._impl.device_selected}}


def leg_c1(hip, cpu):
    from openr_amd.facade import load_topology
    from openr_amd.topology import bench_grid
    adj, pfx = bench_grid(10, 1)
    als, ps = load_topology(hip, adj, pfx)
    out = {"workload": "C1 createGrid(10) buildRouteDb('1')",
           "build_route_db_ms": round(_route_ms(hip.spf_solver("1", True), "1", als, ps, 9), 4)}
    if cpu:
        o = _oracle()
        als_o, ps_o = load_topology(o, adj, pfx)
        out["cpu_build_route_db_ms"] = round(_route_ms(o.spf_solver("1", True), "1", als_o, ps_o, 9), 4)
    return out


def leg_c2w(hip, cpu, reps=10):
    """C2 with integer metrics (workloads.c2_weighted_grid: the 100x100 grid,
    a seeded metric in [1, 64] per link): all 10,000 sources swept, dist +
    first-hop rows written to HBM (runSpf semantics, LinkState.cpp:808-882,
    getMetricFromNode :851-852). Wall time of back-to-back sweeps, the HIP-event
    device time of one sweep alone, and its roofline by the same algorithmic
    bytes per source as C2."""
    from openr_amd.facade import load_topology
    from openr_amd.types import K_TESTING_AREA as A
    from openr_amd.workloads import C2W_MAX_METRIC, c2_weighted_grid
    adj, pfx = c2_weighted_grid()
    als, _ = load_topology(hip, adj, pfx)
    names = [db.thisNodeName for db in adj]
    sw = als[A]._impl.sweep(names, True)
    sw.run()
    sw.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        sw.run()
    sw.sync()
    dt = (time.perf_counter() - t0) / reps
    dev, ph = [], []
    for _ in range(5):
        sw.run()
        dev.append(sw.last_ms())
        ph.append(sw.phase_ms())
    kms = statistics.median(dev)
    N, E, W = sw.nodes, sw.edges, sw.words
    b_src = 4 * (N + 1) + 8 * E + N * (4 + 4 * W)
    gbs = b_src * len(names) / (kms * 1e-3) / 1e9
    info = sw.info()
    out = {"workload": f"C2w {N}-node grid, link metrics uniform in [1, {C2W_MAX_METRIC}] (E={E})",
           "sweep_spf_sources_per_s": round(len(names) / dt, 1),
           "sweep_ms": round(dt * 1e3, 3),
           "kernel_ms": round(kms, 3),
           "phase_ms": {"distances": round(statistics.median(p[0] for p in ph), 3),
                        "first_hops": round(statistics.median(p[1] for p in ph), 3)},
           "plan": {"variant": info["variant"], "rows": info["rows"]},
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                        "frac": round(gbs / 8000.0, 4), "algorithmic_bytes_per_source": b_src,
                        "sources_per_launch": len(names)}}
    if cpu:
        o = _oracle()
        als_o, _ = load_topology(o, adj, pfx)
        sample = names[::max(1, len(names) // 128)]
        sec, _ = als_o[A]._impl.time_spf_sources(sample, 1)
        out["cpu_sweep_spf_sources_per_s"] = round(len(sample) / sec, 2)
        out["cpu_sample"] = f"{len(sample)} runSpf calls (evenly spaced sources), 1 thread"
    return out


def leg_c3(hip, cpu):
    from openr_amd.facade import load_topology
    from openr_amd.types import K_TESTING_AREA as A
    from openr_amd.workloads import c3_fabric
    adj, pfx = c3_fabric()
    als, ps = load_topology(hip, adj, pfx)
    names = [db.thisNodeName for db in adj]
    sweep = als[A]._impl.sweep(names, True)
    sweep.run()
    sweep.sync()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        sweep.run()
    sweep.sync()
    dt = (time.perf_counter() - t0) / reps
    me = "2-0-0"
    out = {"workload": f"C3 Clos N={len(names)} E={sweep.edges}, {len(pfx)} prefix advertisements",
           "sweep_spf_sources_per_s": round(len(names) / dt, 1),
           "sweep_ms": round(dt * 1e3, 4),
           "build_route_db_best_route_ms": round(_route_ms(
               hip.spf_solver(me, True, enable_best_route_selection=True), me, als, ps, 5), 3)}
    c3_ms, out["build_route_db_runs"] = _route_runs(hip.spf_solver(me, True), me, als, ps, 7)
    out["build_route_db_ms"] = round(statistics.median(c3_ms), 3)
    out.update(_select_roofline(hip.spf_solver(me, True, enable_best_route_selection=True),
                                me, als, ps))
    # prefix-sharded build (route selection sharded over 8
    # GPUs): ShardedRouteBuilder on 8 device contexts (on this one-GPU box,
    # contexts of device 0). Each shard built alone is the per-GPU time of an
    # 8-GPU node; the concurrent library build (every shard on its own
    # thread, unicast maps spliced into one DecisionRouteDb) is timed too
    ras = hip.module.ReplicatedAreaLinkStates([0] * 8)
    for db in adj:
        ras.update_adjacency_database(db.to_wire())
    sb = ras.route_builder(me, True)
    sb.time_build_route_db(me, ps._impl)  # warm: mirrors, rows, selection buffers
    shard_ms = [statistics.median(sb.time_build_shard(r, me, ps._impl)[0] * 1e3 for _ in range(5))
                for r in range(8)]
    whole = [sb.time_build_route_db(me, ps._impl) for _ in range(5)]
    out["build_route_db_8_prefix_shards_max_ms"] = round(max(shard_ms), 3)
    out["build_route_db_8_prefix_shards_ms"] = [round(x, 3) for x in shard_ms]
    out["build_route_db_8_prefix_shards_frac_of_whole"] = round(max(shard_ms) / out["build_route_db_ms"], 3)
    out["sharded_builder_merged_ms"] = round(statistics.median(w[0] for w in whole) * 1e3, 3)
    out["sharded_builder_merge_ms"] = round(statistics.median(w[3] for w in whole), 3)
    out["build_route_db_8_prefix_shards_note"] = (
        "ShardedRouteBuilder over 8 contexts: max_ms = slowest shard built alone (the per-GPU time on "
        "8 GPUs); merged_ms = all 8 shards concurrently on this one GPU and its host pool, spliced into "
        "one DecisionRouteDb")
    sb.release_prefix_mirrors(ps._impl)  # the 7 extra contexts' copies of the prefix mirror
    del sb, ras
    if cpu:
        o = _oracle()
        als_o, ps_o = load_topology(o, adj, pfx)
        sample = names[::max(1, len(names) // 64)]
        sec, _ = als_o[A]._impl.time_spf_sources(sample, 1)
        out["cpu_sweep_spf_sources_per_s"] = round(len(sample) / sec, 2)
        out["cpu_sample"] = f"{len(sample)} runSpf calls, 1 thread"
        out["cpu_build_route_db_ms"] = round(_route_ms(o.spf_solver(me, True), me, als_o, ps_o, 1), 2)
    return out


def leg_c4(hip, cpu, reps=3, chunk=None):
    """C4 at BASELINE.md's shape: 4,096 links x 64 sources = 262,144
    runSpf(src, true, {link}) as one what-if job (64 plain searches, then the
    requests in chunks of C4_WHATIF_CHUNK into one device row buffer: every request's
    full dist + first-hop row is written to HBM, chunk after chunk), and 1,024
    KSP2 (src, dst) pairs."""
    from openr_amd.facade import load_topology
    from openr_amd.types import K_TESTING_AREA as A
    from openr_amd.workloads import (C4_KSP2_PAIRS, C4_SEED, C4_WHATIF_CHUNK, c4_ksp2_pairs, c4_wan,
                                     c4_what_if_job)
    adj, _ = c4_wan()
    als, _ = load_topology(hip, adj, [])
    ls = als[A]._impl
    names = ls.node_names()
    links = ls.link_ids()
    srcs, idx, sets = c4_what_if_job([lid for lid, _ in links], names)
    chunk = chunk or C4_WHATIF_CHUNK
    batch = ls.what_if_batch(srcs, idx, sets, chunk)
    batch.run()
    batch.sync()
    walls, devs = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        batch.run()
        batch.sync()
        walls.append(time.perf_counter() - t0)
        devs.append(batch.last_ms())
    dt, dev_ms = statistics.median(walls), statistics.median(devs)
    info = batch.info()
    n_req = len(idx)
    n_nodes, n_edges = batch.nodes, batch.edges
    # per what-if SPF the same B_spf as a plain source
    b_spf = 4 * (n_nodes + 1) + 8 * n_edges + n_nodes * (4 + 4)
    out_bytes = n_req * n_nodes * 8  # the rows alone (the output floor)
    tiers = {int(t): int((info & 7 == t).sum()) for t in range(5)}
    aff = info >> 3
    # the same job with ORH_WHATIF_SHARE_BASE: a source-row request's row is
    # the job's base row (referenced, not copied); only repaired rows land
    # in the row buffer
    del batch
    shared = ls.what_if_batch(srcs, idx, sets, chunk, share_base=True)
    shared.run()
    shared.sync()
    s_walls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        shared.run()
        shared.sync()
        s_walls.append(time.perf_counter() - t0)
    s_dt = statistics.median(s_walls)
    del shared
    kp = c4_ksp2_pairs(names, C4_KSP2_PAIRS)
    ls.prefetch_kth_paths(c4_ksp2_pairs(names, 64, seed=C4_SEED + 99))  # warm-up pairs (not memoized for kp)
    # LinkState::prefetchKthPaths timed in C++ around the call (the pairs
    # converted from Python beforehand), cold each time (memo dropped as a
    # topology change drops it); median of 3
    ksp_walls = ls.time_prefetch_kth_paths(kp, 3)
    kdt = statistics.median(ksp_walls)
    out = {"workload": f"C4 WAN N={len(names)} E={n_edges}, log-normal metrics",
           # copy-on-write is the job mode for a caller that reads the tiers
           # (a tier-0 request's row IS its source's base row); the dense
           # mode, every row copied out, is kept beside it
           "what_if_spfs_per_s": round(n_req / s_dt, 1),
           "what_if_mode": "copy-on-write (ORH_WHATIF_SHARE_BASE); dense below",
           "what_if_dense_spfs_per_s": round(n_req / dt, 1),
           "what_if_batch": (f"{n_req} runSpf(src, true, {{link}}) = {len(sets) // len(srcs)} links x "
                             f"{len(srcs)} sources: one what-if job (the sources' plain searches + "
                             f"{(n_req + chunk - 1) // chunk} chunks of {chunk:,} requests into one device row buffer)"),
           "what_if_batch_ms": round(dt * 1e3, 3),
           "what_if_device_ms": round(dev_ms, 3),
           "what_if_tiers": {"source_row": tiers[0], "lds_small": tiers[1], "lds_large": tiers[2],
                             "global_slot": tiers[3], "full_search": tiers[4]},
           "what_if_affected_nodes": {"mean": round(float(aff.mean()), 2), "max": int(aff.max())},
           # the rows are the floor: 8 B/node/request must reach HBM whatever
           # the plan; B_spf per request credits work the
           # repair plan skips, so it is reported as an equivalent only
           "what_if_roofline": {"bound": "hbm", "bytes": out_bytes,
                                "achieved_gbs": round(out_bytes / (dev_ms * 1e-3) / 1e9, 1),
                                "frac": round(out_bytes / (dev_ms * 1e-3) / 1e9 / 8000.0, 4),
                                "b_spf_equivalent": {"bytes_per_spf": b_spf,
                                                     "gbs": round(n_req * b_spf / (dev_ms * 1e-3) / 1e9, 1)}},
           "what_if_shared_base": {"what_if_spfs_per_s": round(n_req / s_dt, 1),
                                   "batch_ms": round(s_dt * 1e3, 3),
                                   "rows_written": n_req - tiers[0],
                                   "note": "ORH_WHATIF_SHARE_BASE: the 50 % of requests whose source row stands "
                                           "reference the job's base row instead of a copy (same tiers, rows "
                                           "bit-identical: test_c4_shared_base_rows)"},
           "ksp2_pairs_per_s": round(len(kp) / kdt, 1),
           "ksp2_batch": f"{len(kp)} (src, dst) getKthPaths k=1,2 (prefetchKthPaths)",
           "ksp2_batch_ms": [round(x * 1e3, 3) for x in ksp_walls],
           "ksp2_note": "wall time of the C++ prefetchKthPaths call, cold (memo dropped), median of 3"}
    if cpu:
        o = _oracle()
        als_o, _ = load_topology(o, adj, [])
        k = 8
        threads = min(k, os.cpu_count() or 1)
        desc = dict(links)
        pick = [i * (n_req // k) for i in range(k)]
        q = [srcs[idx[i]] for i in pick]
        t0 = time.perf_counter()
        als_o[A]._impl.spf_tables(q, names, [ls.neighbors(s) for s in q], threads,
                                  [[desc[sets[i][0]][:3]] for i in pick])
        sec = time.perf_counter() - t0
        out["cpu_spfs_per_s"] = round(k / sec, 4)
        out["cpu_sample"] = (f"{k} what-if runSpf(src, true, {{link}}) of the same batch on {threads} threads "
                             "(reference DijkstraQ re-heap), per-thread LinkState copies")
        # KSP2 on the CPU: the oracle's getKthPaths k = 1, 2 (two fresh SPFs
        # and the traces per pair) on `threads` threads, a sample of the pairs
        kq = kp[::max(1, len(kp) // 8)][:8]
        t0 = time.perf_counter()
        als_o[A]._impl.kth_paths_threaded(kq, threads, [db.thisNodeName for db in adj])
        ksec = time.perf_counter() - t0
        out["cpu_ksp2_pairs_per_s"] = round(len(kq) / ksec, 4)
        out["cpu_ksp2_sample"] = (f"{len(kq)} of the benched pairs, getKthPaths k = 1, 2 on {threads} threads "
                                  "(per-thread LinkState copies, their load included)")
    return out


def leg_c5(hip, cpu):
    from openr_amd.facade import load_topology
    from openr_amd.rib_policy import RibPolicy, RibPolicyStatement, RibRouteActionWeight
    from openr_amd.workloads import C5_AREAS, C5_TAG, c5_multi_area
    areas, pfx = c5_multi_area()
    adj = [db for a in C5_AREAS for db in areas[a]]
    # load = the product's ingest of the topology and the 1M advertisements
    # (LinkState::updateAdjacencyDatabase, PrefixState::updatePrefix per
    # advertisement, in order); the generator's Python objects are turned
    # into wire records before the clock starts
    adj_wire = [db.to_wire() for db in adj]
    pfx_wire = [(node, area, e.to_wire()) for node, area, e in pfx]
    t0 = time.perf_counter()
    als = hip.area_link_states(*C5_AREAS)
    for db, w in zip(adj, adj_wire):
        als[db.area]._impl.update_adjacency_database(w, 0, 0)
    ps = hip.prefix_state()
    for i in range(0, len(pfx_wire), 1 << 16):
        ps._impl.update_prefixes(pfx_wire[i:i + (1 << 16)])
    load_s = time.perf_counter() - t0
    del adj_wire, pfx_wire
    solver = hip.spf_solver("me", True, enable_best_route_selection=True)
    out = {"workload": f"C5 4 areas x {len(areas['A'])} nodes, {len(pfx)} prefix advertisements",
           "load_s": round(load_s, 2),
           "load_note": "adjacency + 1M prefix advertisements ingested from wire records (updateAdjacencyDatabase / "
                        "updatePrefix in order); the generator's Python-to-wire conversion is not timed",
           "build_route_db_ms": None}
    c5_ms, out["build_route_db_runs"] = _route_runs(solver, "me", als, ps, 5)
    out["build_route_db_ms"] = round(statistics.median(c5_ms), 2)
    out.update(_select_roofline(solver, "me", als, ps))
    policy = RibPolicy([RibPolicyStatement("ucmp", None, [C5_TAG], RibRouteActionWeight(
        0, {"A": 1, "B": 2, "C": 3, "D": 4}, {}))], 3600)
    # Decision::rebuildRoutes over Decision::routeDb_ (DecisionRib,
    # Decision.cpp:1865-1930), RibPolicy applied: the first full rebuild
    # builds everything; the full rebuild after the incremental stress runs as
    # a delta against routeDb_ (device selection compared on the device with
    # the previous snapshot; only changed routes built, policy-applied and
    # compared); calculateUpdate semantics either way
    import random
    from openr_amd.types import PrefixEntry, PrefixMetrics
    rib = hip.module.DecisionRib()
    _, first_s = rib.rebuild_routes(solver._impl, "me", als._impl, ps._impl, True, [], policy._impl, wire=False)
    # incremental stress: 10k prefix add / withdraw
    # advertisements plus 100 adjacency-metric changes, then one full rebuild
    rng = random.Random(55)
    t0 = time.perf_counter()
    changed = set()
    for i in range(10_000):
        node, area, e = pfx[rng.randrange(len(pfx))]
        if i % 2:
            got = ps.delete_prefix(node, area, e.prefix)
        else:
            got = ps.update_prefix(node, area, PrefixEntry(e.prefix, metrics=PrefixMetrics(
                1, rng.randint(0, 3), rng.randint(0, 3), rng.randint(0, 3)), tags=e.tags))
        changed |= {(p.prefixAddress.addr, p.prefixLength) for p in got}
    for _ in range(100):
        a = rng.choice(C5_AREAS)
        db = areas[a][rng.randrange(len(areas[a]) - 1)]
        db.adjacencies[rng.randrange(len(db.adjacencies))].metric = rng.randint(1, 4)
        als[a].update_adjacency_database(db)
    upd_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    (uu, ud, mu, md), reb_s = rib.rebuild_routes(solver._impl, "me", als._impl, ps._impl, True, sorted(changed),
                                                policy._impl, wire=False)
    wall_s = time.perf_counter() - t0
    # the same state built whole (buildRouteDb alone, no policy) for comparison
    whole_s, _ = solver._impl.time_build_route_db("me", als._impl, ps._impl)
    out["incremental"] = {"updates": "10k prefix add/withdraw + 100 adjacency metric changes",
                          "apply_s": round(upd_s, 3),
                          "first_full_rebuild_ms": round(first_s * 1e3, 2),
                          "rebuild_ms": round(reb_s * 1e3, 2),
                          "rebuild_wall_ms": round(wall_s * 1e3, 2),
                          "ran_as": "delta" if rib.delta_rebuilds else "whole build",
                          "routes_updated": uu, "routes_deleted": ud,
                          "mpls_updated": mu, "mpls_deleted": md,
                          "whole_build_route_db_ms": round(whole_s * 1e3, 2),
                          "note": "Decision::rebuildRoutes with RibPolicy: buildRouteDb + applyPolicy + "
                                  "calculateUpdate + routeDb_.update, the delta freed inside"}
    # Decision::rebuildRoutes after prefix-only updates (Decision.cpp:1902-1924):
    # only the updated prefixes are rebuilt (one device selection pass over
    # the prefix mirror + host materialisation of those routes)
    changed = set()
    for i in range(10_000):
        node, area, e = pfx[rng.randrange(len(pfx))]
        if i % 2:
            got = ps.delete_prefix(node, area, e.prefix)
        else:
            got = ps.update_prefix(node, area, PrefixEntry(e.prefix, metrics=PrefixMetrics(
                1, rng.randint(0, 3), rng.randint(0, 3), rng.randint(0, 3)), tags=e.tags))
        changed |= {(p.prefixAddress.addr, p.prefixLength) for p in got}
    (uu, ud, _, _), sec = rib.rebuild_routes(solver._impl, "me", als._impl, ps._impl, False, sorted(changed),
                                            policy._impl, wire=False)
    out["incremental_prefix_only"] = {"updates": "10k prefix add/withdraw, no topology change",
                                      "prefixes_rebuilt": len(changed),
                                      "rebuild_ms": round(sec * 1e3, 2),
                                      "routes_updated": uu, "routes_deleted": ud}
    # buildRouteDb + RibPolicy::applyPolicy (the full rebuild's two steps):
    # the policy decided per route on the device (route_policy_kernel) and
    # its weights set as the routes materialise. rib_policy_ms = the policy's
    # own step (tables + kernel + copy-out); the build's difference with and
    # without the policy (medians of 3, same state) is reported beside it
    runs = [solver._impl.time_build_route_db_with_policy("me", als._impl, ps._impl, policy._impl)
            for _ in range(3)]
    plain_ms = _route_ms(solver, "me", als, ps, 3)
    both_ms = statistics.median(r[0] for r in runs) * 1e3
    _, routes, updated, invalidated, on_device, dev_ms = runs[-1]
    host_s, _ = solver._impl.time_host_apply_policy("me", als._impl, ps._impl, policy._impl)
    out.update({"build_plus_policy_ms": round(both_ms, 2),
                "rib_policy_ms": round(dev_ms, 3),
                "build_policy_delta_ms": round(both_ms - plain_ms, 2),
                "build_route_db_same_state_ms": round(plain_ms, 2),
                "routes": routes, "policy_updated_routes": updated,
                "policy_invalidated": invalidated, "policy_decided_on_device": on_device,
                "host_apply_policy_ms": round(host_s * 1e3, 2),
                "policy_note": "rib_policy_ms = policy tables + route_policy_kernel + copy-out (the "
                               "weights are set as routes materialise, inside the build); "
                               "build_policy_delta_ms = median(build + policy) - median(build) on the same "
                               "state (noise-level, may be negative); host_apply_policy_ms = A/B: RibPolicy::applyPolicy over the "
                               "built map on the host pool"})
    if cpu:
        o = _oracle()
        als_o, ps_o = load_topology(o, adj, pfx)
        so = o.spf_solver("me", True, enable_best_route_selection=True)
        out["cpu_build_route_db_ms"] = round(_route_ms(so, "me", als_o, ps_o, 1), 1)
    return out


LEGS = {"c1": leg_c1, "c2w": leg_c2w, "c3": leg_c3, "c4": leg_c4, "c5": leg_c5}


def run(names, hip, cpu):
    out = {}
    for n in names:
        n = n.strip()
        if not n:
            continue
        t0 = time.perf_counter()
        try:
            out[n] = LEGS[n](hip, cpu)
        except Exception as e:  # a failed leg is reported, not hidden
            out[n] = {"error": f"{type(e).__name__}: {e}"}
        out[n]["leg_wall_s"] = round(time.perf_counter() - t0, 1)
    return out


# ---------------------------------------------------------------------------
# N-rank legs (bench.py --gpus N, N > 1): one process per GPU, rank r runs
# block r of configs[2] (C3 prefix shard) and configs[3] (C4 what-if + KSP2
# blocks) on its own device; bench.py reports the max over ranks. The blocks
# are the library's own cuts: SpfSolver::setPrefixShard (ShardedRouteBuilder),
# equalWorkCuts of the sources by request / pair count (MultiDeviceWhatIf,
# MultiDeviceKthPaths). Every block is independent given the topology: no
# data-path collective.
# ---------------------------------------------------------------------------
def c3_rank_state(hip):
    from openr_amd.facade import load_topology
    from openr_amd.workloads import c3_fabric
    adj, pfx = c3_fabric()
    als, ps = load_topology(hip, adj, pfx)
    return als, ps


def rank_c3(hip, rank, world, state=None, reps=7, digest=False):
    """Prefix block `rank` of `world` of the C3 100k-prefix buildRouteDb
    (Decision.cpp:615-792) on this process's device: the shard's SPF, route
    selection and materialisation (shard 0 adds the MPLS routes)."""
    als, ps = state or c3_rank_state(hip)
    me = "2-0-0"
    solver = hip.spf_solver(me, True)
    solver._impl.set_prefix_shard(rank, world)
    solver._impl.time_build_route_db(me, als._impl, ps._impl)  # warm: mirrors, rows, buffers
    ms, runs = _route_runs(solver, me, als, ps, reps)
    out = {"build_route_db_shard_ms": round(statistics.median(ms), 3), "runs": runs}
    if digest:
        out["digest"] = solver._impl.build_route_db_digest(me, als._impl, ps._impl)
    return out


def c4_rank_state(hip):
    from openr_amd.facade import load_topology
    from openr_amd.types import K_TESTING_AREA as A
    from openr_amd.workloads import C4_KSP2_PAIRS, c4_ksp2_pairs, c4_wan, c4_what_if_job
    adj, _ = c4_wan()
    als, _ = load_topology(hip, adj, [])
    ls = als[A]._impl
    names = ls.node_names()
    srcs, idx, sets = c4_what_if_job([lid for lid, _ in ls.link_ids()], names)
    return als, ls, srcs, idx, sets, c4_ksp2_pairs(names, C4_KSP2_PAIRS)


def c4_what_if_block(srcs, idx, sets, rank, world):
    """Block `rank` of the C4 what-if job cut as MultiDeviceWhatIf cuts it:
    contiguous source blocks of equal request counts. Returns (the caller's
    request indices, the block's sources, per request its source index in the
    block, ignore sets)."""
    from openr_amd.sharding import weighted_blocks
    w = [0.0] * len(srcs)
    for i in idx:
        w[i] += 1.0
    lo, hi = weighted_blocks(w, world)[rank]
    reqs = [i for i, s in enumerate(idx) if lo <= s < hi]
    return reqs, srcs[lo:hi], [idx[i] - lo for i in reqs], [sets[i] for i in reqs]


def c4_ksp2_block(pairs, rank, world):
    """Block `rank` of the KSP2 pairs cut as MultiDeviceKthPaths cuts it: the
    pairs of one source together, sources in first-appearance order cut into
    blocks of equal pair counts. Returns the caller's pair indices."""
    from openr_amd.sharding import weighted_blocks
    order, by_src = [], {}
    for i, (s, _) in enumerate(pairs):
        if s not in by_src:
            by_src[s] = []
            order.append(s)
        by_src[s].append(i)
    lo, hi = weighted_blocks([float(len(by_src[s])) for s in order], world)[rank]
    return [i for s in order[lo:hi] for i in by_src[s]]


SEARCH_LARGE_BLOCKS = 4  # MultiDeviceWhatIf::kSearchLargeBlocks


def rank_c4(hip, rank, world, state=None, reps=3, digest=False):
    """Block `rank` of `world` of the C4 what-if job (copy-on-write, the
    bench's mode) and of the 1,024-pair KSP2 batch (prefetchKthPaths, cold)
    on this process's device."""
    from openr_amd.workloads import C4_WHATIF_CHUNK
    als, ls, srcs, idx, sets, pairs = state or c4_rank_state(hip)
    reqs, bsrcs, bidx, bsets = c4_what_if_block(srcs, idx, sets, rank, world)
    out = {"what_if_requests": len(reqs), "what_if_sources": len(bsrcs)}
    if reqs:
        # the single job's chunking scaled to the block (four chunks of the
        # block: the two row buffers stay 1/world of the single job's)
        chunk = min(C4_WHATIF_CHUNK, max(1024, -(-len(reqs) // 4)))
        # a 4-way or wider split: the block searches its largest repairs in
        # full (MultiDeviceWhatIf's rule, ORH_WHATIF_SEARCH_LARGE)
        job = ls.what_if_batch(bsrcs, bidx, bsets, chunk, share_base=True,
                               search_large=world >= SEARCH_LARGE_BLOCKS)
        if digest:
            job.set_digests()
        job.run()
        job.sync()
        walls = []
        for _ in range(reps):
            t0 = time.perf_counter()
            job.run()
            job.sync()
            walls.append(time.perf_counter() - t0)
        out["what_if_block_ms"] = round(statistics.median(walls) * 1e3, 3)
        if digest:
            out["what_if_reqs"] = reqs
            out["what_if_info"] = job.info()
            out["what_if_digests"] = job.digests()
        job.release()
        del job
    else:
        out["what_if_block_ms"] = 0.0
    kp = c4_ksp2_block(pairs, rank, world)
    out["ksp2_pairs"] = len(kp)
    if kp:
        bp = [pairs[i] for i in kp]
        walls = ls.time_prefetch_kth_paths(bp, reps)
        out["ksp2_block_ms"] = round(statistics.median(walls) * 1e3, 3)
        if digest:
            out["ksp2_idx"] = kp
            out["ksp2_paths"] = [(ls.get_kth_path_ids(s, d, 1), ls.get_kth_path_ids(s, d, 2)) for s, d in bp]
    else:
        out["ksp2_block_ms"] = 0.0
    return out


def run_ranks(names, hip, rank, world):
    """This rank's block of every N-rank leg (bench.py gathers them)."""
    out = {}
    for n in names:
        n = n.strip()
        t0 = time.perf_counter()
        try:
            if n == "c3":
                out[n] = rank_c3(hip, rank, world)
            elif n == "c4":
                out[n] = rank_c4(hip, rank, world)
            else:
                continue
        except Exception as e:  # a failed leg is reported, not hidden
            out[n] = {"error": f"{type(e).__name__}: {e}"}
        out[n]["leg_wall_s"] = round(time.perf_counter() - t0, 1)
    return out


def merge_ranks(per_rank, world):
    """Rank 0's report of the N-rank legs: per leg the max over ranks (the
    per-GPU time of an N-GPU node) and every rank's own numbers."""
    out = {}
    for leg in sorted({k for r in per_rank for k in r}):
        rows = [r.get(leg, {}) for r in per_rank]
        err = [r["error"] for r in rows if "error" in r]
        if err:
            out[leg] = {"error": err[0]}
            continue
        if leg == "c3":
            ms = [r["build_route_db_shard_ms"] for r in rows]
            out[leg] = {"workload": f"C3 100k-prefix buildRouteDb, prefix block r of {world} on GPU r",
                        "build_route_db_max_ms": max(ms), "build_route_db_ms_by_rank": ms}
        elif leg == "c4":
            wi = [r["what_if_block_ms"] for r in rows]
            kp = [r["ksp2_block_ms"] for r in rows]
            n_req = sum(r["what_if_requests"] for r in rows)
            n_kp = sum(r["ksp2_pairs"] for r in rows)
            out[leg] = {"workload": f"C4 what-if job ({n_req} requests) and KSP2 ({n_kp} pairs), "
                                    f"source block r of {world} on GPU r",
                        "what_if_max_ms": max(wi), "what_if_ms_by_rank": wi,
                        "what_if_spfs_per_s": round(n_req / (max(wi) * 1e-3), 1) if max(wi) else None,
                        "ksp2_max_ms": max(kp), "ksp2_ms_by_rank": kp,
                        "ksp2_pairs_per_s": round(n_kp / (max(kp) * 1e-3), 1) if max(kp) else None}
        out[leg]["leg_wall_s_by_rank"] = [r.get("leg_wall_s") for r in rows]
    return out
