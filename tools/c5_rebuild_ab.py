"""C5 (1M prefixes, 4 areas, best-route, the UCMP RibPolicy) first
Decision::rebuildRoutes (build + policy + calculateUpdate against an empty
routeDb_) and buildRouteDb alone, under env A/B specs, each spec in its own
child process, alternating, twice:
  python tools/c5_rebuild_ab.py "ORH_NH_LOCAL=1" "ORH_NH_LOCAL=0"
Per child: the ingest time, medians of 5 builds and of 5 first rebuilds
(a fresh DecisionRib each)."""
import os
import statistics
import subprocess
import sys
import time

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from openr_amd import host_backend
    from openr_amd.rib_policy import RibPolicy, RibPolicyStatement, RibRouteActionWeight
    from openr_amd.workloads import C5_AREAS, C5_TAG, c5_multi_area
    hip = host_backend()
    areas, pfx = c5_multi_area()
    adj = [db for a in C5_AREAS for db in areas[a]]
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
    solver = hip.spf_solver("me", True, enable_best_route_selection=True)
    policy = RibPolicy([RibPolicyStatement("ucmp", None, [C5_TAG], RibRouteActionWeight(
        0, {"A": 1, "B": 2, "C": 3, "D": 4}, {}))], 3600)
    build = [solver._impl.time_build_route_db("me", als._impl, ps._impl)[0] * 1e3 for _ in range(6)][1:]
    first = []
    for _ in range(5):
        rib = hip.module.DecisionRib()
        _, s = rib.rebuild_routes(solver._impl, "me", als._impl, ps._impl, True, [], policy._impl, wire=False)
        first.append(s * 1e3)
        del rib
    host_s, _ = solver._impl.time_host_apply_policy("me", als._impl, ps._impl, policy._impl)
    print(f"load {load_s:.2f} s | build ms {[round(x, 1) for x in build]} median {statistics.median(build):.1f} | "
          f"first rebuild ms {[round(x, 1) for x in first]} median {statistics.median(first):.1f} | "
          f"host applyPolicy {host_s * 1e3:.1f} ms", flush=True)
    sys.exit(0)
for rep in range(2):
    for spec in sys.argv[1:]:
        env = dict(os.environ)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                           timeout=500)
        print(f"[{spec}] {r.stdout.strip()} {r.stderr.strip()[-300:] if r.returncode else ''}", flush=True)
